// rt_render -- headless C++ driver of the render loop in src/main.cpp:170-206,
// written against include/rtamd.hpp only (the C++ surface a reference user
// switches to). Loads a .obj / .grid / .octree the way main.cpp does (mesh:
// LoadMeshFromObj + loadAndScale, ground plane at the model's bbox min y;
// SDFs: plane at y = -1), renders `frames` frames with FrameBuffer::clear()
// before each, and prints one JSON line with the FNV-1a-64 of the last colour
// buffer (word-wise, as SURVEY.md 8(c)'s golden hashes), its coverage and the
// mean kernel milliseconds. --ppm writes the last frame.
//
//   rt_render <input> [--size W H] [--pos x y z] [--mode normal|lambert|color]
//             [--plane 0|1] [--shadows 0|1] [--reflections 0|1] [--frames N]
//             [--ppm out.ppm] [--png out.png] [--drag dx dy] [--zoom notches]
//             [--save-obj out.obj]   (the loaded, scaled mesh via SaveMeshToObj)
//             [--devices d0,d1,...] [--band-rows R]  (one process, several GPUs:
//                                     Renderer::devices, rt_multi_*)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "rtamd.hpp"

namespace {

bool ends_with(const std::string &s, const char *suf) {
  const size_t n = std::strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

void write_ppm(const char *path, const rtamd::FrameBuffer &fb) {
  FILE *f = std::fopen(path, "wb");
  if (!f) throw std::runtime_error(std::string("cannot write ") + path);
  std::fprintf(f, "P6\n%u %u\n255\n", fb.width(), fb.height());
  for (uint32_t c : fb.color) {
    const unsigned char rgb[3] = {(unsigned char)(c & 0xFF), (unsigned char)((c >> 8) & 0xFF),
                                  (unsigned char)((c >> 16) & 0xFF)};
    std::fwrite(rgb, 1, 3, f);
  }
  std::fclose(f);
}

int usage() {
  std::fprintf(stderr,
               "usage: rt_render <input.obj|.grid|.octree> [--size W H] [--pos x y z]\n"
               "       [--mode normal|lambert|color] [--plane 0|1] [--shadows 0|1]\n"
               "       [--reflections 0|1] [--frames N] [--ppm out.ppm] [--png out.png]\n"
               "       [--drag dx dy] [--zoom notches] [--save-obj out.obj]\n"
               "       [--devices d0,d1,...] [--band-rows R]\n");
  return 2;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) return usage();
  const std::string input = argv[1];
  uint32_t W = 1920, H = 1080;
  rtamd::float3 pos{0.0f, 0.0f, 2.5f};  // main.cpp:89-91
  rtamd::Renderer renderer;             // light (2,2,2), shadows + reflections on
  renderer.shadingMode = rtamd::ShadingMode::Lambert;
  bool plane = true;
  int frames = 1;
  const char *ppm = nullptr, *png = nullptr, *save_obj = nullptr;
  float drag_dx = 0.0f, drag_dy = 0.0f, zoom = 0.0f;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    auto need = [&](int k) {
      if (i + k >= argc) throw std::runtime_error("missing value for " + a);
    };
    if (a == "--size") {
      need(2);
      W = (uint32_t)std::atoi(argv[++i]);
      H = (uint32_t)std::atoi(argv[++i]);
    } else if (a == "--pos") {
      need(3);
      pos.x = std::strtof(argv[++i], nullptr);
      pos.y = std::strtof(argv[++i], nullptr);
      pos.z = std::strtof(argv[++i], nullptr);
    } else if (a == "--mode") {
      need(1);
      const std::string m = argv[++i];
      renderer.shadingMode = m == "normal"    ? rtamd::ShadingMode::Normal
                             : m == "color"   ? rtamd::ShadingMode::Color
                                              : rtamd::ShadingMode::Lambert;
    } else if (a == "--plane") {
      need(1);
      plane = std::atoi(argv[++i]) != 0;
    } else if (a == "--shadows") {
      need(1);
      renderer.enableShadows = std::atoi(argv[++i]) != 0;
    } else if (a == "--reflections") {
      need(1);
      renderer.enableReflections = std::atoi(argv[++i]) != 0;
    } else if (a == "--frames") {
      need(1);
      frames = std::max(1, std::atoi(argv[++i]));
    } else if (a == "--ppm") {
      need(1);
      ppm = argv[++i];
    } else if (a == "--png") {
      need(1);
      png = argv[++i];
    } else if (a == "--save-obj") {
      need(1);
      save_obj = argv[++i];
    } else if (a == "--drag") {  // a mouse drag in the viewer: Camera::rotate(-dx, -dy)
      need(2);
      drag_dx = std::strtof(argv[++i], nullptr);
      drag_dy = std::strtof(argv[++i], nullptr);
    } else if (a == "--zoom") {  // mouse-wheel notches
      need(1);
      zoom = std::strtof(argv[++i], nullptr);
    } else if (a == "--devices") {  // e.g. 0,1,2,3 (a device may repeat: 0,0)
      need(1);
      renderer.devices.clear();
      for (const char *q = argv[++i]; *q;) {
        char *end = nullptr;
        renderer.devices.push_back((int32_t)std::strtol(q, &end, 10));
        if (end == q) return usage();
        q = *end == ',' ? end + 1 : end;
      }
    } else if (a == "--band-rows") {
      need(1);
      renderer.bandRows = std::atoi(argv[++i]);
    } else {
      return usage();
    }
  }
  if (W == 0 || H == 0) return usage();

  try {
    if (!renderer.devices.empty()) rtamd::check(rt_set_device(renderer.devices[0]));  // the scene lives on devices[0]
    std::unique_ptr<rtamd::IScene> scene;
    float planeY = -1.0f;  // SDF model box is [-1,1]^3 (main.cpp:176-184)
    if (ends_with(input, ".obj")) {
      const rtamd::SimpleMesh mesh = rtamd::LoadMeshFromObj(input, true);
      float ymin = INFINITY;
      for (size_t v = 0; v < mesh.vPos4f.size(); v += 4) ymin = std::min(ymin, mesh.vPos4f[v + 1]);
      planeY = ymin;
      if (save_obj) rtamd::SaveMeshToObj(save_obj, mesh);
      auto b = std::make_unique<rtamd::BVHBuilder>();
      b->perform(mesh);
      scene = std::move(b);
    } else if (ends_with(input, ".grid")) {
      auto g = std::make_unique<rtamd::SDFGrid>();
      rtamd::loadSDFGrid(*g, input);
      scene = std::move(g);
    } else if (ends_with(input, ".octree")) {
      auto o = std::make_unique<rtamd::SDFOctree>();
      rtamd::loadSDFOctree(*o, input);
      scene = std::move(o);
    } else {
      return usage();
    }

    rtamd::FrameBuffer fb;
    fb.resize(W, H);
    rtamd::Camera camera(pos, {0.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f});
    if (drag_dx != 0.0f || drag_dy != 0.0f) camera.rotate(-drag_dx, -drag_dy);
    if (zoom != 0.0f) camera.zoom(zoom);
    const rtamd::float4x4 projInv = rtamd::projInverse(45.0f, (float)W / (float)H, 0.01f, 100.0f);
    const rtamd::SceneUnion full(*scene, rtamd::Plane{{0.0f, 1.0f, 0.0f}, planeY});
    double total_ms = 0.0;
    for (int f = 0; f < frames; ++f) {
      fb.clear();
      total_ms += plane ? renderer.draw(full, fb, camera, projInv) : renderer.draw(*scene, fb, camera, projInv);
    }

    uint64_t h = 1469598103934665603ull;
    int64_t covered = 0;
    for (size_t i = 0; i < fb.color.size(); ++i) {
      h = (h ^ (uint64_t)fb.color[i]) * 1099511628211ull;
      covered += std::isfinite(fb.t[i]) ? 1 : 0;
    }
    if (ppm) write_ppm(ppm, fb);
    if (png) fb.savePNG(png);
    std::printf(
        "{\"input\": \"%s\", \"width\": %u, \"height\": %u, \"frames\": %d, \"hash\": \"%016llx\", "
        "\"covered\": %lld, \"kernel_ms\": %.4f, \"devices\": %zu}\n",
        input.c_str(), W, H, frames, (unsigned long long)h, (long long)covered, total_ms / frames,
        std::max<size_t>(renderer.devices.size(), 1));
    return 0;
  } catch (const std::exception &e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
}
