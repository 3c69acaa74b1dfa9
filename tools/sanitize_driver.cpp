// sanitize_driver.cpp -- host-side driver for the sanitizer builds (`make
// sanitize`, triangles-sdf-cpu-raytracing_amd/Makefile). Not product code.
//
// Exercises the multi-threaded host code of librtamd -- the OpenMP-task BVH8
// builder (rt_host.cpp: replicated introsort with task-parallel partitions,
// concurrent SAH axes, task-built children; the reference's
// triangles_raytracing.cpp:182-244), the loaders and the mesh operations
// (rt_meshops.cpp) -- under ThreadSanitizer (clang + libomp + archer) or
// AddressSanitizer/UBSan (gcc), and checks that every build of a mesh gives
// the same canonical tree at 1 thread and at N threads.
//
// usage: sanitize_driver DATA_DIR [threads]
#include <omp.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "../triangles-sdf-cpu-raytracing_amd/csrc/rt_bvhstage.h"
#include "../triangles-sdf-cpu-raytracing_amd/csrc/rt_host.h"

namespace {

int g_fail = 0;

void check(bool ok, const std::string &what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    ++g_fail;
  }
}

bool same_build(const char *name, const std::vector<float> &v, const std::vector<uint32_t> &idx, int threads) {
  rth::BVHGpu a, b;
  std::string err;
  omp_set_num_threads(1);
  if (!rth::build_bvh8(v.data(), (int64_t)v.size() / 4, idx.data(), (int64_t)idx.size(), a, err)) {
    check(false, std::string(name) + ": 1-thread build: " + err);
    return false;
  }
  omp_set_num_threads(threads);
  if (!rth::build_bvh8(v.data(), (int64_t)v.size() / 4, idx.data(), (int64_t)idx.size(), b, err)) {
    check(false, std::string(name) + ": parallel build: " + err);
    return false;
  }
  const bool same = a.canon == b.canon && a.perm_tri == b.perm_tri && a.max_depth == b.max_depth;
  check(same, std::string(name) + ": tree differs between 1 and " + std::to_string(threads) + " threads");
  // the device builder's stage loop (rt_bvhstage.cpp, parallel passes) with
  // its device steps emulated on the host
  rth::BVHGpu e;
  const bool emu = rth::bvhs::emulate_device_build(v.data(), (int64_t)v.size() / 4, idx.data(),
                                                   (int64_t)idx.size(), e, err) &&
                   e.canon == b.canon && e.perm_tri == b.perm_tri;
  check(emu, std::string(name) + ": emulated device stage loop differs: " + err);
  std::printf("%-28s %8zu tris  %7lld nodes  depth %d  %s%s\n", name, idx.size() / 3, (long long)b.host_nodes,
              b.max_depth, same ? "same tree at 1 and N threads" : "DIFFERENT",
              emu ? ", and from the device stage loop" : ", STAGE LOOP DIFFERS");
  return same && emu;
}

// test_host.py's tie-heavy meshes: duplicate triangles, integer lattices, flat
std::vector<float> synth(const char *mode, int ntri, unsigned seed) {
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.0f, 1.0f);
  std::uniform_int_distribution<int> ud(0, 5);
  std::vector<float> v;
  v.reserve((size_t)ntri * 12);
  float base[9];
  for (float &x : base) x = nd(rng);
  for (int t = 0; t < ntri; ++t) {
    float p[9];
    if (std::string(mode) == "same") {
      for (int k = 0; k < 9; ++k) p[k] = base[k];
    } else if (std::string(mode) == "grid") {
      const float g[3] = {(float)ud(rng), (float)ud(rng), (float)ud(rng)};
      const float off[9] = {0, 0, 0, 1, 0, 0, 0, 1, 0};
      for (int k = 0; k < 9; ++k) p[k] = g[k % 3] + off[k];
    } else {
      const float c[3] = {nd(rng), nd(rng), nd(rng)};
      for (int k = 0; k < 9; ++k) p[k] = c[k % 3] + 0.05f * nd(rng);
    }
    for (int k = 0; k < 3; ++k) {
      v.push_back(p[3 * k]);
      v.push_back(p[3 * k + 1]);
      v.push_back(p[3 * k + 2]);
      v.push_back(1.0f);
    }
  }
  return v;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s DATA_DIR [threads]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
  std::string err;
  for (const char *f : {"cube.obj", "spot.obj", "stanford-bunny.obj"}) {
    rth::Mesh m;
    if (!rth::load_obj((dir + "/" + f).c_str(), true, m, err)) {
      check(false, std::string(f) + ": " + err);
      continue;
    }
    same_build(f, m.vpos4, m.idx, threads);
    if (std::string(f) == "stanford-bunny.obj") {  // the config-5 stand-in's subdivision, one level
      rth::Mesh sub;
      check(rth::subdivide_mesh(m.vpos4.data(), (int64_t)m.vpos4.size() / 4, m.idx.data(), (int64_t)m.idx.size(), 1,
                                sub, err),
            "subdivide: " + err);
      same_build("stanford-bunny subdivided", sub.vpos4, sub.idx, threads);
    }
  }
  for (auto [mode, n, seed] : {std::tuple{"same", 12000, 10u}, std::tuple{"grid", 30000, 9u},
                               std::tuple{"rand", 40000, 11u}}) {
    std::vector<float> v = synth(mode, n, seed);
    std::vector<uint32_t> idx(v.size() / 4);
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (uint32_t)i;
    same_build((std::string("synthetic ") + mode).c_str(), v, idx, threads);
  }
  uint32_t size[3];
  std::vector<float> vals;
  check(rth::load_grid((dir + "/example_grid.grid").c_str(), size, vals, err), "grid: " + err);
  std::vector<uint8_t> nodes;
  check(rth::load_octree((dir + "/sdf_6.octree").c_str(), nodes, err), "octree: " + err);
  rth::OctGpu og;
  check(rth::flatten_octree(nodes.data(), (int64_t)nodes.size() / 36, og, err), "flatten: " + err);
  std::printf("loaders: grid %ux%ux%u, octree %zu nodes\n", size[0], size[1], size[2], nodes.size() / 36);
  std::printf("%s\n", g_fail ? "SANITIZE DRIVER FAILED" : "sanitize driver ok");
  return g_fail ? 1 : 0;
}
