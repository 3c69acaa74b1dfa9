// rtamd.hpp -- header-only C++ mirror of the reference's render surface over
// the C ABI in rtamd.h. A user of iMacsimus/Triangles-SDF-CPU-RayTracing can
// keep the shape of their code:
//
//   reference (src/...)                            here (namespace rtamd)
//   --------------------------------------------   ------------------------------------
//   cmesh4::LoadMeshFromObj + loadAndScale          LoadMeshFromObj(path, /*scale=*/true)
//   cmesh4::SaveMeshToObj(path, mesh)               SaveMeshToObj(path, mesh)
//   BVHBuilder b; b.perform(std::move(mesh));       BVHBuilder b; b.perform(mesh);
//   SDFGrid g; loadSDFGrid(g, path);                SDFGrid g; loadSDFGrid(g, path);
//   SDFOctree o; loadSDFOctree(o, path);            SDFOctree o; loadSDFOctree(o, path);
//   Plane(float3{0,1,0}, y)                         Plane{{0,1,0}, y}
//   SceneUnion(scene, plane)                        SceneUnion(scene, plane)
//   Camera(pos, target, up)                         Camera(pos, target, up)
//   FrameBuffer fb; fb.resize(W,H); fb.clear();     FrameBuffer fb; fb.resize(W,H); fb.clear();
//   inverse4x4(perspectiveMatrix(45, W/H, .01,100)) projInverse(45, W/H, .01, 100)
//   renderer.draw(scene, fb, camera, projInv)       renderer.draw(scene, fb, camera, projInv)
//   IScene::intersect(o, d, tNear, tFar)            scene.intersect(o, d, tNear, tFar)
//
// (raytracing.hpp:9-213, triangles_raytracing.hpp:38-67, grid_raytracing.hpp,
// octree_raytracing.hpp, camera.hpp, main.cpp:198-206.) Everything runs on the
// current HIP device through librtamd.so; errors throw rtamd::Error.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rtamd.h"

namespace rtamd {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
inline void check(int rc) {
  if (rc != RT_OK) throw Error(rc, std::string("rtamd: ") + rt_last_error());
}

struct float3 {
  float x = 0, y = 0, z = 0;
};
using float4x4 = std::array<float, 16>;  // column-major, LiteMath m_col layout

enum class ShadingMode { Normal = RT_SHADING_NORMAL, Lambert = RT_SHADING_LAMBERT, Color = RT_SHADING_COLOR };

// HitInfo (raytracing.hpp:67-73) + this build's primitive id.
struct HitInfo {
  bool hitten = false;
  float t = 0.0f;
  float3 normal{0.0f, 1.0f, 0.0f};
  int64_t prim = -1;
};

struct SimpleMesh {  // cmesh4::SimpleMesh positions + indices (core/mesh.h:15-55)
  std::vector<float> vPos4f;      // 4 floats per vertex
  std::vector<uint32_t> indices;  // 3 per triangle
  size_t TrianglesNum() const { return indices.size() / 3; }
};

inline SimpleMesh LoadMeshFromObj(const std::string &path, bool scale = true) {
  int64_t nv = 0, ni = 0;
  check(rt_load_obj(path.c_str(), scale ? 1 : 0, nullptr, &nv, nullptr, &ni));
  SimpleMesh m;
  m.vPos4f.resize((size_t)nv * 4);
  m.indices.resize((size_t)ni);
  check(rt_load_obj(path.c_str(), scale ? 1 : 0, m.vPos4f.data(), &nv, m.indices.data(), &ni));
  return m;
}

// cmesh4::SaveMeshToObj (core/mesh.cpp:14-63); normals / texcoords default as fix_missing.
inline void SaveMeshToObj(const std::string &path, const SimpleMesh &m) {
  check(rt_save_obj(path.c_str(), m.vPos4f.data(), (int64_t)(m.vPos4f.size() / 4), m.indices.data(),
                    (int64_t)m.indices.size(), nullptr, nullptr));
}

// FrameBuffer {Image2D<uint32_t> color; Image2D<float> t;} (raytracing.hpp:9-20)
struct FrameBuffer {
  std::vector<uint32_t> color;
  std::vector<float> t;
  uint32_t w = 0, h = 0;
  // true while the buffers hold clear()'s values (set by clear() / resize(),
  // reset by Renderer::draw): draw then tells the library so (RT_FLAG_CLEAR |
  // RT_FLAG_HITS_ONLY) -- the same image as the tPrev draw over a cleared
  // frame, with nothing uploaded. A caller that writes color / t directly
  // after clear() sets it to false.
  bool cleared = false;
  void resize(uint32_t width, uint32_t height) {
    w = width;
    h = height;
    color.assign((size_t)w * h, 0u);
    t.assign((size_t)w * h, std::numeric_limits<float>::infinity());
    cleared = true;
  }
  void clear() {
    std::fill(color.begin(), color.end(), 0u);
    std::fill(t.begin(), t.end(), std::numeric_limits<float>::infinity());
    cleared = true;
  }
  uint32_t width() const { return w; }
  uint32_t height() const { return h; }
  // the colour buffer as an 8-bit RGBA PNG
  void savePNG(const std::string &path) const {
    check(rt_write_png(path.c_str(), color.data(), (int32_t)w, (int32_t)h));
  }
};

// Camera (camera.hpp:7-61, camera.cpp:1-72): the viewer's orbit camera over
// rt_camera_state -- the reference's quaternion math, bit for bit.
class Camera {
 public:
  Camera() : Camera(float3{0.0f, 0.0f, 2.5f}, float3{}) {}
  Camera(float3 position, float3 target, float3 up = {0.0f, 1.0f, 0.0f}) {
    check(rt_camera_init(&position.x, &target.x, &up.x, &s_));
  }
  float3 position() const { return {s_.position[0], s_.position[1], s_.position[2]}; }
  float3 target() const { return {s_.target[0], s_.target[1], s_.target[2]}; }
  float3 up() const { float3 u, r, f; basis(u, r, f); return u; }
  float3 right() const { float3 u, r, f; basis(u, r, f); return r; }
  float3 forward() const { float3 u, r, f; basis(u, r, f); return f; }
  float sensetivity() const { return s_.sensitivity; }  // (sic) camera.hpp:38
  void rotate(float dx, float dy) { check(rt_camera_rotate(&s_, dx, dy)); }
  void resetPosition(float3 p) { check(rt_camera_reset_position(&s_, &p.x)); }
  void resetTarget(float3 t) { check(rt_camera_reset_target(&s_, &t.x)); }
  void setLockUp(bool on) { check(rt_camera_set_lock_up(&s_, on ? 1 : 0)); }
  bool isLockedUp() const { return s_.lock_up != 0; }
  void zoom(float wheel) { check(rt_camera_zoom(&s_, wheel)); }  // the viewer's mouse wheel
  // inverse4x4(lookAtMatrix())
  float4x4 viewInverse() const {
    float4x4 vi{};
    check(rt_camera_view_inverse(&s_, vi.data()));
    return vi;
  }
  const rt_camera_state &state() const { return s_; }

 private:
  void basis(float3 &u, float3 &r, float3 &f) const { check(rt_camera_basis(&s_, &u.x, &r.x, &f.x)); }
  rt_camera_state s_{};
};

// inverse4x4(perspectiveMatrix(fovy, aspect, zNear, zFar)) (main.cpp:198-201)
inline float4x4 projInverse(float fovy, float aspect, float znear, float zfar) {
  float4x4 vi{}, pi{};
  const float p[3] = {0, 0, 1}, t[3] = {0, 0, 0}, u[3] = {0, 1, 0};
  check(rt_camera(p, t, u, fovy, aspect, znear, zfar, vi.data(), pi.data()));
  return pi;
}

struct Plane {  // Plane(normal, offset): dot(p, normal) = offset (raytracing.hpp:121-124)
  float3 normal{0.0f, 1.0f, 0.0f};
  float offset = 0.0f;
};

// A scene resident on the current HIP device (IScene, raytracing.hpp:75-81).
class IScene {
 public:
  IScene() = default;
  IScene(const IScene &) = delete;
  IScene &operator=(const IScene &) = delete;
  virtual ~IScene() = default;

  rt_scene *handle() const {
    if (!h_) throw Error(RT_E_STATE, "rtamd: scene not built");
    return h_.get();
  }
  // Identity of the current device scene: a process-wide counter value taken
  // at every (re)build, so a scene rebuilt at a freed scene's address is
  // never mistaken for the old one (Renderer's multi-GPU handle keys on it).
  uint64_t generation() const { return gen_; }
  // IScene::intersect for one ray (for many rays use intersect(n, ...)).
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const {
    HitInfo r;
    intersect(1, &o.x, &d.x, tNear, tFar, &r);
    return r;
  }
  void intersect(int64_t n, const float *o3, const float *d3, float tNear, float tFar, HitInfo *out) const {
    std::vector<int32_t> hit((size_t)n);
    std::vector<float> t((size_t)n), nrm((size_t)n * 3);
    std::vector<int64_t> prim((size_t)n);
    check(rt_intersect_rays(handle(), o3, d3, n, tNear, tFar, hit.data(), t.data(), nrm.data(), prim.data()));
    for (int64_t i = 0; i < n; ++i)
      out[i] = HitInfo{hit[(size_t)i] != 0, t[(size_t)i],
                       {nrm[3 * (size_t)i], nrm[3 * (size_t)i + 1], nrm[3 * (size_t)i + 2]}, prim[(size_t)i]};
  }
  void setPlane(const Plane *p) const {
    const float n[3] = {p ? p->normal.x : 0.0f, p ? p->normal.y : 1.0f, p ? p->normal.z : 0.0f};
    check(rt_scene_set_plane(handle(), p ? 1 : 0, n, p ? p->offset : 0.0f));
  }

 protected:
  struct Del {
    void operator()(rt_scene *s) const { rt_scene_destroy(s); }
  };
  void reset(rt_scene *s) {
    static std::atomic<uint64_t> next{1};
    h_.reset(s);
    gen_ = next.fetch_add(1);
  }
  std::unique_ptr<rt_scene, Del> h_;
  uint64_t gen_ = 0;
};

// BVHBuilder::perform (triangles_raytracing.cpp:227-258): same SAH BVH8.
class BVHBuilder : public IScene {
 public:
  void perform(const SimpleMesh &mesh) {
    rt_scene *s = nullptr;
    check(rt_scene_create_mesh(mesh.vPos4f.data(), (int64_t)(mesh.vPos4f.size() / 4), mesh.indices.data(),
                               (int64_t)mesh.indices.size(), &s));
    reset(s);
  }
  size_t nodesCount() const {
    int64_t n = 0, inner = 0;
    int32_t d = 0;
    check(rt_scene_bvh_stats(handle(), &n, &inner, &d));
    return (size_t)n;
  }
};

class SDFGrid : public IScene {  // grid_raytracing.hpp:10-21
 public:
  uint32_t size[3] = {0, 0, 0};
  std::vector<float> values;  // host copy, x-major (x*sy+y)*sz+z
  void upload() {
    rt_scene *s = nullptr;
    check(rt_scene_create_grid(size, values.data(), &s));
    reset(s);
  }
};
inline void loadSDFGrid(SDFGrid &g, const std::string &path) {  // grid_raytracing.cpp:127-134
  check(rt_load_grid(path.c_str(), g.size, nullptr));
  g.values.resize((size_t)g.size[0] * g.size[1] * g.size[2]);
  check(rt_load_grid(path.c_str(), g.size, g.values.data()));
  g.upload();
}

class SDFOctree : public IScene {  // octree_raytracing.hpp:20-47
 public:
  std::vector<uint8_t> nodes;  // count x 36-byte SDFOctreeNode
  void upload() {
    rt_scene *s = nullptr;
    check(rt_scene_create_octree(nodes.data(), (int64_t)(nodes.size() / 36), &s));
    reset(s);
  }
};
inline void loadSDFOctree(SDFOctree &o, const std::string &path) {  // octree_raytracing.cpp:8-16
  int64_t n = 0;
  check(rt_load_octree(path.c_str(), &n, nullptr));
  o.nodes.resize((size_t)n * 36);
  check(rt_load_octree(path.c_str(), &n, o.nodes.data()));
  o.upload();
}

// SceneUnion(scene, plane) (raytracing.hpp:83-97): the reference application
// only ever unions a scene with the ground plane (main.cpp:64, 190).
struct SceneUnion {
  const IScene &first;
  Plane second;
  SceneUnion(const IScene &a, Plane p) : first(a), second(p) {}
};

// Renderer (raytracing.hpp:101-117).
struct Renderer {
  float3 lightPos{2.0f, 2.0f, 2.0f};  // main.cpp:60
  bool enableShadows = true;
  bool enableReflections = true;
  ShadingMode shadingMode = ShadingMode::Lambert;
  // GPUs a frame is split over (one process; rt_multi_*): empty renders on the
  // scene's device with rt_render. Otherwise the scene (which must live on
  // devices[0]) is replicated on the others at the first draw, each device
  // renders every n-th band of bandRows rows (the reference's draw splits
  // rows over OpenMP threads, raytracing.cpp:77-96), and one gather per frame
  // (RCCL ncclGather; peer copies when a device repeats) assembles it on
  // devices[0]. The frame is bitwise the single-device frame.
  std::vector<int32_t> devices;
  int32_t bandRows = 8;

  // Renderer::draw: t is read as tPrev, pixels written only on hit
  // (raytracing.cpp:67-102). Returns the kernel time in milliseconds.
  float draw(const IScene &scene, FrameBuffer &fb, const Camera &camera, const float4x4 &projInv) const {
    scene.setPlane(nullptr);
    return drawImpl(scene, fb, camera, projInv);
  }
  float draw(const SceneUnion &u, FrameBuffer &fb, const Camera &camera, const float4x4 &projInv) const {
    u.first.setPlane(&u.second);
    return drawImpl(u.first, fb, camera, projInv);
  }

 private:
  float drawImpl(const IScene &scene, FrameBuffer &fb, const Camera &camera, const float4x4 &projInv) const {
    rt_render_params p{};
    const float3 c = camera.position();
    p.camera_pos[0] = c.x; p.camera_pos[1] = c.y; p.camera_pos[2] = c.z;
    const float4x4 vi = camera.viewInverse();
    for (int i = 0; i < 16; ++i) { p.view_inv[i] = vi[(size_t)i]; p.proj_inv[i] = projInv[(size_t)i]; }
    p.light_pos[0] = lightPos.x; p.light_pos[1] = lightPos.y; p.light_pos[2] = lightPos.z;
    p.shading_mode = (int32_t)shadingMode;
    p.enable_shadows = enableShadows;
    p.enable_reflections = enableReflections;
    float ms = 0.0f;
    // over a frame that still holds clear()'s values (the viewer's loop,
    // main.cpp:197-206) nothing needs uploading: the cleared-frame call
    const uint32_t flags = fb.cleared ? (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY) : 0u;
    if (!devices.empty()) {
      check(rt_multi_render(multi(scene), &p, fb.color.data(), fb.t.data(), (int32_t)fb.width(),
                            (int32_t)fb.height(), flags, &ms));
    } else {
      check(rt_render(scene.handle(), &p, fb.color.data(), fb.t.data(), (int32_t)fb.width(),
                      (int32_t)fb.height(), flags, &ms));
    }
    fb.cleared = false;
    return ms;
  }
  // the multi-GPU handle of (scene build, devices, bandRows), made at first
  // use. Keyed on the scene's generation, not its address: its replicas on
  // devices[1..] are copies of the scene as it was, so a rebuilt scene (a new
  // perform / upload, possibly at a freed scene's address) gets a new handle.
  rt_multi *multi(const IScene &scene) const {
    if (!multi_ || multi_gen_ != scene.generation() || multi_devices_ != devices || multi_rows_ != bandRows) {
      multi_.reset();
      rt_multi *m = nullptr;
      check(rt_multi_create(scene.handle(), devices.data(), (int32_t)devices.size(), bandRows, &m));
      multi_.reset(m, MultiDel{});
      multi_gen_ = scene.generation();
      multi_devices_ = devices;
      multi_rows_ = bandRows;
    }
    return multi_.get();
  }
  struct MultiDel {
    void operator()(rt_multi *m) const { rt_multi_destroy(m); }
  };
  mutable std::shared_ptr<rt_multi> multi_;
  mutable uint64_t multi_gen_ = 0;
  mutable std::vector<int32_t> multi_devices_;
  mutable int32_t multi_rows_ = 0;
};

}  // namespace rtamd
