// rt_host.h -- host-side scene preparation for the MI355X renderer.
// Loaders, the BVH8 SAH builder (same tree as BVHBuilder::perform,
// triangles_raytracing.cpp:227-258) and its GPU layout, octree flattening,
// and the reference camera math. Compiled by g++ with -ffp-contract=off.
#pragma once
#include <stdint.h>

#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

#include "rt_layout.h"

// A/B and diagnostic switches (RTAMD_* environment variables) are read only
// by variant builds (tools/build_variant.sh compiles with -DRT_AB_ENV=1): the
// shipping librtamd.so ignores the environment, so a host application that
// inherits one of them cannot change the render path. Run-time settings the
// tests need have rtx_* setters instead.
#ifndef RT_AB_ENV
#define RT_AB_ENV 0
#endif
inline const char *ab_env(const char *name) {
#if RT_AB_ENV
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

namespace rth {

struct Mesh {
  std::vector<float> vpos4;     // 4 floats per vertex (x, y, z, w)
  std::vector<uint32_t> idx;    // 3 per triangle
};

bool load_obj(const char *path, bool scale, Mesh &out, std::string &err);
bool load_grid(const char *path, uint32_t size[3], std::vector<float> &values, std::string &err);
bool load_octree(const char *path, std::vector<uint8_t> &nodes36, std::string &err);

// What a BVH build returns besides the inner nodes, root and depth (BVHGpu).
enum : unsigned {
  kBvhCanon = 1,       // BVHGpu::canon (rt_bvh_export)
  kBvhPerm = 2,        // BVHGpu::perm_tri (rt_bvh_export)
  kBvhTris = 4,        // the leaf triangles (BVHGpu::tris)
  kBvhDeviceTris = 8,  // with kBvhTris: the device builder may leave them on the device (BVHGpu::dev_tris)
  kBvhAll = kBvhCanon | kBvhPerm | kBvhTris,
};
// A device allocation handed from the builder to the scene (move-only).
struct DevBuffer {
  void *p = nullptr;
  size_t bytes = 0;
  void (*release)(void *) = nullptr;
  DevBuffer() = default;
  DevBuffer(const DevBuffer &) = delete;
  DevBuffer &operator=(const DevBuffer &) = delete;
  DevBuffer(DevBuffer &&o) noexcept { swap(o); }
  DevBuffer &operator=(DevBuffer &&o) noexcept {
    DevBuffer t(std::move(o));
    swap(t);
    return *this;
  }
  ~DevBuffer() {
    if (p && release) release(p);
  }
  void swap(DevBuffer &o) noexcept {
    std::swap(p, o.p);
    std::swap(bytes, o.bytes);
    std::swap(release, o.release);
  }
  void *take() {  // the caller owns (and frees) it from here on
    void *q = p;
    p = nullptr;
    return q;
  }
};
struct BVHGpu {
  std::vector<rtl::GNode> nodes;   // inner nodes, BFS order, root = 0
  std::vector<rtl::GTri> tris;     // leaf triangles, leaves in BFS order of their parents
  DevBuffer dev_tris;              // or these on the device (kBvhDeviceTris), followed by 8 zero triangles
  uint32_t n_tris = 0;             // triangle slots (either form)
  uint32_t root_word = rtl::kInvalidChild;
  float root_box[6] = {0, 0, 0, 0, 0, 0};  // union of the root's child boxes (inner root)
  int32_t max_depth = 0;           // inner nodes on the deepest root->leaf path
  int64_t host_nodes = 0, host_inner = 0;
  // canonical pre-order export (52 x u32 per node), for parity with the oracle
  std::vector<uint32_t> canon;
  std::vector<uint32_t> perm_tri;  // original triangle id per triangle slot
  // leaves whose triangles bvh_layout did not write (no kBvhTris on the host):
  // (first slot, first triangle position, count) per leaf
  std::vector<uint32_t> leaf_tab;
};
bool build_bvh8(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                std::string &err, unsigned want = kBvhAll);

// The tree BVHBuilder::perform builds (triangles_raytracing.cpp:155-225), as
// either builder produces it: nodes (node 0 = root; children anywhere) and the
// final triangle order (BVHBuilder's reordered mesh.indices / 3).
struct BvhBox {
  float mn[3], mx[3];
};
struct BvhHostNode {
  bool leaf = false;
  uint32_t start = 0, count = 0;  // leaf: range in indices (reference units)
  uint32_t nchild = 0;
  int32_t child[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  BvhBox box[8];
};
// libstdc++ std::sort of ids by K[id] (< 0 depth: std::sort's own limit).
void host_introsort(uint32_t *ids, size_t n, const float *K, int64_t depth_limit);
// A built tree's nodes, wherever they are stored (std::vector for the host
// builder, a huge-page arena for the device builder).
struct HostNodes {
  const BvhHostNode *p;
  size_t n;
  HostNodes(const std::vector<BvhHostNode> &v) : p(v.data()), n(v.size()) {}
  HostNodes(const BvhHostNode *ptr, size_t count) : p(ptr), n(count) {}
  size_t size() const { return n; }
  const BvhHostNode &operator[](size_t i) const { return p[i]; }
};
// Canonical export + GPU layout (GNode / GTri, BFS over inner nodes) of a
// built tree; `cur` (the triangle order) is read for kBvhPerm and host kBvhTris
// only. host_tris false: the leaf table instead of BVHGpu::tris.
void bvh_layout(const float *vpos4, const uint32_t *idx, int64_t nidx, HostNodes H,
                const std::vector<uint32_t> &cur, BVHGpu &out, unsigned want, bool host_tris);
// The same tree built on the current HIP device (rt_bvhgpu.hip): libstdc++'s
// introsort replicated with parallel Hoare partitions, SAH sweeps as device
// scans. Identical output to build_bvh8.
bool build_bvh8_gpu(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                    std::string &err, unsigned want = kBvhAll);

struct OctGpu {
  std::vector<rtl::OctWord> child;    // per node: {0 leaf, kOctNeverHits or childrenOffset; child masks}
  std::vector<rtl::OctVals> vals;     // per node corner values
  int32_t max_depth = 0;
};
bool flatten_octree(const uint8_t *nodes36, int64_t count, OctGpu &out, std::string &err);

// ---- mesh -> SDF construction (rt_meshops.cpp) ----
// Feature order of the closest-point regions (Ericson, RTCD 5.1.5):
// 0..2 vertex a,b,c; 3 edge ab; 4 edge ac; 5 edge bc; 6 face.
constexpr int kSdfFeatures = 7;
struct SdfMeshHost {
  BVHGpu bvh;               // the renderer's BVH8 over the same triangles
  std::vector<float> tri;   // per GPU leaf-order triangle: a.xyz,id | b.xyz,0 | c.xyz,0
  std::vector<float> pn;    // per ORIGINAL triangle: 7 x float4 angle-weighted pseudonormals
};
bool prep_sdf_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                   SdfMeshHost &out, std::string &err);

// Loop-free midpoint subdivision, `levels` times (config-5 stand-in mesh).
bool subdivide_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, int levels,
                    Mesh &out, std::string &err);

// Sparse SDF octree in the reference's 36-byte node format, built top-down:
// a node at depth d < depth is refined when |sdf(centre)| <= half-diagonal;
// unrefined nodes become empty leaves (values 1000), nodes at `depth` become
// leaves holding the SDF at their 8 corners; inner nodes hold zeros. Nodes are
// in BFS order with the 8 children of a node contiguous (id (x<<2)|(y<<1)|z).
// `query(points xyz, n, out)` evaluates the SDF at n points.
using SdfQuery = bool (*)(void *ctx, const float *p3, int64_t n, float *out, std::string &err);
bool build_sdf_octree(SdfQuery query, void *ctx, int depth, std::vector<uint8_t> &nodes36,
                      std::string &err);

// Camera (camera.hpp:7-61, camera.cpp:1-72): the viewer's orbit camera.
// Same memory layout as rt_camera_state (include/rtamd.h).
struct CamState {
  float pos[3], target[3], q[4];
  float sens;
  int32_t lock;
  float locked[3];
};
void cam_init(CamState &c, const float pos[3], const float target[3], const float up[3]);
void cam_rotate(CamState &c, float dx, float dy);
void cam_reset_position(CamState &c, const float pos[3]);
void cam_reset_target(CamState &c, const float target[3]);
void cam_set_lock_up(CamState &c, bool on);
void cam_zoom(CamState &c, float wheel);
void cam_basis(const CamState &c, float up[3], float right[3], float forward[3]);
void cam_view_inverse(const CamState &c, float view_inv[16]);

// cmesh4::SaveMeshToObj (core/mesh.cpp:14-63); vnorm4 / vtex2 may be NULL.
bool save_obj(const char *path, const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
              const float *vnorm4, const float *vtex2, std::string &err);

// 8-bit RGBA PNG (stored deflate blocks: no compression library needed).
bool write_png(const char *path, const uint32_t *rgba, int32_t W, int32_t H, std::string &err);

void camera_matrices(const float pos[3], const float target[3], const float up[3], float fovy,
                     float aspect, float znear, float zfar, float view_inv[16], float proj_inv[16]);

// rt_render's staged download of a cleared frame: rows [y0, y1] x columns
// [x0, x1] of two W-wide frames copied from the staging frame (sc, st) to the
// caller's buffers (dc, dt); rows split over up to `threads` OpenMP threads
// (<= 0: one per 32 rows, at most the OpenMP default and 16).
void copy_rect(uint32_t *dc, float *dt, const uint32_t *sc, const float *st, int64_t W, int32_t x0, int32_t x1,
               int32_t y0, int32_t y1, int threads);
// The same for per-row spans: row y's columns [span[2y], -span[2y+1]] (rows
// with span[2y] > -span[2y+1] are skipped); rt_render's zero-copy cleared
// frames on pageable buffers (FrameArgs::row_span). clear_src: each copied
// span of the source is then reset to the cleared frame (0, +inf).
void copy_spans(uint32_t *dc, float *dt, uint32_t *sc, float *st, int64_t W, int32_t H, const int32_t *span,
                int threads, bool clear_src = false);
// FrameBuffer::clear() of n pixels (0, +inf), over up to `threads` threads.
void clear_frame(uint32_t *c, float *t, int64_t n, int threads);

}  // namespace rth
