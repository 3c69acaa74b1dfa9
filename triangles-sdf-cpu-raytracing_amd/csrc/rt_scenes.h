// rt_scenes.h -- per-ray scene intersection on the device (the IScene
// implementations of the reference, re-expressed as stackful loops).
//
// Each scene exposes
//   intersect(o, d, tNear, tFar)  -> Hit  (HitInfo: hitten, t, normal, prim)
//   occluded (o, d, tNear, tFar)  -> bool (HitInfo::hitten only: shadow rays)
// Traversal state lives in a per-lane LDS stack (lane-interleaved: slot s of
// lane l at word s*BLOCK + l, so a wave's stack accesses are conflict-free).
#pragma once
#include "rt_layout.h"
#include "rt_math.h"

namespace rtd {

// Work counters (compile-time optional). Index map = oracle's cpuref_counters:
// 0 bvh_inner 1 bvh_leaf 2 bvh_tri 3 grid_sdf 4 oct_node 5 oct_leaf 6 oct_step
// 7 oct_normal 8 rays. NoCnt compiles away; LaneCnt is used only by the
// counting kernel variant that feeds the algorithmic-bytes model.
enum { C_BVH_INNER = 0, C_BVH_LEAF, C_BVH_TRI, C_GRID_SDF, C_OCT_NODE, C_OCT_LEAF, C_OCT_STEP,
       C_OCT_NORMAL, C_RAYS, C_NUM };
struct NoCnt {
  __device__ __forceinline__ void add(int, uint32_t) {}
};
struct LaneCnt {
  uint32_t v[C_NUM];
  __device__ __forceinline__ void add(int i, uint32_t n) { v[i] += n; }
};

struct Hit {
  bool hit;
  float t;
  f3 n;
  int64_t prim;  // mesh: original triangle id; grid: c0 cell; octree: leaf node; plane: -2
};
__device__ __forceinline__ Hit miss_hit() { return Hit{false, kInf, f3{0.0f, 1.0f, 0.0f}, -1}; }

// ------------------------------------------------------------------- mesh --
// BVHBuilder::traverseNode (triangles_raytracing.cpp:266-335) without
// recursion. Semantics reproduced exactly:
//  * at an inner node the 8 child entry distances come from the ISPC slab test
//    and are ordered by the sort8 network; children with t < 0 are skipped;
//  * a child is skipped when the LOCAL best of its parent's recursion frame is
//    < its entry distance (the reference's `result` is per call frame), so each
//    frame keeps its own best t and folds it into its parent's on return;
//  * leaf hits are kept with no t-range check (the reference's negative-t
//    quirk) and the smallest t wins, ties to the first found in DFS order.
// Frames hold (node, remaining child ids, best t); the entry distance of a
// frame's next child is recomputed from that child's box when the frame
// resumes (the same slab formula on the same floats: the same bits).
struct MeshDev {
  const rtl::GNode *__restrict__ nodes;
  const rtl::GTri *__restrict__ tris;
  uint32_t root;
};

__device__ __forceinline__ void tri_test(const rtl::GTri *__restrict__ tris, uint32_t k, f3 o, f3 d,
                                         float &best, uint32_t &best_k) {
  // triangle_intersection (ray_pack.ispc:132-165); e1/e2 precomputed (exact)
  const float4 *q = reinterpret_cast<const float4 *>(tris + k);
  const float4 a = q[0], b = q[1], c = q[2];
  const f3 v0{a.x, a.y, a.z}, e1{b.x, b.y, b.z}, e2{c.x, c.y, c.z};
  const f3 pvec = cross(d, e2);
  const float det = dot(e1, pvec);
  if (det < 1e-8f && det > -1e-8f) return;
  const float inv_det = 1 / det;
  const f3 tvec = o - v0;
  const float u = dot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return;
  const f3 qvec = cross(tvec, e1);
  const float v = dot(d, qvec) * inv_det;
  if (v < 0.0f || u + v > 1.0f) return;
  const float t = dot(e2, qvec) * inv_det;
  if (best > t) { best = t; best_k = k; }
}

__device__ __forceinline__ f3 tri_normal(const rtl::GTri *__restrict__ tris, uint32_t k) {
  const float4 *q = reinterpret_cast<const float4 *>(tris + k);
  const float4 b = q[1], c = q[2];
  return normalize(cross(f3{b.x, b.y, b.z}, f3{c.x, c.y, c.z}));
}

// One leaf: its local best (first wins among equal t, triangle order).
template <class CT>
__device__ __forceinline__ void leaf_test(const rtl::GTri *__restrict__ tris, uint32_t w, f3 o,
                                          f3 d, float &lt, uint32_t &lk, CT &cnt) {
  const uint32_t first = (w >> 3) & rtl::kMaxLeafFirstTri;
  const uint32_t n = (w & 7u) + 1u;
  cnt.add(C_BVH_LEAF, 1);
  cnt.add(C_BVH_TRI, n);
  for (uint32_t k = 0; k < n; ++k) tri_test(tris, first + k, o, d, lt, lk);
}

// Expand an inner node: slab-test its 8 children, sort8, keep t >= 0 entries
// (a suffix of the sorted order) as a packed list of 3-bit ids + count.
__device__ __forceinline__ void expand_node(const rtl::GNode *__restrict__ node, f3 o, f3 inv,
                                            float tNear, float tFar, uint32_t &list,
                                            uint32_t &cnt, float &tfirst) {
  const float4 *p = reinterpret_cast<const float4 *>(node);
  float bx[48];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const float4 v = p[i];
    bx[4 * i] = v.x; bx[4 * i + 1] = v.y; bx[4 * i + 2] = v.z; bx[4 * i + 3] = v.w;
  }
  float t[8];
  uint32_t id[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    t[c] = slab_ispc(bx[6 * c], bx[6 * c + 1], bx[6 * c + 2], bx[6 * c + 3], bx[6 * c + 4],
                     bx[6 * c + 5], o, inv, tNear, tFar);
    id[c] = (uint32_t)c;
  }
  sort8(t, id);
  list = 0;
  cnt = 0;
  tfirst = 0.0f;
#pragma unroll
  for (int i = 7; i >= 0; --i) {  // build from the back so the first visit ends in the low bits
    if (!(t[i] < 0.0f)) {
      list = (list << 3) | id[i];
      cnt += 1;
      tfirst = t[i];
    }
  }
}

template <int BLOCK>
struct LdsStack {
  uint32_t *base;  // lane-interleaved words
  __device__ __forceinline__ uint32_t &at(int slot, int field) {
    return base[(slot * 3 + field) * BLOCK];
  }
};

// ANY = true: shadow-ray query, stop at the first leaf hit (only hitten is used).
template <int BLOCK, bool ANY, class CT>
__device__ __forceinline__ bool mesh_trace(const MeshDev &sc, f3 o, f3 d, float tNear, float tFar,
                                           LdsStack<BLOCK> st, float &out_t, uint32_t &out_k,
                                           CT &cnt) {
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};  // 1.0f / rayDir (:273)
  float gbest = kInf;
  uint32_t gk = rtl::kInvalidChild;
  uint32_t word = sc.root;
  // top frame in registers; frames below it in LDS slots [0, depth-2]
  uint32_t fnode = 0, flist = 0, fcnt = 0;
  float fbest = kInf;
  int depth = 0;
  float tnext = 0.0f;
  bool have_t = false;
  for (;;) {
    if (word != rtl::kInvalidChild) {
      if (word & rtl::kLeafBit) {
        float lt = kInf;
        uint32_t lk = rtl::kInvalidChild;
        leaf_test(sc.tris, word, o, d, lt, lk, cnt);
        if (lk != rtl::kInvalidChild) {
          if (ANY) { out_t = lt; out_k = lk; return true; }
          if (lt < fbest) fbest = lt;
          if (lt < gbest) { gbest = lt; gk = lk; }
        }
      } else {
        uint32_t l, c;
        float tf;
        cnt.add(C_BVH_INNER, 1);
        expand_node(sc.nodes + word, o, inv, tNear, tFar, l, c, tf);
        if (c != 0) {
          if (depth >= 1) {
            st.at(depth - 1, 0) = fnode;
            st.at(depth - 1, 1) = flist | (fcnt << 24);
            st.at(depth - 1, 2) = __float_as_uint(fbest);
          }
          ++depth;
          fnode = word; flist = l; fcnt = c; fbest = kInf;
          tnext = tf;
          have_t = true;
        }
      }
      word = rtl::kInvalidChild;
    }
    if (depth == 0) break;
    if (fcnt == 0) {  // frame done: fold its best into the parent frame
      --depth;
      if (depth == 0) break;
      const float child_best = fbest;
      fnode = st.at(depth - 1, 0);
      const uint32_t lc = st.at(depth - 1, 1);
      flist = lc & 0xFFFFFFu;
      fcnt = lc >> 24;
      fbest = __uint_as_float(st.at(depth - 1, 2));
      if (child_best < fbest) fbest = child_best;
      have_t = false;
      continue;
    }
    const uint32_t j = flist & 7u;
    flist >>= 3;
    fcnt -= 1;
    const rtl::GNode *nd = sc.nodes + fnode;
    if (!have_t) {
      const float *b = nd->box[j];
      tnext = slab_ispc(b[0], b[1], b[2], b[3], b[4], b[5], o, inv, tNear, tFar);
    }
    have_t = false;
    if (fbest < tnext) { fcnt = 0; continue; }  // pruned; later siblings have larger t
    word = nd->child[j];
  }
  out_t = gbest;
  out_k = gk;
  return gk != rtl::kInvalidChild;
}

template <int BLOCK, class CT>
__device__ __forceinline__ Hit mesh_intersect(const MeshDev &sc, f3 o, f3 d, float tNear, float tFar,
                                              LdsStack<BLOCK> st, CT &cnt) {
  float t;
  uint32_t k;
  Hit h = miss_hit();
  if (mesh_trace<BLOCK, false>(sc, o, d, tNear, tFar, st, t, k, cnt)) {
    h.hit = true;
    h.t = t;
    h.n = tri_normal(sc.tris, k);
    h.prim = (int64_t)sc.tris[k].orig_id;
  }
  return h;
}
template <int BLOCK, class CT>
__device__ __forceinline__ bool mesh_occluded(const MeshDev &sc, f3 o, f3 d, float tNear, float tFar,
                                              LdsStack<BLOCK> st, CT &cnt) {
  float t;
  uint32_t k;
  return mesh_trace<BLOCK, true>(sc, o, d, tNear, tFar, st, t, k, cnt);
}

// ------------------------------------------------------------------- grid --
// SDFGrid (grid_raytracing.cpp:1-125): trilinear sdf over 8 taps of an
// x-major grid, sphere tracing inside [-1,1]^3 until sdf < 1e-3.
struct GridDev {
  const float *__restrict__ v;
  uint32_t sx, sy, sz;
};

template <class CT>
__device__ __forceinline__ float grid_sdf(const GridDev &g, f3 p, uint32_t *cell, CT &cnt) {
  cnt.add(C_GRID_SDF, 1);
  p = f3{(p.x + 1.0f) / 2.0f, (p.y + 1.0f) / 2.0f, (p.z + 1.0f) / 2.0f};
  p = p * f3{(float)(g.sx - 1), (float)(g.sy - 1), (float)(g.sz - 1)};
  const float c0x = __builtin_floorf(p.x), c0y = __builtin_floorf(p.y), c0z = __builtin_floorf(p.z);
  const float c1x = __builtin_ceilf(p.x), c1y = __builtin_ceilf(p.y), c1z = __builtin_ceilf(p.z);
  const uint32_t i0x = (uint32_t)c0x, i0y = (uint32_t)c0y, i0z = (uint32_t)c0z;
  const uint32_t i1x = (uint32_t)c1x, i1y = (uint32_t)c1y, i1z = (uint32_t)c1z;
  float ax = p.x - c0x, ay = p.y - c0y, az = p.z - c0z;  // p_c0f
  float bx = c1x - p.x, by = c1y - p.y, bz = c1z - p.z;  // c1f_p
  if (i1x == i0x) { ax = 1.0f; bx = 0.0f; }
  if (i1y == i0y) { ay = 1.0f; by = 0.0f; }
  if (i1z == i0z) { az = 1.0f; bz = 0.0f; }
  const uint32_t r00 = (i0x * g.sy + i0y) * g.sz, r01 = (i0x * g.sy + i1y) * g.sz;
  const uint32_t r10 = (i1x * g.sy + i0y) * g.sz, r11 = (i1x * g.sy + i1y) * g.sz;
  const float p0 = g.v[r00 + i0z], p1 = g.v[r00 + i1z], p2 = g.v[r01 + i0z], p3 = g.v[r01 + i1z];
  const float p4 = g.v[r10 + i0z], p5 = g.v[r10 + i1z], p6 = g.v[r11 + i0z], p7 = g.v[r11 + i1z];
  float res = 0.0f;
  res += p0 * bx * by * bz;
  res += p1 * bx * by * az;
  res += p2 * bx * ay * bz;
  res += p3 * bx * ay * az;
  res += p4 * ax * by * bz;
  res += p5 * ax * by * az;
  res += p6 * ax * ay * bz;
  res += p7 * ax * ay * az;
  if (cell) *cell = r00 + i0z;
  return res;
}

template <class CT>
__device__ __forceinline__ f3 grid_normal(const GridDev &g, f3 p, CT &cnt) {  // grid_raytracing.cpp:64-89
  const float E = 1e-3f;
  const float xl = (p.x - E >= -1.0f) ? p.x - E : p.x, xr = (p.x + E <= 1.0f) ? p.x + E : p.x;
  const float yl = (p.y - E >= -1.0f) ? p.y - E : p.y, yr = (p.y + E <= 1.0f) ? p.y + E : p.y;
  const float zl = (p.z - E >= -1.0f) ? p.z - E : p.z, zr = (p.z + E <= 1.0f) ? p.z + E : p.z;
  const float dx = grid_sdf(g, f3{xr, p.y, p.z}, nullptr, cnt) - grid_sdf(g, f3{xl, p.y, p.z}, nullptr, cnt);
  const float dy = grid_sdf(g, f3{p.x, yr, p.z}, nullptr, cnt) - grid_sdf(g, f3{p.x, yl, p.z}, nullptr, cnt);
  const float dz = grid_sdf(g, f3{p.x, p.y, zr}, nullptr, cnt) - grid_sdf(g, f3{p.x, p.y, zl}, nullptr, cnt);
  return normalize(f3{dx, dy, dz});
}

// grid_raytracing.cpp:93-125. Returns hit and leaves the hit point in *hp.
template <class CT>
__device__ __forceinline__ bool grid_march(const GridDev &g, f3 o, f3 d, float tNear, float tFar,
                                           float &out_t, f3 &hp, uint32_t &cell, CT &cnt) {
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
  float t1, t2;
  bbox_intersection(f3{-1.0f, -1.0f, -1.0f}, f3{1.0f, 1.0f, 1.0f}, o, inv, tNear, tFar, t1, t2);
  if (t1 > t2) return false;
  float t = t1;
  f3 p = o + t * d;
  p = vstd_max(p, f3{-1.0f, -1.0f, -1.0f});
  p = vstd_min(p, f3{1.0f, 1.0f, 1.0f});
  while (p.x <= 1.0f && p.y <= 1.0f && p.z <= 1.0f && p.x >= -1.0f && p.y >= -1.0f && p.z >= -1.0f) {
    const float s = grid_sdf(g, p, &cell, cnt);
    if (s < 1e-3f) {
      out_t = t + s;
      hp = p;
      return true;
    }
    t += s;
    p = o + t * d;
  }
  return false;
}

template <class CT>
__device__ __forceinline__ Hit grid_intersect(const GridDev &g, f3 o, f3 d, float tNear, float tFar,
                                              CT &cnt) {
  Hit h = miss_hit();
  f3 p;
  uint32_t cell;
  if (grid_march(g, o, d, tNear, tFar, h.t, p, cell, cnt)) {
    h.hit = true;
    h.n = grid_normal(g, p, cnt);
    h.prim = (int64_t)cell;
  } else {
    h.t = kInf;
  }
  return h;
}
template <class CT>
__device__ __forceinline__ bool grid_occluded(const GridDev &g, f3 o, f3 d, float tNear, float tFar,
                                              CT &cnt) {
  float t;
  f3 p;
  uint32_t cell;
  return grid_march(g, o, d, tNear, tFar, t, p, cell, cnt);
}

// ----------------------------------------------------------------- octree --
// SDFOctree (octree_raytracing.cpp:18-208): front-to-back recursion over an
// implicit octree on [-1,1]^3; the FIRST child (in sort8 order of the slab
// entry distances, t > 0 only) whose subtree hits wins. Node boxes: the
// reference derives them by repeated divide_box_8 float arithmetic; every
// value on that chain is a dyadic rational (min = -1 + i*2^(1-k), size
// 2^(1-k)), so each add/halve is exact and the box of a node at depth k with
// integer coordinates i equals [-1 + i*s, -1 + i*s + s], s = 2^(1-k).
// (tests/test_host.py checks this against the float chain for every node.)
struct OctDev {
  const uint32_t *__restrict__ child;
  const rtl::OctVals *__restrict__ vals;
};

__device__ __forceinline__ void oct_box(uint32_t ix, uint32_t iy, uint32_t iz, int depth, f3 &bmin,
                                        f3 &bmax) {
  const float s = __builtin_ldexpf(2.0f, -depth);
  bmin = f3{-1.0f + (float)ix * s, -1.0f + (float)iy * s, -1.0f + (float)iz * s};
  bmax = f3{bmin.x + s, bmin.y + s, bmin.z + s};
}

struct OctCorners {
  float v[8];
};

__device__ __forceinline__ void oct_local(f3 bmin, f3 bmax, f3 p, f3 &a, f3 &b) {
  // point = (p - boxMin) / (boxMax - boxMin); clamp to [1e-7, 0.9999999]
  p = (p - bmin) / (bmax - bmin);
  p = vstd_min(vstd_max(p, f3{0.0000001f, 0.0000001f, 0.0000001f}),
               f3{0.9999999f, 0.9999999f, 0.9999999f});
  const f3 c0{__builtin_floorf(p.x), __builtin_floorf(p.y), __builtin_floorf(p.z)};
  const f3 c1{__builtin_ceilf(p.x), __builtin_ceilf(p.y), __builtin_ceilf(p.z)};
  a = p - c0;  // p_c0f  (c0 = 0 and c1 = 1 after the clamp)
  b = c1 - p;  // c1f_p
}

__device__ __forceinline__ float oct_sdf(const OctCorners &c, f3 bmin, f3 bmax, f3 p) {
  f3 a, b;
  oct_local(bmin, bmax, p, a, b);
  float res = 0.0f;  // octree_raytracing.cpp:36-55, values[(x<<2)+(y<<1)+z]
  res += c.v[0] * b.x * b.y * b.z;
  res += c.v[1] * b.x * b.y * a.z;
  res += c.v[2] * b.x * a.y * b.z;
  res += c.v[3] * b.x * a.y * a.z;
  res += c.v[4] * a.x * b.y * b.z;
  res += c.v[5] * a.x * b.y * a.z;
  res += c.v[6] * a.x * a.y * b.z;
  res += c.v[7] * a.x * a.y * a.z;
  return res;
}

__device__ __forceinline__ f3 oct_normal(const OctCorners &c, f3 bmin, f3 bmax, f3 p) {
  f3 a, b;
  oct_local(bmin, bmax, p, a, b);
  const float da = 1.0f, db = -1.0f;  // dp_c0f, dc1f_p (octree_raytracing.cpp:79-80)
  const float *v = c.v;
  const float dfdx = v[0] * db * b.y * b.z + v[1] * db * b.y * a.z + v[2] * db * a.y * b.z +
                     v[3] * db * a.y * a.z + v[4] * da * b.y * b.z + v[5] * da * b.y * a.z +
                     v[6] * da * a.y * b.z + v[7] * da * a.y * a.z;
  const float dfdy = v[0] * b.x * db * b.z + v[1] * b.x * db * a.z + v[2] * b.x * da * b.z +
                     v[3] * b.x * da * a.z + v[4] * a.x * db * b.z + v[5] * a.x * db * a.z +
                     v[6] * a.x * da * b.z + v[7] * a.x * da * a.z;
  const float dfdz = v[0] * b.x * b.y * db + v[1] * b.x * b.y * da + v[2] * b.x * a.y * db +
                     v[3] * b.x * a.y * da + v[4] * a.x * b.y * db + v[5] * a.x * b.y * da +
                     v[6] * a.x * a.y * db + v[7] * a.x * a.y * da;
  return normalize(f3{dfdx, dfdy, dfdz});
}

// intersectLeaf (octree_raytracing.cpp:122-164) for a leaf that may hit.
template <bool NEED_NORMAL, class CT>
__device__ __forceinline__ bool oct_leaf(const OctDev &sc, uint32_t node, f3 bmin, f3 bmax, f3 o,
                                         f3 d, f3 inv, float tNear, float tFar, float &out_t,
                                         f3 &out_n, CT &cnt) {
  float t1, t2;
  bbox_intersection(bmin, bmax, o, inv, tNear, tFar, t1, t2);
  if (t1 > t2) return false;
  OctCorners c;
  const float4 *q = reinterpret_cast<const float4 *>(sc.vals + node);
  const float4 a = q[0], b = q[1];
  c.v[0] = a.x; c.v[1] = a.y; c.v[2] = a.z; c.v[3] = a.w;
  c.v[4] = b.x; c.v[5] = b.y; c.v[6] = b.z; c.v[7] = b.w;
  float t = t1;
  f3 p = o + t * d;
  p = vstd_max(p, bmin);
  p = vstd_min(p, bmax);
  while (p.x <= bmax.x && p.y <= bmax.y && p.z <= bmax.z && p.x >= bmin.x && p.y >= bmin.y &&
         p.z >= bmin.z) {
    const float s = oct_sdf(c, bmin, bmax, p);
    cnt.add(C_OCT_STEP, 1);
    if (s < 1e-4f) {
      out_t = t + s;
      if (NEED_NORMAL) { out_n = oct_normal(c, bmin, bmax, p); cnt.add(C_OCT_NORMAL, 1); }
      return true;
    }
    t += s;
    p = o + t * d;
  }
  return false;
}

// Expand an octree inner node: divide_box_8 + intersect_box_8 + sort8, keep
// entries with t > 0 (octree_raytracing.cpp:185).
__device__ __forceinline__ void oct_expand(f3 bmin, f3 bmax, f3 o, f3 inv, float tNear, float tFar,
                                           uint32_t &list, uint32_t &cnt) {
  const f3 center{(bmin.x + bmax.x) / 2.0f, (bmin.y + bmax.y) / 2.0f, (bmin.z + bmax.z) / 2.0f};
  const f3 diff = center - bmin;
  float t[8];
  uint32_t id[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int x = c >> 2, y = (c & 3) >> 1, z = c & 1;
    const float x0 = x == 0 ? bmin.x : center.x, y0 = y == 0 ? bmin.y : center.y,
                z0 = z == 0 ? bmin.z : center.z;
    t[c] = slab_ispc(x0, y0, z0, x0 + diff.x, y0 + diff.y, z0 + diff.z, o, inv, tNear, tFar);
    id[c] = (uint32_t)c;
  }
  sort8(t, id);
  list = 0;
  cnt = 0;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    if (t[i] > 0.0f) {
      list = (list << 3) | id[i];
      cnt += 1;
    }
  }
}

template <int BLOCK, bool NEED_NORMAL, class CT>
__device__ __forceinline__ bool oct_trace(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                          LdsStack<BLOCK> st, float &out_t, f3 &out_n,
                                          uint32_t &out_node, CT &cnt) {
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
  const uint32_t root = sc.child[0];
  cnt.add(C_OCT_NODE, 1);
  if (root == 0 || root == rtl::kOctNeverHits) {
    cnt.add(C_OCT_LEAF, 1);
    if (root == rtl::kOctNeverHits) return false;
    out_node = 0;
    return oct_leaf<NEED_NORMAL>(sc, 0, f3{-1.0f, -1.0f, -1.0f}, f3{1.0f, 1.0f, 1.0f}, o, d, inv,
                                 tNear, tFar, out_t, out_n, cnt);
  }
  // top frame: node whose children are being visited, its coords and list
  uint32_t fnode = 0, flist, fcnt;
  uint32_t ix = 0, iy = 0, iz = 0;
  int depth = 0;  // depth of fnode (root = 0); frames below the top live in LDS
  {
    f3 bmin, bmax;
    oct_box(0, 0, 0, 0, bmin, bmax);
    oct_expand(bmin, bmax, o, inv, tNear, tFar, flist, fcnt);
  }
  for (;;) {
    if (fcnt == 0) {
      if (depth == 0) return false;
      --depth;
      fnode = st.at(depth, 0);
      const uint32_t lc = st.at(depth, 1);
      flist = lc & 0xFFFFFFu;
      fcnt = lc >> 24;
      ix >>= 1; iy >>= 1; iz >>= 1;
      continue;
    }
    const uint32_t j = flist & 7u;
    flist >>= 3;
    fcnt -= 1;
    const uint32_t cn = sc.child[fnode] + j;
    const uint32_t cx = (ix << 1) | (j >> 2), cy = (iy << 1) | ((j >> 1) & 1u), cz = (iz << 1) | (j & 1u);
    const uint32_t cw = sc.child[cn];
    cnt.add(C_OCT_NODE, 1);
    if (cw == rtl::kOctNeverHits) { cnt.add(C_OCT_LEAF, 1); continue; }
    f3 bmin, bmax;
    oct_box(cx, cy, cz, depth + 1, bmin, bmax);
    if (cw == 0) {
      cnt.add(C_OCT_LEAF, 1);
      if (oct_leaf<NEED_NORMAL>(sc, cn, bmin, bmax, o, d, inv, tNear, tFar, out_t, out_n, cnt)) {
        out_node = cn;
        return true;
      }
      continue;
    }
    uint32_t l, c;
    oct_expand(bmin, bmax, o, inv, tNear, tFar, l, c);
    if (c == 0) continue;
    st.at(depth, 0) = fnode;
    st.at(depth, 1) = flist | (fcnt << 24);
    ++depth;
    fnode = cn; flist = l; fcnt = c;
    ix = cx; iy = cy; iz = cz;
  }
}

template <int BLOCK, class CT>
__device__ __forceinline__ Hit oct_intersect(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                             LdsStack<BLOCK> st, CT &cnt) {
  Hit h = miss_hit();
  uint32_t node;
  if (oct_trace<BLOCK, true>(sc, o, d, tNear, tFar, st, h.t, h.n, node, cnt)) {
    h.hit = true;
    h.prim = (int64_t)node;
  } else {
    h.t = kInf;
  }
  return h;
}
template <int BLOCK, class CT>
__device__ __forceinline__ bool oct_occluded(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                             LdsStack<BLOCK> st, CT &cnt) {
  float t;
  f3 n;
  uint32_t node;
  return oct_trace<BLOCK, false>(sc, o, d, tNear, tFar, st, t, n, node, cnt);
}

// ------------------------------------------------------------------ plane --
// Plane (raytracing.hpp:119-186): checkerboard, albedo 0/1, reflectiveness 0.3.
struct PlaneDev {
  int on;
  f3 n;
  float off;
  f3 b1, b2;
};
__device__ __forceinline__ bool plane_hit(const PlaneDev &pl, f3 o, f3 d, float tNear, float tFar,
                                          float &t, float &albedo) {
  const float div = dot(d, pl.n);
  if (__builtin_fabsf(div) < 1e-8f) return false;
  t = (pl.off - dot(o, pl.n)) / div;
  if (t < tNear || t > tFar) return false;
  const f3 p = o + t * d;
  const int x = (int)__builtin_ceilf(dot(p, pl.b1));
  const int y = (int)__builtin_ceilf(dot(p, pl.b2));
  albedo = ((x + y) % 2 == 0) ? 0.0f : 1.0f;
  return true;
}

}  // namespace rtd
