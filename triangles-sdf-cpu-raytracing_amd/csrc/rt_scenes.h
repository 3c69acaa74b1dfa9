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
#include "rt_rcp.h"

namespace rtd {

// Work counters (compile-time optional). Index map = oracle's cpuref_counters:
// 0 bvh_inner 1 bvh_leaf 2 bvh_tri 3 grid_sdf 4 oct_node 5 oct_leaf 6 oct_step
// 7 oct_normal 8 rays. NoCnt compiles away; LaneCnt is used only by the
// counting kernel variant that feeds the algorithmic-bytes model.
enum { C_BVH_INNER = 0, C_BVH_LEAF, C_BVH_TRI, C_GRID_SDF, C_OCT_NODE, C_OCT_LEAF, C_OCT_STEP,
       C_OCT_NORMAL, C_RAYS, C_NUM };
struct NoCnt {
  static constexpr bool kCounts = false;
  __device__ __forceinline__ void add(int, uint32_t) {}
};
struct LaneCnt {
  static constexpr bool kCounts = true;
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
  // union of the root's child boxes (exact min/max of their floats): a ray that
  // misses it under the slab formula misses every child (the formula is
  // monotone in the box bounds when 1/d is finite), so the root node need not
  // be fetched. Used only when all three 1/d components are finite.
  float rbox[6];
  bool coop;  // primary rays: cooperative tail enabled (diagnostic switch rtx_set_coop)
  uint32_t n_inner;  // inner nodes (BFS order: the first ones are the top levels)
  // top-of-tree copy in LDS (render_persist_kernel, RT_LDS_NODES): inner nodes
  // [0, n_lds) are read from lnodes (a block's LDS), the rest from nodes
  const rtl::GNode *lnodes;
  uint32_t n_lds;
  // rays with dot(d, d) <= dmax2 cannot make any triangle's |det| reach 2^125
  // (|det| <= 1.5 |e1| |e2| |d| in float arithmetic, max |e1| |e2| of the
  // scene measured at creation, mesh_dmax2): they take the triangle test with
  // the fast reciprocal (tri_t<true>). 0: every ray takes the division.
  float dmax2;
};

// Inner nodes of the top BVH levels kept in each persistent block's LDS (0:
// off; A/B switch, e.g. 73 = the top three levels, 16 KiB per block). Node
// reads then go through a per-lane choice of the LDS or the global copy (flat
// loads). Bit-exact, and measured level to 1 % slower:
// the vector L1 already serves 96-99 % of the node lines, so off.
#ifndef RT_LDS_NODES
#define RT_LDS_NODES 0
#endif
__device__ __forceinline__ const rtl::GNode *mesh_node(const MeshDev &sc, uint32_t i) {
#if RT_LDS_NODES
  return i < sc.n_lds ? sc.lnodes + i : sc.nodes + i;
#else
  return sc.nodes + i;
#endif
}

// triangle_intersection (ray_pack.ispc:132-165) on one triangle already in
// registers (v0, e1 = v1-v0, e2 = v2-v0; the subtractions are exact host-side
// float ops, identical to the reference's). Returns t, or +inf on a miss.
// FR (fast reciprocal): 1 / det as rtm::rcp_rn (rt_rcp.h), the same bits as
// the division for every 1e-8 <= |det| < 2^126; taken by rays whose direction
// keeps every |det| of the scene below 2^125 (MeshDev::dmax2; |det| < 1e-8 is
// a miss below whatever inv_det is). RT_FAST_RCP=0: the division always (A/B
// switch).
#ifndef RT_FAST_RCP
#define RT_FAST_RCP 1
#endif
template <bool FR>
__device__ __forceinline__ float tri_t(float4 a, float4 b, float4 c, f3 o, f3 d) {
  const f3 v0{a.x, a.y, a.z}, e1{b.x, b.y, b.z}, e2{c.x, c.y, c.z};
  const f3 pvec = cross(d, e2);
  const float det = dot(e1, pvec);
  float inv_det;
  if constexpr (FR && RT_FAST_RCP) {
    inv_det = rtm::rcp_rn(det);
  } else {
    inv_det = 1 / det;
  }
  const f3 tvec = o - v0;
  const float u = dot(tvec, pvec) * inv_det;
  const f3 qvec = cross(tvec, e1);
  const float v = dot(d, qvec) * inv_det;
  const float t = dot(e2, qvec) * inv_det;
  const bool miss = (det < 1e-8f && det > -1e-8f) || u < 0.0f || u > 1.0f || v < 0.0f || u + v > 1.0f;
  return miss ? kInf : t;
}

__device__ __forceinline__ f3 tri_normal(const rtl::GTri *__restrict__ tris, uint32_t k) {
  const float4 *q = reinterpret_cast<const float4 *>(tris + k);
  const float4 b = q[1], c = q[2];
  return normalize(cross(f3{b.x, b.y, b.z}, f3{c.x, c.y, c.z}));
}

// One leaf: its local best, first wins among equal t (strict `>` in triangle
// order, triangles_raytracing.cpp:324-331). The leaf's triangles are read in
// batches of B with all their loads in flight together (the triangle array is
// padded by 8 entries, so reading past a short leaf is in bounds and the extra
// lanes are discarded), instead of one memory round trip per triangle. The
// primary-ray kernels take batches of RT_LEAF_BATCH_PRIMARY = 4 (127 VGPRs, 4
// waves; bunny 0.1088 -> 0.1074, 1.1 M tris 4K 0.4292 -> 0.4244 ms/frame
// against 2); the shading kernels keep RT_LEAF_BATCH = 2, where 4 takes them
// from 3 waves (136 VGPRs) to 2 (181).
#ifndef RT_LEAF_BATCH
#define RT_LEAF_BATCH 2
#endif
#ifndef RT_LEAF_BATCH_PRIMARY
#define RT_LEAF_BATCH_PRIMARY 4
#endif
template <uint32_t B = RT_LEAF_BATCH, bool FR = false, class CT>
__device__ __forceinline__ void leaf_test(const rtl::GTri *__restrict__ tris, uint32_t w, f3 o,
                                          f3 d, float &lt, uint32_t &lk, CT &cnt) {
  const uint32_t first = (w >> 3) & rtl::kMaxLeafFirstTri;
  const uint32_t n = (w & 7u) + 1u;
  cnt.add(C_BVH_LEAF, 1);
  cnt.add(C_BVH_TRI, n);
  const float4 *q = reinterpret_cast<const float4 *>(tris + first);
  for (uint32_t base = 0; base < n; base += B) {
    float4 a[B], b[B], c[B];
#pragma unroll
    for (uint32_t k = 0; k < B; ++k) {
      a[k] = q[3 * (base + k)];
      b[k] = q[3 * (base + k) + 1];
      c[k] = q[3 * (base + k) + 2];
    }
    float tk[B];
#pragma unroll
    for (uint32_t k = 0; k < B; ++k) tk[k] = tri_t<FR>(a[k], b[k], c[k], o, d);
#pragma unroll
    for (uint32_t k = 0; k < B; ++k)
      if (base + k < n && lt > tk[k]) { lt = tk[k]; lk = first + base + k; }
  }
}

// Expand an inner node: slab-test its 8 children, sort8, keep t >= 0 entries
// (a suffix of the sorted order) as a packed list of 3-bit ids + count. Also
// returns the entry distance and child word of the first child to visit (the
// child words arrive with the boxes: descending needs no extra load).
// 1: expand_node skips sort8 in waves whose rays all enter <= 2 children with
// distinct t (A/B switch; 0 always runs the network)
#ifndef RT_EXPAND_FAST
#define RT_EXPAND_FAST 1
#endif
template <bool FAST>
__device__ __forceinline__ void expand_node(const rtl::GNode *__restrict__ node, f3 o, f3 inv,
                                            float tNear, float tFar, uint32_t &list,
                                            uint32_t &cnt, float &tfirst, uint32_t &cwfirst) {
  const float4 *p = reinterpret_cast<const float4 *>(node);
  float bx[48];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const float4 v = p[i];
    bx[4 * i] = v.x; bx[4 * i + 1] = v.y; bx[4 * i + 2] = v.z; bx[4 * i + 3] = v.w;
  }
  const uint4 cw0 = reinterpret_cast<const uint4 *>(node->child)[0];
  const uint4 cw1 = reinterpret_cast<const uint4 *>(node->child)[1];
  const uint32_t cws[8] = {cw0.x, cw0.y, cw0.z, cw0.w, cw1.x, cw1.y, cw1.z, cw1.w};
  float t[8];
  uint32_t id[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    t[c] = slab<FAST>(bx[6 * c], bx[6 * c + 2], bx[6 * c + 4], bx[6 * c + 1], bx[6 * c + 3],
                      bx[6 * c + 5], o, inv, tNear, tFar);  // box: xMin xMax yMin yMax zMin zMax
    id[c] = (uint32_t)c;
  }
  uint32_t first_id = 0;
  bool sorted = false;
  if constexpr (FAST && RT_EXPAND_FAST) {
    // At most two children entered with distinct t: the network's output order
    // of the entered children is plain ascending t (any correct sort gives
    // it), so the wave skips sort8 when every lane is in that case. Ties (or
    // three or more children) take the network: its order among equal keys
    // is its own.
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) m |= (t[c] < 0.0f) ? 0u : (1u << c);
    const uint32_t pc = (uint32_t)__builtin_popcount(m);
    const uint32_t ia = (uint32_t)__builtin_ctz(m | 0x100u), ib = 31u - (uint32_t)__builtin_clz(m | 1u);
    float ta = t[0], tb = t[0];
#pragma unroll
    for (int c = 1; c < 8; ++c) {
      ta = (ia == (uint32_t)c) ? t[c] : ta;
      tb = (ib == (uint32_t)c) ? t[c] : tb;
    }
    const bool slow = pc > 2 || (pc == 2 && !(ta != tb));
    if (__ballot(slow) == 0) {
      sorted = true;
      const bool sw = pc == 2 && tb < ta;
      first_id = sw ? ib : ia;
      tfirst = pc == 0 ? 0.0f : (sw ? tb : ta);
      cnt = pc;
      list = pc == 0 ? 0u : pc == 1 ? ia : (sw ? (ib | (ia << 3)) : (ia | (ib << 3)));
    }
  }
  if (!sorted) {
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
        first_id = id[i];
      }
    }
  }
  uint32_t cf = cws[0];
#pragma unroll
  for (int c = 1; c < 8; ++c) cf = (first_id == (uint32_t)c) ? cws[c] : cf;
  cwfirst = cf;
}

template <int BLOCK, int F = 3>
struct LdsStack {
  uint32_t *base;  // lane-interleaved words, F words per frame slot
  __device__ __forceinline__ uint32_t &at(int slot, int field) {
    // slot * F * BLOCK as a full-rate 24-bit multiply (slots are small): the
    // plain form compiles to the quarter-rate v_mul_lo_u32
    return base[__umul24((uint32_t)slot, (uint32_t)(F * BLOCK)) + (uint32_t)(field * BLOCK)];
  }
};

// ANY = true: shadow-ray query, stop at the first leaf hit (only hitten is used).
// Slab test of the root union box: true iff the ray certainly misses it.
__device__ __forceinline__ bool root_box_miss(const float *b, f3 o, f3 inv, float tNear, float tFar) {
  if (!(__builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z)))
    return false;  // 1/d = inf: NaN slabs possible, take the exact path
  const float t1x = (b[0] - o.x) * inv.x, t1y = (b[1] - o.y) * inv.y, t1z = (b[2] - o.z) * inv.z;
  const float t2x = (b[3] - o.x) * inv.x, t2y = (b[4] - o.y) * inv.y, t2z = (b[5] - o.z) * inv.z;
  float tMin = isp_max(isp_min(t1x, t2x), isp_max(isp_min(t1y, t2y), isp_min(t1z, t2z)));
  float tMax = isp_min(isp_max(t1x, t2x), isp_min(isp_max(t1y, t2y), isp_max(t1z, t2z)));
  tMin = isp_max(tMin, tNear);
  tMax = isp_min(tMax, tFar);
  return tMax < 0.0f || tMin > tMax;
}

// Root stage of BVHBuilder::traverseNode(0): the union-box pretest and the
// root's 8-child expansion (wave-uniform node: scalar loads). Returns false if
// the traversal ends here (no child entered); otherwise the root frame.
template <bool FAST = false, class CT>
__device__ __forceinline__ bool mesh_root(const MeshDev &sc, f3 o, f3 inv, float tNear, float tFar,
                                          uint32_t &l, uint32_t &c, float &tf, uint32_t &cwf,
                                          CT &cnt) {
  cnt.add(C_BVH_INNER, 1);
  if (root_box_miss(sc.rbox, o, inv, tNear, tFar)) return false;
  expand_node<FAST>(sc.nodes + sc.root, o, inv, tNear, tFar, l, c, tf, cwf);
  return c != 0;
}

// Traversal below the root frame (or from a root leaf when root_is_leaf).
// Traversal state of one ray below its root frame. The top frame lives in
// registers, the frames below it in LDS slots [0, depth-2].
struct MState {
  uint32_t word;    // next node/leaf to process (kInvalidChild: none)
  uint32_t flist;   // top frame: remaining child ids, 3 bits each, next in the low bits
  uint32_t fcnt;    // top frame: remaining child count
  uint32_t fnode;   // top frame: node index
  uint32_t cwnext;  // child word of the next child (valid with have_t)
  uint32_t gk;      // best triangle slot so far (kInvalidChild: none)
  float fbest;      // top frame's LOCAL best t
  float tnext;      // entry t of the next child (valid with have_t)
  float gbest;      // best t so far
  int32_t depth;    // frames on the stack, incl. the top one
  bool have_t;
};

// Frame ends by pruning handled per traversal iteration (1: one; the next
// iteration pops the ended frame; A/B switch)
#ifndef RT_MESH_PRUNE_PASSES
#define RT_MESH_PRUNE_PASSES 1
#endif

// Rays still looping in a wave at or below which the primary mesh path hands
// its remaining rays to 8-lane groups (mesh_run_coop).
#ifndef RT_COOP_RAYS
#define RT_COOP_RAYS 8  // A/B switch (0: never hand over)
#endif
constexpr int kCoopRays = RT_COOP_RAYS;
// Persistent primary-mesh waves still traversing a tile after this many
// iterations (a silhouette tile: the chains that end a launch) raise their
// issue priority on their SIMD until the tile is done (0: off; A/B switch)
#ifndef RT_HEAVY_PRIO
#define RT_HEAVY_PRIO 16
#endif
#ifndef RT_HEAVY_PRIO_LEVEL
#define RT_HEAVY_PRIO_LEVEL 3
#endif

// Primary mesh traversal (MAJ, mesh_primary_wave): an iteration whose lanes
// split between leaf tests and inner expansions runs only the side with more
// lanes -- the lanes of the side with fewer than 1/K as many wait one
// iteration, their visit order unchanged -- so the wave mostly runs one of the
// two branches per iteration instead of both. Modelled first on the CPU
// (tools/trav_sim.cpp, bunny 1080p: 38 % of the kernel's iterations ran both
// branches; waiting at K = 1 takes 14 % of the wave instructions for 15 % more
// iterations), then measured (section 4, round 6): bunny 10 x 2 0.0808 /
// 0.0800 -> 0.0777 / 0.0776, one frame 0.1806 -> 0.1594 / 0.1588 ms/frame. K =
// 2 was level; the shading kernels (MAJ off) were ~2 % slower with it.
// RT_MESH_MAJ = K (0: off everywhere; A/B switch).
#ifndef RT_MESH_MAJ
#define RT_MESH_MAJ 1
#endif
#ifndef RT_MESH_MAJ_DEN  // K = RT_MESH_MAJ / RT_MESH_MAJ_DEN
#define RT_MESH_MAJ_DEN 1
#endif

// The traversal loop. One iteration = one unit of this lane's work (expand a
// node, test a leaf, or resume/pop a frame). (Measured and rejected: the
// "while-while" split into an inner-node phase and a leaf phase: bunny
// 0.342 -> 0.523 ms.) TAIL: before each iteration, if kCoopRays or fewer lanes
// of the wave are still looping, store the state and return true (suspended).
template <int BLOCK, bool ANY, bool FAST, bool TAIL, uint32_t LB = RT_LEAF_BATCH, bool MAJ = false, class CT>
__device__ __forceinline__ bool mesh_run(const MeshDev &sc, f3 o, f3 d, f3 inv, float tNear, float tFar,
                                         LdsStack<BLOCK> st, MState &S, CT &cnt, int coop_rays = kCoopRays,
                                         int prio_iters = 0) {
  uint32_t word = S.word, flist = S.flist, fcnt = S.fcnt, fnode = S.fnode, cwnext = S.cwnext, gk = S.gk;
  float fbest = S.fbest, tnext = S.tnext, gbest = S.gbest;
  int depth = S.depth;
  bool have_t = S.have_t;
  bool suspended = false;
  int it = 0;  // wave-uniform iteration count (prio_iters)
  for (;;) {
    if (TAIL && __popcll(__ballot(1)) <= coop_rays) { suspended = true; break; }
    if (TAIL && prio_iters > 0) {
      it = __builtin_amdgcn_readfirstlane(it + 1);
      if (it == prio_iters) __builtin_amdgcn_s_setprio(RT_HEAVY_PRIO_LEVEL);
    }
#if RT_MESH_MAJ
    if constexpr (MAJ && !ANY) {
      // one branch per iteration where the lanes disagree by more than K to 1:
      // the minority side's lanes wait (their visit order is unchanged, only
      // later), so the wave runs the leaf test or the expansion, not both
      const bool isL = word != rtl::kInvalidChild && (word & rtl::kLeafBit);
      const bool isI = word != rtl::kInvalidChild && !(word & rtl::kLeafBit);
      const uint32_t nL = (uint32_t)__popcll(__ballot(isL)), nI = (uint32_t)__popcll(__ballot(isI));
      // wave-uniform: at most one side waits, so every iteration advances
      const bool waitL = nL * RT_MESH_MAJ < nI * RT_MESH_MAJ_DEN;
      const bool waitI = !waitL && nI * RT_MESH_MAJ < nL * RT_MESH_MAJ_DEN;
      if ((isL && waitL) || (isI && waitI)) continue;
    }
#endif
    if (word != rtl::kInvalidChild) {
      if (word & rtl::kLeafBit) {
        float lt = kInf;
        uint32_t lk = rtl::kInvalidChild;
        leaf_test<LB, FAST>(sc.tris, word, o, d, lt, lk, cnt);
        if (lk != rtl::kInvalidChild) {
          if (ANY) { gbest = lt; gk = lk; break; }
          if (lt < fbest) fbest = lt;
          if (lt < gbest) { gbest = lt; gk = lk; }
        }
      } else {
        uint32_t l, c, cwf;
        float tf;
        cnt.add(C_BVH_INNER, 1);
        expand_node<FAST>(mesh_node(sc, word), o, inv, tNear, tFar, l, c, tf, cwf);
        if (c != 0) {
          if (depth >= 1 && fcnt == 0) {
            // tail call: the top frame has no child left, so it is replaced,
            // not pushed; its best folds into the frame below now (that frame
            // reads it only when it resumes, after this whole subtree, and
            // min is associative: the same best as folding on return)
            if (depth >= 2) {
              const float below = __uint_as_float(st.at(depth - 2, 2));
              if (fbest < below) st.at(depth - 2, 2) = __float_as_uint(fbest);
            }
          } else {
            if (depth >= 1) {
              st.at(depth - 1, 0) = fnode;
              st.at(depth - 1, 1) = flist | (fcnt << 24);
              st.at(depth - 1, 2) = __float_as_uint(fbest);
            }
            ++depth;
          }
          fnode = word; flist = l; fcnt = c; fbest = kInf;
          tnext = tf;
          cwnext = cwf;
          have_t = true;
        }
      }
      word = rtl::kInvalidChild;
    }
    // choose the next child; a pruned child ends its frame, and up to
    // RT_MESH_PRUNE_PASSES - 1 such ends are popped in this same iteration
    bool done = false;
#pragma unroll
    for (int pass = 0; pass < RT_MESH_PRUNE_PASSES; ++pass) {
      if (depth == 0) { done = true; break; }
      if (fcnt == 0) {  // frame done: fold its best into the parent frame
        --depth;
        if (depth == 0) { done = true; break; }
        const float child_best = fbest;
        fnode = st.at(depth - 1, 0);
        const uint32_t lc = st.at(depth - 1, 1);
        flist = lc & 0xFFFFFFu;
        fcnt = lc >> 24;
        fbest = __uint_as_float(st.at(depth - 1, 2));
        if (child_best < fbest) fbest = child_best;
        have_t = false;
        // stacked frames always have a child left: go on to it
      }
      const uint32_t j = flist & 7u;
      flist >>= 3;
      fcnt -= 1;
      if (!have_t) {  // resumed frame: child box and word, loaded together
        const rtl::GNode *nd = mesh_node(sc, fnode);
        const float *b = nd->box[j];
        cwnext = nd->child[j];
        tnext = slab<FAST>(b[0], b[2], b[4], b[1], b[3], b[5], o, inv, tNear, tFar);
      }
      have_t = false;
      if (!(fbest < tnext)) { word = cwnext; break; }
      fcnt = 0;  // pruned; later siblings have larger t
    }
    if (done) break;
  }
  S.word = word; S.flist = flist; S.fcnt = fcnt; S.fnode = fnode; S.cwnext = cwnext; S.gk = gk;
  S.fbest = fbest; S.tnext = tnext; S.gbest = gbest; S.depth = depth; S.have_t = have_t;
  return suspended;
}

template <int BLOCK, bool ANY, bool FAST = false, class CT>
__device__ __forceinline__ bool mesh_continue(const MeshDev &sc, f3 o, f3 d, f3 inv, float tNear,
                                              float tFar, LdsStack<BLOCK> st, uint32_t word,
                                              uint32_t flist, uint32_t fcnt, float tnext,
                                              uint32_t cwnext, bool have_t, int depth,
                                              float &out_t, uint32_t &out_k, CT &cnt) {
  MState S{word, flist, fcnt, sc.root, cwnext, rtl::kInvalidChild, kInf, tnext, kInf, depth, have_t};
  mesh_run<BLOCK, ANY, FAST, false>(sc, o, d, inv, tNear, tFar, st, S, cnt);
  out_t = S.gbest;
  out_k = S.gk;
  return S.gk != rtl::kInvalidChild;
}

// ---- 8-lane groups: the cooperative tail of the primary mesh path ---------
// When at most kCoopRays rays of a wave are still traversing (the long,
// grazing ones that otherwise run alone on an idle wave), each gets a group of
// 8 lanes -- one DPP half-row, lanes 8g..8g+7, k = lane & 7 -- and the group
// runs the SAME traversal (same visiting order, same local-best pruning, same
// arithmetic) with the per-node work spread over its lanes: lane k slab-tests
// child k, the sort8 network runs across the lanes (its 19 comparators in 7
// layers, exchanged through DPP), and lane k tests triangle k of a leaf
// followed by a first-wins min reduction. Everything else (frame push/pop,
// resume, prune) is executed identically by the 8 lanes on the owner lane's
// LDS stack.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __uint_as_float(dpp_u<CTRL>(__float_as_uint(v)));
}
// DPP controls: quad_perm [1,0,3,2], [2,3,0,1], [0,2,1,3]; row_shl:n (lane i
// reads lane i+n) = 0x100+n, row_shr:n (lane i reads lane i-n) = 0x110+n.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppSwap12 = 0xD8;
template <int N> constexpr int kDppShl = 0x100 + N;
template <int N> constexpr int kDppShr = 0x110 + N;

// One comparator of sort8 seen from one of its two lanes: swap iff
// t[lower] > t[upper] (RTD_CSWAP), identical on both lanes.
__device__ __forceinline__ void grp_cswap(float &t, uint32_t &id, float pt, uint32_t pid, bool in,
                                          bool lower) {
  const bool sw = in && (lower ? (t > pt) : (pt > t));
  t = sw ? pt : t;
  id = sw ? pid : id;
}
// A comparator layer whose pairs are (k, k+N) for the lanes in it.
template <int N>
__device__ __forceinline__ void grp_layer_shift(float &t, uint32_t &id, bool in, bool lower) {
  const float tl = dpp_f<kDppShl<N>>(t), tr = dpp_f<kDppShr<N>>(t);
  const uint32_t il = dpp_u<kDppShl<N>>(id), ir = dpp_u<kDppShr<N>>(id);
  grp_cswap(t, id, lower ? tl : tr, lower ? il : ir, in, lower);
}
// sort8 (raytracing.hpp:188-213) over the group: lane k holds entry k.
__device__ __forceinline__ void grp_sort8(float &t, uint32_t &id, int k) {
  // (0,1)(2,3)(4,5)(6,7)
  grp_cswap(t, id, dpp_f<kDppXor1>(t), dpp_u<kDppXor1>(id), true, (k & 1) == 0);
  // (0,2)(1,3)(4,6)(5,7)
  grp_cswap(t, id, dpp_f<kDppXor2>(t), dpp_u<kDppXor2>(id), true, (k & 2) == 0);
  {  // (1,2)(5,6)(0,4)(3,7)
    const bool mid = k == 1 || k == 2 || k == 5 || k == 6;
    const float tq = dpp_f<kDppSwap12>(t), tl = dpp_f<kDppShl<4>>(t), tr = dpp_f<kDppShr<4>>(t);
    const uint32_t iq = dpp_u<kDppSwap12>(id), il = dpp_u<kDppShl<4>>(id), ir = dpp_u<kDppShr<4>>(id);
    const float pt = mid ? tq : (k < 4 ? tl : tr);
    const uint32_t pi = mid ? iq : (k < 4 ? il : ir);
    grp_cswap(t, id, pt, pi, true, mid ? (k == 1 || k == 5) : k < 4);
  }
  grp_layer_shift<4>(t, id, k == 1 || k == 2 || k == 5 || k == 6, k < 4);  // (1,5)(2,6)
  grp_layer_shift<3>(t, id, k == 1 || k == 3 || k == 4 || k == 6, k == 1 || k == 3);  // (1,4)(3,6)
  grp_layer_shift<2>(t, id, k >= 2 && k <= 5, k == 2 || k == 3);  // (2,4)(3,5)
  grp_layer_shift<1>(t, id, k == 3 || k == 4, k == 3);  // (3,4)
}
// Exchange with lane k^4 of the group.
__device__ __forceinline__ uint32_t grp_xor4_u(uint32_t v, int k) {
  const uint32_t l = dpp_u<kDppShl<4>>(v), r = dpp_u<kDppShr<4>>(v);
  return k < 4 ? l : r;
}
// Group-wide min of (t, k), ties to the lower k: the first triangle of a leaf
// with the smallest t, as the reference's strict `>` scan keeps it.
__device__ __forceinline__ void grp_min_first(float &t, uint32_t &kk, int k) {
  float pt;
  uint32_t pk;
  bool tk;
  pt = dpp_f<kDppXor1>(t); pk = dpp_u<kDppXor1>(kk);
  tk = pt < t || (pt == t && pk < kk); t = tk ? pt : t; kk = tk ? pk : kk;
  pt = dpp_f<kDppXor2>(t); pk = dpp_u<kDppXor2>(kk);
  tk = pt < t || (pt == t && pk < kk); t = tk ? pt : t; kk = tk ? pk : kk;
  pt = __uint_as_float(grp_xor4_u(__float_as_uint(t), k)); pk = grp_xor4_u(kk, k);
  tk = pt < t || (pt == t && pk < kk); t = tk ? pt : t; kk = tk ? pk : kk;
}
__device__ __forceinline__ uint32_t grp_or(uint32_t v, int k) {
  v |= dpp_u<kDppXor1>(v);
  v |= dpp_u<kDppXor2>(v);
  v |= grp_xor4_u(v, k);
  return v;
}

// mesh_run (non-ANY) executed by an 8-lane group on one ray; S is the same in
// all 8 lanes and stays so. st = the owner lane's LDS stack column.
template <int BLOCK, bool FAST>
__device__ __forceinline__ void mesh_run_coop(const MeshDev &sc, f3 o, f3 d, f3 inv, float tNear,
                                              float tFar, LdsStack<BLOCK> st, MState &S, int k) {
  uint32_t word = S.word, flist = S.flist, fcnt = S.fcnt, fnode = S.fnode, cwnext = S.cwnext, gk = S.gk;
  float fbest = S.fbest, tnext = S.tnext, gbest = S.gbest;
  int depth = S.depth;
  bool have_t = S.have_t;
  const int gbase = (threadIdx.x & 63) & ~7;
  for (;;) {
    if (word != rtl::kInvalidChild) {
      if (word & rtl::kLeafBit) {
        const uint32_t first = (word >> 3) & rtl::kMaxLeafFirstTri;
        const uint32_t n = (word & 7u) + 1u;
        float tk = kInf;
        if ((uint32_t)k < n) {
          const float4 *q = reinterpret_cast<const float4 *>(sc.tris + first + k);
          tk = tri_t<FAST>(q[0], q[1], q[2], o, d);
          if (!(tk < kInf)) tk = kInf;  // a NaN t never wins the strict scan
        }
        uint32_t kk = (uint32_t)k;
        grp_min_first(tk, kk, k);
        if (tk < kInf) {
          if (tk < fbest) fbest = tk;
          if (tk < gbest) { gbest = tk; gk = first + kk; }
        }
      } else {
        const rtl::GNode *nd = mesh_node(sc, word);
        const float2 *bp = reinterpret_cast<const float2 *>(nd->box[k]);
        const float2 bxx = bp[0], byy = bp[1], bzz = bp[2];  // (min, max) per axis
        const uint32_t cwk = nd->child[k];
        float t = slab<FAST>(bxx.x, byy.x, bzz.x, bxx.y, byy.y, bzz.y, o, inv, tNear, tFar);
        uint32_t id = (uint32_t)k;
        grp_sort8(t, id, k);
        // misses (-1) sort first; the entries to visit are the suffix from i0
        const uint32_t i0 = (uint32_t)__popcll((__ballot(t < 0.0f) >> gbase) & 0xFFull);
        const uint32_t c = 8u - i0;
        const uint32_t l = grp_or(t < 0.0f ? 0u : id << (3u * ((uint32_t)k - i0)), k);
        const float tf = __shfl(t, gbase + (int)(i0 & 7u), 64);
        const uint32_t idf = __shfl(id, gbase + (int)(i0 & 7u), 64);
        const uint32_t cwf = __shfl(cwk, gbase + (int)idf, 64);
        if (c != 0) {
          if (depth >= 1 && fcnt == 0) {  // tail call, as in mesh_run
            if (depth >= 2) {
              const float below = __uint_as_float(st.at(depth - 2, 2));
              if (fbest < below) st.at(depth - 2, 2) = __float_as_uint(fbest);
            }
          } else {
            if (depth >= 1) {
              st.at(depth - 1, 0) = fnode;
              st.at(depth - 1, 1) = flist | (fcnt << 24);
              st.at(depth - 1, 2) = __float_as_uint(fbest);
            }
            ++depth;
          }
          fnode = word; flist = l; fcnt = c; fbest = kInf;
          tnext = tf;
          cwnext = cwf;
          have_t = true;
        }
      }
      word = rtl::kInvalidChild;
    }
    if (depth == 0) break;
    if (fcnt == 0) {
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
    }
    const uint32_t j = flist & 7u;
    flist >>= 3;
    fcnt -= 1;
    if (!have_t) {
      const rtl::GNode *nd = mesh_node(sc, fnode);
      const float *b = nd->box[j];
      cwnext = nd->child[j];
      tnext = slab<FAST>(b[0], b[2], b[4], b[1], b[3], b[5], o, inv, tNear, tFar);
    }
    have_t = false;
    if (fbest < tnext) { fcnt = 0; continue; }
    word = cwnext;
  }
  S.gk = gk;
  S.gbest = gbest;
}

// Primary-ray mesh intersection for a whole wave (every lane of the wave must
// call it, with active = false for lanes without a pixel): each lane traverses
// its own ray until at most kCoopRays rays remain, then those finish in 8-lane
// groups. The result is the same as mesh_trace's, bit for bit.
template <int BLOCK>
__device__ __forceinline__ bool mesh_primary_wave(const MeshDev &sc, f3 o, f3 d, float tNear, float tFar,
                                                  bool active, uint32_t *stk_block, float &out_t,
                                                  uint32_t &out_k, int coop_rays = kCoopRays,
                                                  int prio_iters = 0) {
  if (prio_iters > 0) __builtin_amdgcn_s_setprio(0);  // a new tile starts at normal priority
  NoCnt cnt;
  const int lane = threadIdx.x & 63;
  LdsStack<BLOCK> st{stk_block + threadIdx.x};
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};  // 1.0f / rayDir (:273)
  // fast: the finite-1/d slab forms and the fast reciprocal (MeshDev::dmax2)
  const bool fast = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z) &&
                    dot(d, d) <= sc.dmax2;
  MState S{rtl::kInvalidChild, 0u, 0u, sc.root, rtl::kInvalidChild, rtl::kInvalidChild, kInf, 0.0f, kInf, 0,
           false};
  bool pending = false;
  if (active && sc.root != rtl::kInvalidChild) {
    if (sc.root & rtl::kLeafBit) {
      S.word = sc.root;
      pending = true;
    } else {
      uint32_t l, c, cwf;
      float tf;
      const bool entered = fast ? mesh_root<true>(sc, o, inv, tNear, tFar, l, c, tf, cwf, cnt)
                                : mesh_root<false>(sc, o, inv, tNear, tFar, l, c, tf, cwf, cnt);
      if (entered) {
        S.flist = l; S.fcnt = c; S.tnext = tf; S.cwnext = cwf; S.depth = 1; S.have_t = true;
        pending = true;
      }
    }
  }
  bool suspended = false;
  if (pending && sc.coop)
    suspended = fast ? mesh_run<BLOCK, false, true, true, RT_LEAF_BATCH_PRIMARY, true>(sc, o, d, inv, tNear, tFar, st, S,
                                                                                        cnt, coop_rays, prio_iters)
                     : mesh_run<BLOCK, false, false, true, RT_LEAF_BATCH_PRIMARY, true>(sc, o, d, inv, tNear, tFar, st, S,
                                                                                         cnt, coop_rays, prio_iters);
  else if (pending)
    (void)(fast ? mesh_run<BLOCK, false, true, false, RT_LEAF_BATCH_PRIMARY, true>(sc, o, d, inv, tNear, tFar, st, S, cnt)
                : mesh_run<BLOCK, false, false, false, RT_LEAF_BATCH_PRIMARY, true>(sc, o, d, inv, tNear, tFar, st, S, cnt));
  // Rays still traversing: at most kCoopRays per branch of the fast/exact
  // dispatch above (each branch suspends on its own lane count), so up to
  // 2 * kCoopRays; they are finished 8 at a time (one per 8-lane group; a
  // threshold above 8 means several rounds).
  uint64_t U = __ballot(suspended);  // wave-uniform
  while (U != 0) {
    uint64_t R = 0, rest = U;  // the lowest 8 rays of U
    for (int i = 0; i < 8 && rest != 0; ++i) {
      R |= rest & (~rest + 1ull);
      rest &= rest - 1ull;
    }
    U &= ~R;
    const int g = lane >> 3, k = lane & 7;
    const int n = __popcll(R);
    uint64_t m = R;
    for (int i = 0; i < g && i < n; ++i) m &= m - 1;
    const int owner = g < n ? (int)__builtin_ctzll(m) : lane;
    // gather the owner's ray and state (all 64 lanes active here)
    const f3 go{__shfl(o.x, owner, 64), __shfl(o.y, owner, 64), __shfl(o.z, owner, 64)};
    const f3 gd{__shfl(d.x, owner, 64), __shfl(d.y, owner, 64), __shfl(d.z, owner, 64)};
    const f3 ginv{__shfl(inv.x, owner, 64), __shfl(inv.y, owner, 64), __shfl(inv.z, owner, 64)};
    const float gtf = __shfl(tFar, owner, 64);
    const bool gfast = __shfl((int)fast, owner, 64) != 0;
    MState G;
    G.word = __shfl(S.word, owner, 64);
    G.flist = __shfl(S.flist, owner, 64);
    G.fcnt = __shfl(S.fcnt, owner, 64);
    G.fnode = __shfl(S.fnode, owner, 64);
    G.cwnext = __shfl(S.cwnext, owner, 64);
    G.gk = __shfl(S.gk, owner, 64);
    G.fbest = __shfl(S.fbest, owner, 64);
    G.tnext = __shfl(S.tnext, owner, 64);
    G.gbest = __shfl(S.gbest, owner, 64);
    G.depth = __shfl(S.depth, owner, 64);
    G.have_t = __shfl((int)S.have_t, owner, 64) != 0;
    if (g < n) {
      const LdsStack<BLOCK> gst{stk_block + (threadIdx.x & ~63) + owner};
      if (gfast)
        mesh_run_coop<BLOCK, true>(sc, go, gd, ginv, tNear, gtf, gst, G, k);
      else
        mesh_run_coop<BLOCK, false>(sc, go, gd, ginv, tNear, gtf, gst, G, k);
    }
    // each ray of this round takes the result of its group (group = rank of its bit in R)
    const int mg = __popcll(R & ((1ull << lane) - 1ull));
    const float rb = __shfl(G.gbest, (mg & 7) * 8, 64);
    const uint32_t rk = __shfl(G.gk, (mg & 7) * 8, 64);
    if ((R >> lane) & 1ull) { S.gbest = rb; S.gk = rk; }
  }
  out_t = S.gbest;
  out_k = S.gk;
  return S.gk != rtl::kInvalidChild;
}

template <int BLOCK, bool ANY, class CT>
__device__ __forceinline__ bool mesh_trace(const MeshDev &sc, f3 o, f3 d, float tNear, float tFar,
                                           LdsStack<BLOCK> st, float &out_t, uint32_t &out_k,
                                           CT &cnt) {
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};  // 1.0f / rayDir (:273)
  if (sc.root == rtl::kInvalidChild) return false;
  if (sc.root & rtl::kLeafBit)
    return mesh_continue<BLOCK, ANY>(sc, o, d, inv, tNear, tFar, st, sc.root, 0u, 0u, 0.0f,
                                     rtl::kInvalidChild, false, 0, out_t, out_k, cnt);
  uint32_t l, c, cwf;
  float tf;
  if (__builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z) &&
      dot(d, d) <= sc.dmax2) {  // (see mesh_primary_wave)
    if (!mesh_root<true>(sc, o, inv, tNear, tFar, l, c, tf, cwf, cnt)) return false;
    return mesh_continue<BLOCK, ANY, true>(sc, o, d, inv, tNear, tFar, st, rtl::kInvalidChild, l, c, tf,
                                           cwf, true, 1, out_t, out_k, cnt);
  }
  if (!mesh_root<false>(sc, o, inv, tNear, tFar, l, c, tf, cwf, cnt)) return false;
  return mesh_continue<BLOCK, ANY, false>(sc, o, d, inv, tNear, tFar, st, rtl::kInvalidChild, l, c, tf,
                                          cwf, true, 1, out_t, out_k, cnt);
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
//
// Device layouts (values are the reference's, bit for bit; only addresses
// change):
//  - linear: the reference's x-major array, index (x*sy + y)*sz + z. Grids
//    that fit one XCD's L2 (<= 4 MiB) keep it.
//  - bricked: 4x4x4 bricks of 256 B (two 128 B lines), bricks x-major like
//    the reference array, samples inside a brick (lx, ly, lz) at
//    lx*16 + ly*4 + lz. The x-major array puts the 2x2x2 taps of one
//    evaluation on 4 different lines (x and y neighbours are a plane / a row
//    apart), and a wave's footprint of k^3 cells on ~k^2 mostly unused lines;
//    a brick holds a 4^3 neighbourhood, so the same evaluations touch ~2.3
//    lines and neighbouring lanes and steps share them (256^3 grid, 1080p:
//    0.0646 -> 0.0507 ms per frame). The padding up to a multiple of 4 per
//    axis is never read (taps are at most size-1).
#ifndef RT_GRID_TAP_CACHE
#define RT_GRID_TAP_CACHE 1  // A/B switch: 0 reloads the 8 taps at every march step
#endif
#ifndef RT_GRID_MUL24
#define RT_GRID_MUL24 1  // A/B switch: 0 keeps 32-bit multiplies in the tap addressing
#endif
#ifndef RT_GRID_MARCH
#define RT_GRID_MARCH 1  // A/B switch: 1 the march as a one-exit loop (grid_march), 0 the two-exit form
#endif
constexpr uint32_t kBrick = 4;
constexpr uint64_t kGridLinearMaxBytes = 4ull << 20;
struct GridDev {
  const float *__restrict__ v;
  uint32_t sx, sy, sz;  // reference sizes
  uint32_t ys, xs;      // linear: sz, sy*sz; bricked: samples per brick step along y, x
  uint32_t bytes;       // buffer num_records: device bytes (<= 4 GiB, saturated), else 0
};

__host__ __device__ __forceinline__ uint32_t grid_bricks(uint32_t n) { return (n + kBrick - 1) / kBrick; }

// grid kernel modes: bit 0 = buffer loads with 32-bit byte offsets (else 64-bit
// addresses), bit 1 = bricked (else linear). Separate kernel instantiations,
// so the rare 64-bit path does not set the common one's register budget.
// (A per-wave LDS block cache of the march was built in round 4 and measured
// 2.8-5x slower; it was removed in round 5)
constexpr int kGridBuf = 1, kGridBricked = 2;

// a * b for sample offsets. In buffer mode both factors are below 2^24
// (grid_mode checks the strides) and the product below 2^30 (a sample
// offset in a < 4 GiB buffer), so the full-rate 24-bit multiply is exact;
// the 32-bit form compiles to the multi-pass v_mad_u64_u32, and the march is
// VALU-bound (four of them per sdf evaluation).
template <int kMode>
__device__ __forceinline__ uint32_t grid_mul(uint32_t a, uint32_t b) {
  if constexpr ((kMode & kGridBuf) != 0 && RT_GRID_MUL24) return __umul24(a, b);
  return a * b;
}
// sample offsets of coordinate i along each axis (their sum addresses sample (x, y, z))
template <int kMode>
__device__ __forceinline__ uint32_t grid_ox(const GridDev &g, uint32_t i) {
  if constexpr (kMode & kGridBricked) return grid_mul<kMode>(i >> 2, g.xs) + ((i & 3u) << 4);
  return grid_mul<kMode>(i, g.xs);
}
template <int kMode>
__device__ __forceinline__ uint32_t grid_oy(const GridDev &g, uint32_t i) {
  if constexpr (kMode & kGridBricked) return grid_mul<kMode>(i >> 2, g.ys) + ((i & 3u) << 2);
  return grid_mul<kMode>(i, g.ys);
}
template <int kMode>
__device__ __forceinline__ uint32_t grid_oz(uint32_t i) {
  if constexpr (kMode & kGridBricked) return ((i >> 2) << 6) + (i & 3u);
  return i;
}

// gfx9 buffer resource word 3 (raw dword access, no swizzle)
constexpr int kBufWord3 = 0x00020000;

// The 8 taps of one evaluation and the cell they belong to. The march keeps
// the last cell's taps: a step that lands in the same cell (the same c0 and
// c1 on every axis; near the surface steps are short) reuses them instead of
// reloading 8 values, so it costs only the weights and the trilinear sum.
// The values are the same samples, so the result is bitwise the same.
struct GridTaps {
  uint32_t i0x = 0xFFFFFFFFu, i0y = 0, i0z = 0, i1x = 0, i1y = 0, i1z = 0;
  float v[8];
};

template <int kMode>
__device__ __forceinline__ void grid_fetch(const GridDev &g, uint32_t i0x, uint32_t i0y, uint32_t i0z,
                                           uint32_t i1x, uint32_t i1y, uint32_t i1z, float v[8]) {
  // the 8 taps sdf(c0/c1 per axis) in the reference's order (grid_raytracing.cpp:41-49)
  const uint32_t x0 = grid_ox<kMode>(g, i0x), x1 = grid_ox<kMode>(g, i1x);
  const uint32_t y0 = grid_oy<kMode>(g, i0y), y1 = grid_oy<kMode>(g, i1y);
  const uint32_t z0 = grid_oz<kMode>(i0z), z1 = grid_oz<kMode>(i1z);
  const uint32_t o00 = x0 + y0, o01 = x0 + y1, o10 = x1 + y0, o11 = x1 + y1;
  if constexpr ((kMode & kGridBuf) != 0) {  // buffer loads: 32-bit byte offsets, no 64-bit address arithmetic
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.v), 0, (int)g.bytes, kBufWord3);
    v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o00 + z0) << 2, 0, 0));
    v[1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o00 + z1) << 2, 0, 0));
    v[2] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o01 + z0) << 2, 0, 0));
    v[3] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o01 + z1) << 2, 0, 0));
    v[4] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o10 + z0) << 2, 0, 0));
    v[5] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o10 + z1) << 2, 0, 0));
    v[6] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o11 + z0) << 2, 0, 0));
    v[7] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (o11 + z1) << 2, 0, 0));
  } else {
    const float *__restrict__ gv = g.v;
    v[0] = gv[(size_t)o00 + z0]; v[1] = gv[(size_t)o00 + z1]; v[2] = gv[(size_t)o01 + z0]; v[3] = gv[(size_t)o01 + z1];
    v[4] = gv[(size_t)o10 + z0]; v[5] = gv[(size_t)o10 + z1]; v[6] = gv[(size_t)o11 + z0]; v[7] = gv[(size_t)o11 + z1];
  }
}

// SDFGrid::sdf(float3) (grid_raytracing.cpp:7-62). CACHE: taps from / into tc.
template <int kMode, bool CACHE, class CT>
__device__ __forceinline__ float grid_sdf_t(const GridDev &g, f3 p, uint32_t *cell, GridTaps &tc, CT &cnt) {
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
  float v[8];
  if constexpr (CACHE) {
    if (!(i0x == tc.i0x && i0y == tc.i0y && i0z == tc.i0z && i1x == tc.i1x && i1y == tc.i1y && i1z == tc.i1z)) {
      grid_fetch<kMode>(g, i0x, i0y, i0z, i1x, i1y, i1z, tc.v);
      tc.i0x = i0x; tc.i0y = i0y; tc.i0z = i0z; tc.i1x = i1x; tc.i1y = i1y; tc.i1z = i1z;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tc.v[k];
  } else {
    grid_fetch<kMode>(g, i0x, i0y, i0z, i1x, i1y, i1z, v);
  }
  float res = 0.0f;
  res += v[0] * bx * by * bz;
  res += v[1] * bx * by * az;
  res += v[2] * bx * ay * bz;
  res += v[3] * bx * ay * az;
  res += v[4] * ax * by * bz;
  res += v[5] * ax * by * az;
  res += v[6] * ax * ay * bz;
  res += v[7] * ax * ay * az;
  if (cell) *cell = (i0x * g.sy + i0y) * g.sz + i0z;  // hit primitive: the c0 sample's reference index
  return res;
}

template <int kMode, class CT>
__device__ __forceinline__ float grid_sdf(const GridDev &g, f3 p, uint32_t *cell, CT &cnt) {
  GridTaps unused;
  return grid_sdf_t<kMode, false>(g, p, cell, unused, cnt);
}

template <int kMode, class CT>
__device__ __forceinline__ f3 grid_normal(const GridDev &g, f3 p, CT &cnt) {  // grid_raytracing.cpp:64-89
  const float E = 1e-3f;
  const float xl = (p.x - E >= -1.0f) ? p.x - E : p.x, xr = (p.x + E <= 1.0f) ? p.x + E : p.x;
  const float yl = (p.y - E >= -1.0f) ? p.y - E : p.y, yr = (p.y + E <= 1.0f) ? p.y + E : p.y;
  const float zl = (p.z - E >= -1.0f) ? p.z - E : p.z, zr = (p.z + E <= 1.0f) ? p.z + E : p.z;
  // one axis pair per iteration (not unrolled): 16 taps in flight instead of
  // 48 keeps the kernel's register peak at the march's, not the normal's
  float dx = 0.0f, dy = 0.0f, dz = 0.0f;
#pragma unroll 1
  for (int k = 0; k < 3; ++k) {
    const f3 pr{k == 0 ? xr : p.x, k == 1 ? yr : p.y, k == 2 ? zr : p.z};
    const f3 pl{k == 0 ? xl : p.x, k == 1 ? yl : p.y, k == 2 ? zl : p.z};
    const float dk = grid_sdf<kMode>(g, pr, nullptr, cnt) - grid_sdf<kMode>(g, pl, nullptr, cnt);
    dx = k == 0 ? dk : dx;
    dy = k == 1 ? dk : dy;
    dz = k == 2 ? dk : dz;
  }
  return normalize(f3{dx, dy, dz});
}

// ray status: still traversing (suspended), finished without a hit, with a hit
enum { RAY_PENDING = 0, RAY_MISS = 1, RAY_HIT = 2 };

// grid_raytracing.cpp:93-125. Returns hit and leaves the hit point in *hp.
template <int kMode, class CT>
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
  GridTaps tc;
#if RT_GRID_MARCH
  // One exit per step, as the octree's leaf march (oct_leaf): t advances by s
  // on every step (the reference returns t + s at a hit), the next point and
  // its in-box test are computed on the hit step too, and the hit point is
  // rebuilt after the loop from the t it was computed at, clamped as above
  // (the first step's point exactly; a later one passed the in-box test, so
  // the clamp leaves it -- at most a zero's sign, which grid_normal's p +- E
  // and the sdf's (p + 1) / 2 never see). The hit cell is the last step's c0
  // sample, read from the tap cache's key after the loop.
  // in the box: med3(q, -1, 1) == q on every axis (false for a NaN coordinate)
  auto inside = [](f3 q) {
    return clamp_med3(q.x, -1.0f, 1.0f) == q.x && clamp_med3(q.y, -1.0f, 1.0f) == q.y &&
           clamp_med3(q.z, -1.0f, 1.0f) == q.z;
  };
  constexpr bool kCache = RT_GRID_TAP_CACHE != 0;
  bool hit = false;
  float tp = t;
  if (inside(p)) {
    bool in;
    do {
      const float s = grid_sdf_t<kMode, kCache>(g, p, kCache ? nullptr : &cell, tc, cnt);
      hit = s < 1e-3f;
      tp = t;
      t += s;
      p = o + t * d;
      in = inside(p);
    } while (!hit && in);
  }
  if (hit) {
    out_t = t;
    hp = vstd_min(vstd_max(o + tp * d, f3{-1.0f, -1.0f, -1.0f}), f3{1.0f, 1.0f, 1.0f});
    if (kCache) cell = (tc.i0x * g.sy + tc.i0y) * g.sz + tc.i0z;
  }
  return hit;
#else
  while (p.x <= 1.0f && p.y <= 1.0f && p.z <= 1.0f && p.x >= -1.0f && p.y >= -1.0f && p.z >= -1.0f) {
    const float s = grid_sdf_t<kMode, RT_GRID_TAP_CACHE != 0>(g, p, &cell, tc, cnt);
    if (s < 1e-3f) {
      out_t = t + s;
      hp = p;
      return true;
    }
    t += s;
    p = o + t * d;
  }
  return false;
#endif
}

template <int kMode, class CT>
__device__ __forceinline__ Hit grid_intersect(const GridDev &g, f3 o, f3 d, float tNear, float tFar,
                                              CT &cnt) {
  Hit h = miss_hit();
  f3 p;
  uint32_t cell;
  if (grid_march<kMode>(g, o, d, tNear, tFar, h.t, p, cell, cnt)) {
    h.hit = true;
    h.n = grid_normal<kMode>(g, p, cnt);  // the normal's 6 evaluations load their taps
    h.prim = (int64_t)cell;
  } else {
    h.t = kInf;
  }
  return h;
}
template <int kMode, class CT>
__device__ __forceinline__ bool grid_occluded(const GridDev &g, f3 o, f3 d, float tNear, float tFar,
                                              CT &cnt) {
  float t;
  f3 p;
  uint32_t cell;
  return grid_march<kMode>(g, o, d, tNear, tFar, t, p, cell, cnt);
}

// SDFGrid::intersect (grid_raytracing.cpp:93-125) split for the ray pump
// (render_pump_kernel): grid_start is the box entry and the clamp of the first
// march point, grid_run the sphere march, which can suspend between two steps
// and continue later in the same lane. The state between steps is the
// reference's (t, p) pair; the tap cache is not carried over (a resumed step
// reloads its 8 taps: the same samples, the same bits).
struct GridRay {
  float t;
  f3 p;
};
__device__ __forceinline__ int grid_start(f3 o, f3 d, f3 inv, float tNear, float tFar, GridRay &R) {
  float t1, t2;
  bbox_intersection(f3{-1.0f, -1.0f, -1.0f}, f3{1.0f, 1.0f, 1.0f}, o, inv, tNear, tFar, t1, t2);
  if (t1 > t2) return RAY_MISS;
  f3 p = o + t1 * d;
  p = vstd_max(p, f3{-1.0f, -1.0f, -1.0f});
  p = vstd_min(p, f3{1.0f, 1.0f, 1.0f});
  R = GridRay{t1, p};
  return RAY_PENDING;
}
// SUSPEND: before each step, if `limit` or fewer lanes of the wave are still
// marching, save (t, p) and return RAY_PENDING.
template <int kMode, bool SUSPEND, class CT>
__device__ __forceinline__ int grid_run(const GridDev &g, f3 o, f3 d, GridRay &R, int limit, float &out_t,
                                        f3 &hp, CT &cnt) {
  float t = R.t;
  f3 p = R.p;
  GridTaps tc;
  uint32_t cell;
  while (p.x <= 1.0f && p.y <= 1.0f && p.z <= 1.0f && p.x >= -1.0f && p.y >= -1.0f && p.z >= -1.0f) {
    if (SUSPEND && __popcll(__ballot(1)) <= limit) {
      R = GridRay{t, p};
      return RAY_PENDING;
    }
    const float s = grid_sdf_t<kMode, RT_GRID_TAP_CACHE != 0>(g, p, &cell, tc, cnt);
    if (s < 1e-3f) {
      out_t = t + s;
      hp = p;
      return RAY_HIT;
    }
    t += s;
    p = o + t * d;
  }
  return RAY_MISS;
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
  const rtl::OctWord *__restrict__ node;  // child word + child masks (rt_layout.h)
  const rtl::OctVals *__restrict__ vals;
};
constexpr int kOctFields = 3;  // LDS words per octree frame: children block, list | count, leaf mask

__device__ __forceinline__ void oct_box(uint32_t ix, uint32_t iy, uint32_t iz, int depth, f3 &bmin,
                                        f3 &bmax, float &inv_s) {
  const float s = __builtin_ldexpf(2.0f, -depth);
  bmin = f3{-1.0f + (float)ix * s, -1.0f + (float)iy * s, -1.0f + (float)iz * s};
  bmax = f3{bmin.x + s, bmin.y + s, bmin.z + s};
  inv_s = __builtin_ldexpf(0.5f, depth);
}

struct OctCorners {
  float v[8];
};

// point = (p - boxMin) / (boxMax - boxMin), clamped to [1e-7, 0.9999999]
// (octree_raytracing.cpp:24-25). boxMax - boxMin is exactly the node size s, a
// power of two (exact dyadic box arithmetic), and x / 2^k == x * 2^-k bit for
// bit (both round the exact value once, subnormals included), so the three
// divisions become multiplications by inv_s = 1/s. p is finite here (a point
// inside the leaf box), so the clamp is one v_med3 per axis; after it
// floor(p) = 0 and ceil(p) = 1 on every axis, so p - c0 = p and c1 - p = 1 - p
// (the reference's subtractions with those operands, the same bits).
__device__ __forceinline__ void oct_local(f3 bmin, float inv_s, f3 p, f3 &a, f3 &b) {
  p = (p - bmin) * inv_s;
  p = f3{clamp_med3(p.x, 0.0000001f, 0.9999999f), clamp_med3(p.y, 0.0000001f, 0.9999999f),
         clamp_med3(p.z, 0.0000001f, 0.9999999f)};
  a = p;                                      // p_c0f = p - 0
  b = f3{1.0f - p.x, 1.0f - p.y, 1.0f - p.z};  // c1f_p = 1 - p
}

__device__ __forceinline__ float oct_sdf(const OctCorners &c, f3 bmin, float inv_s, f3 p) {
  f3 a, b;
  oct_local(bmin, inv_s, p, a, b);
  // octree_raytracing.cpp:36-55, values[(x<<2)+(y<<1)+z]: each term is
  // ((v * X) * Y) * Z, the reference's product order; the two terms that
  // differ only in Z (b.z / a.z) go through the packed-math unit together
  // (v2f: the same IEEE multiplies per element), and the sum keeps the
  // reference's order
  const v2f zz{b.z, a.z};
  const v2f t01 = v2f{c.v[0], c.v[1]} * b.x * b.y * zz;
  const v2f t23 = v2f{c.v[2], c.v[3]} * b.x * a.y * zz;
  const v2f t45 = v2f{c.v[4], c.v[5]} * a.x * b.y * zz;
  const v2f t67 = v2f{c.v[6], c.v[7]} * a.x * a.y * zz;
  // (the reference starts the sum from 0: 0 + x differs from x only for
  // x = -0, and then only in the sign of an all-zero sum, which the march
  // never sees -- s < 1e-4 either way, and t + s with t >= tNear > 0)
  float res = t01.x;
  res += t01.y;
  res += t23.x;
  res += t23.y;
  res += t45.x;
  res += t45.y;
  res += t67.x;
  res += t67.y;
  return res;
}

__device__ __forceinline__ f3 oct_normal(const OctCorners &c, f3 bmin, float inv_s, f3 p) {
  f3 a, b;
  oct_local(bmin, inv_s, p, a, b);
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

// intersectLeaf (octree_raytracing.cpp:122-164) for a leaf that may hit. The
// normal (nodeNormal, :60-118) is NOT evaluated here: a hit returns the march
// point, and oct_normal_at evaluates it after the traversal loop, where the
// stack state is dead -- the same arithmetic on the same values, outside the
// loop's register peak.
// FAST (1/d finite, tNear > 0): the box entry with hardware min/max and the
// start clamp as one v_med3 per axis (t1 is finite, so p is; the clamp's
// result differs from std's only in the sign of a zero coordinate, which the
// march's comparisons and oct_local's clamp never see).
// 1: the leaf march as a one-exit loop (A/B switch; 0 the two-exit form)
#ifndef RT_OCT_MARCH
#define RT_OCT_MARCH 1
#endif

// The box entry / exit of a node for FAST rays (bbox_intersection_fast), once
// per visit: the leaf march starts from them and the inner expansion's
// crossing-order path takes them as its P / Q (the same max / min of the same
// slab distances, in another order: max and min are exact). 0 otherwise.
template <bool FAST>
__device__ __forceinline__ void oct_entry(f3 bmin, f3 bmax, f3 o, f3 inv, float tNear, float tFar, float &P,
                                          float &Q) {
  P = 0.0f;
  Q = 0.0f;
  if constexpr (FAST) bbox_intersection_fast(bmin, bmax, o, inv, tNear, tFar, P, Q);
}

// P, Q: oct_entry's values (FAST; ignored otherwise)
template <bool FAST, class CT>
__device__ __forceinline__ bool oct_leaf(const OctDev &sc, uint32_t node, f3 bmin, f3 bmax,
                                         float inv_s, f3 o, f3 d, f3 inv, float tNear, float tFar,
                                         float P, float Q, float &out_t, f3 &out_p, CT &cnt) {
  float t1 = P, t2 = Q;
  if constexpr (!FAST) bbox_isect<FAST>(bmin, bmax, o, inv, tNear, tFar, t1, t2);
  if (t1 > t2) return false;
  OctCorners c;
  const float4 *q = reinterpret_cast<const float4 *>(sc.vals + node);
  const float4 a = q[0], b = q[1];
  c.v[0] = a.x; c.v[1] = a.y; c.v[2] = a.z; c.v[3] = a.w;
  c.v[4] = b.x; c.v[5] = b.y; c.v[6] = b.z; c.v[7] = b.w;
  float t = t1;
  f3 p = o + t * d;
  if constexpr (FAST) {
    p = f3{clamp_med3(p.x, bmin.x, bmax.x), clamp_med3(p.y, bmin.y, bmax.y), clamp_med3(p.z, bmin.z, bmax.z)};
  } else {
    p = vstd_max(p, bmin);
    p = vstd_min(p, bmax);
  }
  // p inside the box on every axis, as med3(p, min, max) == p: false for a NaN
  // coordinate, true exactly when min <= p <= max (3 med3 + 3 compares instead
  // of 6 compares and their mask ands)
  auto inside = [&](f3 q) {
    return clamp_med3(q.x, bmin.x, bmax.x) == q.x && clamp_med3(q.y, bmin.y, bmax.y) == q.y &&
           clamp_med3(q.z, bmin.z, bmax.z) == q.z;
  };
  // The march's state (t, p, s) is all the loop carries; the hit is read off
  // it after the loop, so no output is a loop-carried value (the outputs
  // written inside the loop made the compiler copy ~13 registers per step).
#if RT_OCT_MARCH
  // One exit per step: the reference returns t + s at a hit and continues
  // from t + s otherwise, so t advances on every step; the next point and
  // its in-box test are computed on the hit step too (unused there). The
  // point the hit was found at is rebuilt once after the loop from the t it
  // was computed from: o + tp * d, clamped to the box -- on the first step
  // that is the entry point as computed above, on a later one the clamp
  // leaves it as it is (that point passed the in-box test; at most a zero
  // coordinate's sign changes, which oct_local's clamp never sees). The
  // two-exit form (a break on the hit, the box test as the loop condition)
  // made the compiler carry the exit state in extra masks and copy t and p
  // through 8 v_mov per step.
  bool hit = false;
  float tp = t;
  // FAST: p is the med3 clamp of a finite point into the box, which the
  // in-box test (the same med3, compared) always passes
  if (FAST || inside(p)) {
    bool in;
    do {
      const float s = oct_sdf(c, bmin, inv_s, p);
      cnt.add(C_OCT_STEP, 1);
      hit = s < 1e-4f;
      tp = t;
      t += s;
      p = o + t * d;
      in = inside(p);
    } while (!hit && in);
  }
  if (hit) {
    out_t = t;
    const f3 q = o + tp * d;
    if constexpr (FAST) {
      out_p = f3{clamp_med3(q.x, bmin.x, bmax.x), clamp_med3(q.y, bmin.y, bmax.y), clamp_med3(q.z, bmin.z, bmax.z)};
    } else {
      out_p = vstd_min(vstd_max(q, bmin), bmax);
    }
  }
  return hit;
#else
  float s = 0.0f;
  bool in = inside(p);
  while (in) {
    s = oct_sdf(c, bmin, inv_s, p);
    cnt.add(C_OCT_STEP, 1);
    if (s < 1e-4f) break;  // hit: `in` stays true
    t += s;
    p = o + t * d;
    in = inside(p);
  }
  if (in) {
    out_t = t + s;
    out_p = p;
  }
  return in;
#endif
}

// Where a leaf march hit: the leaf (node index, integer box coordinates at
// its depth) and the march point, for nodeNormal after the traversal.
struct OctHitPt {
  f3 p;
  uint32_t node, ix, iy, iz;
  int32_t depth;
};
// nodeNormal at a hit (octree_raytracing.cpp:60-118): the leaf's corner
// values reloaded, its box rebuilt from the coordinates (exact dyadics, the
// same bits as during the march).
template <class CT>
__device__ __forceinline__ f3 oct_normal_at(const OctDev &sc, const OctHitPt &h, CT &cnt) {
  f3 bmin, bmax;
  float inv_s;
  oct_box(h.ix, h.iy, h.iz, h.depth, bmin, bmax, inv_s);
  OctCorners c;
  const float4 *q = reinterpret_cast<const float4 *>(sc.vals + h.node);
  const float4 a = q[0], b = q[1];
  c.v[0] = a.x; c.v[1] = a.y; c.v[2] = a.z; c.v[3] = a.w;
  c.v[4] = b.x; c.v[5] = b.y; c.v[6] = b.z; c.v[7] = b.w;
  cnt.add(C_OCT_NORMAL, 1);
  return oct_normal(c, bmin, inv_s, h.p);
}

// the entries of a sorted child list (oct_expand) whose bit is set in keep
__device__ __forceinline__ void oct_filter(uint32_t &list, uint32_t &cnt, uint32_t keep) {
  uint32_t out = 0, n = 0, l = list;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t id = l & 7u;
    if ((uint32_t)i < cnt && ((keep >> id) & 1u)) {
      out |= id << (3 * n);
      ++n;
    }
    l >>= 3;
  }
  list = out;
  cnt = n;
}

// 1: oct_expand takes the crossing-order path when it provably gives sort8's
// list (A/B switch; 0 always runs the 8-child slab test and sort8)
#ifndef RT_OCT_PATH
#define RT_OCT_PATH 1
#endif

// Expand an octree inner node: divide_box_8 + intersect_box_8 + sort8, keep
// entries with t > 0 (octree_raytracing.cpp:175-199), then only the children
// whose bit is set in `keep` (the child masks; 0xFF keeps all). The 8 child
// boxes have only 3 distinct bounds per axis (min, centre, max: centre + diff
// == max and min + diff == centre exactly), so the 24 slab distances of the
// reference are 9 distinct values, computed once each with the reference's
// operations.
//
// Crossing-order path (FAST, i.e. 1/d finite). Per axis the ray's interval in
// the half it meets first ("near") is [entry, s] and in the other [s, exit],
// s = the centre-plane distance, so a child's reference values are
//   tMin = max(P, s_a over its far axes), tMax = min(Q, s_a over its near axes)
// with P = max(the 3 entries, tNear), Q = min(the 3 exits, tFar) -- the same
// floats the reference's max/min chains select. With the three s strictly
// ordered s_1 < s_2 < s_3, a child whose far axes are not a prefix of that
// order has tMin >= s_b > s_a >= tMax for some pair, so it is never entered;
// the candidates are the 4 children met by flipping the axes in order of s.
// If the kept ones (t > 0) have strictly increasing t, every correct sort
// lists them in that order, so the result equals sort8's. Equal s values or
// equal kept t (a ray through a centre edge or entering on a centre plane)
// take the exact slab + sort8 path.
template <bool FAST>
__device__ __forceinline__ void oct_expand(f3 bmin, f3 bmax, f3 o, f3 inv, float tNear, float tFar,
                                           float P, float Q, uint32_t keep, uint32_t &list, uint32_t &cnt) {
  const f3 center{(bmin.x + bmax.x) / 2.0f, (bmin.y + bmax.y) / 2.0f, (bmin.z + bmax.z) / 2.0f};
  // divide_box_8's upper child max, center + (center - boxMin), IS bmax: every
  // value on the chain is an exact dyadic (oct_box), so the add is exact; the
  // slab distances below use bmax directly (the same operands, the same
  // bits), which the child visit's leaf test computes too
  const f3 hi = bmax;
  const float x0 = (bmin.x - o.x) * inv.x, x1 = (center.x - o.x) * inv.x, x2 = (hi.x - o.x) * inv.x;
  const float y0 = (bmin.y - o.y) * inv.y, y1 = (center.y - o.y) * inv.y, y2 = (hi.y - o.y) * inv.y;
  const float z0 = (bmin.z - o.z) * inv.z, z1 = (center.z - o.z) * inv.z, z2 = (hi.z - o.z) * inv.z;
  bool exact = !FAST || !RT_OCT_PATH;
  if constexpr (FAST && RT_OCT_PATH) {
    // near half per axis: 0 when the ray runs towards +axis (1/d > 0), else 1.
    // P = max(the 3 entries, tNear), Q = min(the 3 exits, tFar): oct_entry's
    // t1 / t2 (an entry is the smaller of an axis' two slab distances)
    const bool px = inv.x > 0.0f, py = inv.y > 0.0f, pz = inv.z > 0.0f;
    // the centre-plane distances in ascending order, with their child-id bits
    float s0 = x1, s1 = y1, s2 = z1;
    uint32_t b0 = 4u, b1 = 2u, b2 = 1u;
    auto cswap = [](float &sa, uint32_t &ba, float &sb, uint32_t &bb) {
      const bool sw = sb < sa;
      const float t = sa; sa = sw ? sb : sa; sb = sw ? t : sb;
      const uint32_t u = ba; ba = sw ? bb : ba; bb = sw ? u : bb;
    };
    cswap(s0, b0, s1, b1);
    cswap(s1, b1, s2, b2);
    cswap(s0, b0, s1, b1);
    // max / min of these finite values as the bare v_max_f32 / v_min_f32: the
    // same value, without the operand canonicalisation the compiler puts in
    // front of fmaxf / fminf (it cannot prove the selects' results canonical)
    const float k0 = P, k1 = vmax_f32(P, s0), k2 = vmax_f32(P, s1), k3 = vmax_f32(P, s2);
    const float m0 = vmin_f32(Q, s0), m1 = vmin_f32(Q, s1), m2 = vmin_f32(Q, s2), m3 = Q;
    // entered and kept: the reference's !(tMax < 0 || tMin > tMax) && t > 0;
    // with no NaN, k > 0 and k <= m imply m >= 0, and k >= P >= tNear > 0
    // (FAST rays have tNear > 0, oct_trace), so k <= m is the whole test
    const bool e0 = m0 >= k0, e1 = m1 >= k1;
    const bool e2 = m2 >= k2, e3 = m3 >= k3;
    // Ties among the kept entries: with s0 < s1 < s2, k_i = max(P, s_{i-1}) is
    // non-decreasing and k_i == k_{i+1} only when both are P, i.e. s_i <= P;
    // entry i also needs m_i = min(Q, s_i) >= k_i = P, so a tie of two kept
    // entries implies s_i == P. Testing s_i == P directly is therefore a
    // superset of the tie test (a spare exact expansion is still exact).
    exact = !(s0 < s1 && s1 < s2) || s0 == P || s1 == P || s2 == P;
    const uint32_t c0 = (px ? 0u : 4u) | (py ? 0u : 2u) | (pz ? 0u : 1u);
    const uint32_t c1 = c0 ^ b0, c2 = c1 ^ b1, c3 = c2 ^ b2;
    // pack from the back so the first visit ends in the low bits
    uint32_t l = 0, n = 0;
    if (e3 && ((keep >> c3) & 1u)) { l = c3; n = 1; }
    if (e2 && ((keep >> c2) & 1u)) { l = (l << 3) | c2; ++n; }
    if (e1 && ((keep >> c1) & 1u)) { l = (l << 3) | c1; ++n; }
    if (e0 && ((keep >> c0) & 1u)) { l = (l << 3) | c0; ++n; }
    list = l;
    cnt = n;
  }
  if (exact) {
    // per axis and half: (min, max) of the two slab distances, ISPC operand order
    // FAST (1/d finite, so no NaN operand): IEEE min/max equal ISPC's forms (see slab_fast)
    auto mn = [](float a, float b) { return FAST ? __builtin_fminf(a, b) : isp_min(a, b); };
    auto mx = [](float a, float b) { return FAST ? __builtin_fmaxf(a, b) : isp_max(a, b); };
    const float mnx[2] = {mn(x0, x1), mn(x1, x2)}, mxx[2] = {mx(x0, x1), mx(x1, x2)};
    const float mny[2] = {mn(y0, y1), mn(y1, y2)}, mxy[2] = {mx(y0, y1), mx(y1, y2)};
    const float mnz[2] = {mn(z0, z1), mn(z1, z2)}, mxz[2] = {mx(z0, z1), mx(z1, z2)};
    float t[8];
    uint32_t id[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int x = c >> 2, y = (c & 3) >> 1, z = c & 1;
      float tMin = mx(mnx[x], mx(mny[y], mnz[z]));
      float tMax = mn(mxx[x], mn(mxy[y], mxz[z]));
      tMin = mx(tMin, tNear);
      tMax = mn(tMax, tFar);
      t[c] = (tMax < 0.0f || tMin > tMax) ? -1.0f : tMin;
      id[c] = (uint32_t)c;
    }
    sort8(t, id);
    uint32_t l = 0, n = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      if (t[i] > 0.0f) {
        l = (l << 3) | id[i];
        n += 1;
      }
    }
    if (keep != 0xFFu) oct_filter(l, n, keep);
    list = l;
    cnt = n;
  }
}

// Traversal state of one octree ray below the root expansion: the top frame
// (the children block (childrenOffset) of the node whose children are being
// visited, its remaining list, the leaf mask of that block and its
// coordinates) lives here, the frames below it in LDS slots [0, sp-1]. A frame
// whose list is used up is not pushed (the descent into a block's last child
// is a tail call), so a frame records its depth, and a pop always finds a
// child to visit: it falls through to that visit in the same iteration.
// Frames keep the block, not the node, so visiting a child costs one dependent
// load (its word, or a leaf's corner values), not two. The state is
// resumable: oct_run can suspend a ray between two iterations and continue it
// later in the same lane (the ray pump, render_pump_kernel).
//
// Child masks (rtl::OctWord, the timed kernels; the counting variant, CT =
// LaneCnt, walks every child as the reference does, so its work units are the
// reference's): an inner node's sorted child list keeps only children whose
// subtree can produce a hit -- a skipped child is a leaf intersectLeaf rejects
// before marching (isEmpty() or every corner >= HIT_EPS,
// octree_raytracing.cpp:125-133) or an inner node with only such leaves below
// it, whose recursion returns false for every ray, so the first child that
// hits is the same -- and a child flagged as a leaf that can hit is marched
// straight away, without loading its word.
// Integer box coordinates of the top frame's node in the traversal loop.
// PACK (trees of depth <= 10, which is every tree of up to 7 stack slots): x,
// y, z in 10-bit fields of one register -- a child is the parent shifted left
// by one with the child-id bits or'ed in, a pop shifts right and masks -- so
// the loop carries one register instead of three. Otherwise three words.
template <bool PACK>
struct OctXYZ {
  uint32_t x, y, z;
  __device__ __forceinline__ OctXYZ(uint32_t ix, uint32_t iy, uint32_t iz) : x(ix), y(iy), z(iz) {}
  __device__ __forceinline__ OctXYZ child(uint32_t j) const {
    return OctXYZ((x << 1) | (j >> 2), (y << 1) | ((j >> 1) & 1u), (z << 1) | (j & 1u));
  }
  __device__ __forceinline__ void up(uint32_t sh) { x >>= sh; y >>= sh; z >>= sh; }
  __device__ __forceinline__ uint32_t ix() const { return x; }
  __device__ __forceinline__ uint32_t iy() const { return y; }
  __device__ __forceinline__ uint32_t iz() const { return z; }
};
template <>
struct OctXYZ<true> {
  uint32_t w;  // x | y << 10 | z << 20
  __device__ __forceinline__ OctXYZ(uint32_t ix, uint32_t iy, uint32_t iz) : w(ix | (iy << 10) | (iz << 20)) {}
  __device__ __forceinline__ explicit OctXYZ(uint32_t packed, int) : w(packed) {}
  __device__ __forceinline__ OctXYZ child(uint32_t j) const {
    return OctXYZ((w << 1) | (j >> 2) | (((j >> 1) & 1u) << 10) | ((j & 1u) << 20), 0);
  }
  __device__ __forceinline__ void up(uint32_t sh) {
    const uint32_t m = 0x3FFu >> sh;
    w = (w >> sh) & (m | (m << 10) | (m << 20));
  }
  __device__ __forceinline__ uint32_t ix() const { return w & 0x3FFu; }
  __device__ __forceinline__ uint32_t iy() const { return (w >> 10) & 0x3FFu; }
  __device__ __forceinline__ uint32_t iz() const { return w >> 20; }
};

struct OctRay {
  uint32_t fbase;
  uint32_t lc;  // remaining child ids (3 bits each, next in the low bits) | count << 24
  uint32_t leafm;  // children of the top frame that are leaves that can hit (masked walk)
  uint32_t ix, iy, iz;
  int32_t depth;  // depth of the top frame's node (root = 0)
  int32_t sp;     // frames on the LDS stack
};

// SDFOctree::intersect -> intersectNode(0) (octree_raytracing.cpp:166-208), root stage.
template <bool FAST, class CT>
__device__ __forceinline__ int oct_start(const OctDev &sc, f3 o, f3 d, f3 inv, float tNear, float tFar,
                                         OctRay &R, float &out_t, OctHitPt &hp, CT &cnt) {
  const rtl::OctWord rw = sc.node[0];
  const uint32_t root = rw.child;
  cnt.add(C_OCT_NODE, 1);
  if (root == 0 || root == rtl::kOctNeverHits) {
    cnt.add(C_OCT_LEAF, 1);
    if (root == rtl::kOctNeverHits) return RAY_MISS;
    float lt, P, Q;
    f3 lp;
    oct_entry<FAST>(f3{-1.0f, -1.0f, -1.0f}, f3{1.0f, 1.0f, 1.0f}, o, inv, tNear, tFar, P, Q);
    if (!oct_leaf<FAST>(sc, 0, f3{-1.0f, -1.0f, -1.0f}, f3{1.0f, 1.0f, 1.0f}, 0.5f, o, d, inv, tNear, tFar, P, Q,
                        lt, lp, cnt))
      return RAY_MISS;
    out_t = lt;
    hp.p = lp;
    hp.node = 0; hp.ix = 0; hp.iy = 0; hp.iz = 0; hp.depth = 0;
    return RAY_HIT;
  }
  f3 bmin, bmax;
  float inv_s;
  oct_box(0, 0, 0, 0, bmin, bmax, inv_s);
  uint32_t l, c;
  float P, Q;
  oct_entry<FAST>(bmin, bmax, o, inv, tNear, tFar, P, Q);
  oct_expand<FAST>(bmin, bmax, o, inv, tNear, tFar, P, Q, CT::kCounts ? 0xFFu : (rw.masks & 0xFFu), l, c);
  R = OctRay{root, l | (c << 24), rw.masks >> 8, 0u, 0u, 0u, 0, 0};
  return c == 0 ? RAY_MISS : RAY_PENDING;
}

// The front-to-back loop of intersectNode below the root. SUSPEND: before each
// iteration, if `limit` or fewer lanes of the wave are still in the loop, save
// the state and return RAY_PENDING.
// Octree loop iterations whose lanes split between leaf marches and inner
// expansions run only the side with more lanes (the others keep their chosen
// child pending for the next iteration, their visit order unchanged), as the
// mesh's primary loop does (RT_MESH_MAJ). 0: off (A/B switch).
#ifndef RT_OCT_MAJ
#define RT_OCT_MAJ 0
#endif

template <int BLOCK, bool FAST, bool SUSPEND, bool PACK, class CT>
__device__ __forceinline__ int oct_run(const OctDev &sc, f3 o, f3 d, f3 inv, float tNear, float tFar,
                                       LdsStack<BLOCK, kOctFields> st, OctRay &R, int limit, float &out_t,
                                       OctHitPt &hp, CT &cnt) {
  constexpr bool MASKS = !CT::kCounts;
  constexpr bool MAJ = RT_OCT_MAJ && MASKS && !SUSPEND;
  uint32_t fbase = R.fbase, flist = R.lc & 0xFFFFFFu, fcnt = R.lc >> 24, leafm = R.leafm;
  OctXYZ<PACK> xyz(R.ix, R.iy, R.iz);
  int depth = R.depth, sp = R.sp;
  uint32_t pj = 8;  // MAJ: the chosen child not visited yet (8: none)
  for (;;) {
    if (SUSPEND && __popcll(__ballot(1)) <= limit) {
      R = OctRay{fbase, flist | (fcnt << 24), leafm, xyz.ix(), xyz.iy(), xyz.iz(), depth, sp};
      return RAY_PENDING;
    }
    if (!MAJ || pj == 8) {
      if (fcnt == 0) {
        if (sp == 0) return RAY_MISS;
        --sp;
        fbase = st.at(sp, 0);
        const uint32_t lc = st.at(sp, 1);
        const uint32_t w2 = st.at(sp, 2);  // leaf mask | depth << 8
        if (MASKS) leafm = w2 & 0xFFu;
        const int d2 = (int)(w2 >> 8);
        xyz.up((uint32_t)(depth - d2));
        depth = d2;
        flist = lc & 0xFFFFFFu;
        fcnt = lc >> 24;  // >= 1: empty frames are never pushed
      }
      pj = flist & 7u;
      flist >>= 3;
      fcnt -= 1;
    }
    const uint32_t j = pj;
    if constexpr (MAJ) {
      const bool lf = (leafm >> j) & 1u;
      const uint32_t nL = (uint32_t)__popcll(__ballot(lf)), nI = (uint32_t)__popcll(__ballot(!lf));
      if (lf ? nL < nI : nI < nL) continue;  // wait: j stays pending
    }
    pj = 8;
    const uint32_t cn = fbase + j;
    const OctXYZ<PACK> cxyz = xyz.child(j);
    rtl::OctWord cw{0u, 0u};
    bool leaf;
    if (MASKS) {
      leaf = (leafm >> j) & 1u;  // a leaf that can hit: no word to load
      if (!leaf) cw = sc.node[cn];
    } else {
      cw = sc.node[cn];
      cnt.add(C_OCT_NODE, 1);
      if (cw.child == rtl::kOctNeverHits) { cnt.add(C_OCT_LEAF, 1); continue; }
      leaf = cw.child == 0;
    }
    f3 bmin, bmax;
    float inv_s;
    oct_box(cxyz.ix(), cxyz.iy(), cxyz.iz(), depth + 1, bmin, bmax, inv_s);
    // the box entry / exit, shared by the leaf and the inner-node paths (a
    // wave whose lanes take both computes it once)
    float P, Q;
    oct_entry<FAST>(bmin, bmax, o, inv, tNear, tFar, P, Q);
    if (leaf) {
      cnt.add(C_OCT_LEAF, 1);
      float lt;
      f3 lp;
      if (oct_leaf<FAST>(sc, cn, bmin, bmax, inv_s, o, d, inv, tNear, tFar, P, Q, lt, lp, cnt)) {
        out_t = lt;
        hp.p = lp;
        hp.node = cn; hp.ix = cxyz.ix(); hp.iy = cxyz.iy(); hp.iz = cxyz.iz(); hp.depth = depth + 1;
        return RAY_HIT;
      }
      continue;
    }
    uint32_t l, c;
    oct_expand<FAST>(bmin, bmax, o, inv, tNear, tFar, P, Q, MASKS ? (cw.masks & 0xFFu) : 0xFFu, l, c);
    if (c == 0) continue;
    if (fcnt != 0) {
      st.at(sp, 0) = fbase;
      st.at(sp, 1) = flist | (fcnt << 24);
      st.at(sp, 2) = (MASKS ? leafm : 0u) | ((uint32_t)depth << 8);
      ++sp;
    }
    ++depth;
    fbase = cw.child; flist = l; fcnt = c;
    leafm = cw.masks >> 8;
    xyz = cxyz;
  }
}

template <int BLOCK, bool NEED_NORMAL, bool FAST, bool PACK, class CT>
__device__ __forceinline__ bool oct_trace_t(const OctDev &sc, f3 o, f3 d, f3 inv, float tNear,
                                            float tFar, LdsStack<BLOCK, kOctFields> st, float &out_t, f3 &out_n,
                                            uint32_t &out_node, CT &cnt) {
  OctRay R;
  OctHitPt hp;
  int s = oct_start<FAST>(sc, o, d, inv, tNear, tFar, R, out_t, hp, cnt);
  if (s == RAY_PENDING) s = oct_run<BLOCK, FAST, false, PACK>(sc, o, d, inv, tNear, tFar, st, R, 0, out_t, hp, cnt);
  if (s != RAY_HIT) return false;
  out_node = hp.node;
  if (NEED_NORMAL) out_n = oct_normal_at(sc, hp, cnt);
  return true;
}

template <int BLOCK, bool NEED_NORMAL, bool PACK, class CT>
__device__ __forceinline__ bool oct_trace(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                          LdsStack<BLOCK, kOctFields> st, float &out_t, f3 &out_n,
                                          uint32_t &out_node, CT &cnt) {
  const f3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
  // FAST: every 1/d finite and tNear > 0 (the render paths' 0.01;
  // rt_intersect_rays callers may pass any tNear)
  if (__builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z) && tNear > 0.0f)
    return oct_trace_t<BLOCK, NEED_NORMAL, true, PACK>(sc, o, d, inv, tNear, tFar, st, out_t, out_n, out_node, cnt);
  return oct_trace_t<BLOCK, NEED_NORMAL, false, PACK>(sc, o, d, inv, tNear, tFar, st, out_t, out_n, out_node, cnt);
}

template <int BLOCK, bool PACK, class CT>
__device__ __forceinline__ Hit oct_intersect(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                             LdsStack<BLOCK, kOctFields> st, CT &cnt) {
  Hit h = miss_hit();
  uint32_t node;
  if (oct_trace<BLOCK, true, PACK>(sc, o, d, tNear, tFar, st, h.t, h.n, node, cnt)) {
    h.hit = true;
    h.prim = (int64_t)node;
  } else {
    h.t = kInf;
  }
  return h;
}
template <int BLOCK, bool PACK, class CT>
__device__ __forceinline__ bool oct_occluded(const OctDev &sc, f3 o, f3 d, float tNear, float tFar,
                                             LdsStack<BLOCK, kOctFields> st, CT &cnt) {
  float t;
  f3 n;
  uint32_t node;
  return oct_trace<BLOCK, false, PACK>(sc, o, d, tNear, tFar, st, t, n, node, cnt);
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
