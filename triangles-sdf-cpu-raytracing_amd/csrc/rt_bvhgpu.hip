// rt_bvhgpu.hip -- BVHBuilder::perform (triangles_raytracing.cpp:12-258) on the
// GPU: the SAME tree as the host build (rt_host.cpp build_bvh8), bit for bit.
//
// The tree depends on the order std::sort leaves triangles with equal keys
// (their bbox max on the split axis; triangles sharing a vertex tie), so the
// device sort replicates libstdc++'s introsort exactly instead of using a
// radix or merge sort:
//  * a segment longer than kSerialMax is partitioned by the whole grid: the
//    median of three moves to the front (std::__move_median_to_first), and
//    the unguarded Hoare partition is evaluated in parallel: the k-th swap
//    pairs the k-th element >= pivot from the left with the k-th element <=
//    pivot from the right while they have not crossed, so ranks from two
//    prefix sums (rounds of global scans) give every swap and the cut at once;
//  * shorter segments run libstdc++'s introsort loop (heapsort at depth 0)
//    and the final insertion sort in one thread each;
//  * the final insertion sort never moves an element across a partition
//    boundary, so sorting each leaf segment separately gives the same order.
// The SAH sweeps (triangles_raytracing.cpp:53-98) cut every (candidate, axis)
// range into chunks of 2048 triangles, one workgroup each: chunk unions, their
// prefix / suffix per range, then each chunk's right boxes (reverse scan),
// left boxes (forward scan), costs and first minimum. The breadth-first
// candidate queue of createNode (:155-225, at most 7 splits) is driven from
// the host, one candidate layer of every open node per stage; candidates the
// reference never reaches once a node has 7 splits are evaluated
// speculatively and rolled back (their range restored), because tryDivide
// re-sorts its range even when it does not split.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtamd.h"
#include "rt_error.h"
#include "rt_host.h"
#include "rt_layout.h"

namespace {

#ifndef RT_SERIAL_MAX
#define RT_SERIAL_MAX 256  // A/B switch
#endif
constexpr uint32_t kSerialMax = RT_SERIAL_MAX;  // segments at most this long: one wave, serial introsort in LDS
constexpr int kScanT = 256, kScanI = 8, kScanBlk = kScanT * kScanI;

struct Seg {
  uint32_t first, last;  // position range in the 3n-element space (axis a: [a*n, (a+1)*n))
  int32_t depth;         // remaining introsort depth
  uint32_t pad;
};

// ---- libstdc++'s sort algorithms --------------------------------------------
// On an LDS array of (key, id) pairs compared by key: moving the pairs is
// moving the ids std::sort moves, so the permutation is the same.
struct KI {
  float k;
  uint32_t id;
};
__device__ __forceinline__ bool lt(const KI &a, const KI &b) { return a.k < b.k; }
__device__ __forceinline__ void d_swap(KI *a, KI *b) {
  const KI t = *a;
  *a = *b;
  *b = t;
}
// std::__insertion_sort
__device__ void d_insertion(KI *first, KI *last) {
  if (first == last) return;
  for (KI *i = first + 1; i != last; ++i) {
    const KI v = *i;
    if (lt(v, *first)) {
      for (KI *j = i; j != first; --j) *j = *(j - 1);
      *first = v;
    } else {  // std::__unguarded_linear_insert
      KI *l = i, *nx = i - 1;
      while (lt(v, *nx)) {
        *l = *nx;
        l = nx;
        --nx;
      }
      *l = v;
    }
  }
}
// std::__move_median_to_first
template <class T, class LT>
__device__ void d_median_to_first(T *r, T *a, T *b, T *c, LT less) {
  auto sw = [](T *x, T *y) {
    const T t = *x;
    *x = *y;
    *y = t;
  };
  if (less(*a, *b)) {
    if (less(*b, *c)) sw(r, b);
    else if (less(*a, *c)) sw(r, c);
    else sw(r, a);
  } else if (less(*a, *c)) sw(r, a);
  else if (less(*b, *c)) sw(r, c);
  else sw(r, b);
}
// std::__unguarded_partition
__device__ KI *d_partition(KI *first, KI *last, KI *pivot) {
  for (;;) {
    while (lt(*first, *pivot)) ++first;
    --last;
    while (lt(*pivot, *last)) --last;
    if (!(first < last)) return first;
    d_swap(first, last);
    ++first;
  }
}
// std::__adjust_heap (with std::__push_heap), on elements of type T
template <class T, class LT>
__device__ void d_adjust_heap(T *first, int64_t hole, int64_t len, T value, LT less) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (less(first[child], first[child - 1])) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  int64_t parent = (hole - 1) / 2;
  while (hole > top && less(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}
// std::__partial_sort(first, last, last): std::__make_heap, then std::__sort_heap
template <class T, class LT>
__device__ void d_heapsort(T *first, T *last, LT less) {
  const int64_t len = last - first;
  if (len >= 2) {
    for (int64_t parent = (len - 2) / 2;; --parent) {
      d_adjust_heap(first, parent, len, first[parent], less);
      if (parent == 0) break;
    }
  }
  while (last - first > 1) {  // std::__pop_heap(first, last - 1, last - 1)
    --last;
    const T v = *last;
    *last = *first;
    d_adjust_heap(first, 0, last - first, v, less);
  }
}
// std::__introsort_loop; the recursion on the right part on a stack in LDS
// (one entry per level descended: at most the initial depth limit, <= 62)
__device__ void d_introsort(KI *base, uint32_t len, int depth, uint32_t *stk) {
  uint32_t f = 0, l = len;
  int sp = 0;
  for (;;) {
    while (l - f > 16) {
      if (depth == 0) {
        d_heapsort(base + f, base + l, [](const KI &a, const KI &b) { return a.k < b.k; });
        break;
      }
      --depth;
      KI *first = base + f, *last = base + l;
      KI *mid = first + (last - first) / 2;
      d_median_to_first(first, first + 1, mid, last - 1, [](const KI &a, const KI &b) { return a.k < b.k; });
      const uint32_t cut = (uint32_t)(d_partition(first + 1, last, first) - base);
      stk[sp++] = (cut << 16) | l;  // positions < 2^16 (kSerialMax)
      stk[sp++] = (uint32_t)depth;
      l = cut;
    }
    if (sp == 0) break;
    depth = (int)stk[--sp];
    const uint32_t w = stk[--sp];
    f = w >> 16;
    l = w & 0xFFFFu;
  }
}

// one wave per short segment (<= kSerialMax): (key, id) pairs staged in LDS,
// the rest of the introsort and the final insertion sort by lane 0
__global__ __launch_bounds__(64) void k_serial(const Seg *segs, uint32_t *ids, const float *K3, uint32_t n) {
  __shared__ KI a[kSerialMax];
  __shared__ uint32_t stk[2 * 64];
  const Seg s = segs[blockIdx.x];
  const float *K = K3 + (size_t)(s.first / n) * n;
  const uint32_t len = s.last - s.first;
  if (len > kSerialMax) {  // a long segment whose depth ran out (k_prep): heapsort in place
    if (threadIdx.x == 0)
      d_heapsort(ids + s.first, ids + s.last, [K](uint32_t x, uint32_t y) { return K[x] < K[y]; });
    return;  // sorted: the final insertion sort leaves it unchanged
  }
  for (uint32_t i = threadIdx.x; i < len; i += 64) {
    const uint32_t id = ids[s.first + i];
    a[i] = KI{K[id], id};
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    d_introsort(a, len, s.depth, stk);
    d_insertion(a, a + len);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < len; i += 64) ids[s.first + i] = a[i].id;
}

// ---- inclusive scan of u32 (three launches) --------------------------------
// blockIdx.y (k_scan1, k_scan3) / blockIdx.x (k_scan2) selects one of two
// independent arrays, so the partition round's two flag scans share launches
struct ScanPair {
  const uint32_t *in[2];
  uint32_t *out[2];
  uint32_t *bsum[2];
};
__global__ __launch_bounds__(kScanT) void k_scan1(ScanPair sp, uint32_t n) {
  const uint32_t *in = sp.in[blockIdx.y];
  uint32_t *out = sp.out[blockIdx.y], *bsum = sp.bsum[blockIdx.y];
  __shared__ uint32_t sm[kScanT];
  const uint32_t base = blockIdx.x * kScanBlk + threadIdx.x * kScanI;
  uint32_t v[kScanI], acc = 0;
#pragma unroll
  for (int k = 0; k < kScanI; ++k) {
    acc += (base + k < n) ? in[base + k] : 0u;
    v[k] = acc;
  }
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 1; o < kScanT; o <<= 1) {
    const uint32_t x = threadIdx.x >= (uint32_t)o ? sm[threadIdx.x - o] : 0u;
    __syncthreads();
    sm[threadIdx.x] += x;
    __syncthreads();
  }
  const uint32_t ex = threadIdx.x ? sm[threadIdx.x - 1] : 0u;
#pragma unroll
  for (int k = 0; k < kScanI; ++k)
    if (base + k < n) out[base + k] = v[k] + ex;
  if (threadIdx.x == kScanT - 1) bsum[blockIdx.x] = sm[kScanT - 1];
}
__global__ __launch_bounds__(1024) void k_scan2(ScanPair sp, uint32_t nb) {
  uint32_t *bsum = sp.bsum[blockIdx.x];
  __shared__ uint32_t sm[1024];
  const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nb) acc += bsum[b0 + k];
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t x = threadIdx.x >= (uint32_t)o ? sm[threadIdx.x - o] : 0u;
    __syncthreads();
    sm[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? sm[threadIdx.x - 1] : 0u;
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nb) {
      run += bsum[b0 + k];
      bsum[b0 + k] = run;
    }
}
__global__ __launch_bounds__(kScanT) void k_scan3(ScanPair sp, uint32_t n) {
  uint32_t *out = sp.out[blockIdx.y];
  const uint32_t *bsum = sp.bsum[blockIdx.y];
  if (blockIdx.x == 0) return;
  const uint32_t add = bsum[blockIdx.x - 1], base = blockIdx.x * kScanBlk + threadIdx.x * kScanI;
#pragma unroll
  for (int k = 0; k < kScanI; ++k)
    if (base + k < n) out[base + k] += add;
}

// ---- one round of parallel introsort partitions ----------------------------
// per segment: median to the front, pivot key, size (0: depth exhausted, the
// segment goes to the serial list, whose introsort loop heapsorts it)
__global__ void k_prep(const Seg *segs, uint32_t m, uint32_t *ids, const float *K3, uint32_t n, float *kp,
                       uint32_t *size, Seg *serial, uint32_t *nserial) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const Seg s = segs[i];
  if (s.depth == 0) {
    serial[atomicAdd(nserial, 1u)] = s;
    size[i] = 0;
    return;
  }
  const float *K = K3 + (size_t)(s.first / n) * n;
  uint32_t *f = ids + s.first, *l = ids + s.last;
  d_median_to_first(f, f + 1, f + (l - f) / 2, l - 1, [K](uint32_t x, uint32_t y) { return K[x] < K[y]; });
  kp[i] = K[*f];
  size[i] = s.last - s.first;
}

__device__ __forceinline__ uint32_t seg_of(const uint32_t *offs, uint32_t m, uint32_t v) {
  uint32_t lo = 0, hi = m;  // largest i with offs[i] <= v
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (offs[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// flags over the active elements (virtual index v, segments back to back):
// a = stops the left scan of the partition (!(key < pivot), the pivot itself
// excluded), b = stops the right scan (!(pivot < key), the pivot included)
__global__ void k_flags(const Seg *segs, const uint32_t *offs, uint32_t m, const uint32_t *ids, const float *K3,
                        uint32_t n, const float *kp, uint32_t *af, uint32_t *bf, uint32_t *segv, uint32_t E) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= E || v >= offs[m]) return;  // E: host bound; offs[m]: elements of this round
  const uint32_t i = seg_of(offs, m, v);
  const Seg s = segs[i];
  const uint32_t p = s.first + (v - offs[i]);
  const float *K = K3 + (size_t)(s.first / n) * n;
  const float k = K[ids[p]], pk = kp[i];
  af[v] = (p != s.first && !(k < pk)) ? 1u : 0u;
  bf[v] = (p == s.first || !(pk < k)) ? 1u : 0u;
  segv[v] = i;
}

// ranks of the a-elements from the left and the b-elements from the right,
// scattered into per-segment position lists L, R (v-space, offs[i] + rank - 1)
__global__ void k_ranks(const Seg *segs, const uint32_t *offs, uint32_t m, const uint32_t *af, const uint32_t *bf,
                        const uint32_t *Ai, const uint32_t *Bi, const uint32_t *segv, uint32_t *Lpos,
                        uint32_t *Rpos, uint32_t E) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= E || v >= offs[m]) return;
  const uint32_t i = segv[v], o = offs[i], oe = offs[i + 1];
  const uint32_t p = segs[i].first + (v - o);
  const uint32_t abase = o ? Ai[o - 1] : 0u, bbase = o ? Bi[o - 1] : 0u;
  if (af[v]) Lpos[o + (Ai[v] - abase) - 1] = p;
  if (bf[v]) {
    const uint32_t btot = Bi[oe - 1] - bbase;
    Rpos[o + (btot - (Bi[v] - bbase) + 1) - 1] = p;
  }
}

// number of swaps s: the a-element of rank k swaps with the b-element of rank
// k from the right while it lies left of it, i.e. while at least k b-elements
// lie strictly right of it (monotone in k); the a-element where that stops
// writes s (one writer per segment; s stays 0 if the first one fails)
__device__ __forceinline__ bool pred_at(const Seg &s, uint32_t o, uint32_t oe, uint32_t p, uint32_t rank,
                                        const uint32_t *Bi) {
  const uint32_t v = o + (p - s.first);
  const uint32_t nright = Bi[oe - 1] - Bi[v];  // b-elements strictly right of p
  return nright >= rank;
}
__global__ void k_swaps_count(const Seg *segs, const uint32_t *offs, uint32_t m, const uint32_t *af,
                              const uint32_t *Ai, const uint32_t *Bi, const uint32_t *segv, const uint32_t *Lpos,
                              uint32_t *sw, uint32_t E) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= E || v >= offs[m] || !af[v]) return;
  const uint32_t i = segv[v], o = offs[i], oe = offs[i + 1];
  const Seg s = segs[i];
  const uint32_t abase = o ? Ai[o - 1] : 0u, na = Ai[oe - 1] - abase, rank = Ai[v] - abase;
  const uint32_t p = s.first + (v - o);
  if (!pred_at(s, o, oe, p, rank, Bi)) return;
  if (rank == na || !pred_at(s, o, oe, Lpos[o + rank], rank + 1, Bi)) sw[i] = rank;
}

// the swaps themselves: one thread per pair (its a-element)
__global__ void k_swap(const Seg *segs, const uint32_t *offs, uint32_t m, const uint32_t *af, const uint32_t *Ai,
                       const uint32_t *segv, const uint32_t *Rpos, const uint32_t *sw, uint32_t *ids, uint32_t E) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= E || v >= offs[m] || !af[v]) return;
  const uint32_t i = segv[v], o = offs[i];
  const uint32_t rank = Ai[v] - (o ? Ai[o - 1] : 0u);
  if (rank > sw[i]) return;
  const uint32_t p = segs[i].first + (v - o), q = Rpos[o + rank - 1];
  const uint32_t t = ids[p];
  ids[p] = ids[q];
  ids[q] = t;
}

// the cut (where the left scan stops after the last swap) and the two parts:
// longer than kSerialMax -> next round, else the serial list
__global__ void k_split(const Seg *segs, const uint32_t *offs, uint32_t m, const uint32_t *size, const uint32_t *Ai,
                        const uint32_t *Lpos, const uint32_t *Rpos, const uint32_t *sw, Seg *next,
                        uint32_t *nnext, uint32_t *Enext, Seg *serial, uint32_t *nserial) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || size[i] == 0) return;
  const Seg s = segs[i];
  const uint32_t o = offs[i], oe = offs[i + 1];
  const uint32_t na = Ai[oe - 1] - (o ? Ai[o - 1] : 0u), k = sw[i];
  uint32_t cut;
  if (k == 0) cut = Lpos[o];  // the median of three guarantees an element >= pivot
  else {
    const uint32_t rk = Rpos[o + k - 1];
    cut = (k < na) ? min(Lpos[o + k], rk) : rk;
  }
  const Seg parts[2] = {Seg{cut, s.last, s.depth - 1, 0}, Seg{s.first, cut, s.depth - 1, 0}};
  for (const Seg &q : parts) {
    if (q.last - q.first > kSerialMax) {
      next[atomicAdd(nnext, 1u)] = q;
      atomicAdd(Enext, q.last - q.first);
    } else if (q.last - q.first > 1) {
      serial[atomicAdd(nserial, 1u)] = q;
    }
  }
}

// ---- SAH sweeps: one workgroup per (candidate, axis) -----------------------
struct TBox {
  float mn[3], mx[3];
};
__device__ __forceinline__ TBox tb_empty() {
  const float inf = __builtin_huge_valf();
  return TBox{{inf, inf, inf}, {-inf, -inf, -inf}};
}
// std::min / std::max as the reference's update_box / calc_bbox use them
__device__ __forceinline__ TBox tb_union(const TBox &a, const TBox &b) {
  TBox r;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    r.mn[k] = (b.mn[k] < a.mn[k]) ? b.mn[k] : a.mn[k];
    r.mx[k] = (a.mx[k] < b.mx[k]) ? b.mx[k] : a.mx[k];
  }
  return r;
}
__device__ __forceinline__ float tb_area(const TBox &b) {  // surfaceArea (raytracing.hpp:62-65)
  const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
  return 2 * (dx * dy + dx * dz + dy * dz);
}

constexpr int kSahT = 256, kSahI = 8, kSahChunk = kSahT * kSahI;
// exclusive scan of box unions over the block in thread order (earlier threads
// first, so among equal bounds the earlier operand is kept); returns the
// union of the threads before this one, *tot the union of all
__device__ TBox block_excl_box(const TBox &b, TBox *sm, TBox *tot) {
  sm[threadIdx.x] = b;
  __syncthreads();
  for (int o = 1; o < kSahT; o <<= 1) {
    TBox x = tb_empty();
    if (threadIdx.x >= (uint32_t)o) x = sm[threadIdx.x - o];
    __syncthreads();
    sm[threadIdx.x] = tb_union(x, sm[threadIdx.x]);
    __syncthreads();
  }
  const TBox ex = threadIdx.x ? sm[threadIdx.x - 1] : tb_empty();
  *tot = sm[kSahT - 1];
  __syncthreads();
  return ex;
}

struct Task {
  uint32_t s, e;  // triangle range [s, e) of one candidate
};

// ---- SAH sweeps over chunks: many workgroups per (candidate, axis) ----------
// The sweep above walks a whole candidate range in ONE workgroup, so the top
// stages (a handful of candidates over up to 3n triangles) ran on 3-6
// workgroups. Here a (candidate, axis) range is cut into chunks of kSahChunk
// triangles: (1) every chunk's box union, (2) per (candidate, axis) the
// exclusive prefix and suffix unions of its chunks (one thread walks them),
// (3) every chunk's dividers -- right boxes by a reverse scan inside the chunk
// plus the suffix of the chunks after it, left boxes by a forward scan plus
// the prefix -- and the chunk's first minimum; the host takes the first
// minimum over the chunks. Box unions are exact min / max, so the areas, and
// with them every cost, are the sequential sweep's values.
struct SahChunk {
  uint32_t task, axis, lo, hi;  // triangle range [lo, hi) of candidate `task` on `axis`
  uint32_t group;               // task * 3 + axis
};
struct SahGroup {
  uint32_t first, count;  // its chunks
};

__global__ __launch_bounds__(kSahT) void k_sah_chunk_box(const SahChunk *chunks, const uint32_t *ids3,
                                                         const TBox *tbox, uint32_t n, TBox *cbox) {
  __shared__ TBox sm[kSahT];
  const SahChunk c = chunks[blockIdx.x];
  const uint32_t *ids = ids3 + c.axis * n;
  TBox acc = tb_empty();
  const uint32_t t0 = c.lo + threadIdx.x * kSahI;
#pragma unroll
  for (int q = 0; q < kSahI; ++q)
    if (t0 + q < c.hi) acc = tb_union(acc, tbox[ids[t0 + q]]);
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t o = 1; o < (uint32_t)kSahT; o <<= 1) {
    if ((threadIdx.x & (2 * o - 1)) == 0) sm[threadIdx.x] = tb_union(sm[threadIdx.x], sm[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) cbox[blockIdx.x] = sm[0];
}

// one thread per (candidate, axis): exclusive prefix / suffix unions of its
// chunks, and the parent's surface area (:84, the union of the whole range)
__global__ void k_sah_carry(const SahGroup *groups, uint32_t ng, const TBox *cbox, TBox *cpre, TBox *csuf,
                            float *psa) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const SahGroup G = groups[g];
  TBox a = tb_empty();
  for (uint32_t k = 0; k < G.count; ++k) {
    cpre[G.first + k] = a;
    a = tb_union(a, cbox[G.first + k]);
  }
  psa[g] = tb_area(a);
  TBox b = tb_empty();
  for (uint32_t k = G.count; k-- > 0;) {
    csuf[G.first + k] = b;
    b = tb_union(cbox[G.first + k], b);
  }
}

__global__ __launch_bounds__(kSahT) void k_sah_chunk_cost(const SahChunk *chunks, const Task *tasks,
                                                          const uint32_t *ids3, const TBox *tbox, uint32_t n,
                                                          const TBox *cpre, const TBox *csuf, const float *psa_g,
                                                          float *ccost, uint32_t *cdiv) {
  __shared__ TBox sm[kSahT];
  __shared__ float s_cost[kSahT];
  __shared__ uint32_t s_div[kSahT];
  const SahChunk c = chunks[blockIdx.x];
  const Task tk = tasks[c.task];
  const uint32_t *ids = ids3 + c.axis * n;
  const float psa = psa_g[c.group];
  const uint32_t t0 = c.lo + threadIdx.x * kSahI;
  TBox tb[kSahI];
  TBox loc = tb_empty();
#pragma unroll
  for (int q = 0; q < kSahI; ++q) {
    tb[q] = (t0 + q < c.hi) ? tbox[ids[t0 + q]] : tb_empty();
    loc = tb_union(loc, tb[q]);
  }
  // right boxes: the union of everything after triangle t, t = t0 + q
  // (threads after this one in the chunk: a reverse exclusive scan; chunks
  // after this one: csuf)
  sm[threadIdx.x] = loc;
  __syncthreads();
  for (int o = 1; o < kSahT; o <<= 1) {
    TBox x = tb_empty();
    if (threadIdx.x + (uint32_t)o < (uint32_t)kSahT) x = sm[threadIdx.x + o];
    __syncthreads();
    sm[threadIdx.x] = tb_union(sm[threadIdx.x], x);
    __syncthreads();
  }
  TBox r = tb_union(threadIdx.x + 1 < (uint32_t)kSahT ? sm[threadIdx.x + 1] : tb_empty(), csuf[blockIdx.x]);
  float rarea[kSahI];
#pragma unroll
  for (int q = kSahI - 1; q >= 0; --q) {
    rarea[q] = tb_area(r);
    r = tb_union(tb[q], r);
  }
  __syncthreads();
  // left boxes: everything up to and including triangle t (chunks before:
  // cpre; threads before this one: an exclusive scan)
  TBox tot;
  TBox left = tb_union(cpre[blockIdx.x], block_excl_box(loc, sm, &tot));
  float best = __builtin_huge_valf();
  uint32_t bdiv = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 0; q < kSahI; ++q) {
    const uint32_t t = t0 + q, d = t + 1;  // divider after triangle t (index units: 3 d)
    if (t < c.hi) left = tb_union(left, tb[q]);
    if (t < c.hi && d < tk.e) {
      const float lc = static_cast<float>(3u * (d - tk.s)) / 3.0f;
      const float rc = static_cast<float>(3u * (tk.e - tk.s)) / 3.0f - lc;
      const float cost = 0.2f + tb_area(left) / psa * lc + rarea[q] / psa * rc;
      if (cost < best) {  // NaN never wins, as `curSAH < result.sah`; a thread's dividers ascend
        best = cost;
        bdiv = d;
      }
    }
  }
  s_cost[threadIdx.x] = best;
  s_div[threadIdx.x] = bdiv;
  __syncthreads();
  for (int o = kSahT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < (uint32_t)o) {
      const float c2 = s_cost[threadIdx.x + o];
      const uint32_t d2 = s_div[threadIdx.x + o];
      if (c2 < s_cost[threadIdx.x] || (c2 == s_cost[threadIdx.x] && d2 < s_div[threadIdx.x])) {
        s_cost[threadIdx.x] = c2;
        s_div[threadIdx.x] = d2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ccost[blockIdx.x] = s_cost[0];
    cdiv[blockIdx.x] = s_div[0];
  }
}

// stage start: every candidate range saved (rollback) and copied to the Y / Z
// scratch; one workgroup per kSahChunk-triangle chunk of a candidate (the axis-0
// chunks of the SAH table), so a stage of a few huge candidates is not left to
// a few workgroups
__global__ void k_stage_copy(const SahChunk *chunks, uint32_t *ids3, uint32_t *backup, uint32_t n) {
  const SahChunk c = chunks[blockIdx.x];
  for (uint32_t t = c.lo + threadIdx.x; t < c.hi; t += blockDim.x) {
    const uint32_t v = ids3[t];
    backup[t] = v;
    ids3[n + t] = v;
    ids3[2 * n + t] = v;
  }
}
// stage end: 1 = take the Y order, 2 = the Z order, 3 = restore (never evaluated by the reference)
__global__ void k_stage_apply(const SahChunk *chunks, const uint32_t *action, uint32_t *ids3, const uint32_t *backup,
                              uint32_t n) {
  const SahChunk c = chunks[blockIdx.x];
  const uint32_t a = action[c.task];
  if (a == 0) return;
  const uint32_t *src = a == 1 ? ids3 + n : a == 2 ? ids3 + 2 * n : backup;
  for (uint32_t t = c.lo + threadIdx.x; t < c.hi; t += blockDim.x) ids3[t] = src[t];
}
// child boxes (calc_bbox, :199): the ordered fold of a range's chunk unions
// (k_sah_chunk_box on its chunks), earlier chunk on the left
__global__ void k_group_fold(const SahGroup *groups, uint32_t ng, const TBox *cbox, TBox *out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const SahGroup G = groups[g];
  TBox a = tb_empty();
  for (uint32_t k = 0; k < G.count; ++k) a = tb_union(a, cbox[G.first + k]);
  out[g] = a;
}

// per-triangle box (calc_bbox of the /w-divided vertices, raytracing.hpp:51-60) and keys
__global__ void k_tribox(const float4 *vpos, const uint32_t *idx, uint32_t n, TBox *tbox, float *K3) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  TBox b = tb_empty();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float4 v = vpos[idx[3 * t + k]];
    const float x = v.x / v.w, y = v.y / v.w, z = v.z / v.w;
    b = tb_union(b, TBox{{x, y, z}, {x, y, z}});
  }
  tbox[t] = b;
  K3[t] = b.mx[0];
  K3[n + t] = b.mx[1];
  K3[2 * n + t] = b.mx[2];
}

// ---- host side ---------------------------------------------------------------
// RTAMD_BVH_TIMING=1: per-phase wall time of a device build on stderr (the
// phases are synchronised for the measurement)
struct PhaseTimer {
  bool on = std::getenv("RTAMD_BVH_TIMING") != nullptr;
  double acc[8] = {};
  double host[4] = {};  // wall time of host-side stage sections (no syncs): prologue, FIFO, apply+boxes
  std::chrono::steady_clock::time_point h0;
  void hstart() { h0 = std::chrono::steady_clock::now(); }
  void hstop(int k) { host[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count(); }
  int rounds = 0, stages = 0, serial_launches = 0;
  std::chrono::steady_clock::time_point t0;
  hipStream_t st = nullptr;
  void start() {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    t0 = std::chrono::steady_clock::now();
  }
  void stop(int k) {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    acc[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
};

template <class T>
struct DBuf {
  T *p = nullptr;
  size_t cap = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  // grows geometrically: the per-stage buffers widen with the tree, and a
  // hipFree / hipMalloc pair at every stage for each of them synchronises the
  // device each time
  int reserve(size_t n) {
    if (n <= cap) return RT_OK;
    const size_t want = std::max<size_t>({n, 2 * cap, 1024});
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(&p, want * sizeof(T)));
    cap = want;
    return RT_OK;
  }
};

// rtx_bvh_inject_failure: the next N device builds fail as a device error would
std::atomic<int> g_inject_fail{0};

inline int lg2(uint64_t n) { return 63 - __builtin_clzll(n); }

struct Sorter {
  uint32_t n = 0;  // triangles (one axis block of the 3n space)
  uint32_t *ids = nullptr;
  const float *K3 = nullptr;
  DBuf<Seg> segA, segB, serial;
  DBuf<uint32_t> size, offs, sw, af, bf, Ai, Bi, segv, Lpos, Rpos, bsum, ctr;
  DBuf<float> kp;
  size_t bsum_half = 0;  // bsum: two halves, one per array of a paired scan
  hipStream_t st = nullptr;
  PhaseTimer own_pt;             // per build: concurrent builds share no state
  PhaseTimer *pt = &own_pt;

  int init(uint32_t ntri, uint32_t *ids3, const float *keys3) {
    n = ntri;
    ids = ids3;
    K3 = keys3;
    const size_t N = 3 * (size_t)n, segcap = N / kSerialMax + 16, sercap = N / 2 + 4096;
    int rc;
    if ((rc = segA.reserve(segcap)) || (rc = segB.reserve(segcap)) || (rc = serial.reserve(sercap)) ||
        (rc = size.reserve(segcap + 1)) || (rc = offs.reserve(segcap + 1)) || (rc = sw.reserve(segcap)) ||
        (rc = kp.reserve(segcap)) || (rc = af.reserve(N)) || (rc = bf.reserve(N)) || (rc = Ai.reserve(N)) ||
        (rc = Bi.reserve(N)) || (rc = segv.reserve(N)) || (rc = Lpos.reserve(N)) || (rc = Rpos.reserve(N)) ||
        (rc = bsum.reserve(2 * (N / kScanBlk + 2))) || (rc = ctr.reserve(4)))
      return rc;
    bsum_half = N / kScanBlk + 2;
    return RT_OK;
  }

  // inclusive scans of one array (in1 == nullptr) or of two at once
  int scan(const uint32_t *in, uint32_t *out, uint32_t cnt, const uint32_t *in1 = nullptr,
           uint32_t *out1 = nullptr) {
    if (cnt == 0) return RT_OK;
    const uint32_t nb = (cnt + kScanBlk - 1) / kScanBlk, na = in1 ? 2u : 1u;
    const ScanPair sp{{in, in1}, {out, out1}, {bsum.p, bsum.p + bsum_half}};
    k_scan1<<<dim3(nb, na), kScanT, 0, st>>>(sp, cnt);
    if (nb > 1) {
      k_scan2<<<na, 1024, 0, st>>>(sp, nb);
      k_scan3<<<dim3(nb, na), kScanT, 0, st>>>(sp, cnt);
    }
    HIP_TRY(hipGetLastError());
    return RT_OK;
  }

  // sort every segment of `init` (host list): exactly std::sort on each
  int sort(const std::vector<Seg> &init) {
    std::vector<Seg> act, ser;
    for (const Seg &s : init) {
      if (s.last - s.first <= 1) continue;
      (s.last - s.first > kSerialMax ? act : ser).push_back(s);
    }
    uint32_t nser = (uint32_t)ser.size(), m = (uint32_t)act.size(), E = 0;
    for (const Seg &s : act) E += s.last - s.first;
    if (nser) HIP_TRY(hipMemcpyAsync(serial.p, ser.data(), nser * sizeof(Seg), hipMemcpyHostToDevice, st));
    if (m) HIP_TRY(hipMemcpyAsync(segA.p, act.data(), m * sizeof(Seg), hipMemcpyHostToDevice, st));
    uint32_t hc[3] = {0, 0, nser};  // next count, next E, serial count
    HIP_TRY(hipMemcpyAsync(ctr.p + 2, &hc[2], 4, hipMemcpyHostToDevice, st));
    Seg *cur = segA.p, *nxt = segB.p;
    pt->start();
    while (m > 0) {
      ++pt->rounds;
      HIP_TRY(hipMemsetAsync(ctr.p, 0, 8, st));
      HIP_TRY(hipMemsetAsync(sw.p, 0, (size_t)m * 4, st));
      const uint32_t gm = (m + 255) / 256;
      k_prep<<<gm, 256, 0, st>>>(cur, m, ids, K3, n, kp.p, size.p + 1, serial.p, ctr.p + 2);
      HIP_TRY(hipMemsetAsync(size.p, 0, 4, st));
      if (int rc = scan(size.p, offs.p, m + 1)) return rc;  // offs[i] = sum of sizes before segment i
      const uint32_t ge = (E + 255) / 256;
      if (E) {
        k_flags<<<ge, 256, 0, st>>>(cur, offs.p, m, ids, K3, n, kp.p, af.p, bf.p, segv.p, E);
        if (int rc = scan(af.p, Ai.p, E, bf.p, Bi.p)) return rc;
        k_ranks<<<ge, 256, 0, st>>>(cur, offs.p, m, af.p, bf.p, Ai.p, Bi.p, segv.p, Lpos.p, Rpos.p, E);
        k_swaps_count<<<ge, 256, 0, st>>>(cur, offs.p, m, af.p, Ai.p, Bi.p, segv.p, Lpos.p, sw.p, E);
        k_swap<<<ge, 256, 0, st>>>(cur, offs.p, m, af.p, Ai.p, segv.p, Rpos.p, sw.p, ids, E);
        k_split<<<gm, 256, 0, st>>>(cur, offs.p, m, size.p + 1, Ai.p, Lpos.p, Rpos.p, sw.p, nxt, ctr.p, ctr.p + 1,
                                    serial.p, ctr.p + 2);
      }
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(hc, ctr.p, 12, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      m = hc[0];
      E = hc[1];
      std::swap(cur, nxt);
    }
    HIP_TRY(hipMemcpyAsync(&nser, ctr.p + 2, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    pt->stop(0);
    pt->start();
    if (nser) k_serial<<<nser, 64, 0, st>>>(serial.p, ids, K3, n);
    ++pt->serial_launches;
    HIP_TRY(hipGetLastError());
    pt->stop(1);
    return RT_OK;
  }
};

// The device build's host-side node array (createNode's m_nodes). Up to 2n - 1
// nodes of ~240 B are written once each as the build proceeds; backed by an
// anonymous mapping of that bound with transparent huge pages requested, so a
// 1.1 M-triangle build's ~40 MB of nodes are ~20 page faults instead of ~10^4
// (untouched pages of the reservation cost nothing).
struct NodeArena {
  rth::BvhHostNode *p = nullptr;
  size_t n = 0, cap = 0, bytes = 0;
  NodeArena() = default;
  NodeArena(const NodeArena &) = delete;
  NodeArena &operator=(const NodeArena &) = delete;
  ~NodeArena() {
    if (p) munmap(p, bytes);
  }
  bool reserve(size_t c) {
    const size_t huge = (size_t)2 << 20;
    bytes = (c * sizeof(rth::BvhHostNode) + huge - 1) / huge * huge;
    void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) return false;
    (void)madvise(m, bytes, MADV_HUGEPAGE);
    p = static_cast<rth::BvhHostNode *>(m);
    cap = c;
    return true;
  }
  size_t size() const { return n; }
  rth::BvhHostNode &operator[](size_t i) { return p[i]; }
  void emplace_back() { new (p + n++) rth::BvhHostNode(); }  // n < cap: at most 2 ntri - 1 nodes
};

// createNode's ChipQueue contents (FIFO). A node splits at most 7 times and
// its queue is dropped at the 7th split, so it never holds more than 8
// candidates (a layer of 4 that all split reaches 7 splits); kept inline, so
// the ~10^5 open nodes of a large build allocate nothing
struct CandQueue {
  std::pair<uint32_t, uint32_t> a[16];
  uint32_t n = 0;
  const std::pair<uint32_t, uint32_t> *begin() const { return a; }
  const std::pair<uint32_t, uint32_t> *end() const { return a + n; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const std::pair<uint32_t, uint32_t> &operator[](size_t i) const { return a[i]; }
  void push_back(std::pair<uint32_t, uint32_t> c) { a[n < 16 ? n++ : 15] = c; }
  static CandQueue of(uint32_t lo, uint32_t hi) {
    CandQueue q;
    q.push_back({lo, hi});
    return q;
  }
};
// BVHBuilder::createNode state of one node (triangles_raytracing.cpp:155-225)
struct Open {
  int32_t node;
  uint32_t start, end;  // index units
  CandQueue queue;
  uint32_t div[8];
  int nd = 0;
};

}  // namespace

namespace rth {

bool build_bvh8_gpu(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                    std::string &err, bool with_canon) {
  // every device-side failure is reported as "GPU BVH build: <step>: <HIP
  // error>" (RT_E_DEVICE at the C ABI; in AUTO mode the host builder takes
  // over); input errors carry no prefix (RT_E_INVALID)
  auto fail = [&](const char *what) {
    err = std::string("GPU BVH build: ") + what + ": " + rterr::get();
    return false;
  };
  auto hfail = [&](const char *what, hipError_t e) {
    err = std::string("GPU BVH build: ") + what + ": " + hipGetErrorString(e);
    return false;
  };
#define BVH_DEV(expr, what)                     \
  do {                                          \
    const hipError_t e_ = (expr);               \
    if (e_ != hipSuccess) return hfail(what, e_); \
  } while (0)
  if (nidx < 0 || nidx % 3 != 0) { err = "index count must be a multiple of 3"; return false; }
  for (int64_t i = 0; i < nidx; ++i)
    if ((int64_t)idx[i] >= nverts) { err = "vertex index out of range"; return false; }
  const uint32_t n = (uint32_t)(nidx / 3);
  if ((uint64_t)n > rtl::kMaxLeafFirstTri || 3ull * n >= (1ull << 31)) { err = "too many triangles"; return false; }
  out = BVHGpu();
  if (n == 0) { out.root_word = rtl::kInvalidChild; return true; }
  if (g_inject_fail.load() > 0) {  // rtx_bvh_inject_failure: a simulated device failure
    g_inject_fail.fetch_sub(1);
    return hfail("injected failure", hipErrorOutOfMemory);
  }

  const auto tb0 = std::chrono::steady_clock::now();
  PhaseTimer pt;
  pt.start();
  DBuf<float4> dv;
  DBuf<uint32_t> didx, ids3, backup, ddiv, dact;
  DBuf<float> K3, dcost;
  DBuf<TBox> tbox, boxes, cbox, cpre, csuf;
  DBuf<Task> dtasks;
  DBuf<SahChunk> dchunks, drch;
  DBuf<SahGroup> dgroups, drgrp;
  DBuf<TBox> rcbox;
  std::vector<SahChunk> ch, rch;  // per-stage chunk tables (host copies)
  std::vector<SahGroup> grp, rgrp;
  uint32_t NC = 0, NC0 = 0;
  DBuf<float> ccost, dpsa;
  DBuf<uint32_t> cdivv;
  Sorter S;
  if (dv.reserve((size_t)nverts) || didx.reserve((size_t)nidx) || ids3.reserve(3 * (size_t)n) ||
      backup.reserve(n) || K3.reserve(3 * (size_t)n) || tbox.reserve(n) ||
      S.init(n, nullptr, nullptr))
    return fail("allocation");
  S.ids = ids3.p;
  S.K3 = K3.p;
  S.pt = &pt;
  hipStream_t st = nullptr;
  BVH_DEV(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  S.st = st;
  pt.st = st;
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  std::vector<uint32_t> iota(n);
  for (uint32_t t = 0; t < n; ++t) iota[t] = t;
  BVH_DEV(hipMemcpyAsync(dv.p, vpos4, (size_t)nverts * 16, hipMemcpyHostToDevice, st), "upload");
  BVH_DEV(hipMemcpyAsync(didx.p, idx, (size_t)nidx * 4, hipMemcpyHostToDevice, st), "upload");
  BVH_DEV(hipMemcpyAsync(ids3.p, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice, st), "upload");
  k_tribox<<<(n + 255) / 256, 256, 0, st>>>(dv.p, didx.p, n, tbox.p, K3.p);
  BVH_DEV(hipGetLastError(), "triangle boxes");
  pt.stop(7);  // allocation, upload, triangle boxes

  // host state reused across the stages (cleared, never freed: fresh pages
  // of per-stage vectors cost more than the stage logic itself)
  NodeArena H;
  if (!H.reserve(2 * (size_t)n + 1)) return hfail("node arena", hipErrorOutOfMemory);
  H.emplace_back();
  std::vector<Open> open, next;
  std::vector<Task> tasks;
  std::vector<int> task_of;
  std::vector<uint32_t> task_off, dvd, action;
  std::vector<float> cost, hcc;
  std::vector<uint32_t> hcd;
  std::vector<Seg> segs;
  open.push_back(Open{0, 0, 3 * n, CandQueue::of(0u, 3 * n), {}, 0});
  // child ranges (triangle units) and their boxes: a node's child boxes are
  // computed in the stage that completes the node, over the triangle order at
  // that point (calc_bbox at creation, triangles_raytracing.cpp:199), before
  // the children's own sorts reorder their ranges (first-kept among equal
  // bounds, so -0.0 / +0.0 come out as the reference's sequential min / max)
  std::vector<Task> ranges;
  std::vector<std::pair<int32_t, int>> range_of;  // (node, child slot) per range
  const size_t max_ranges = 2 * (size_t)n + 8;    // every node but the root is a child range
  ranges.reserve(max_ranges);
  range_of.reserve(max_ranges);
  if (boxes.reserve(max_ranges)) return fail("allocation");
  const auto ts0 = std::chrono::steady_clock::now();
  while (!open.empty()) {
    ++pt.stages;
    pt.hstart();
    const size_t r0 = ranges.size();
    // this stage: every queued candidate of every open node that tryDivide sorts (> 8 triangles)
    tasks.clear();
    // task index of open node o's candidate c: task_of[task_off[o] + c] (-1: not sorted)
    task_of.clear();
    task_off.resize(open.size());
    for (size_t o = 0; o < open.size(); ++o) {
      task_off[o] = (uint32_t)task_of.size();
      for (auto &c : open[o].queue) {
        const bool gpu = c.second - c.first > 24;
        task_of.push_back(gpu ? (int)tasks.size() : -1);
        if (gpu) tasks.push_back(Task{c.first / 3, c.second / 3});
      }
    }
    const uint32_t T = (uint32_t)tasks.size();
    cost.assign(3 * (size_t)T, 0.0f);
    dvd.assign(3 * (size_t)T, 0u);
    action.assign(T, 0u);
    if (T) {
      if (dtasks.reserve(T) || dcost.reserve(3 * (size_t)T) || ddiv.reserve(3 * (size_t)T) || dact.reserve(T))
        return fail("allocation");
      BVH_DEV(hipMemcpyAsync(dtasks.p, tasks.data(), T * sizeof(Task), hipMemcpyHostToDevice, st), "upload");
      // chunks of every (candidate, axis) range: [axis-0 chunks of all candidates | axis 1 | axis 2]
      ch.clear();
      grp.assign(3 * (size_t)T, SahGroup{});
      for (uint32_t a = 0; a < 3; ++a)
        for (uint32_t ti = 0; ti < T; ++ti) {
          SahGroup &G = grp[3 * ti + a];
          G.first = (uint32_t)ch.size();
          for (uint32_t lo = tasks[ti].s; lo < tasks[ti].e; lo += kSahChunk)
            ch.push_back(SahChunk{ti, a, lo, std::min<uint32_t>(tasks[ti].e, lo + kSahChunk), 3 * ti + a});
          G.count = (uint32_t)ch.size() - G.first;
        }
      NC = (uint32_t)ch.size();
      NC0 = NC / 3;  // the axis-0 chunks come first
      const uint32_t NG = 3 * T;
      if (dchunks.reserve(NC) || dgroups.reserve(NG) || cbox.reserve(NC) || cpre.reserve(NC) || csuf.reserve(NC) ||
          ccost.reserve(NC) || cdivv.reserve(NC) || dpsa.reserve(NG))
        return fail("allocation");
      BVH_DEV(hipMemcpyAsync(dchunks.p, ch.data(), NC * sizeof(SahChunk), hipMemcpyHostToDevice, st), "upload");
      BVH_DEV(hipMemcpyAsync(dgroups.p, grp.data(), NG * sizeof(SahGroup), hipMemcpyHostToDevice, st), "upload");
      k_stage_copy<<<NC0, 256, 0, st>>>(dchunks.p, ids3.p, backup.p, n);
      segs.clear();
      segs.reserve(3 * (size_t)T);
      for (int a = 0; a < 3; ++a)
        for (const Task &tk : tasks)
          segs.push_back(Seg{a * n + tk.s, a * n + tk.e, 2 * lg2(tk.e - tk.s), 0});
      pt.hstop(0);
      if (S.sort(segs)) return fail("sort");
      pt.start();
      k_sah_chunk_box<<<NC, kSahT, 0, st>>>(dchunks.p, ids3.p, tbox.p, n, cbox.p);
      k_sah_carry<<<(NG + 63) / 64, 64, 0, st>>>(dgroups.p, NG, cbox.p, cpre.p, csuf.p, dpsa.p);
      k_sah_chunk_cost<<<NC, kSahT, 0, st>>>(dchunks.p, dtasks.p, ids3.p, tbox.p, n, cpre.p, csuf.p, dpsa.p, ccost.p,
                                             cdivv.p);
      BVH_DEV(hipGetLastError(), "SAH sweep");
      hcc.resize(NC);
      hcd.resize(NC);
      BVH_DEV(hipMemcpyAsync(hcc.data(), ccost.p, NC * 4, hipMemcpyDeviceToHost, st), "SAH sweep");
      BVH_DEV(hipMemcpyAsync(hcd.data(), cdivv.p, NC * 4, hipMemcpyDeviceToHost, st), "SAH sweep");
      BVH_DEV(hipStreamSynchronize(st), "SAH sweep");
      pt.stop(2);
      // first minimum over the chunks of each (candidate, axis): (cost, divider) lexicographic
      for (uint32_t g = 0; g < NG; ++g) {
        float bc = __builtin_huge_valf();
        uint32_t bd = 0xFFFFFFFFu;
        for (uint32_t k = grp[g].first; k < grp[g].first + grp[g].count; ++k)
          if (hcc[k] < bc || (hcc[k] == bc && hcd[k] < bd)) {
            bc = hcc[k];
            bd = hcd[k];
          }
        // cost/dvd are indexed [3 * task + axis], as the single-workgroup sweep wrote them
        cost[g] = bc;
        dvd[g] = bd;
      }
    }
    pt.hstart();
    // createNode's FIFO, candidate by candidate (triangles_raytracing.cpp:162-173)
    next.clear();
    for (size_t o = 0; o < open.size(); ++o) {
      Open &N = open[o];
      CandQueue q2;
      bool capped = false;
      for (size_t c = 0; c < N.queue.size(); ++c) {
        const auto cand = N.queue[c];
        const int ti = task_of[task_off[o] + c];
        if (N.nd == 7) {  // the reference stops here: this candidate is never tried
          capped = true;
          if (ti >= 0) action[ti] = 3;
          continue;
        }
        if (ti < 0) continue;  // <= 8 triangles: tryDivide returns at once
        // tryDivide(start, end) (:119-153) from the three tryDivide(indices, start, end, axis)
        const uint32_t start = cand.first, end = cand.second;
        const float curSAH = static_cast<float>(end - start) / 3.0f;
        float sah[3];
        bool divided[3];
        uint32_t dv3[3];
        for (int a = 0; a < 3; ++a) {
          const float cst = cost[(size_t)3 * ti + a];
          divided[a] = cst < curSAH;
          sah[a] = divided[a] ? cst : curSAH;
          uint32_t d = dvd[(size_t)3 * ti + a] * 3;
          if (divided[a] && (d - start) % 24 != 0) {  // align to 8 (:100-114)
            const uint32_t d1 = (d - 1) / 24 * 24, d2 = ((d - 1) / 24 + 1) * 24;
            const uint32_t nearest = (d - d1 <= d2 - d) ? d1 : d2, other = d1 + d2 - nearest;
            if (start < nearest && nearest < end) d = nearest;
            else if (start < other && other < end) d = other;
          }
          dv3[a] = d;
        }
        const float mn = std::min({curSAH, sah[0], sah[1], sah[2]});
        int win = -1;
        if (sah[0] == mn) win = 0;
        else if (sah[1] == mn) win = 1;
        else if (sah[2] == mn) win = 2;
        action[ti] = win == 1 ? 1u : win == 2 ? 2u : 0u;
        if (win >= 0 && divided[win]) {
          N.div[N.nd++] = dv3[win];
          q2.push_back({start, dv3[win]});
          q2.push_back({dv3[win], end});
        }
      }
      N.queue = (capped || N.nd == 7) ? CandQueue{} : q2;
      if (!N.queue.empty()) {
        next.push_back(std::move(N));
        continue;
      }
      // node complete (:175-224)
      BvhHostNode node;
      if (N.nd == 0) {
        if (N.end - N.start > 24) {
          N.div[N.nd++] = ((N.start / 3 + N.end / 3) / 2) * 3;
        } else {
          node.leaf = true;
          node.start = N.start;
          node.count = N.end - N.start;
          H[N.node] = node;
          continue;
        }
      }
      std::sort(N.div, N.div + N.nd);
      node.nchild = (uint32_t)(N.nd + 1);
      for (int c = 0; c <= N.nd; ++c) {
        const uint32_t lo = c == 0 ? N.start : N.div[c - 1], hi = c == N.nd ? N.end : N.div[c];
        node.child[c] = (int32_t)H.size();
        H.emplace_back();
        ranges.push_back(Task{lo / 3, hi / 3});
        range_of.push_back({N.node, c});
        next.push_back(Open{node.child[c], lo, hi, CandQueue::of(lo, hi), {}, 0});
      }
      H[N.node] = node;
    }
    pt.hstop(1);
    pt.hstart();
    if (T) {
      BVH_DEV(hipMemcpyAsync(dact.p, action.data(), T * 4, hipMemcpyHostToDevice, st), "upload");
      k_stage_apply<<<NC0, 256, 0, st>>>(dchunks.p, dact.p, ids3.p, backup.p, n);
      BVH_DEV(hipGetLastError(), "stage apply");
    }
    if (ranges.size() > r0) {  // boxes of the children of the nodes completed in this stage
      if (ranges.size() > max_ranges) return hfail("child range bound", hipErrorInvalidValue);
      const uint32_t nr = (uint32_t)(ranges.size() - r0);
      rch.clear();
      rgrp.resize(nr);
      for (uint32_t r = 0; r < nr; ++r) {
        const Task &R = ranges[r0 + r];
        rgrp[r].first = (uint32_t)rch.size();
        for (uint32_t lo = R.s; lo < R.e; lo += kSahChunk)
          rch.push_back(SahChunk{r, 0u, lo, std::min<uint32_t>(R.e, lo + kSahChunk), r});
        rgrp[r].count = (uint32_t)rch.size() - rgrp[r].first;
      }
      const uint32_t nrc = (uint32_t)rch.size();
      if (drch.reserve(nrc) || drgrp.reserve(nr) || rcbox.reserve(nrc)) return fail("allocation");
      BVH_DEV(hipMemcpyAsync(drch.p, rch.data(), nrc * sizeof(SahChunk), hipMemcpyHostToDevice, st), "upload");
      BVH_DEV(hipMemcpyAsync(drgrp.p, rgrp.data(), nr * sizeof(SahGroup), hipMemcpyHostToDevice, st), "upload");
      k_sah_chunk_box<<<nrc, kSahT, 0, st>>>(drch.p, ids3.p, tbox.p, n, rcbox.p);
      k_group_fold<<<(nr + 63) / 64, 64, 0, st>>>(drgrp.p, nr, rcbox.p, boxes.p + r0);
      BVH_DEV(hipGetLastError(), "child boxes");
      BVH_DEV(hipStreamSynchronize(st), "child boxes");  // rch / rgrp are reused by the next stage
    }
    pt.hstop(2);
    open.swap(next);
  }
  if (pt.on) {
    (void)hipStreamSynchronize(st);
    pt.acc[5] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
  }
  pt.start();
  // the child boxes, and the final triangle order
  std::vector<uint32_t> cur(n);
  if (!ranges.empty()) {
    std::vector<TBox> hb(ranges.size());
    BVH_DEV(hipMemcpyAsync(hb.data(), boxes.p, hb.size() * sizeof(TBox), hipMemcpyDeviceToHost, st), "child boxes");
    BVH_DEV(hipStreamSynchronize(st), "child boxes");
    for (size_t r = 0; r < ranges.size(); ++r) {
      BvhBox &b = H[range_of[r].first].box[range_of[r].second];
      std::memcpy(b.mn, hb[r].mn, 12);
      std::memcpy(b.mx, hb[r].mx, 12);
    }
  }
  BVH_DEV(hipMemcpyAsync(cur.data(), ids3.p, (size_t)n * 4, hipMemcpyDeviceToHost, st), "download");
  BVH_DEV(hipStreamSynchronize(st), "download");
  pt.stop(6);
  pt.start();
  bvh_layout(vpos4, idx, nidx, HostNodes(H.p, H.size()), cur, out, with_canon);
  pt.stop(3);
  if (pt.on)
    std::fprintf(stderr,
                 "[bvh gpu] %u tris: total %.1f ms | alloc+upload+tri boxes %.1f, stages %.1f (partition rounds %.1f "
                 "(%d rounds), serial sorts %.1f (%d launches), SAH %.1f, other %.1f), boxes+download %.1f, layout "
                 "%.1f; %d stages; host sections: stage prologue %.1f, FIFO %.1f, apply+boxes %.1f\n",
                 n, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count(),
                 pt.acc[7], pt.acc[5], pt.acc[0], pt.rounds, pt.acc[1], pt.serial_launches, pt.acc[2],
                 pt.acc[5] - pt.acc[0] - pt.acc[1] - pt.acc[2], pt.acc[6], pt.acc[3], pt.stages, pt.host[0],
                 pt.host[1], pt.host[2]);
  return true;
#undef BVH_DEV
}

}  // namespace rth

// ---- diagnostics (not part of include/rtamd.h) ------------------------------
extern "C" {

// Fault injection for the builder fallback test: the next `n` device builds
// fail with a device error before touching the GPU.
int rtx_bvh_inject_failure(int32_t n) {
  g_inject_fail.store(n < 0 ? 0 : n);
  return RT_OK;
}

// The device sort against libstdc++ std::sort (host_introsort) on n keys:
// ids[] receives the device permutation; returns RT_OK and *mismatch = number
// of positions that differ from the host permutation. depth < 0: std::sort's
// own depth limit (2 lg n); smaller limits force the heapsort fallback.
int rtx_sort_check(const float *keys, int64_t n, int32_t depth, uint32_t *ids_out, int64_t *mismatch) {
  if (!keys || n <= 0 || n >= (1ll << 30) || !mismatch) return rterr::set(RT_E_INVALID, "bad arguments");
  const uint32_t nn = (uint32_t)n;
  std::vector<uint32_t> host(nn);
  for (uint32_t i = 0; i < nn; ++i) host[i] = i;
  rth::host_introsort(host.data(), nn, keys, depth);
  // the sort works on a 3n space; the test uses axis block 0 only
  DBuf<uint32_t> ids3;
  DBuf<float> K3;
  Sorter S;
  if (int rc = ids3.reserve(3 * (size_t)nn)) return rc;
  if (int rc = K3.reserve(3 * (size_t)nn)) return rc;
  if (int rc = S.init(nn, ids3.p, K3.p)) return rc;
  HIP_TRY(hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking));
  std::vector<uint32_t> iota(nn);
  for (uint32_t i = 0; i < nn; ++i) iota[i] = i;
  int rc = RT_OK;
  if (hipMemcpy(ids3.p, iota.data(), (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(K3.p, keys, (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess)
    rc = rterr::set(RT_E_DEVICE, "upload");
  if (!rc) rc = S.sort({Seg{0, nn, depth < 0 ? 2 * lg2(nn) : depth, 0}});
  std::vector<uint32_t> dev(nn);
  if (!rc && (hipStreamSynchronize(S.st) != hipSuccess ||
              hipMemcpy(dev.data(), ids3.p, (size_t)nn * 4, hipMemcpyDeviceToHost) != hipSuccess))
    rc = rterr::set(RT_E_DEVICE, "download");
  (void)hipStreamDestroy(S.st);
  if (rc) return rc;
  int64_t bad = 0;
  for (uint32_t i = 0; i < nn; ++i) bad += dev[i] != host[i];
  *mismatch = bad;
  if (ids_out) std::memcpy(ids_out, dev.data(), (size_t)nn * 4);
  return RT_OK;
}

}  // extern "C"
