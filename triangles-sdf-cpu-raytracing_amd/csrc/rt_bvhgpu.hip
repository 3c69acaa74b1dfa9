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
#include <sys/resource.h>

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
#include "rt_bvhstage.h"
#include "rt_host.h"
#include "rt_layout.h"

namespace {

using rth::bvhs::SahChunk;
using rth::bvhs::SahGroup;
using rth::bvhs::Seg;
using rth::bvhs::Task;

#ifndef RT_SERIAL_MAX
#define RT_SERIAL_MAX 1024  // A/B switch (256: 2.9 ms short sorts + 14.9 ms rounds; 1024: 5.7 + 10.3, 1.1 M tris)
#endif
constexpr uint32_t kSerialMax = RT_SERIAL_MAX;  // segments at most this long: one wave, serial introsort in LDS


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

// set bits of m below this lane
__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// std::__introsort_loop by one wave (a 64-thread block) on LDS. Each
// std::__unguarded_partition_pivot runs as in the partition rounds: the
// a-elements (stop the left scan) and b-elements (stop the right scan) are
// listed by ballots, and the k-th a from the left swaps with the k-th b from
// the right while it lies left of it -- all such pairs at once (every left
// one lies left of every right one). The ranges of <= 16 left for the final
// insertion sort are listed in `leaf` (first | last << 16); returns their
// count. Heapsorted ranges (depth 0) are already sorted and not listed.
__device__ uint32_t wave_introsort(KI *a, uint32_t len, int depth, uint16_t *Lp, uint16_t *Bp, uint32_t *stk,
                                   uint32_t *leaf) {
  const uint32_t lane = threadIdx.x;
  const auto less = [](const KI &x, const KI &y) { return x.k < y.k; };
  uint32_t f = 0, l = len, nleaf = 0;
  int sp = 0;
  for (;;) {
    bool heaped = false;
    while (l - f > 16) {
      if (depth == 0) {
        if (lane == 0) d_heapsort(a + f, a + l, less);
        heaped = true;
        break;
      }
      --depth;
      if (lane == 0) d_median_to_first(a + f, a + f + 1, a + f + (l - f) / 2, a + l - 1, less);
      __syncthreads();
      const float pk = a[f].k;
      uint32_t na = 0, nb = 0;
      for (uint32_t base = f; base < l; base += 64) {
        const uint32_t p = base + lane;
        const bool v = p < l;
        const float k = v ? a[p].k : 0.0f;
        const bool fa = v && p != f && !(k < pk), fb = v && (p == f || !(pk < k));
        const uint64_t ma = __ballot(fa), mb = __ballot(fb);
        if (fa) Lp[na + lane_prefix(ma)] = (uint16_t)p;
        if (fb) Bp[nb + lane_prefix(mb)] = (uint16_t)p;
        na += (uint32_t)__popcll(ma);
        nb += (uint32_t)__popcll(mb);
      }
      __syncthreads();
      uint32_t sw = 0;  // pairs that swap: L_k < R_k, monotone in k
      for (uint32_t kb = 0; kb < na; kb += 64) {
        const uint32_t k = kb + lane + 1;
        sw += (uint32_t)__popcll(__ballot(k <= na && k <= nb && Lp[k - 1] < Bp[nb - k]));
      }
      for (uint32_t kb = 0; kb < sw; kb += 64) {
        const uint32_t k = kb + lane + 1;
        if (k <= sw) {
          const uint32_t x = Lp[k - 1], y = Bp[nb - k];
          const KI t = a[x];
          a[x] = a[y];
          a[y] = t;
        }
      }
      // where the left scan stops after the last swap (the median of three
      // guarantees an a-element)
      const uint32_t cut = sw == 0 ? Lp[0] : (sw < na ? min((uint32_t)Lp[sw], (uint32_t)Bp[nb - sw])
                                                       : (uint32_t)Bp[nb - sw]);
      __syncthreads();
      if (lane == 0) {
        stk[2 * sp] = (cut << 16) | l;
        stk[2 * sp + 1] = (uint32_t)depth;
      }
      ++sp;
      l = cut;
    }
    if (!heaped && l - f > 1) {
      if (lane == 0) leaf[nleaf] = f | (l << 16);
      ++nleaf;
    }
    __syncthreads();
    if (sp == 0) break;
    --sp;
    const uint32_t w = stk[2 * sp];
    depth = (int)stk[2 * sp + 1];
    f = w >> 16;
    l = w & 0xFFFFu;
  }
  return nleaf;
}

// one wave per short segment (<= kSerialMax): (key, id) pairs staged in LDS,
// the introsort loop by the wave, then the final insertion sort as one
// insertion sort per leaf range, a lane each (it never moves an element
// across a partition boundary, so the order is std::sort's)
__global__ __launch_bounds__(64) void k_serial(const Seg *segs, uint32_t *ids, float *kv, const float *K3,
                                               uint32_t n) {
  __shared__ KI a[kSerialMax];
  __shared__ uint16_t Lp[kSerialMax], Bp[kSerialMax];
  __shared__ uint32_t stk[2 * 64], leaf[kSerialMax];
  const Seg s = segs[blockIdx.x];
  const uint32_t len = s.last - s.first;
  if (len > kSerialMax) {  // a long segment whose depth ran out (k_prep): heapsort in place
    const float *K = K3 + (size_t)(s.first / n) * n;
    if (threadIdx.x == 0)
      d_heapsort(ids + s.first, ids + s.last, [K](uint32_t x, uint32_t y) { return K[x] < K[y]; });
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += 64) kv[s.first + i] = K[ids[s.first + i]];
    return;  // sorted: the final insertion sort leaves it unchanged
  }
  for (uint32_t i = threadIdx.x; i < len; i += 64) a[i] = KI{kv[s.first + i], ids[s.first + i]};
  __syncthreads();
  const uint32_t nl = wave_introsort(a, len, s.depth, Lp, Bp, stk, leaf);
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nl; j += 64) d_insertion(a + (leaf[j] & 0xFFFFu), a + (leaf[j] >> 16));
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < len; i += 64) {
    ids[s.first + i] = a[i].id;
    kv[s.first + i] = a[i].k;
  }
}

// ---- one round of parallel introsort partitions ----------------------------
// A round is six launches that read the round's segment count m and element
// count E from device memory (the ctl words), so the host enqueues several
// rounds back to back with upper bounds for the grids and synchronises once
// per batch (a round whose m is 0 exits at once). Element space of a round:
// the active segments back to back (virtual index v; segment i covers
// [offs[i], offs[i+1])). Keys travel with the ids (kv[p] = K[ids[p]], swapped
// together), so a round reads them coalesced instead of gathering K[id].
constexpr int kRoundT = 256, kRoundI = 8, kRoundTile = kRoundT * kRoundI;
constexpr int kMaxRounds = 64;  // > the introsort depth limit 2 lg2(3n) + 1: a sort never needs more
// ctl words: [0] serial-list count, [1..3] unused, then (m, E) of round r at [4 + 2 r]
constexpr int kCtlWords = 4 + 2 * (kMaxRounds + 1);

// exclusive scan of cnt u32 values by one 256-thread block, out[cnt] = total
// (in == out allowed: each thread reads its values before writing them)
__device__ void block_excl_scan(const uint32_t *in, uint32_t *out, uint32_t cnt, uint32_t *sm) {
  uint32_t carry = 0;
  for (uint32_t base = 0; base < cnt; base += kRoundTile) {
    const uint32_t b0 = base + threadIdx.x * kRoundI;
    uint32_t v[kRoundI], acc = 0;
#pragma unroll
    for (int k = 0; k < kRoundI; ++k) {
      v[k] = acc;
      acc += (b0 + k < cnt) ? in[b0 + k] : 0u;
    }
    sm[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 1; o < kRoundT; o <<= 1) {
      const uint32_t x = threadIdx.x >= (uint32_t)o ? sm[threadIdx.x - o] : 0u;
      __syncthreads();
      sm[threadIdx.x] += x;
      __syncthreads();
    }
    const uint32_t ex = carry + (threadIdx.x ? sm[threadIdx.x - 1] : 0u);
#pragma unroll
    for (int k = 0; k < kRoundI; ++k)
      if (b0 + k < cnt) out[b0 + k] = ex + v[k];
    carry += sm[kRoundT - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[cnt] = carry;
}

struct Round {
  const Seg *cur;
  Seg *nxt;
  uint32_t *ctl;
  int r;  // (m, E) of this round at ctl[4 + 2 r], of the next at ctl[6 + 2 r]
  __device__ uint32_t m() const { return ctl[4 + 2 * r]; }
};

// per segment: median to the front, pivot key, size (0: depth exhausted, the
// segment goes to the serial list, whose introsort loop heapsorts it)
__global__ __launch_bounds__(kRoundT) void k_prep(Round R, uint32_t *ids, float *kv, float *kp, uint32_t *size,
                                                  Seg *serial) {
  const uint32_t m = R.m(), i = blockIdx.x * kRoundT + threadIdx.x;
  if (i >= m) return;
  const Seg s = R.cur[i];
  if (s.depth == 0) {
    serial[atomicAdd(&R.ctl[0], 1u)] = s;
    size[i] = 0;
    return;
  }
  // std::__move_median_to_first on (id, key) pairs
  const uint32_t f = s.first, l = s.last, mid = f + (l - f) / 2;
  const uint32_t pos[3] = {f + 1, mid, l - 1};
  const float a = kv[pos[0]], b = kv[pos[1]], c = kv[pos[2]];
  int w;  // which of the three moves to the front
  if (a < b) w = (b < c) ? 1 : (a < c) ? 2 : 0;
  else w = (a < c) ? 0 : (b < c) ? 2 : 1;
  const uint32_t q = pos[w];
  const uint32_t t = ids[f];
  const float tk = kv[f], pk = kv[q];
  ids[f] = ids[q];
  kv[f] = pk;
  ids[q] = t;
  kv[q] = tk;
  kp[i] = pk;
  size[i] = l - f;
}
// one block: the segment sizes into offs[0..m] (exclusive, offs[m] = E)
__global__ __launch_bounds__(kRoundT) void k_scan_sizes(Round R, const uint32_t *size, uint32_t *offs) {
  __shared__ uint32_t sm[kRoundT];
  block_excl_scan(size, offs, R.m(), sm);
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

// Prefix counts of the two flag kinds over the round's elements:
// a = stops the left scan of the partition (!(key < pivot), the pivot itself
// excluded), b = stops the right scan (!(pivot < key), the pivot included).
// Per tile of kRoundTile elements the in-tile inclusive counts (AB: a in bits
// 0-15, b in 16-31), the tile totals (exclusive-scanned over the tiles by
// k_scan_tiles), and per segment the in-tile count before its first element
// (startA / startB) and through its last (endA / endB).
struct Prefix {
  uint32_t *AB, *tileA, *tileB, *startA, *startB, *endA, *endB;
  __device__ uint32_t a_at(uint32_t v) const { return tileA[v / kRoundTile] + (AB[v] & 0xFFFFu); }
  __device__ uint32_t b_at(uint32_t v) const { return tileB[v / kRoundTile] + (AB[v] >> 16); }
  // a / b elements before segment i (o = its first element) and through it (oe = one past its last)
  __device__ uint32_t a_before(uint32_t i, uint32_t o) const { return tileA[o / kRoundTile] + startA[i]; }
  __device__ uint32_t b_before(uint32_t i, uint32_t o) const { return tileB[o / kRoundTile] + startB[i]; }
  __device__ uint32_t b_through(uint32_t i, uint32_t oe) const { return tileB[(oe - 1) / kRoundTile] + endB[i]; }
  __device__ uint32_t a_through(uint32_t i, uint32_t oe) const { return tileA[(oe - 1) / kRoundTile] + endA[i]; }
};

// A tile is 4 waves x 512 elements; a wave walks its 512 in 8 coalesced
// chunks of 64 (lane = element), counting the flags with ballots.
__global__ __launch_bounds__(kRoundT) void k_flags(Round R, const uint32_t *offs, const float *kv, const float *kp,
                                                   uint8_t *fl, uint32_t *segv, Prefix P) {
  constexpr uint32_t kWaveSpan = kRoundTile / (kRoundT / 64);
  __shared__ uint32_t wsum[kRoundT / 64];
  const uint32_t m = R.m(), E = offs[m];
  const uint32_t t0 = blockIdx.x * kRoundTile;
  if (t0 >= E) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u, wb = t0 + w * kWaveSpan;
  uint32_t i = wb < E ? seg_of(offs, m, wb) : 0;  // segment of this chunk's first element (wave-uniform)
  uint32_t inc[kRoundI], seg[kRoundI], run = 0;   // in-wave inclusive packed counts (a | b << 16)
  uint8_t fk[kRoundI];
#pragma unroll
  for (int c = 0; c < kRoundI; ++c) {
    const uint32_t v = wb + c * 64 + lane;
    bool fa = false, fb = false;
    uint32_t il = i;
    if (v < E) {
      while (offs[il + 1] <= v) ++il;  // zero-size segments (serial) are skipped
      const uint32_t o = offs[il];
      const float key = kv[R.cur[il].first + (v - o)], pk = kp[il];
      fa = v != o && !(key < pk);
      fb = v == o || !(pk < key);
      segv[v] = il;
      fl[v] = (uint8_t)((fa ? 1u : 0u) | (fb ? 2u : 0u));
    }
    const uint64_t ma = __ballot(fa), mb = __ballot(fb);
    inc[c] = run + ((lane_prefix(ma) + (fa ? 1u : 0u)) | ((lane_prefix(mb) + (fb ? 1u : 0u)) << 16));
    run += (uint32_t)__popcll(ma) | ((uint32_t)__popcll(mb) << 16);
    fk[c] = (uint8_t)((fa ? 1u : 0u) | (fb ? 2u : 0u));
    seg[c] = il;
    i = (uint32_t)__shfl((int)il, 63);
  }
  if (lane == 0) wsum[w] = run;
  __syncthreads();
  uint32_t woff = 0;
  for (uint32_t k = 0; k < w; ++k) woff += wsum[k];
#pragma unroll
  for (int c = 0; c < kRoundI; ++c) {
    const uint32_t v = wb + c * 64 + lane;
    if (v >= E) continue;
    const uint32_t in = woff + inc[c], il = seg[c];
    P.AB[v] = in;
    if (v == offs[il]) {
      const uint32_t ex = in - ((fk[c] & 1u) | ((uint32_t)(fk[c] >> 1) << 16));
      P.startA[il] = ex & 0xFFFFu;
      P.startB[il] = ex >> 16;
    }
    if (v + 1 == offs[il + 1]) {
      P.endA[il] = in & 0xFFFFu;
      P.endB[il] = in >> 16;
    }
  }
  if (threadIdx.x == 0) {
    const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    P.tileA[blockIdx.x] = tot & 0xFFFFu;
    P.tileB[blockIdx.x] = tot >> 16;
  }
}
// one block: the tile totals into exclusive prefixes
__global__ __launch_bounds__(kRoundT) void k_scan_tiles(Round R, const uint32_t *offs, Prefix P) {
  __shared__ uint32_t sm[kRoundT];
  const uint32_t nt = (offs[R.m()] + kRoundTile - 1) / kRoundTile;
  block_excl_scan(P.tileA, P.tileA, nt, sm);
  block_excl_scan(P.tileB, P.tileB, nt, sm);
}

// Element blocks: ranks of the a-elements from the left and the b-elements
// from the right, scattered into per-segment position lists L, R (v-space,
// offs[i] + rank - 1). Segment blocks (after the element blocks, one wave per
// segment): the swap count s. The a-element of rank k swaps with the
// b-element of rank k from the right while it lies left of it, i.e. while at
// least k b-elements lie strictly right of it: B_end - B(v) >= A(v) - A_before,
// i.e. A(v) + B(v) <= B_end + A_before. A + B never decreases along the
// segment, so the positions where that holds are a prefix [o, v*], and
// s = A(v*) - A_before (0 when even o fails); a 64-way search finds v*.
__global__ __launch_bounds__(kRoundT) void k_ranks(Round R, const uint32_t *offs, const uint8_t *fl,
                                                   const uint32_t *segv, Prefix P, uint32_t *Lpos, uint32_t *Rpos,
                                                   uint32_t *sw, uint32_t eblocks) {
  const uint32_t m = R.m(), E = offs[m];
  if (blockIdx.x < eblocks) {
    const uint32_t v = blockIdx.x * kRoundT + threadIdx.x;
    if (v >= E) return;
    const uint8_t f = fl[v];
    if (!f) return;
    const uint32_t i = segv[v], o = offs[i], p = R.cur[i].first + (v - o);
    if (f & 1u) Lpos[o + (P.a_at(v) - P.a_before(i, o)) - 1] = p;
    if (f & 2u) {
      const uint32_t bb = P.b_before(i, o);
      const uint32_t btot = P.b_through(i, offs[i + 1]) - bb, rank = P.b_at(v) - bb;
      Rpos[o + (btot - rank)] = p;
    }
    return;
  }
  const uint32_t i = (blockIdx.x - eblocks) * (kRoundT / 64) + threadIdx.x / 64, lane = threadIdx.x & 63u;
  if (i >= m) return;
  const uint32_t o = offs[i], oe = offs[i + 1];
  if (o == oe) return;  // depth exhausted: serial
  const uint32_t ab = P.a_before(i, o), C = P.b_through(i, oe) + ab;
  // largest v in [o, oe) with A(v) + B(v) <= C; the candidates are [lo, hi]
  uint32_t lo = o, hi = oe - 1;
  if (P.a_at(lo) + P.b_at(lo) > C) {
    if (lane == 0) sw[i] = 0;
    return;
  }
  while (hi > lo) {  // invariant: F(lo) <= C
    const uint32_t len = hi - lo, step = (len + 63) / 64;
    const uint32_t pr = min(hi, lo + (lane + 1) * step);
    const bool ok = P.a_at(pr) + P.b_at(pr) <= C;
    const uint64_t bm = __ballot(ok);  // a prefix of the lanes (F is monotone; clamped probes repeat hi)
    const int j = bm ? 63 - __clzll((unsigned long long)bm) : -1;  // last lane that holds
    if (j < 0) {
      hi = min(hi, lo + step) - 1;  // the answer lies in [lo, lo + step - 1]
    } else {
      const uint32_t at = min(hi, lo + (uint32_t)(j + 1) * step);
      lo = at;
      hi = (j == 63 || at == hi) ? hi : min(hi, at + step - 1);
    }
  }
  if (lane == 0) sw[i] = P.a_at(lo) - ab;
}

// the swaps (one thread per pair: its a-element, ids and keys together) and,
// per segment, the cut (where the left scan stops after the last swap) and
// the two parts: longer than kSerialMax -> the next round, else the serial list
__global__ __launch_bounds__(kRoundT) void k_swap_split(Round R, const uint32_t *offs, const uint32_t *size,
                                                        const uint8_t *fl, const uint32_t *segv, Prefix P,
                                                        const uint32_t *Lpos, const uint32_t *Rpos,
                                                        const uint32_t *sw, uint32_t *ids, float *kv, Seg *serial) {
  const uint32_t m = R.m(), E = offs[m];
  const uint32_t t = blockIdx.x * kRoundT + threadIdx.x;
  if (t < E && (fl[t] & 1u)) {
    const uint32_t i = segv[t], o = offs[i];
    const uint32_t rank = P.a_at(t) - P.a_before(i, o);
    if (rank <= sw[i]) {
      const uint32_t p = R.cur[i].first + (t - o), q = Rpos[o + rank - 1];
      const uint32_t x = ids[p];
      const float xk = kv[p];
      ids[p] = ids[q];
      kv[p] = kv[q];
      ids[q] = x;
      kv[q] = xk;
    }
  }
  if (t >= m || size[t] == 0) return;
  const Seg s = R.cur[t];
  const uint32_t o = offs[t], oe = offs[t + 1];
  const uint32_t na = P.a_through(t, oe) - P.a_before(t, o), k = sw[t];
  uint32_t cut;
  if (k == 0) cut = Lpos[o];  // the median of three guarantees an element >= pivot
  else {
    const uint32_t rk = Rpos[o + k - 1];
    cut = (k < na) ? min(Lpos[o + k], rk) : rk;
  }
  uint32_t *next_mE = R.ctl + 6 + 2 * R.r;
  const Seg parts[2] = {Seg{cut, s.last, s.depth - 1, 0}, Seg{s.first, cut, s.depth - 1, 0}};
  for (const Seg &q : parts) {
    if (q.last - q.first > kSerialMax) {
      R.nxt[atomicAdd(&next_mE[0], 1u)] = q;
      atomicAdd(&next_mE[1], q.last - q.first);
    } else if (q.last - q.first > 1) {
      serial[atomicAdd(&R.ctl[0], 1u)] = q;
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
__global__ void k_stage_copy(const SahChunk *chunks, uint32_t *ids3, float *kv3, const float *K3, uint32_t *backup,
                             uint32_t n) {
  const SahChunk c = chunks[blockIdx.x];
  for (uint32_t t = c.lo + threadIdx.x; t < c.hi; t += blockDim.x) {
    const uint32_t v = ids3[t];
    backup[t] = v;
    ids3[n + t] = v;
    ids3[2 * n + t] = v;
    kv3[n + t] = K3[n + v];
    kv3[2 * n + t] = K3[2 * n + v];
  }
}
// stage end: 1 = take the Y order, 2 = the Z order, 3 = restore (never evaluated by the reference)
__global__ void k_stage_apply(const SahChunk *chunks, const uint32_t *action, uint32_t *ids3, float *kv3,
                              const float *K3, const uint32_t *backup, uint32_t n) {
  const SahChunk c = chunks[blockIdx.x];
  const uint32_t a = action[c.task];
  if (a == 0) return;
  const uint32_t *src = a == 1 ? ids3 + n : a == 2 ? ids3 + 2 * n : backup;
  for (uint32_t t = c.lo + threadIdx.x; t < c.hi; t += blockDim.x) {
    const uint32_t v = src[t];
    ids3[t] = v;
    kv3[t] = K3[v];
  }
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
__global__ void k_tribox(const float4 *vpos, const uint32_t *idx, uint32_t n, TBox *tbox, float *K3, float *kv3) {
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
  kv3[t] = b.mx[0];  // the X order starts as the identity
  K3[n + t] = b.mx[1];
  K3[2 * n + t] = b.mx[2];
}

// the leaf triangles in slot order (bvh_layout's fill_tris, rt_host.cpp; the
// vertices /= w as triangles_raytracing.cpp:307-309): one thread per leaf,
// tab = (first slot, first position in the final order, count)
__global__ void k_fill_tris(const uint32_t *tab, uint32_t nl, const float4 *vpos, const uint32_t *idx,
                            const uint32_t *order, rtl::GTri *tris) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  const uint32_t first = tab[3 * l], pos = tab[3 * l + 1], cnt = tab[3 * l + 2];
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t id = order[pos + k];
    float v[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float4 p = vpos[idx[3 * id + j]];
      v[j][0] = p.x / p.w;
      v[j][1] = p.y / p.w;
      v[j][2] = p.z / p.w;
    }
    rtl::GTri g;
    g.v0x = v[0][0]; g.v0y = v[0][1]; g.v0z = v[0][2];
    g.orig_id = id;
    g.e1x = v[1][0] - v[0][0]; g.e1y = v[1][1] - v[0][1]; g.e1z = v[1][2] - v[0][2];
    g.e2x = v[2][0] - v[0][0]; g.e2y = v[2][1] - v[0][1]; g.e2z = v[2][2] - v[0][2];
    g.pad1 = g.pad2 = 0.0f;
    tris[first + k] = g;
  }
}

// ---- host side ---------------------------------------------------------------
// RTAMD_BVH_TIMING=1: per-phase wall time of a device build on stderr (the
// phases are synchronised for the measurement)
struct PhaseTimer {
  bool on = ab_env("RTAMD_BVH_TIMING") != nullptr;
  double acc[8] = {};
  double host[4] = {};  // wall time of host-side stage sections (no syncs): prologue, FIFO, apply+boxes
  long faults[4] = {};  // minor page faults in those sections
  std::chrono::steady_clock::time_point h0;
  long f0 = 0;
  static long minflt() {
    rusage u;
    getrusage(RUSAGE_THREAD, &u);
    return u.ru_minflt;
  }
  void hstart() {
    h0 = std::chrono::steady_clock::now();
    if (on) f0 = minflt();
  }
  void hstop(int k) {
    host[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
    if (on) faults[k] += minflt() - f0;
  }
  int rounds = 0, stages = 0, serial_launches = 0;
  std::chrono::steady_clock::time_point t0;
  hipStream_t st = nullptr;
  void start() {
    if (!on) return;
    HIP_NOTE(hipStreamSynchronize(st));
    t0 = std::chrono::steady_clock::now();
  }
  void stop(int k) {
    if (!on) return;
    HIP_NOTE(hipStreamSynchronize(st));
    acc[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
};

// One device allocation for a whole build, carved into the build's buffers
// (a hipMalloc / hipFree pair per buffer costs more than the launches of a
// small stage). Buffers that outgrow their share fall back to hipMalloc.
struct DevArena {
  char *base = nullptr;
  size_t cap = 0, off = 0;
  ~DevArena() {
    if (base) HIP_NOTE(hipFree(base));
  }
  static size_t round(size_t b) { return (b + 255) & ~(size_t)255; }
  void *take(size_t bytes) {
    if (!base || off + round(bytes) > cap) return nullptr;
    void *q = base + off;
    off += round(bytes);
    return q;
  }
};
thread_local DevArena *t_arena = nullptr;  // the arena of the build running on this thread

template <class T>
struct DBuf {
  T *p = nullptr;
  size_t cap = 0;
  bool owned = false;
  ~DBuf() {
    if (p && owned) HIP_NOTE(hipFree(p));
  }
  static size_t first_cap(size_t n) { return std::max<size_t>(n, 1024); }  // what the first reserve(n) takes
  // grows geometrically: the per-stage buffers widen with the tree, and a
  // hipFree / hipMalloc pair at every stage for each of them synchronises the
  // device each time
  int reserve(size_t n) {
    if (n <= cap) return RT_OK;
    const size_t want = std::max<size_t>({n, 2 * cap, 1024});
    if (p && owned) HIP_NOTE(hipFree(p));
    p = nullptr;
    cap = 0;
    owned = false;
    if (t_arena)
      if (void *q = t_arena->take(want * sizeof(T))) {
        p = static_cast<T *>(q);
        cap = want;
        return RT_OK;
      }
    HIP_TRY(hipMalloc(&p, want * sizeof(T)));
    owned = true;
    cap = want;
    return RT_OK;
  }
};
template <class T>
size_t dbytes(size_t n) {  // arena bytes of a DBuf<T> whose first reserve is n
  return DevArena::round(DBuf<T>::first_cap(n) * sizeof(T));
}

// rtx_bvh_inject_failure: the next N device builds fail as a device error would
std::atomic<int> g_inject_fail{0};

inline int lg2(uint64_t n) { return 63 - __builtin_clzll(n); }

struct Sorter {
  uint32_t n = 0;  // triangles (one axis block of the 3n space)
  uint32_t *ids = nullptr;
  float *kv = nullptr;  // kv[p] = K3[block of p][ids[p]], kept in step with ids
  const float *K3 = nullptr;
  DBuf<Seg> segA, segB, serial;
  DBuf<uint32_t> size, offs, sw, AB, tiles, bnd, segv, Lpos, Rpos, ctl;
  DBuf<uint8_t> fl;
  DBuf<float> kp;
  size_t segcap = 0, tilecap = 0;
  hipStream_t st = nullptr;
  PhaseTimer own_pt;             // per build: concurrent builds share no state
  PhaseTimer *pt = &own_pt;

  // arena bytes of init(ntri)'s buffers (the same list)
  static size_t arena_bytes(uint32_t ntri) {
    const size_t N = 3 * (size_t)ntri, sercap = N / 2 + 4096, sc = N / (kSerialMax + 1) + 16,
                 tc = N / kRoundTile + 2;
    return 2 * dbytes<Seg>(sc) + dbytes<Seg>(sercap) + 2 * dbytes<uint32_t>(sc + 1) +
           dbytes<uint32_t>(sc) + dbytes<float>(sc) + dbytes<uint32_t>(N) + dbytes<uint8_t>(N) +
           dbytes<uint32_t>(2 * tc) + dbytes<uint32_t>(4 * sc) + 3 * dbytes<uint32_t>(N) + dbytes<uint32_t>(kCtlWords);
  }
  int init(uint32_t ntri, uint32_t *ids3, float *kv3, const float *keys3) {
    n = ntri;
    ids = ids3;
    kv = kv3;
    K3 = keys3;
    const size_t N = 3 * (size_t)n, sercap = N / 2 + 4096;
    segcap = N / (kSerialMax + 1) + 16;
    tilecap = N / kRoundTile + 2;
    int rc;
    if ((rc = segA.reserve(segcap)) || (rc = segB.reserve(segcap)) || (rc = serial.reserve(sercap)) ||
        (rc = size.reserve(segcap + 1)) || (rc = offs.reserve(segcap + 1)) || (rc = sw.reserve(segcap)) ||
        (rc = kp.reserve(segcap)) || (rc = AB.reserve(N)) || (rc = fl.reserve(N)) ||
        (rc = tiles.reserve(2 * tilecap)) || (rc = bnd.reserve(4 * segcap)) || (rc = segv.reserve(N)) ||
        (rc = Lpos.reserve(N)) || (rc = Rpos.reserve(N)) || (rc = ctl.reserve(kCtlWords)))
      return rc;
    return RT_OK;
  }

  // sort every segment of `init` (host list): exactly std::sort on each
  int sort(const std::vector<Seg> &init) {
    std::vector<Seg> act, ser;
    uint32_t maxlen = 0;
    for (const Seg &s : init) {
      if (s.last - s.first <= 1) continue;
      (s.last - s.first > kSerialMax ? act : ser).push_back(s);
      if (s.last - s.first > kSerialMax) maxlen = std::max(maxlen, s.last - s.first);
    }
    uint32_t m = (uint32_t)act.size(), E = 0;
    for (const Seg &s : act) E += s.last - s.first;
    if (m > segcap || ser.size() > serial.cap) return rterr::set(RT_E_DEVICE, "bound: sort segment list");
    uint32_t hc[kCtlWords] = {};
    hc[0] = (uint32_t)ser.size();
    hc[4] = m;
    hc[5] = E;
    if (!ser.empty()) HIP_TRY(hipMemcpyAsync(serial.p, ser.data(), ser.size() * sizeof(Seg), hipMemcpyHostToDevice, st));
    if (m) HIP_TRY(hipMemcpyAsync(segA.p, act.data(), m * sizeof(Seg), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctl.p, hc, sizeof(hc), hipMemcpyHostToDevice, st));
    const Prefix P{AB.p, tiles.p, tiles.p + tilecap, bnd.p, bnd.p + segcap, bnd.p + 2 * segcap, bnd.p + 3 * segcap};
    pt->start();
    // rounds are enqueued in batches, with grid bounds: E never grows, m at
    // most doubles and each active segment holds more than kSerialMax elements;
    // the first batch is the round count of even splits of the longest segment
    int r = 0, batch = m ? std::max(1, lg2(maxlen / kSerialMax) + 1) : 0;
    uint32_t mb = m, Eb = E;
    while (mb > 0) {
      for (int b = 0; b < batch && mb > 0; ++b, ++r) {
        if (r >= kMaxRounds) return rterr::set(RT_E_DEVICE, "bound: sort partition rounds");
        ++pt->rounds;
        const Round R{(r & 1) ? segB.p : segA.p, (r & 1) ? segA.p : segB.p, ctl.p, r};
        const uint32_t gm = (mb + kRoundT - 1) / kRoundT, gt = (Eb + kRoundTile - 1) / kRoundTile,
                       ge = (std::max(Eb, mb) + kRoundT - 1) / kRoundT, eb = (Eb + kRoundT - 1) / kRoundT,
                       gs = (mb + kRoundT / 64 - 1) / (kRoundT / 64);
        k_prep<<<std::max(gm, 1u), kRoundT, 0, st>>>(R, ids, kv, kp.p, size.p, serial.p);
        k_scan_sizes<<<1, kRoundT, 0, st>>>(R, size.p, offs.p);
        k_flags<<<std::max(gt, 1u), kRoundT, 0, st>>>(R, offs.p, kv, kp.p, fl.p, segv.p, P);
        k_scan_tiles<<<1, kRoundT, 0, st>>>(R, offs.p, P);
        k_ranks<<<eb + gs, kRoundT, 0, st>>>(R, offs.p, fl.p, segv.p, P, Lpos.p, Rpos.p, sw.p, eb);
        k_swap_split<<<std::max(ge, 1u), kRoundT, 0, st>>>(R, offs.p, size.p, fl.p, segv.p, P, Lpos.p, Rpos.p,
                                                           sw.p, ids, kv, serial.p);
        HIP_TRY(hipGetLastError());
        mb = std::min<uint64_t>(2ull * mb, Eb / (kSerialMax + 1));
      }
      HIP_TRY(hipMemcpyAsync(hc, ctl.p, (size_t)(6 + 2 * r) * 4, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      mb = hc[4 + 2 * r];
      Eb = hc[5 + 2 * r];
      batch = 2;
    }
    if (r == 0) {
      HIP_TRY(hipMemcpyAsync(hc, ctl.p, 4, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
    }
    const uint32_t nser = hc[0];
    pt->stop(0);
    pt->start();
    if (nser) k_serial<<<nser, 64, 0, st>>>(serial.p, ids, kv, K3, n);
    ++pt->serial_launches;
    HIP_TRY(hipGetLastError());
    pt->stop(1);
    return RT_OK;
  }
};

}  // namespace

namespace rth {

bool build_bvh8_gpu(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                    std::string &err, unsigned want) {
  // every device-side failure is reported as "GPU BVH build: <step>: <HIP
  // error>" (RT_E_DEVICE at the C ABI; in AUTO mode the host builder takes
  // over unless the fault is sticky); a bound of the builder's own stage logic
  // that is exceeded is "GPU BVH builder bound: <what>" (RT_E_DEVICE, never
  // hidden by the fallback: it is a builder bug, not a device failure); input
  // errors carry no prefix (RT_E_INVALID)
  auto fail = [&](const char *what) {
    const std::string m = rterr::get();
    err = m.rfind("bound: ", 0) == 0 ? "GPU BVH builder bound: " + std::string(what) + ": " + m.substr(7)
                                     : std::string("GPU BVH build: ") + what + ": " + m;
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
  // wall time of the whole call, teardown included (RTAMD_BVH_TIMING)
  struct WallClock {
    bool on = ab_env("RTAMD_BVH_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), tv = t0, te = t0;
    static double ms(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    }
    ~WallClock() {
      if (on) {
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[bvh gpu] wall %.1f ms (validation %.1f, teardown %.1f)\n", ms(t0, t1), ms(t0, tv),
                     ms(te, t1));
      }
    }
  } wall;
  if (nidx < 0 || nidx % 3 != 0) { err = "index count must be a multiple of 3"; return false; }
  uint32_t imax = 0;  // a max reduction vectorises; an early-exit loop does not
  for (int64_t i = 0; i < nidx; ++i) imax = std::max(imax, idx[i]);
  if (nidx && (int64_t)imax >= nverts) { err = "vertex index out of range"; return false; }
  wall.tv = std::chrono::steady_clock::now();
  const uint32_t n = (uint32_t)(nidx / 3);
  if ((uint64_t)n > rtl::kMaxLeafFirstTri || 3ull * n >= (1ull << 31)) { err = "too many triangles"; return false; }
  out = BVHGpu();
  if (n == 0) { out.root_word = rtl::kInvalidChild; return true; }
  if (const int inj = g_inject_fail.load(); inj != 0) {  // rtx_bvh_inject_failure
    g_inject_fail.fetch_add(inj > 0 ? -1 : 1);
    if (inj < 0) {  // a simulated builder bug: never hidden by the host fallback
      err = "GPU BVH builder bound: injected bound";
      return false;
    }
    return hfail("injected failure", hipErrorOutOfMemory);  // a simulated device failure
  }

  const auto tb0 = std::chrono::steady_clock::now();
  PhaseTimer pt;
  pt.start();
  DBuf<float4> dv;
  DBuf<uint32_t> didx, ids3, backup, dact;
  DBuf<float> K3, KV3;
  DBuf<TBox> tbox, boxes, cbox, cpre, csuf;
  DBuf<Task> dtasks;
  DBuf<SahChunk> dchunks, drch;
  DBuf<SahGroup> dgroups, drgrp;
  DBuf<TBox> rcbox;
  std::vector<SahChunk> rch;  // per-stage child-box chunk table (host copy)
  std::vector<SahGroup> rgrp;
  uint32_t NC = 0, NC0 = 0;
  DBuf<float> ccost, dpsa;
  DBuf<uint32_t> cdivv;
  Sorter S;
  // every buffer at its bound, from one allocation. Per stage: the candidates
  // are disjoint ranges of > 8 triangles (tasks <= n / 9), each cut into
  // chunks of kSahChunk on 3 axes; completed nodes' child ranges are disjoint
  // (<= n); leaves <= n.
  const size_t Tmax = n / 9 + 2, NCmax = 3 * (Tmax + n / kSahChunk + 2), NGmax = 3 * Tmax,
               NRmax = (size_t)n + 1, NRCmax = NRmax + n / kSahChunk + 2, maxranges = 2 * (size_t)n + 8;
  DevArena arena;
  {
    const size_t bytes = dbytes<float4>((size_t)nverts) + dbytes<uint32_t>((size_t)nidx) +
                         dbytes<uint32_t>(3 * (size_t)n) + dbytes<uint32_t>(n) + 2 * dbytes<float>(3 * (size_t)n) +
                         dbytes<TBox>(n) + Sorter::arena_bytes(n) + 2 * dbytes<uint32_t>(Tmax) +
                         dbytes<Task>(Tmax) + dbytes<SahChunk>(NCmax) + dbytes<SahGroup>(NGmax) +
                         3 * dbytes<TBox>(NCmax) + dbytes<float>(NCmax) + dbytes<uint32_t>(NCmax) +
                         dbytes<float>(NGmax) + dbytes<TBox>(maxranges) + dbytes<SahChunk>(NRCmax) +
                         dbytes<SahGroup>(NRmax) + dbytes<TBox>(NRCmax) + dbytes<uint32_t>(3 * (size_t)n);
    BVH_DEV(hipMalloc(&arena.base, bytes), "allocation");
    arena.cap = bytes;
  }
  struct ArenaScope {
    explicit ArenaScope(DevArena *a) { t_arena = a; }
    ~ArenaScope() { t_arena = nullptr; }
  } arena_scope(&arena);
  if (dv.reserve((size_t)nverts) || didx.reserve((size_t)nidx) || ids3.reserve(3 * (size_t)n) ||
      backup.reserve(n) || K3.reserve(3 * (size_t)n) || KV3.reserve(3 * (size_t)n) || tbox.reserve(n) ||
      S.init(n, ids3.p, KV3.p, K3.p) || dact.reserve(Tmax) || cdivv.reserve(NCmax) || dtasks.reserve(Tmax) ||
      dchunks.reserve(NCmax) || dgroups.reserve(NGmax) || cbox.reserve(NCmax) || cpre.reserve(NCmax) ||
      csuf.reserve(NCmax) || ccost.reserve(NCmax) || dpsa.reserve(NGmax) || boxes.reserve(maxranges) ||
      drch.reserve(NRCmax) || drgrp.reserve(NRmax) || rcbox.reserve(NRCmax))
    return fail("allocation");
  S.pt = &pt;
  hipStream_t st = nullptr;
  BVH_DEV(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  S.st = st;
  pt.st = st;
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { HIP_NOTE(hipStreamDestroy(s)); }
  } sg{st};
  std::vector<uint32_t> iota(n);
  for (uint32_t t = 0; t < n; ++t) iota[t] = t;
  // (the caller's arrays through rtdma: pinned memory only ever reaches the DMA)
  BVH_DEV(rtdma::h2d(dv.p, vpos4, (size_t)nverts * 16, st), "upload");
  BVH_DEV(rtdma::h2d(didx.p, idx, (size_t)nidx * 4, st), "upload");
  BVH_DEV(hipMemcpyAsync(ids3.p, iota.data(), (size_t)n * 4, hipMemcpyHostToDevice, st), "upload");
  k_tribox<<<(n + 255) / 256, 256, 0, st>>>(dv.p, didx.p, n, tbox.p, K3.p, KV3.p);
  BVH_DEV(hipGetLastError(), "triangle boxes");
  pt.stop(7);  // allocation, upload, triangle boxes

  // host side of the stages (rt_bvhstage.cpp): nodes, per-node FIFO state,
  // open lists, child ranges. A node's child boxes are computed in the stage
  // that completes the node, over the triangle order at that point (calc_bbox
  // at creation, triangles_raytracing.cpp:199), before the children's own
  // sorts reorder their ranges (first-kept among equal bounds, so -0.0 / +0.0
  // come out as the reference's sequential min / max)
  bvhs::Stage SG;
  if (!SG.init(n, kSahChunk)) return hfail("host arrays", hipErrorOutOfMemory);
  if (boxes.reserve(SG.ranges.cap)) return fail("allocation");
  std::vector<float> hcc;
  std::vector<uint32_t> hcd;
  const auto ts0 = std::chrono::steady_clock::now();
  while (SG.n_open) {
    ++pt.stages;
    pt.hstart();
    const size_t r0 = SG.n_ranges;
    SG.prologue();
    const uint32_t T = (uint32_t)SG.tasks.size();
    if (T) {
      NC = (uint32_t)SG.ch.size();
      NC0 = SG.nc_axis;  // the axis-0 chunks come first
      const uint32_t NG = 3 * T;
      if (dtasks.reserve(T) || dact.reserve(T) || dchunks.reserve(NC) || dgroups.reserve(NG) || cbox.reserve(NC) ||
          cpre.reserve(NC) || csuf.reserve(NC) || ccost.reserve(NC) || cdivv.reserve(NC) || dpsa.reserve(NG))
        return fail("allocation");
      BVH_DEV(hipMemcpyAsync(dtasks.p, SG.tasks.data(), T * sizeof(Task), hipMemcpyHostToDevice, st), "upload");
      BVH_DEV(hipMemcpyAsync(dchunks.p, SG.ch.data(), NC * sizeof(SahChunk), hipMemcpyHostToDevice, st), "upload");
      BVH_DEV(hipMemcpyAsync(dgroups.p, SG.grp.data(), NG * sizeof(SahGroup), hipMemcpyHostToDevice, st), "upload");
      k_stage_copy<<<NC0, 256, 0, st>>>(dchunks.p, ids3.p, KV3.p, K3.p, backup.p, n);
      pt.hstop(0);
      if (S.sort(SG.segs)) return fail("sort");
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
      pt.hstart();
      SG.reduce_sah(hcc.data(), hcd.data());
    }
    // createNode's FIFO, candidate by candidate (triangles_raytracing.cpp:162-173)
    std::string ferr;
    if (!SG.fifo(ferr)) {
      err = "GPU BVH builder bound: createNode FIFO: " + ferr;
      return false;
    }
    pt.hstop(1);
    pt.hstart();
    if (T) {
      BVH_DEV(hipMemcpyAsync(dact.p, SG.action.data(), T * 4, hipMemcpyHostToDevice, st), "upload");
      k_stage_apply<<<NC0, 256, 0, st>>>(dchunks.p, dact.p, ids3.p, KV3.p, K3.p, backup.p, n);
      BVH_DEV(hipGetLastError(), "stage apply");
    }
    if (SG.n_ranges > r0) {  // boxes of the children of the nodes completed in this stage
      const uint32_t nr = (uint32_t)(SG.n_ranges - r0);
      rch.clear();
      rgrp.resize(nr);
      for (uint32_t r = 0; r < nr; ++r) {
        const Task &R = SG.ranges[r0 + r];
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
    }
    // the tables uploaded above are rewritten by the next stage's host code
    BVH_DEV(hipStreamSynchronize(st), "stage end");
    pt.hstop(2);
    SG.advance();
  }
  if (pt.on) {
    HIP_NOTE(hipStreamSynchronize(st));
    pt.acc[5] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
  }
  pt.start();
  // the child boxes, and the final triangle order when the host needs it
  const bool dev_tris = (want & kBvhTris) && (want & kBvhDeviceTris);
  std::vector<uint32_t> cur;
  if (SG.n_ranges) {
    std::vector<TBox> hb(SG.n_ranges);
    BVH_DEV(hipMemcpyAsync(hb.data(), boxes.p, hb.size() * sizeof(TBox), hipMemcpyDeviceToHost, st), "child boxes");
    BVH_DEV(hipStreamSynchronize(st), "child boxes");
    for (size_t r = 0; r < SG.n_ranges; ++r) {
      BvhBox &b = SG.H[SG.range_of[r].first].box[SG.range_of[r].second];
      std::memcpy(b.mn, hb[r].mn, 12);
      std::memcpy(b.mx, hb[r].mx, 12);
    }
  }
  if ((want & kBvhPerm) || ((want & kBvhTris) && !dev_tris)) {
    cur.resize(n);
    BVH_DEV(hipMemcpyAsync(cur.data(), ids3.p, (size_t)n * 4, hipMemcpyDeviceToHost, st), "download");
    BVH_DEV(hipStreamSynchronize(st), "download");
  }
  pt.stop(6);
  pt.start();
  bvh_layout(vpos4, idx, nidx, HostNodes(SG.H.p, SG.n_nodes), cur, out, want, !dev_tris);
  pt.stop(3);
  if (dev_tris) {  // the leaf triangles straight from the device-side order (bvh_layout's fill_tris)
    pt.start();
    const uint32_t nl = (uint32_t)(out.leaf_tab.size() / 3);
    DBuf<uint32_t> dtab;
    void *tp = nullptr;
    const size_t tbytes = ((size_t)out.n_tris + 8) * sizeof(rtl::GTri);
    BVH_DEV(hipMalloc(&tp, tbytes), "triangles");
    out.dev_tris.p = tp;
    out.dev_tris.bytes = tbytes;
    out.dev_tris.release = [](void *q) { HIP_NOTE(hipFree(q)); };
    BVH_DEV(hipMemsetAsync((rtl::GTri *)tp + out.n_tris, 0, 8 * sizeof(rtl::GTri), st), "triangles");
    if (nl) {
      if (dtab.reserve(3 * (size_t)nl)) return fail("allocation");
      BVH_DEV(hipMemcpyAsync(dtab.p, out.leaf_tab.data(), (size_t)nl * 12, hipMemcpyHostToDevice, st), "triangles");
      k_fill_tris<<<(nl + 255) / 256, 256, 0, st>>>(dtab.p, nl, dv.p, didx.p, ids3.p, (rtl::GTri *)tp);
      BVH_DEV(hipGetLastError(), "triangles");
    }
    BVH_DEV(hipStreamSynchronize(st), "triangles");
    out.leaf_tab.clear();
    out.leaf_tab.shrink_to_fit();
    pt.stop(4);
  }
  if (pt.on)
    std::fprintf(stderr,
                 "[bvh gpu] %u tris: total %.1f ms | alloc+upload+tri boxes %.1f, stages %.1f (partition rounds %.1f "
                 "(%d rounds), serial sorts %.1f (%d launches), SAH %.1f, other %.1f), boxes+download %.1f, layout "
                 "%.1f, device triangles %.1f; %d stages; host sections: stage prologue %.1f, FIFO %.1f, apply+boxes %.1f (minor faults %ld / %ld / %ld)\n",
                 n, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count(),
                 pt.acc[7], pt.acc[5], pt.acc[0], pt.rounds, pt.acc[1], pt.serial_launches, pt.acc[2],
                 pt.acc[5] - pt.acc[0] - pt.acc[1] - pt.acc[2], pt.acc[6], pt.acc[3], pt.acc[4], pt.stages, pt.host[0],
                 pt.host[1], pt.host[2], pt.faults[0], pt.faults[1], pt.faults[2]);
  wall.te = std::chrono::steady_clock::now();
  return true;
#undef BVH_DEV
}

}  // namespace rth

// ---- diagnostics (not part of include/rtamd.h) ------------------------------
extern "C" {

// Fault injection for the builder fallback tests: the next |n| device builds
// fail before touching the GPU, with a device error (n > 0) or with an
// exceeded bound of the builder's own stage logic (n < 0).
int rtx_bvh_inject_failure(int32_t n) {
  g_inject_fail.store(n);
  return RT_OK;
}

// The device sort against libstdc++ std::sort (host_introsort) on n keys:
// ids[] receives the device permutation; returns RT_OK and *mismatch = number
// of positions that differ from the host permutation. depth < 0: std::sort's
// own depth limit (2 lg n); smaller limits force the heapsort fallback.
// The device builder's stage loop with the device steps done on the host
// (rth::bvhs::emulate_device_build; no GPU needed): canonical export as
// rt_bvh_export, `threads` OpenMP threads for the stage passes (0: default).
int rtx_bvh_stage_emulate(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, uint32_t *canon,
                          int64_t *nnodes) {
  if (!vpos4 || !idx || !nnodes || nverts <= 0 || nidx <= 0) return rterr::set(RT_E_INVALID, "bad mesh");
  rth::BVHGpu b;
  std::string err;
  if (!rth::bvhs::emulate_device_build(vpos4, nverts, idx, nidx, b, err, rth::kBvhCanon))
    return rterr::set(RT_E_INVALID, err.c_str());
  const int64_t nn = (int64_t)b.canon.size() / 52;
  if (canon) {
    if (*nnodes < nn) return rterr::set(RT_E_INVALID, "buffer too small");
    std::memcpy(canon, b.canon.data(), b.canon.size() * 4);
  }
  *nnodes = nn;
  return RT_OK;
}

int rtx_sort_check(const float *keys, int64_t n, int32_t depth, uint32_t *ids_out, int64_t *mismatch) {
  if (!keys || n <= 0 || n >= (1ll << 30) || !mismatch) return rterr::set(RT_E_INVALID, "bad arguments");
  const uint32_t nn = (uint32_t)n;
  std::vector<uint32_t> host(nn);
  for (uint32_t i = 0; i < nn; ++i) host[i] = i;
  rth::host_introsort(host.data(), nn, keys, depth);
  // the sort works on a 3n space; the test uses axis block 0 only
  DBuf<uint32_t> ids3;
  DBuf<float> K3, KV3;
  Sorter S;
  if (int rc = ids3.reserve(3 * (size_t)nn)) return rc;
  if (int rc = K3.reserve(3 * (size_t)nn)) return rc;
  if (int rc = KV3.reserve(3 * (size_t)nn)) return rc;
  if (int rc = S.init(nn, ids3.p, KV3.p, K3.p)) return rc;
  HIP_TRY(hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking));
  std::vector<uint32_t> iota(nn);
  for (uint32_t i = 0; i < nn; ++i) iota[i] = i;
  int rc = RT_OK;
  if (hipMemcpy(ids3.p, iota.data(), (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(K3.p, keys, (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(KV3.p, keys, (size_t)nn * 4, hipMemcpyHostToDevice) != hipSuccess)
    rc = rterr::set(RT_E_DEVICE, "upload");
  if (!rc) rc = S.sort({Seg{0, nn, depth < 0 ? 2 * lg2(nn) : depth, 0}});
  std::vector<uint32_t> dev(nn);
  std::vector<float> dkv(nn);
  if (!rc && (hipStreamSynchronize(S.st) != hipSuccess ||
              hipMemcpy(dev.data(), ids3.p, (size_t)nn * 4, hipMemcpyDeviceToHost) != hipSuccess ||
              hipMemcpy(dkv.data(), KV3.p, (size_t)nn * 4, hipMemcpyDeviceToHost) != hipSuccess))
    rc = rterr::set(RT_E_DEVICE, "download");
  HIP_NOTE(hipStreamDestroy(S.st));
  if (rc) return rc;
  int64_t bad = 0;
  // a position counts once if its id differs from std::sort's or its carried
  // key is not that id's key
  for (uint32_t i = 0; i < nn; ++i)
    bad += dev[i] != host[i] || dev[i] >= nn || std::memcmp(&dkv[i], &keys[dev[i] < nn ? dev[i] : 0], 4) != 0;
  *mismatch = bad;
  if (ids_out) std::memcpy(ids_out, dev.data(), (size_t)nn * 4);
  return RT_OK;
}

}  // extern "C"
