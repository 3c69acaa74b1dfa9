// rt_bvhstage.cpp -- host side of the device BVH build's stages (rt_bvhstage.h).
// Each stage: prologue() lists the stage's sorts and SAH chunks over all open
// nodes, the device sorts and sweeps them (rt_bvhgpu.hip), reduce_sah() takes
// the first minimum per (candidate, axis), fifo() runs createNode's candidate
// FIFO (triangles_raytracing.cpp:155-225) per open node. Passes over the open
// nodes run in parallel; exclusive prefix sums of per-node counts give every
// output the position the serial loop gives it.
#include "rt_bvhstage.h"

#include <sys/mman.h>

#include <algorithm>
#include <new>

namespace rth {
namespace bvhs {

namespace {

constexpr size_t kParMin = 2048;  // open nodes below this: one thread

inline int lg2(uint64_t v) { return 63 - __builtin_clzll(v); }

// in-place exclusive prefix sum; returns the total
uint64_t excl_scan(std::vector<uint32_t> &v, size_t cnt) {
  uint64_t run = 0;
  for (size_t i = 0; i < cnt; ++i) {
    const uint32_t x = v[i];
    v[i] = (uint32_t)run;
    run += x;
  }
  return run;
}

}  // namespace

template <class T>
Arena<T>::~Arena() {
  if (p) munmap(p, bytes);
}
template <class T>
bool Arena<T>::reserve(size_t c) {
  const size_t huge = (size_t)2 << 20;
  bytes = (std::max<size_t>(c, 1) * sizeof(T) + huge - 1) / huge * huge;
  void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (m == MAP_FAILED) {
    bytes = 0;
    return false;
  }
  (void)madvise(m, bytes, MADV_HUGEPAGE);
  p = static_cast<T *>(m);
  cap = c;
  return true;
}
template struct Arena<BvhHostNode>;
template struct Arena<OpenState>;
template struct Arena<int32_t>;
template struct Arena<Task>;
template struct Arena<std::pair<int32_t, int32_t>>;

bool Stage::init(uint32_t ntri, uint32_t chunk_len) {
  n = ntri;
  chunk = chunk_len;
  // at most 2 n - 1 nodes (every node holds >= 1 triangle); every node but
  // the root is one child range and enters one open list
  const size_t maxn = 2 * (size_t)n + 8;
  if (!H.reserve(maxn) || !OS.reserve(maxn) || !open.reserve(maxn) || !next.reserve(maxn) ||
      !ranges.reserve(maxn) || !range_of.reserve(maxn))
    return false;
  new (&H[0]) BvhHostNode();
  OpenState &r = OS[0];
  r.start = 0;
  r.end = 3 * n;
  r.qn = 1;
  r.nd = 0;
  r.q[0] = Cand{0, 3 * n};
  n_nodes = 1;
  open[0] = 0;
  n_open = 1;
  n_next = 0;
  n_ranges = 0;
  return true;
}

void Stage::prologue() {
  const size_t no = n_open;
  task_off.resize(no + 1);
  a_.resize(no + 1);
#pragma omp parallel for schedule(static) if (no >= kParMin)
  for (size_t o = 0; o < no; ++o) {
    const OpenState &N = OS[open[o]];
    uint32_t g = 0;
    for (uint32_t c = 0; c < N.qn; ++c) g += N.q[c].hi - N.q[c].lo > 24;
    task_off[o] = N.qn;
    a_[o] = g;
  }
  const size_t ncand = excl_scan(task_off, no), T = excl_scan(a_, no);
  task_of.resize(ncand);
  tasks.resize(T);
#pragma omp parallel for schedule(static) if (no >= kParMin)
  for (size_t o = 0; o < no; ++o) {
    const OpenState &N = OS[open[o]];
    uint32_t k = a_[o];
    for (uint32_t c = 0; c < N.qn; ++c) {
      const bool gpu = N.q[c].hi - N.q[c].lo > 24;
      task_of[task_off[o] + c] = gpu ? (int32_t)k : -1;
      if (gpu) tasks[k++] = Task{N.q[c].lo / 3, N.q[c].hi / 3};
    }
  }
  // chunks of every (task, axis): [axis-0 chunks of all tasks | axis 1 | axis 2]
  b_.resize(T + 1);
  for (size_t t = 0; t < T; ++t) b_[t] = (tasks[t].e - tasks[t].s + chunk - 1) / chunk;
  nc_axis = (uint32_t)excl_scan(b_, T);
  ch.resize(3 * (size_t)nc_axis);
  grp.resize(3 * T);
  segs.resize(3 * T);
#pragma omp parallel for schedule(static) if (T >= kParMin)
  for (size_t t = 0; t < T; ++t) {
    const Task tk = tasks[t];
    const uint32_t cnt = (tk.e - tk.s + chunk - 1) / chunk;
    for (uint32_t a = 0; a < 3; ++a) {
      SahGroup &G = grp[3 * t + a];
      G.first = a * nc_axis + b_[t];
      G.count = cnt;
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t lo = tk.s + j * chunk;
        ch[G.first + j] = SahChunk{(uint32_t)t, a, lo, std::min<uint32_t>(tk.e, lo + chunk), 3 * (uint32_t)t + a};
      }
      segs[a * T + t] = Seg{a * n + tk.s, a * n + tk.e, 2 * lg2(tk.e - tk.s), 0};
    }
  }
  cost.resize(3 * T);
  dvd.resize(3 * T);
  action.assign(T, 0u);
}

void Stage::reduce_sah(const float *ccost, const uint32_t *cdiv) {
  const size_t NG = grp.size();
#pragma omp parallel for schedule(static) if (NG >= kParMin)
  for (size_t g = 0; g < NG; ++g) {
    float bc = __builtin_huge_valf();
    uint32_t bd = 0xFFFFFFFFu;
    for (uint32_t k = grp[g].first; k < grp[g].first + grp[g].count; ++k)
      if (ccost[k] < bc || (ccost[k] == bc && cdiv[k] < bd)) {
        bc = ccost[k];
        bd = cdiv[k];
      }
    cost[g] = bc;  // indexed [3 * task + axis]
    dvd[g] = bd;
  }
}

bool Stage::fifo(std::string &err) {
  const size_t no = n_open;
  kind_.resize(no + 1);
  a_.resize(no + 1);  // next-list entries per open node
  b_.resize(no + 1);  // new nodes (= child ranges) per open node
  // pass 1: the FIFO of each node, candidate by candidate (:162-173)
  int overflow = 0;  // a queue past 8 candidates (cannot happen: see OpenState)
#pragma omp parallel for schedule(static) if (no >= kParMin) reduction(| : overflow)
  for (size_t o = 0; o < no; ++o) {
    OpenState &N = OS[open[o]];
    Cand q2[8];
    uint32_t qn2 = 0;
    bool capped = false;
    for (uint32_t c = 0; c < N.qn; ++c) {
      const Cand cand = N.q[c];
      const int ti = task_of[task_off[o] + c];
      if (N.nd == 7) {  // the reference stops here: this candidate is never tried
        capped = true;
        if (ti >= 0) action[ti] = 3;
        continue;
      }
      if (ti < 0) continue;  // <= 8 triangles: tryDivide returns at once
      // tryDivide(start, end) (:119-153) from the three tryDivide(indices, start, end, axis)
      const uint32_t start = cand.lo, end = cand.hi;
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
        if (qn2 + 2 <= 8) {
          q2[qn2++] = Cand{start, dv3[win]};
          q2[qn2++] = Cand{dv3[win], end};
        } else {
          overflow = 1;
        }
      }
    }
    if (capped || N.nd == 7) qn2 = 0;
    for (uint32_t c = 0; c < qn2; ++c) N.q[c] = q2[c];
    N.qn = qn2;
    if (qn2) {  // stays open
      kind_[o] = 0;
      a_[o] = 1;
      b_[o] = 0;
      continue;
    }
    // node complete (:175-224)
    if (N.nd == 0) {
      if (N.end - N.start > 24) {
        N.div[N.nd++] = ((N.start / 3 + N.end / 3) / 2) * 3;
      } else {
        kind_[o] = 1;  // leaf
        a_[o] = b_[o] = 0;
        continue;
      }
    }
    std::sort(N.div, N.div + N.nd);
    kind_[o] = 2;
    a_[o] = b_[o] = (uint32_t)N.nd + 1;
  }
  if (overflow) {
    err = "candidate queue bound";
    return false;
  }
  const size_t nn = excl_scan(a_, no), nc = excl_scan(b_, no);
  if (n_nodes + nc > H.cap || n_ranges + nc > ranges.cap || nn > next.cap) {
    err = "node bound";
    return false;
  }
  const size_t h0 = n_nodes, r0 = n_ranges;
  // pass 2: outputs at their serial positions
#pragma omp parallel for schedule(static) if (no >= kParMin)
  for (size_t o = 0; o < no; ++o) {
    const int32_t id = open[o];
    const OpenState &N = OS[id];
    if (kind_[o] == 0) {
      next[a_[o]] = id;
      continue;
    }
    BvhHostNode node;
    if (kind_[o] == 1) {
      node.leaf = true;
      node.start = N.start;
      node.count = N.end - N.start;
    } else {
      node.nchild = (uint32_t)(N.nd + 1);
      for (int c = 0; c <= N.nd; ++c) {
        const uint32_t lo = c == 0 ? N.start : N.div[c - 1], hi = c == N.nd ? N.end : N.div[c];
        const size_t k = b_[o] + (size_t)c;
        const int32_t cid = (int32_t)(h0 + k);
        node.child[c] = cid;
        ranges[r0 + k] = Task{lo / 3, hi / 3};
        range_of[r0 + k] = {id, c};
        next[a_[o] + (size_t)c] = cid;
        OpenState &C = OS[cid];
        C.start = lo;
        C.end = hi;
        C.qn = 1;
        C.nd = 0;
        C.q[0] = Cand{lo, hi};
      }
    }
    new (&H[id]) BvhHostNode(node);
  }
  n_nodes = h0 + nc;
  n_ranges = r0 + nc;
  n_next = nn;
  return true;
}


// ---- the whole stage loop with the device steps emulated on the host --------
namespace {

struct EBox {
  float mn[3], mx[3];
};
inline EBox e_empty() {
  const float inf = __builtin_huge_valf();
  return EBox{{inf, inf, inf}, {-inf, -inf, -inf}};
}
// tb_union of rt_bvhgpu.hip: the earlier operand is kept among equal bounds
inline EBox e_union(const EBox &a, const EBox &b) {
  EBox r;
  for (int k = 0; k < 3; ++k) {
    r.mn[k] = (b.mn[k] < a.mn[k]) ? b.mn[k] : a.mn[k];
    r.mx[k] = (a.mx[k] < b.mx[k]) ? b.mx[k] : a.mx[k];
  }
  return r;
}
inline float e_area(const EBox &b) {
  const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
  return 2 * (dx * dy + dx * dz + dy * dz);
}

}  // namespace

bool emulate_device_build(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                          std::string &err, unsigned want) {
  if (nidx < 0 || nidx % 3 != 0) { err = "index count must be a multiple of 3"; return false; }
  for (int64_t i = 0; i < nidx; ++i)
    if ((int64_t)idx[i] >= nverts) { err = "vertex index out of range"; return false; }
  const uint32_t n = (uint32_t)(nidx / 3);
  out = BVHGpu();
  if (n == 0) { out.root_word = rtl::kInvalidChild; return true; }
  constexpr uint32_t kChunk = 2048;  // kSahChunk
  // k_tribox
  std::vector<EBox> tb(n);
  std::vector<float> K(3 * (size_t)n);
  for (uint32_t t = 0; t < n; ++t) {
    EBox b = e_empty();
    for (int k = 0; k < 3; ++k) {
      const float *v = vpos4 + 4 * (size_t)idx[3 * (size_t)t + k];
      const float x = v[0] / v[3], y = v[1] / v[3], z = v[2] / v[3];
      b = e_union(b, EBox{{x, y, z}, {x, y, z}});
    }
    tb[t] = b;
    for (int a = 0; a < 3; ++a) K[(size_t)a * n + t] = b.mx[a];
  }
  std::vector<uint32_t> ids3(3 * (size_t)n), backup(n);
  for (uint32_t t = 0; t < n; ++t) ids3[t] = t;
  Stage SG;
  if (!SG.init(n, kChunk)) { err = "host arrays"; return false; }
  std::vector<float> hcc;
  std::vector<uint32_t> hcd;
  std::vector<EBox> right;
  while (SG.n_open) {
    const size_t r0 = SG.n_ranges;
    SG.prologue();
    const size_t T = SG.tasks.size();
    if (T) {
      for (const Task &tk : SG.tasks)  // k_stage_copy
        for (uint32_t t = tk.s; t < tk.e; ++t) {
          backup[t] = ids3[t];
          ids3[n + t] = ids3[2 * (size_t)n + t] = ids3[t];
        }
      for (const Seg &sg : SG.segs)  // Sorter::sort: std::sort of each segment
        host_introsort(ids3.data() + sg.first, sg.last - sg.first, K.data() + (size_t)(sg.first / n) * n, sg.depth);
      // the chunked SAH sweeps: each chunk's first minimum over its dividers
      hcc.assign(SG.ch.size(), __builtin_huge_valf());
      hcd.assign(SG.ch.size(), 0xFFFFFFFFu);
      for (size_t g = 0; g < SG.grp.size(); ++g) {
        const Task tk = SG.tasks[g / 3];
        const uint32_t *ids = ids3.data() + (g % 3) * (size_t)n;
        right.assign((size_t)(tk.e - tk.s) + 1, e_empty());
        for (uint32_t t = tk.e; t-- > tk.s;) right[t - tk.s] = e_union(tb[ids[t]], right[t - tk.s + 1]);
        const float psa = e_area(right[0]);
        EBox left = e_empty();
        const SahGroup G = SG.grp[g];
        for (uint32_t k = G.first; k < G.first + G.count; ++k) {
          const SahChunk c = SG.ch[k];
          float best = __builtin_huge_valf();
          uint32_t bdiv = 0xFFFFFFFFu;
          for (uint32_t t = c.lo; t < c.hi; ++t) {
            const uint32_t d = t + 1;
            left = e_union(left, tb[ids[t]]);
            if (d >= tk.e) continue;
            const float lc = static_cast<float>(3u * (d - tk.s)) / 3.0f;
            const float rc = static_cast<float>(3u * (tk.e - tk.s)) / 3.0f - lc;
            const float cost = 0.2f + e_area(left) / psa * lc + e_area(right[d - tk.s]) / psa * rc;
            if (cost < best) {
              best = cost;
              bdiv = d;
            }
          }
          hcc[k] = best;
          hcd[k] = bdiv;
        }
      }
      SG.reduce_sah(hcc.data(), hcd.data());
    }
    if (!SG.fifo(err)) return false;
    for (size_t ti = 0; ti < T; ++ti) {  // k_stage_apply
      const uint32_t a = SG.action[ti];
      if (a == 0) continue;
      const Task tk = SG.tasks[ti];
      for (uint32_t t = tk.s; t < tk.e; ++t)
        ids3[t] = a == 1 ? ids3[n + t] : a == 2 ? ids3[2 * (size_t)n + t] : backup[t];
    }
    for (size_t r = r0; r < SG.n_ranges; ++r) {  // child boxes over the order after the apply
      const Task R = SG.ranges[r];
      EBox b = e_empty();
      for (uint32_t t = R.s; t < R.e; ++t) b = e_union(b, tb[ids3[t]]);
      BvhBox &dst = SG.H[SG.range_of[r].first].box[SG.range_of[r].second];
      for (int k = 0; k < 3; ++k) {
        dst.mn[k] = b.mn[k];
        dst.mx[k] = b.mx[k];
      }
    }
    SG.advance();
  }
  const std::vector<uint32_t> cur(ids3.begin(), ids3.begin() + n);
  bvh_layout(vpos4, idx, nidx, HostNodes(SG.H.p, SG.n_nodes), cur, out, want, true);
  return true;
}

}  // namespace bvhs
}  // namespace rth
