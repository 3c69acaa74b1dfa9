// rt_host.cpp -- host-side scene preparation (not on the per-frame path).
// Build with -ffp-contract=off: the SAH costs and the per-triangle values that
// are handed to the GPU must round exactly as the reference's.
#include "rt_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <unordered_map>
#include <utility>
#include <vector>
#ifdef _OPENMP
#include <immintrin.h>
#include <omp.h>
#endif

namespace rth {

static const float kInf = std::numeric_limits<float>::infinity();

// ------------------------------------------------------------- loaders ---
static bool read_file(const char *path, std::vector<char> &buf, std::string &err) {
  FILE *f = std::fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return false; }
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n < 0) { std::fclose(f); err = "cannot size file"; return false; }
  buf.resize((size_t)n + 1);
  size_t got = n ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if (got != (size_t)n) { err = "short read"; return false; }
  buf[(size_t)n] = '\0';
  return true;
}

// OBJ -> SimpleMesh with the semantics of cmesh4::LoadMeshFromObj
// (core/mesh.cpp:178-287 over tinyobjloader v2): 'v x y z' parsed as
// (float)strtod, face corners 'v', 'v/t', 'v//n', 'v/t/n' with 1-based or
// negative indices, polygons fanned, vertices de-duplicated on the (v, vn, vt)
// index tuple in first-use order, w = 1. Optional loadAndScale
// (main.cpp:326-343): centre the bbox at 0 and divide by |boxMax - center|.
bool load_obj(const char *path, bool scale, Mesh &out, std::string &err) {
  std::vector<char> buf;
  if (!read_file(path, buf, err)) return false;
  std::vector<float> pos;
  int64_t n_vn = 0, n_vt = 0;
  struct Corner { int32_t v, t, n; };
  std::vector<Corner> corners;
  std::vector<Corner> poly;
  auto fix = [](long i, int64_t n) -> int32_t {
    if (i > 0) return (int32_t)(i - 1);
    if (i < 0) return (int32_t)(n + i);
    return -1;
  };
  char *p = buf.data();
  char *end = p + buf.size() - 1;
  while (p < end) {
    char *line = p;
    while (p < end && *p != '\n') ++p;
    char *eol = p;
    if (p < end) ++p;
    *eol = '\0';
    char *q = line;
    while (*q == ' ' || *q == '\t') ++q;
    if (q[0] == 'v' && (q[1] == ' ' || q[1] == '\t')) {
      char *e = q + 2;
      for (int k = 0; k < 3; ++k) { char *s = e; pos.push_back((float)std::strtod(s, &e)); }
    } else if (q[0] == 'v' && q[1] == 'n' && (q[2] == ' ' || q[2] == '\t')) {
      ++n_vn;
    } else if (q[0] == 'v' && q[1] == 't' && (q[2] == ' ' || q[2] == '\t')) {
      ++n_vt;
    } else if (q[0] == 'f' && (q[1] == ' ' || q[1] == '\t')) {
      q += 2;
      poly.clear();
      for (;;) {
        while (*q == ' ' || *q == '\t' || *q == '\r') ++q;
        if (!*q) break;
        Corner c{-1, -1, -1};
        char *e;
        c.v = fix(std::strtol(q, &e, 10), (int64_t)pos.size() / 3);
        q = e;
        if (*q == '/') {
          ++q;
          if (*q != '/') { c.t = fix(std::strtol(q, &e, 10), n_vt); q = e; }
          if (*q == '/') { ++q; c.n = fix(std::strtol(q, &e, 10), n_vn); q = e; }
        }
        while (*q && *q != ' ' && *q != '\t' && *q != '\r') ++q;
        if (c.v < 0 || (int64_t)c.v >= (int64_t)pos.size() / 3) { err = "face index out of range"; return false; }
        poly.push_back(c);
      }
      for (size_t i = 2; i < poly.size(); ++i) {
        corners.push_back(poly[0]);
        corners.push_back(poly[i - 1]);
        corners.push_back(poly[i]);
      }
    }
  }
  struct KH {
    size_t operator()(uint64_t k) const { return (size_t)(k * 0x9E3779B97F4A7C15ull); }
  };
  // key = (v, t, n) packed; indices are < 2^21 for any mesh this loader accepts
  std::unordered_map<uint64_t, uint32_t, KH> uniq;
  uniq.reserve(corners.size());
  out.vpos4.clear();
  out.idx.clear();
  out.idx.reserve(corners.size());
  for (const Corner &c : corners) {
    uint64_t key = ((uint64_t)(uint32_t)(c.v + 1)) | ((uint64_t)(uint32_t)(c.t + 1) << 21) |
                   ((uint64_t)(uint32_t)(c.n + 1) << 42);
    if (c.v + 1 >= (1 << 21) || c.t + 1 >= (1 << 21) || c.n + 1 >= (1 << 21)) {
      err = "OBJ too large for this loader";
      return false;
    }
    auto it = uniq.find(key);
    uint32_t id;
    if (it != uniq.end()) {
      id = it->second;
    } else {
      id = (uint32_t)(out.vpos4.size() / 4);
      uniq.emplace(key, id);
      out.vpos4.push_back(pos[3 * (size_t)c.v]);
      out.vpos4.push_back(pos[3 * (size_t)c.v + 1]);
      out.vpos4.push_back(pos[3 * (size_t)c.v + 2]);
      out.vpos4.push_back(1.0f);
    }
    out.idx.push_back(id);
  }
  if (out.idx.empty()) { err = "OBJ has no faces"; return false; }
  if (scale) {
    // calc_bbox (raytracing.hpp:29-37) then loadAndScale (main.cpp:326-343)
    float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
    size_t nv = out.vpos4.size() / 4;
    for (size_t i = 0; i < nv; ++i) {
      float w = out.vpos4[4 * i + 3];
      for (int k = 0; k < 3; ++k) {
        float c = out.vpos4[4 * i + k] / w;
        mn[k] = std::min(mn[k], c);
        mx[k] = std::max(mx[k], c);
      }
    }
    float center[3], d[3];
    for (int k = 0; k < 3; ++k) center[k] = (mn[k] + mx[k]) / 2.0f;
    for (int k = 0; k < 3; ++k) d[k] = mx[k] - center[k];
    float s = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    for (size_t i = 0; i < nv; ++i) {
      float *v = &out.vpos4[4 * i];
      float w = v[3];
      float x = v[0] / w, y = v[1] / w, z = v[2] / w;  // v /= w (w/w == 1 exactly)
      x = (x - center[0]) / s;
      y = (y - center[1]) / s;
      z = (z - center[2]) / s;
      v[0] = x * w; v[1] = y * w; v[2] = z * w; v[3] = 1.0f * w;
    }
  }
  return true;
}

// loadSDFGrid (grid_raytracing.cpp:127-134), with the size check the
// reference omits (12 + 4*sx*sy*sz bytes).
bool load_grid(const char *path, uint32_t size[3], std::vector<float> &values, std::string &err) {
  FILE *f = std::fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return false; }
  if (std::fread(size, 4, 3, f) != 3) { std::fclose(f); err = "truncated grid header"; return false; }
  uint64_t n = (uint64_t)size[0] * size[1] * size[2];
  if (n == 0 || n > (1ull << 32)) { std::fclose(f); err = "bad grid size"; return false; }
  values.resize(n);
  size_t got = std::fread(values.data(), 4, n, f);
  std::fclose(f);
  if (got != n) { err = "truncated grid values"; return false; }
  return true;
}

// loadSDFOctree (octree_raytracing.cpp:8-16): u32 count + count x 36 B.
bool load_octree(const char *path, std::vector<uint8_t> &nodes36, std::string &err) {
  FILE *f = std::fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return false; }
  uint32_t n = 0;
  if (std::fread(&n, 4, 1, f) != 1) { std::fclose(f); err = "truncated octree header"; return false; }
  nodes36.resize((size_t)n * 36);
  size_t got = n ? std::fread(nodes36.data(), 36, n, f) : 0;
  std::fclose(f);
  if (got != n) { err = "truncated octree nodes"; return false; }
  return true;
}

// ---------------------------------------------------------- BVH8 build ---
// Same tree as BVHBuilder::perform (triangles_raytracing.cpp:12-258):
// full-sweep binary SAH on x, y, z (triangles ordered by their bbox max along
// the axis with std::sort, the reference's par_unseq sort without TBB),
// EMPTY_NODE_TRAVERSE_COST = 0.2, dividers aligned to 8-triangle multiples,
// up to 7 binary splits per node taken breadth-first, median fallback.
// Differences in form only: triangles are sorted as 32-bit ids with
// precomputed keys (the comparator sees the same values, so std::sort makes
// the same comparisons and the same permutation), bbox prefix/suffix unions
// use precomputed per-triangle boxes (min/max are exact), and node storage is
// renumbered afterwards (the reference's OpenMP task order only moves offsets).
namespace {

using Box = BvhBox;
static inline Box empty_box() { return {{kInf, kInf, kInf}, {-kInf, -kInf, -kInf}}; }
static inline void grow(Box &b, const Box &t) {
  for (int k = 0; k < 3; ++k) {
    b.mn[k] = std::min(b.mn[k], t.mn[k]);
    b.mx[k] = std::max(b.mx[k], t.mx[k]);
  }
}
static inline float surface_area(const Box &b) {  // raytracing.hpp:62-65
  float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
  return 2 * (dx * dy + dx * dz + dy * dz);
}

using HNode = BvhHostNode;

// std::sort, in parallel, with the exact permutation libstdc++'s serial
// std::sort produces (introsort: median-of-three pivot moved to the front,
// unguarded Hoare partition, recursion on the right part and a loop on the
// left, heapsort below depth 2*lg(n), ranges of <= 16 left for a final
// insertion sort). The two parts of a partition are independent, so the right
// part becomes an OpenMP task. The final insertion sort is stable and never
// moves an element across a partition boundary (left part <= pivot <= right
// part), so insertion-sorting each <= 16 leaf range where the loop leaves it
// gives the same sequence as the one final pass over the whole range.
// Equal keys therefore end in the same order as the serial sort, which the
// SAH sweeps (and so the tree) depend on. Keys: K[id], compared with <.
namespace psort {
constexpr ptrdiff_t kThreshold = 16;    // libstdc++ _S_threshold
constexpr ptrdiff_t kTaskMin = 4096;    // right parts at least this long become tasks

struct Less {
  const float *K;
  bool operator()(uint32_t a, uint32_t b) const { return K[a] < K[b]; }
};

inline void insertion(uint32_t *first, uint32_t *last, Less c) {  // std::__insertion_sort
  if (first == last) return;
  for (uint32_t *i = first + 1; i != last; ++i) {
    const uint32_t v = *i;
    if (c(v, *first)) {
      std::move_backward(first, i, i + 1);
      *first = v;
    } else {  // std::__unguarded_linear_insert
      uint32_t *l = i, *n = i - 1;
      while (c(v, *n)) { *l = *n; l = n; --n; }
      *l = v;
    }
  }
}

inline void median_to_first(uint32_t *r, uint32_t *a, uint32_t *b, uint32_t *cc, Less c) {
  if (c(*a, *b)) {
    if (c(*b, *cc)) std::iter_swap(r, b);
    else if (c(*a, *cc)) std::iter_swap(r, cc);
    else std::iter_swap(r, a);
  } else if (c(*a, *cc)) std::iter_swap(r, a);
  else if (c(*b, *cc)) std::iter_swap(r, cc);
  else std::iter_swap(r, b);
}

inline uint32_t *partition(uint32_t *first, uint32_t *last, uint32_t *pivot, Less c) {
  for (;;) {
    while (c(*first, *pivot)) ++first;
    --last;
    while (c(*pivot, *last)) --last;
    if (!(first < last)) return first;
    std::iter_swap(first, last);
    ++first;
  }
}

void loop(uint32_t *first, uint32_t *last, ptrdiff_t depth, Less c) {  // std::__introsort_loop
  while (last - first > kThreshold) {
    if (depth == 0) {  // std::__partial_sort(first, last, last): heapsort, output sorted
      std::make_heap(first, last, c);
      std::sort_heap(first, last, c);
      return;
    }
    --depth;
    uint32_t *mid = first + (last - first) / 2;
    median_to_first(first, first + 1, mid, last - 1, c);
    uint32_t *cut = partition(first + 1, last, first, c);
    if (last - cut >= kTaskMin) {
#pragma omp task firstprivate(cut, last, depth, c)
      loop(cut, last, depth, c);
    } else {
      loop(cut, last, depth, c);
    }
    last = cut;
  }
  insertion(first, last, c);
}

inline ptrdiff_t lg(ptrdiff_t n) { return (ptrdiff_t)(sizeof(long long) * 8 - 1 - __builtin_clzll((unsigned long long)n)); }

void sort(uint32_t *first, uint32_t *last, const float *K) {
  if (last - first < 2) return;
  Less c{K};
  if (last - first < kTaskMin) {
    std::sort(first, last, c);
    return;
  }
#pragma omp taskgroup
  loop(first, last, 2 * lg(last - first), c);
}
}  // namespace psort

}  // namespace

// libstdc++'s std::sort on ids by keys K (the permutation the build depends
// on), with an explicit depth limit (< 0: std::sort's own 2 * lg(n)); the host
// reference of the device sort (tests via rtx_sort_check).
void host_introsort(uint32_t *ids, size_t n, const float *K, int64_t depth_limit) {
  if (n < 2) return;
  psort::Less c{K};
  psort::loop(ids, ids + n, depth_limit < 0 ? 2 * psort::lg((ptrdiff_t)n) : (ptrdiff_t)depth_limit, c);
  psort::insertion(ids, ids + n, c);
}

namespace {

struct Builder {
  std::vector<uint32_t> cur, scrY, scrZ;  // triangle ids, 'cur' = mesh.indices order
  std::vector<Box> triBox, rightB[3];
  std::vector<float> key[3];
  std::vector<HNode> nodes;

  struct Div { bool divided = false; size_t divider = (size_t)-1; float sah = kInf; };

  // triangles_raytracing.cpp:30-117 in index units [start, end). The suffix
  // boxes are kept per axis (the three axes may run concurrently); the prefix
  // box is accumulated in the SAH sweep itself. Box unions are min/max, exact
  // in any order, so every box equals the reference's m_leftBoxes /
  // m_rightBoxes entry, and the parent box is the full suffix box.
  Div try_axis(std::vector<uint32_t> &ids, size_t start, size_t end, int axis) {
    psort::sort(ids.data() + start / 3, ids.data() + end / 3, key[axis].data());
    std::vector<Box> &rightB = rightB_for(axis);
    for (size_t r = start / 3; r != end / 3; ++r) {
      size_t b = end / 3 - r + start / 3 - 1;
      Box &box = rightB[b];
      box = (r == start / 3) ? empty_box() : rightB[b + 1];
      grow(box, triBox[ids[b]]);
    }
    Div res;
    res.sah = static_cast<float>(end - start) / 3.0f;
    const float parentSA = surface_area(rightB[start / 3]);
    Box left = empty_box();
    for (size_t d = start + 3; d < end; d += 3) {
      grow(left, triBox[ids[d / 3 - 1]]);
      const float lc = static_cast<float>(d - start) / 3.0f;
      const float rc = static_cast<float>(end - start) / 3.0f - lc;
      const float c = 0.2f + surface_area(left) / parentSA * lc +
                      surface_area(rightB[d / 3]) / parentSA * rc;
      if (c < res.sah) { res.sah = c; res.divider = d; res.divided = true; }
    }
    if (res.divided && (res.divider - start) % 24 != 0) {
      size_t d1 = (res.divider - 1) / 24 * 24, d2 = ((res.divider - 1) / 24 + 1) * 24;
      size_t nearest = (res.divider - d1 <= d2 - res.divider) ? d1 : d2;
      size_t other = d1 + d2 - nearest;
      if (start < nearest && nearest < end) res.divider = nearest;
      else if (start < other && other < end) res.divider = other;
    }
    return res;
  }
  std::vector<Box> &rightB_for(int axis) { return rightB[axis]; }

  static constexpr size_t kAxesTaskMin = 1024;  // triangles

  // triangles_raytracing.cpp:119-153
  Div try_divide(size_t start, size_t end) {
    if (end - start <= 8 * 3) return Div{};
    std::copy(cur.begin() + start / 3, cur.begin() + end / 3, scrY.begin() + start / 3);
    std::copy(cur.begin() + start / 3, cur.begin() + end / 3, scrZ.begin() + start / 3);
    const float curSAH = static_cast<float>(end - start) / 3.0f;
    Div dx, dy, dz;
    if (end - start >= 3 * kAxesTaskMin) {  // the three axes concurrently (disjoint scratch)
#pragma omp task shared(dy)
      dy = try_axis(scrY, start, end, 1);
#pragma omp task shared(dz)
      dz = try_axis(scrZ, start, end, 2);
      dx = try_axis(cur, start, end, 0);
#pragma omp taskwait
    } else {
      dx = try_axis(cur, start, end, 0);
      dy = try_axis(scrY, start, end, 1);
      dz = try_axis(scrZ, start, end, 2);
    }
    const float m = std::min({curSAH, dx.sah, dy.sah, dz.sah});
    if (dx.sah == m) return dx;
    if (dy.sah == m) {
      std::copy(scrY.begin() + start / 3, scrY.begin() + end / 3, cur.begin() + start / 3);
      return dy;
    }
    if (dz.sah == m) {
      std::copy(scrZ.begin() + start / 3, scrZ.begin() + end / 3, cur.begin() + start / 3);
      return dz;
    }
    return Div{};
  }

  int32_t alloc_node() {
    int32_t id;
#pragma omp critical(rt_bvh_nodes)
    {
      id = (int32_t)nodes.size();
      nodes.emplace_back();
    }
    return id;
  }

  // triangles_raytracing.cpp:155-225
  void create(int32_t self, size_t start, size_t end) {
    size_t dividers[20] = {};
    size_t nd = 0;
    std::pair<size_t, size_t> q[40];  // ChipQueue<., 40> (triangles_raytracing.hpp:69-97)
    int qf = 0, qr = -1, qc = 0;
    auto enq = [&](size_t a, size_t b) {
      if (qc == 40) return;
      qr = (qr + 1) % 40;
      q[qr] = {a, b};
      ++qc;
    };
    enq(start, end);
    while (qc) {
      auto c = q[qf];
      qf = (qf + 1) % 40;
      --qc;
      if (nd == 7) break;
      Div r = try_divide(c.first, c.second);
      if (r.divided) {
        dividers[nd++] = r.divider;
        enq(c.first, r.divider);
        enq(r.divider, c.second);
      }
    }
    HNode node;
    if (nd == 0) {
      if (end - start > 24) {
        dividers[nd++] = ((start / 3 + end / 3) / 2) * 3;
      } else {
        node.leaf = true;
        node.start = (uint32_t)start;
        node.count = (uint32_t)(end - start);
#pragma omp critical(rt_bvh_nodes)
        nodes[self] = node;
        return;
      }
    }
    std::sort(dividers, dividers + nd);
    node.nchild = (uint32_t)(nd + 1);
    size_t lo[8], hi[8];
    for (size_t c = 0; c <= nd; ++c) {
      lo[c] = (c == 0) ? start : dividers[c - 1];
      hi[c] = (c == nd) ? end : dividers[c];
      Box b = empty_box();
      for (size_t t = lo[c] / 3; t < hi[c] / 3; ++t) grow(b, triBox[cur[t]]);
      node.box[c] = b;
      node.child[c] = alloc_node();
    }
#pragma omp critical(rt_bvh_nodes)
    nodes[self] = node;
    for (size_t c = 0; c <= nd; ++c) {
      const int32_t ch = node.child[c];
      const size_t a = lo[c], b = hi[c];
      if (b - a > 3 * 2048) {
#pragma omp task firstprivate(ch, a, b)
        create(ch, a, b);
      } else {
        create(ch, a, b);
      }
    }
#pragma omp taskwait
  }
};

}  // namespace

bool build_bvh8(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                std::string &err, unsigned want) {
  if (nidx < 0 || nidx % 3 != 0) { err = "index count must be a multiple of 3"; return false; }
  const size_t ntri = (size_t)nidx / 3;
  for (int64_t i = 0; i < nidx; ++i)
    if ((int64_t)idx[i] >= nverts) { err = "vertex index out of range"; return false; }
  if (ntri > rtl::kMaxLeafFirstTri) { err = "too many triangles"; return false; }
  out = BVHGpu();
  if (ntri == 0) { out.root_word = rtl::kInvalidChild; return true; }

  Builder B;
  B.triBox.resize(ntri);
  for (int a = 0; a < 3; ++a) B.key[a].resize(ntri);
  // per-triangle box of the /w-divided vertices (calc_bbox, raytracing.hpp:51-60)
  for (size_t t = 0; t < ntri; ++t) {
    Box b = empty_box();
    for (int k = 0; k < 3; ++k) {
      const float *v = vpos4 + 4 * (size_t)idx[3 * t + k];
      const float w = v[3];
      Box p{{v[0] / w, v[1] / w, v[2] / w}, {v[0] / w, v[1] / w, v[2] / w}};
      grow(b, p);
    }
    B.triBox[t] = b;
    for (int a = 0; a < 3; ++a) B.key[a][t] = b.mx[a];
  }
  B.cur.resize(ntri);
  for (size_t t = 0; t < ntri; ++t) B.cur[t] = (uint32_t)t;
  B.scrY.resize(ntri);
  B.scrZ.resize(ntri);
  for (int a = 0; a < 3; ++a) B.rightB[a].resize(ntri);
  B.nodes.reserve(ntri + 16);
  B.nodes.emplace_back();
#pragma omp parallel
  {
#pragma omp single
    B.create(0, 0, (size_t)nidx);
  }

  bvh_layout(vpos4, idx, nidx, B.nodes, B.cur, out, want, true);
  return true;
}

void bvh_layout(const float *vpos4, const uint32_t *idx, int64_t nidx, HostNodes H,
                const std::vector<uint32_t> &cur, BVHGpu &out, unsigned want, bool host_tris) {
  (void)nidx;
  out.host_nodes = (int64_t)H.size();
  if (want & kBvhPerm) out.perm_tri = cur;
  if (want & kBvhCanon) {  // canonical pre-order (52 u32 per node), same as the oracle's export
    out.canon.reserve(H.size() * 52);
    std::vector<int32_t> st{0};
    while (!st.empty()) {
      int32_t id = st.back();
      st.pop_back();
      const HNode &n = H[id];
      uint32_t rec[52] = {};
      rec[0] = n.leaf;
      rec[1] = n.leaf ? n.count : n.nchild;
      rec[2] = n.leaf ? n.start : 0;
      if (!n.leaf) {
        float bx[48];
        for (int c = 0; c < 8; ++c) {
          const bool v = (uint32_t)c < n.nchild;
          bx[0 * 8 + c] = v ? n.box[c].mn[0] : kInf;
          bx[1 * 8 + c] = v ? n.box[c].mn[1] : kInf;
          bx[2 * 8 + c] = v ? n.box[c].mn[2] : kInf;
          bx[3 * 8 + c] = v ? n.box[c].mx[0] : kInf;
          bx[4 * 8 + c] = v ? n.box[c].mx[1] : kInf;
          bx[5 * 8 + c] = v ? n.box[c].mx[2] : kInf;
        }
        std::memcpy(rec + 4, bx, 192);
        for (int c = (int)n.nchild - 1; c >= 0; --c) st.push_back(n.child[c]);
      }
      out.canon.insert(out.canon.end(), rec, rec + 52);
    }
  }

  // leaves take consecutive triangle slots in the order they are met; the
  // slots are filled afterwards, in parallel
  std::vector<std::pair<uint32_t, uint32_t>> leaf_fill;  // (first slot, leaf's first triangle position)
  std::vector<uint32_t> leaf_cnt;
  uint32_t next_slot = 0;
  auto leaf_word = [&](const HNode &n) -> uint32_t {
    const uint32_t first = next_slot, nt = n.count / 3;
    if (nt == 0) return rtl::kInvalidChild;
    next_slot += nt;
    leaf_fill.push_back({first, n.start / 3});
    leaf_cnt.push_back(nt);
    return rtl::kLeafBit | (first << 3) | (nt - 1);
  };
  auto fill_tris = [&]() {
    out.n_tris = next_slot;
    if (!(want & kBvhTris)) return;
    if (!host_tris) {  // the caller fills them (the device builder)
      out.leaf_tab.resize(3 * leaf_fill.size());
      for (size_t l = 0; l < leaf_fill.size(); ++l) {
        out.leaf_tab[3 * l] = leaf_fill[l].first;
        out.leaf_tab[3 * l + 1] = leaf_fill[l].second;
        out.leaf_tab[3 * l + 2] = leaf_cnt[l];
      }
      return;
    }
    out.tris.resize(next_slot);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t l = 0; l < (int64_t)leaf_fill.size(); ++l) {
      for (uint32_t k = 0; k < leaf_cnt[l]; ++k) {
        const uint32_t slot = leaf_fill[l].second + k;
        const uint32_t *tv = idx + 3 * (size_t)cur[slot];
        float v[3][3];
        for (int j = 0; j < 3; ++j) {
          const float *p = vpos4 + 4 * (size_t)tv[j];
          const float w = p[3];
          v[j][0] = p[0] / w; v[j][1] = p[1] / w; v[j][2] = p[2] / w;  // v /= v.w (:307-309)
        }
        rtl::GTri &g = out.tris[leaf_fill[l].first + k];
        g.v0x = v[0][0]; g.v0y = v[0][1]; g.v0z = v[0][2];
        g.orig_id = cur[slot];
        g.e1x = v[1][0] - v[0][0]; g.e1y = v[1][1] - v[0][1]; g.e1z = v[1][2] - v[0][2];
        g.e2x = v[2][0] - v[0][0]; g.e2y = v[2][1] - v[0][1]; g.e2z = v[2][2] - v[0][2];
        g.pad1 = g.pad2 = 0.0f;
      }
    }
  };

  if (H[0].leaf) {
    out.root_word = leaf_word(H[0]);
    fill_tris();
    out.max_depth = 0;
    out.host_inner = 0;
    return;
  }
  // BFS over inner nodes; depth = number of inner ancestors incl. itself
  std::vector<int32_t> order{0};
  std::vector<int32_t> depth_of{1};
  std::vector<int32_t> gpu_id(H.size(), -1);
  gpu_id[0] = 0;
  for (size_t i = 0; i < order.size(); ++i) {
    const HNode &n = H[order[i]];
    for (uint32_t c = 0; c < n.nchild; ++c) {
      const int32_t ch = n.child[c];
      if (!H[ch].leaf) {
        gpu_id[ch] = (int32_t)order.size();
        order.push_back(ch);
        depth_of.push_back(depth_of[i] + 1);
      }
    }
  }
  out.host_inner = (int64_t)order.size();
  out.nodes.resize(order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    const HNode &n = H[order[i]];
    rtl::GNode &g = out.nodes[i];
    out.max_depth = std::max(out.max_depth, depth_of[i]);
    for (int c = 0; c < 8; ++c) {
      if ((uint32_t)c < n.nchild) {
        for (int k = 0; k < 3; ++k) { g.box[c][2 * k] = n.box[c].mn[k]; g.box[c][2 * k + 1] = n.box[c].mx[k]; }
        const HNode &ch = H[n.child[c]];
        g.child[c] = ch.leaf ? leaf_word(ch) : (uint32_t)gpu_id[n.child[c]];
      } else {
        for (int k = 0; k < 6; ++k) g.box[c][k] = kInf;
        g.child[c] = rtl::kInvalidChild;
      }
    }
  }
  out.root_word = 0;
  {
    const HNode &r = H[0];
    Box u = empty_box();
    for (uint32_t c = 0; c < r.nchild; ++c) grow(u, r.box[c]);
    for (int k = 0; k < 3; ++k) { out.root_box[k] = u.mn[k]; out.root_box[3 + k] = u.mx[k]; }
  }
  fill_tris();
}

// --------------------------------------------------------------- octree ---
bool flatten_octree(const uint8_t *nodes36, int64_t count, OctGpu &out, std::string &err) {
  out = OctGpu();
  if (count <= 0) { err = "empty octree"; return false; }
  out.child.resize((size_t)count);
  out.vals.resize((size_t)count);
  for (int64_t i = 0; i < count; ++i) {
    float v[8];
    uint32_t off;
    std::memcpy(v, nodes36 + 36 * i, 32);
    std::memcpy(&off, nodes36 + 36 * i + 32, 4);
    std::memcpy(out.vals[(size_t)i].v, v, 32);
    if (off == 0) {
      // octree_raytracing.hpp:12-17 isEmpty(), octree_raytracing.cpp:125-133
      bool all10 = true, all0 = true, allAbove = true;
      for (int k = 0; k < 8; ++k) {
        all10 = all10 && (v[k] > 10.0f);
        all0 = all0 && (v[k] == 0.0f);
        allAbove = allAbove && (v[k] >= 1e-4f);
      }
      out.child[(size_t)i] = rtl::OctWord{(all10 || all0 || allAbove) ? rtl::kOctNeverHits : 0u, 0u};
    } else {
      if ((int64_t)off + 7 >= count || off == rtl::kOctNeverHits) { err = "octree child offset out of range"; return false; }
      out.child[(size_t)i] = rtl::OctWord{off, 0u};
    }
  }
  // depth (levels of inner nodes on the deepest path), with a cycle guard
  std::vector<std::pair<uint32_t, int32_t>> st{{0u, 0}};
  int64_t visited = 0;
  while (!st.empty()) {
    auto [n, d] = st.back();
    st.pop_back();
    if (++visited > count || d > 24) { err = "octree is cyclic or deeper than 24 levels"; return false; }
    const uint32_t c = out.child[n].child;
    if (c != 0 && c != rtl::kOctNeverHits) {
      out.max_depth = std::max(out.max_depth, d + 1);
      for (int k = 0; k < 8; ++k) st.push_back({c + (uint32_t)k, d + 1});
    }
  }
  // child masks (rtl::OctWord), bottom-up: can_hit(node) = a leaf that can hit,
  // or an inner node with a child that can hit. Post-order over the (acyclic,
  // checked above) node graph; nodes reachable along several paths are computed once.
  std::vector<int8_t> can((size_t)count, -1);
  std::vector<std::pair<uint32_t, bool>> post{{0u, false}};
  while (!post.empty()) {
    auto [n, expanded] = post.back();
    post.pop_back();
    if (can[n] >= 0) continue;
    const uint32_t c = out.child[n].child;
    if (c == 0 || c == rtl::kOctNeverHits) {
      can[n] = c == 0 ? 1 : 0;
      continue;
    }
    if (!expanded) {
      post.push_back({n, true});
      for (int k = 0; k < 8; ++k)
        if (can[c + k] < 0) post.push_back({c + (uint32_t)k, false});
      continue;
    }
    uint32_t m = 0;
    for (int k = 0; k < 8; ++k) {
      if (can[c + k] > 0) m |= 1u << k;
      if (out.child[c + k].child == 0) m |= 1u << (8 + k);
    }
    out.child[n].masks = m;
    can[n] = (m & 0xFFu) ? 1 : 0;
  }
  return true;
}

// --------------------------------------------------------------- camera ---
// Reference camera math: Camera(pos, target, up) (camera.cpp:36-62, the
// quaternion left un-normalised, camera.cpp:61), up() (camera.hpp:29-31),
// lookAtMatrix() (camera.hpp:24-26) and the LiteMath restatement recorded in
// SURVEY.md 8(c) for lookAt / perspectiveMatrix / inverse4x4.
namespace {
struct V3 { float x, y, z; };
static inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline float dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 crs(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline V3 nrm(V3 a) { float l = std::sqrt(dot3(a, a)); return {a.x / l, a.y / l, a.z / l}; }
struct M4 { float m[4][4]; float &at(int r, int c) { return m[c][r]; } };
static M4 look_at(V3 eye, V3 center, V3 up) {
  V3 z = nrm(sub(eye, center));
  V3 x = nrm(crs(up, z));
  V3 y = nrm(crs(z, x));
  M4 M{};
  M.at(0, 0) = x.x; M.at(0, 1) = x.y; M.at(0, 2) = x.z; M.at(0, 3) = -dot3(x, eye);
  M.at(1, 0) = y.x; M.at(1, 1) = y.y; M.at(1, 2) = y.z; M.at(1, 3) = -dot3(y, eye);
  M.at(2, 0) = z.x; M.at(2, 1) = z.y; M.at(2, 2) = z.z; M.at(2, 3) = -dot3(z, eye);
  M.at(3, 3) = 1.0f;
  return M;
}
static void invert(M4 &A, float out[16]) {
  double a[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) { a[r][c] = A.at(r, c); a[r][c + 4] = (r == c) ? 1.0 : 0.0; }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r) if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
    if (p != c) for (int k = 0; k < 8; ++k) std::swap(a[p][k], a[c][k]);
    const double piv = a[c][c];
    for (int k = 0; k < 8; ++k) a[c][k] /= piv;
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
      if (f == 0.0) continue;
      for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
    }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out[c * 4 + r] = (float)a[r][c + 4];
}
struct Q { float x, y, z, w; };
static inline Q qmul(Q a, Q b) {  // quaternion.hpp:40-45
  return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
          a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
}  // namespace

namespace {
// Camera::updateOrientation (camera.cpp:36-62): the orientation quaternion of
// lookAt(pos, target, up), left un-normalised (camera.cpp:61 discards the
// normalize result).
Q orientation_of(V3 P, V3 T, V3 U) {
  M4 m = look_at(P, T, U);
  Q q;
  if (m.at(2, 2) < 0) {
    if (m.at(0, 0) > m.at(1, 1)) {
      float t = 1 + m.at(0, 0) - m.at(1, 1) - m.at(2, 2);
      q = {t, m.at(0, 1) + m.at(1, 0), m.at(2, 0) + m.at(0, 2), m.at(1, 2) - m.at(2, 1)};
    } else {
      float t = 1 - m.at(0, 0) + m.at(1, 1) - m.at(2, 2);
      q = {m.at(0, 1) + m.at(1, 0), t, m.at(1, 2) + m.at(2, 1), m.at(2, 0) - m.at(0, 2)};
    }
  } else {
    if (m.at(0, 0) < -m.at(1, 1)) {
      float t = 1 - m.at(0, 0) - m.at(1, 1) + m.at(2, 2);
      q = {m.at(2, 0) + m.at(0, 2), m.at(1, 2) + m.at(2, 1), t, m.at(0, 1) - m.at(1, 0)};
    } else {
      float t = 1 + m.at(0, 0) + m.at(1, 1) + m.at(2, 2);
      q = {m.at(1, 2) - m.at(2, 1), m.at(2, 0) - m.at(0, 2), m.at(0, 1) - m.at(1, 0), t};
    }
  }
  return q;
}
// rotateVector (quaternion.hpp:47-52): q * (v, 0) * conjugate(q)
V3 rotate_vector(V3 v, Q q) {
  const Q p{v.x, v.y, v.z, 0.0f}, c{-q.x, -q.y, -q.z, q.w};
  const Q r = qmul(qmul(q, p), c);
  return {r.x, r.y, r.z};
}
// angleAxis (quaternion.hpp:54-70)
Q angle_axis(float angle, V3 axis) {
  const V3 n = nrm(axis);
  const float half = angle * 0.5f;
  Q q;
  q.w = std::cos(half);
  q.x = n.x * std::sin(half);
  q.y = n.y * std::sin(half);
  q.z = n.z * std::sin(half);
  return q;
}
V3 v3(const float *p) { return {p[0], p[1], p[2]}; }
void put(float *o, V3 v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; }
Q q_of(const CamState &c) { return {c.q[0], c.q[1], c.q[2], c.q[3]}; }
void set_q(CamState &c, Q q) { c.q[0] = q.x; c.q[1] = q.y; c.q[2] = q.z; c.q[3] = q.w; }
V3 cam_up_v(const CamState &c) { return nrm(rotate_vector({0.0f, 1.0f, 0.0f}, q_of(c))); }     // camera.hpp:29-31
V3 cam_right_v(const CamState &c) { return nrm(rotate_vector({1.0f, 0.0f, 0.0f}, q_of(c))); }  // camera.hpp:32-34
V3 cam_forward_v(const CamState &c) { return nrm(sub(v3(c.target), v3(c.pos))); }              // camera.hpp:35-37
float len3(V3 a) { return std::sqrt(dot3(a, a)); }
}  // namespace

void cam_init(CamState &c, const float pos[3], const float target[3], const float up[3]) {
  c = CamState{};
  put(c.pos, v3(pos));
  put(c.target, v3(target));
  set_q(c, orientation_of(v3(pos), v3(target), v3(up)));
  c.sens = 0.01f;  // camera.hpp:55
}

// Camera::rotate + updateVectors (camera.cpp:5-34)
void cam_rotate(CamState &c, float dx, float dy) {
  const float pitch = dy * c.sens, yaw = dx * c.sens;
  const Q q_yaw = angle_axis(yaw, cam_up_v(c));
  const Q q_pitch = angle_axis(pitch, cam_right_v(c));
  const Q r = qmul(qmul(q_pitch, q_yaw), q_of(c));
  // Quaternion::normalized (quaternion.hpp:30-33): / length of the float4
  const float n = std::sqrt(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
  set_q(c, Q{r.x / n, r.y / n, r.z / n, r.w / n});
  // updateVectors: keep the distance to the target, move along the new forward
  const V3 f = nrm(rotate_vector({0.0f, 0.0f, -1.0f}, q_of(c)));
  const V3 T = v3(c.target);
  const float dist = len3(sub(T, v3(c.pos)));
  put(c.pos, sub(T, V3{f.x * dist, f.y * dist, f.z * dist}));
  if (c.lock) set_q(c, orientation_of(v3(c.pos), T, v3(c.locked)));
}

void cam_reset_position(CamState &c, const float pos[3]) {  // camera.cpp:64-67
  const V3 up = cam_up_v(c);
  put(c.pos, v3(pos));
  set_q(c, orientation_of(v3(c.pos), v3(c.target), up));
}

void cam_reset_target(CamState &c, const float target[3]) {  // camera.cpp:69-72
  const V3 up = cam_up_v(c);
  put(c.target, v3(target));
  set_q(c, orientation_of(v3(c.pos), v3(c.target), up));
}

void cam_set_lock_up(CamState &c, bool on) {  // camera.hpp:39-44
  if (!c.lock && on) put(c.locked, cam_up_v(c));
  c.lock = on ? 1 : 0;
}

// The viewer's mouse wheel (main.cpp:283-288): move along forward by
// wheel * distance / 25.
void cam_zoom(CamState &c, float wheel) {
  const float dist = len3(sub(v3(c.target), v3(c.pos)));
  const float r = wheel * dist / 25.0f;
  const V3 f = cam_forward_v(c);
  const V3 P = v3(c.pos);
  const float np[3] = {P.x + f.x * r, P.y + f.y * r, P.z + f.z * r};
  cam_reset_position(c, np);
}

void cam_basis(const CamState &c, float up[3], float right[3], float forward[3]) {
  if (up) put(up, cam_up_v(c));
  if (right) put(right, cam_right_v(c));
  if (forward) put(forward, cam_forward_v(c));
}

// inverse4x4(lookAtMatrix()) (camera.hpp:24-26, raytracing.cpp:74-75)
void cam_view_inverse(const CamState &c, float view_inv[16]) {
  M4 view = look_at(v3(c.pos), v3(c.target), cam_up_v(c));
  invert(view, view_inv);
}

// ------------------------------------------------------------ OBJ writer ---
// cmesh4::SaveMeshToObj (core/mesh.cpp:14-63): "v/vt/vn" records per vertex
// with std::to_string (printf "%f"), faces "f i/i/i" (1-based), in the
// reference's section order. Missing normals / texture coordinates take
// fix_missing's defaults (mesh.cpp:143-160): (0,0,1) and (0,0).
bool save_obj(const char *path, const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
              const float *vnorm4, const float *vtex2, std::string &err) {
  if (!path || (!vpos4 && nverts) || (!idx && nidx) || nidx % 3 != 0) { err = "bad arguments"; return false; }
  FILE *f = std::fopen(path, "wb");
  if (!f) { err = std::string("cannot create ") + path; return false; }
  auto num = [](float x) { return std::to_string(x); };
  std::string v, tc, n, fc;
  for (int64_t i = 0; i < nverts; ++i) {
    const float *p = vpos4 + 4 * i;
    v += "v " + num(p[0]) + " " + num(p[1]) + " " + num(p[2]) + "\n";
    const float nx = vnorm4 ? vnorm4[4 * i] : 0.0f, ny = vnorm4 ? vnorm4[4 * i + 1] : 0.0f,
                nz = vnorm4 ? vnorm4[4 * i + 2] : 1.0f;
    n += "vn " + num(nx) + " " + num(ny) + " " + num(nz) + "\n";
    tc += "vt " + num(vtex2 ? vtex2[2 * i] : 0.0f) + " " + num(vtex2 ? vtex2[2 * i + 1] : 0.0f) + "\n";
  }
  for (int64_t t = 0; t < nidx / 3; ++t) {
    fc += "f";
    for (int k = 0; k < 3; ++k) {
      const std::string q = std::to_string(idx[3 * t + k] + 1);
      fc += " " + q + "/" + q + "/" + q;
    }
    fc += "\n";
  }
  const std::string all = "# obj file created by custom obj loader\no MainModel\n" + v + tc + n + "s off\n" + fc;
  const size_t wrote = std::fwrite(all.data(), 1, all.size(), f);
  std::fclose(f);
  if (wrote != all.size()) { err = "short write"; return false; }
  return true;
}

// ------------------------------------------------------------------ PNG ---
namespace {
uint32_t crc32(const uint8_t *p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t v = i;
      for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
      table[i] = v;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}
void be32(std::vector<uint8_t> &o, uint32_t v) {
  o.push_back((uint8_t)(v >> 24)); o.push_back((uint8_t)(v >> 16));
  o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v);
}
void chunk(std::vector<uint8_t> &o, const char *type, const std::vector<uint8_t> &data) {
  be32(o, (uint32_t)data.size());
  const size_t start = o.size();
  o.insert(o.end(), type, type + 4);
  o.insert(o.end(), data.begin(), data.end());
  be32(o, crc32(o.data() + start, o.size() - start) ^ 0xFFFFFFFFu);
}
}  // namespace

bool write_png(const char *path, const uint32_t *rgba, int32_t W, int32_t H, std::string &err) {
  if (!path || !rgba || W <= 0 || H <= 0) { err = "bad arguments"; return false; }
  std::vector<uint8_t> raw;  // filter byte 0 + RGBA per row
  raw.reserve((size_t)H * (1 + 4 * (size_t)W));
  for (int32_t y = 0; y < H; ++y) {
    raw.push_back(0);
    for (int32_t x = 0; x < W; ++x) {
      const uint32_t c = rgba[(size_t)y * W + x];
      raw.push_back((uint8_t)c); raw.push_back((uint8_t)(c >> 8));
      raw.push_back((uint8_t)(c >> 16)); raw.push_back((uint8_t)(c >> 24));
    }
  }
  std::vector<uint8_t> z{0x78, 0x01};  // zlib header, stored blocks
  uint32_t a = 1, b = 0;
  for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
    const size_t n = std::min<size_t>(65535, raw.size() - off);
    z.push_back(off + n >= raw.size() ? 1 : 0);
    z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
    z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
    if (raw.empty()) break;
  }
  for (uint8_t v : raw) { a = (a + v) % 65521u; b = (b + a) % 65521u; }
  be32(z, (b << 16) | a);
  std::vector<uint8_t> png{0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<uint8_t> ihdr;
  be32(ihdr, (uint32_t)W);
  be32(ihdr, (uint32_t)H);
  const uint8_t rest[5] = {8, 6, 0, 0, 0};  // 8-bit RGBA, deflate, no filter method ext, no interlace
  ihdr.insert(ihdr.end(), rest, rest + 5);
  chunk(png, "IHDR", ihdr);
  chunk(png, "IDAT", z);
  chunk(png, "IEND", {});
  FILE *f = std::fopen(path, "wb");
  if (!f) { err = std::string("cannot write ") + path; return false; }
  const size_t wrote = std::fwrite(png.data(), 1, png.size(), f);
  std::fclose(f);
  if (wrote != png.size()) { err = "short write"; return false; }
  return true;
}

void camera_matrices(const float pos[3], const float target[3], const float up[3], float fovy,
                     float aspect, float znear, float zfar, float view_inv[16], float proj_inv[16]) {
  CamState c;
  cam_init(c, pos, target, up);
  cam_view_inverse(c, view_inv);
  // perspectiveMatrix(fovy, aspect, near, far)
  M4 pr{};
  const float ymax = znear * std::tan(fovy * 3.14159265358979323846f / 360.0f);
  const float xmax = ymax * aspect;
  pr.m[0][0] = 2.0f * znear / (2.0f * xmax);
  pr.m[1][1] = 2.0f * znear / (2.0f * ymax);
  pr.m[2][2] = (-zfar - znear) / (zfar - znear);
  pr.m[2][3] = -1.0f;
  pr.m[3][2] = -2.0f * zfar * znear / (zfar - znear);
  invert(pr, proj_inv);
}

void copy_rect(uint32_t *dc, float *dt, const uint32_t *sc, const float *st, int64_t W, int32_t x0, int32_t x1,
               int32_t y0, int32_t y1, int threads) {
  const size_t w = (size_t)(x1 - x0 + 1);
  if (threads <= 0)  // one thread per 32 rows, at most the OpenMP default and 16
    threads = std::max(1, std::min({(y1 - y0 + 1) / 32, omp_get_max_threads(), 16}));
#pragma omp parallel for schedule(static) num_threads(threads) if (threads > 1)
  for (int32_t y = y0; y <= y1; ++y) {
    const size_t o = (size_t)y * (size_t)W + (size_t)x0;
    std::memcpy(dc + o, sc + o, w * 4);
    std::memcpy(dt + o, st + o, w * 4);
  }
}

// n 4-byte words from s to d, d written with 32-byte streaming stores where it
// is 32-byte aligned (the head and tail with plain stores): the caller's frame
// is not read first (no read-for-ownership), so the copy moves 2 bytes of
// memory traffic per byte instead of 3. The caller issues _mm_sfence().
static void copy_words_stream(uint32_t *d, const uint32_t *s, size_t n) {
  size_t i = 0;
  for (; i < n && ((uintptr_t)(d + i) & 31u); ++i) d[i] = s[i];
  for (; i + 8 <= n; i += 8)
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i)));
  for (; i < n; ++i) d[i] = s[i];
}

void copy_spans(uint32_t *dc, float *dt, uint32_t *sc, float *st, int64_t W, int32_t H, const int32_t *span,
                int threads, bool clear_src) {
  // at most 16 threads (2-24 measured level, profiles/r05/dropin_threads.txt);
  // streaming stores into the caller's frame (measured faster than memcpy,
  // profiles/r05/dropin_copy_nt_ab.txt)
  constexpr int cap = 16;
  constexpr bool nt = true;
  if (threads <= 0) threads = std::max(1, std::min({H / 32, omp_get_max_threads(), cap}));
  auto row = [&](int32_t y) {
    const int32_t lo = span[2 * y], hi = -span[2 * y + 1];
    if (lo > hi || lo < 0 || hi >= W) return;  // (no hit: INT32_MAX, INT32_MAX)
    const size_t o = (size_t)y * (size_t)W + (size_t)lo, w = (size_t)(hi - lo + 1);
    if (nt) {
      copy_words_stream(dc + o, sc + o, w);
      copy_words_stream(reinterpret_cast<uint32_t *>(dt + o), reinterpret_cast<const uint32_t *>(st + o), w);
    } else {
      std::memcpy(dc + o, sc + o, w * 4);
      std::memcpy(dt + o, st + o, w * 4);
    }
    if (clear_src) {  // (the lines were just read: the reset writes into this core's cache)
      std::memset(sc + o, 0, w * 4);
      std::fill(st + o, st + o + w, std::numeric_limits<float>::infinity());
    }
  };
  if (threads <= 1) {
    for (int32_t y = 0; y < H; ++y) row(y);
    _mm_sfence();
    return;
  }
  // the spans sit in the rows the scene covers (the middle of the frame for
  // the app's centred model), so equal row counts per thread leave most
  // threads idle: thread k takes the rows where the running pixel count
  // crosses [k, k+1) / threads of the total
  thread_local std::vector<int64_t> pre;
  pre.assign((size_t)H + 1, 0);
  for (int32_t y = 0; y < H; ++y) {
    const int32_t lo = span[2 * y], hi = -span[2 * y + 1];
    pre[y + 1] = pre[y] + (lo > hi || lo < 0 || hi >= W ? 0 : (int64_t)(hi - lo + 1) + 16);
  }
  const int64_t total = pre[H];
  if (total == 0) return;
  const int64_t *pp = pre.data();
#pragma omp parallel num_threads(threads)
  {
    const int k = omp_get_thread_num(), n = omp_get_num_threads();
    const int64_t a = total * k / n, b = total * (k + 1) / n;
    // rows y with a <= pre[y] < b start in this thread's share
    const int32_t y0 = (int32_t)(std::lower_bound(pp, pp + H, a) - pp);
    const int32_t y1 = (int32_t)(std::lower_bound(pp, pp + H, b) - pp);
    for (int32_t y = y0; y < y1; ++y) row(y);
    _mm_sfence();  // this thread's streaming stores drained before the join
  }
}

void clear_frame(uint32_t *c, float *t, int64_t n, int threads) {
  const float inf = std::numeric_limits<float>::infinity();
  const int64_t chunk = 1 << 16;
#pragma omp parallel for schedule(static) num_threads(threads) if (threads > 1)
  for (int64_t i0 = 0; i0 < n; i0 += chunk) {
    const int64_t m = std::min(chunk, n - i0);
    std::memset(c + i0, 0, (size_t)m * 4);
    std::fill(t + i0, t + i0 + m, inf);
  }
}

}  // namespace rth
