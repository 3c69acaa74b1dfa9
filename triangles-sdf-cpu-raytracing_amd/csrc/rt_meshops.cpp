// rt_meshops.cpp -- host side of mesh -> SDF construction (SURVEY.md 8(f)
// rank 1) and the config-5 mesh stand-in. The reference has no SDF generator
// (its grids/octrees are course data in the formats of grid_raytracing.cpp:
// 127-134 and octree_raytracing.cpp:8-16, octree_raytracing.hpp:8-18); this
// file defines the construction, the GPU evaluates it (rt_sdfgen.hip), and
// oracle/cpuref.cpp restates it by brute force for the parity tests.
//
// Signed distance: d(p) = min over triangles of |p - closest(p, tri)|
// (Ericson, Real-Time Collision Detection 5.1.5; ties -> lowest triangle id);
// sign from the angle-weighted pseudonormal of the closest feature (vertex,
// edge or face; Baerentzen & Aanaes 2005): negative when dot(p - q, N) < 0.
// Vertices are welded by exact position bits so UV seams do not split
// pseudonormals. Built with -ffp-contract=off.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "rt_host.h"

namespace rth {

namespace {

struct P3 {
  float x, y, z;
};
inline P3 sub(P3 a, P3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline P3 cross3(P3 a, P3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float dot3(P3 a, P3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct KeyHash {
  size_t operator()(const std::array<uint32_t, 3> &k) const {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t v : k) h = (h ^ v) * 1099511628211ull;
    return (size_t)h;
  }
};

}  // namespace

bool prep_sdf_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                   SdfMeshHost &out, std::string &err) {
  out = SdfMeshHost();
  if (!build_bvh8(vpos4, nverts, idx, nidx, out.bvh, err, kBvhTris)) return false;
  const size_t ntri = (size_t)nidx / 3;
  if (ntri == 0) { err = "mesh has no triangles"; return false; }

  // positions after the renderer's v /= v.w (triangles_raytracing.cpp:307-309)
  std::vector<P3> P((size_t)nverts);
  for (int64_t v = 0; v < nverts; ++v) {
    const float *q = vpos4 + 4 * v;
    P[(size_t)v] = {q[0] / q[3], q[1] / q[3], q[2] / q[3]};
  }
  // weld by exact bits, ids in order of first appearance
  std::unordered_map<std::array<uint32_t, 3>, uint32_t, KeyHash> wmap;
  std::vector<uint32_t> weld((size_t)nverts);
  for (int64_t v = 0; v < nverts; ++v) {
    std::array<uint32_t, 3> k;
    std::memcpy(k.data(), &P[(size_t)v], 12);
    auto it = wmap.emplace(k, (uint32_t)wmap.size()).first;
    weld[(size_t)v] = it->second;
  }
  std::vector<double> vacc(3 * wmap.size(), 0.0);
  std::unordered_map<uint64_t, std::array<double, 3>> eacc;
  eacc.reserve(ntri * 2);
  std::vector<P3> fn(ntri);
  auto ekey = [&](uint32_t a, uint32_t b) -> uint64_t {
    const uint32_t wa = weld[a], wb = weld[b];
    return wa < wb ? ((uint64_t)wa << 32 | wb) : ((uint64_t)wb << 32 | wa);
  };
  for (size_t t = 0; t < ntri; ++t) {
    const uint32_t vi[3] = {idx[3 * t], idx[3 * t + 1], idx[3 * t + 2]};
    const P3 a = P[vi[0]], b = P[vi[1]], c = P[vi[2]];
    const P3 n = cross3(sub(b, a), sub(c, a));
    const float l = std::sqrt(dot3(n, n));
    const P3 nf = l > 0.0f ? P3{n.x / l, n.y / l, n.z / l} : P3{0.0f, 0.0f, 0.0f};
    fn[t] = nf;
    const P3 vv[3] = {a, b, c};
    for (int k = 0; k < 3; ++k) {  // interior angle at corner k
      const P3 u = vv[(k + 1) % 3], w = vv[(k + 2) % 3], o = vv[k];
      const double ux = (double)u.x - o.x, uy = (double)u.y - o.y, uz = (double)u.z - o.z;
      const double wx = (double)w.x - o.x, wy = (double)w.y - o.y, wz = (double)w.z - o.z;
      const double lu = std::sqrt(ux * ux + uy * uy + uz * uz), lw = std::sqrt(wx * wx + wy * wy + wz * wz);
      double ang = 0.0;
      if (lu > 0.0 && lw > 0.0) {
        const double cs = std::min(1.0, std::max(-1.0, (ux * wx + uy * wy + uz * wz) / (lu * lw)));
        ang = std::acos(cs);
      }
      double *acc = &vacc[3 * (size_t)weld[vi[k]]];
      acc[0] += ang * nf.x;
      acc[1] += ang * nf.y;
      acc[2] += ang * nf.z;
    }
    const uint64_t ek[3] = {ekey(vi[0], vi[1]), ekey(vi[0], vi[2]), ekey(vi[1], vi[2])};
    for (uint64_t k : ek) {
      auto &e = eacc.emplace(k, std::array<double, 3>{0.0, 0.0, 0.0}).first->second;
      e[0] += nf.x;
      e[1] += nf.y;
      e[2] += nf.z;
    }
  }
  out.pn.assign(ntri * 4 * kSdfFeatures, 0.0f);
  for (size_t t = 0; t < ntri; ++t) {
    const uint32_t vi[3] = {idx[3 * t], idx[3 * t + 1], idx[3 * t + 2]};
    float *o = &out.pn[t * 4 * kSdfFeatures];
    for (int k = 0; k < 3; ++k) {
      const double *acc = &vacc[3 * (size_t)weld[vi[k]]];
      o[4 * k + 0] = (float)acc[0];
      o[4 * k + 1] = (float)acc[1];
      o[4 * k + 2] = (float)acc[2];
    }
    const uint64_t ek[3] = {ekey(vi[0], vi[1]), ekey(vi[0], vi[2]), ekey(vi[1], vi[2])};
    for (int k = 0; k < 3; ++k) {
      const auto &e = eacc.at(ek[k]);
      o[4 * (3 + k) + 0] = (float)e[0];
      o[4 * (3 + k) + 1] = (float)e[1];
      o[4 * (3 + k) + 2] = (float)e[2];
    }
    o[24] = fn[t].x;
    o[25] = fn[t].y;
    o[26] = fn[t].z;
  }
  // triangle corners in the BVH's leaf order (GTri order), original id in a.w
  out.tri.resize(out.bvh.tris.size() * 12);
  for (size_t g = 0; g < out.bvh.tris.size(); ++g) {
    const uint32_t id = out.bvh.tris[g].orig_id;
    float *o = &out.tri[12 * g];
    for (int k = 0; k < 3; ++k) {
      const P3 p = P[idx[3 * (size_t)id + k]];
      o[4 * k + 0] = p.x;
      o[4 * k + 1] = p.y;
      o[4 * k + 2] = p.z;
      o[4 * k + 3] = 0.0f;
    }
    std::memcpy(&o[3], &id, 4);
  }
  return true;
}

bool subdivide_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, int levels,
                    Mesh &out, std::string &err) {
  if (nidx < 0 || nidx % 3 != 0) { err = "index count must be a multiple of 3"; return false; }
  if (levels < 0 || levels > 6) { err = "levels must be in [0, 6]"; return false; }
  for (int64_t i = 0; i < nidx; ++i)
    if ((int64_t)idx[i] >= nverts) { err = "vertex index out of range"; return false; }
  std::vector<float> V(vpos4, vpos4 + 4 * nverts);
  std::vector<uint32_t> I(idx, idx + nidx);
  for (int l = 0; l < levels; ++l) {
    const size_t ntri = I.size() / 3;
    if (V.size() / 4 + ntri * 3 > 0xFFFFFFFFull || ntri * 12 > 0xFFFFFFFFull) {
      err = "subdivided mesh too large";
      return false;
    }
    std::unordered_map<uint64_t, uint32_t> mid;
    mid.reserve(ntri * 2);
    auto midpoint = [&](uint32_t a, uint32_t b) -> uint32_t {
      const uint64_t k = a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a);
      auto it = mid.find(k);
      if (it != mid.end()) return it->second;
      const uint32_t id = (uint32_t)(V.size() / 4);
      for (int c = 0; c < 4; ++c) V.push_back((V[4 * (size_t)a + c] + V[4 * (size_t)b + c]) * 0.5f);
      mid.emplace(k, id);
      return id;
    };
    std::vector<uint32_t> J;
    J.reserve(ntri * 12);
    for (size_t t = 0; t < ntri; ++t) {
      const uint32_t a = I[3 * t], b = I[3 * t + 1], c = I[3 * t + 2];
      const uint32_t ab = midpoint(a, b), bc = midpoint(b, c), ca = midpoint(c, a);
      const uint32_t tris[12] = {a, ab, ca, ab, b, bc, ca, bc, c, ab, bc, ca};
      J.insert(J.end(), tris, tris + 12);
    }
    I.swap(J);
  }
  out.vpos4.swap(V);
  out.idx.swap(I);
  return true;
}

bool build_sdf_octree(SdfQuery query, void *ctx, int depth, std::vector<uint8_t> &nodes36,
                      std::string &err) {
  if (depth < 0 || depth > 12) { err = "octree depth must be in [0, 12]"; return false; }
  struct Cell {
    uint32_t x, y, z;
  };
  std::vector<std::vector<Cell>> level(1, std::vector<Cell>{{0, 0, 0}});
  std::vector<std::vector<uint8_t>> refine;
  std::vector<float> pts, s;
  for (int d = 0; d < depth; ++d) {
    const std::vector<Cell> &cur = level[(size_t)d];
    const float half = std::ldexp(1.0f, -d);  // half-size; centre = -1 + (2i+1) * 2^-d (exact)
    pts.resize(cur.size() * 3);
    for (size_t j = 0; j < cur.size(); ++j) {
      pts[3 * j + 0] = (float)(2 * cur[j].x + 1) * half - 1.0f;
      pts[3 * j + 1] = (float)(2 * cur[j].y + 1) * half - 1.0f;
      pts[3 * j + 2] = (float)(2 * cur[j].z + 1) * half - 1.0f;
    }
    s.resize(cur.size());
    if (!query(ctx, pts.data(), (int64_t)cur.size(), s.data(), err)) return false;
    const float hd = 1.7320508f * half;
    std::vector<uint8_t> r(cur.size());
    std::vector<Cell> next;
    for (size_t j = 0; j < cur.size(); ++j) {
      r[j] = std::fabs(s[j]) <= hd;
      if (!r[j]) continue;
      for (uint32_t id = 0; id < 8; ++id)
        next.push_back({2 * cur[j].x + (id >> 2), 2 * cur[j].y + ((id >> 1) & 1), 2 * cur[j].z + (id & 1)});
    }
    refine.push_back(std::move(r));
    level.push_back(std::move(next));
  }
  // corner values of the leaves at full depth
  const std::vector<Cell> &leaves = level[(size_t)depth];
  const float size = std::ldexp(1.0f, 1 - depth);
  pts.resize(leaves.size() * 24);
  for (size_t j = 0; j < leaves.size(); ++j)
    for (uint32_t k = 0; k < 8; ++k) {
      pts[24 * j + 3 * k + 0] = (float)(leaves[j].x + (k >> 2)) * size - 1.0f;
      pts[24 * j + 3 * k + 1] = (float)(leaves[j].y + ((k >> 1) & 1)) * size - 1.0f;
      pts[24 * j + 3 * k + 2] = (float)(leaves[j].z + (k & 1)) * size - 1.0f;
    }
  std::vector<float> corner(leaves.size() * 8);
  if (!leaves.empty() && !query(ctx, pts.data(), (int64_t)leaves.size() * 8, corner.data(), err)) return false;

  size_t total = 0;
  for (const auto &L : level) total += L.size();
  if (total > 0xFFFFFFFFull) { err = "octree too large"; return false; }
  nodes36.assign(total * 36, 0);
  size_t base = 0;
  for (int d = 0; d <= depth; ++d) {
    const size_t n = level[(size_t)d].size();
    size_t child = base + n;  // first node of the next level
    for (size_t j = 0; j < n; ++j) {
      uint8_t *rec = &nodes36[(base + j) * 36];
      float v[8];
      uint32_t off = 0;
      if (d == depth) {
        std::memcpy(v, &corner[8 * j], 32);
      } else if (refine[(size_t)d][j]) {
        std::fill(v, v + 8, 0.0f);
        off = (uint32_t)child;
        child += 8;
      } else {
        std::fill(v, v + 8, 1000.0f);  // empty leaf (SDFOctreeNode::isEmpty, octree_raytracing.hpp:12-17)
      }
      std::memcpy(rec, v, 32);
      std::memcpy(rec + 32, &off, 4);
    }
    base += n;
  }
  return true;
}

}  // namespace rth
