// trav_sim.cpp -- where the headline BVH kernel's idle lanes come from, on the CPU.
//
// Rebuilds the bunny's BVH8 through librtamd's host entry points (rt_load_obj,
// rt_bvh_export with the host builder: no GPU), traces the eye rays of one
// orbit frame with the reference traversal (front-to-back, sort8 order,
// per-frame local best, BVHBuilder::traverseNode, triangles_raytracing.cpp:
// 266-335) and records every ray's sequence of loop iterations: I (expand an
// inner node) or L (test a leaf). Each 8x8 wave tile is then replayed in SIMT
// lockstep under issue policies, with a per-iteration cost model in VALU
// instructions (cI inner, cL leaf, cC the shared choose-next part):
//   P0  every iteration runs both branches if any lane needs them (the kernel);
//   P1  one branch per iteration, the one more lanes need (the others wait);
//   P2  leaves wait until no lane needs an inner node (while-while ordering).
// A lane's own visit order never changes under these policies (they only delay
// it), so the results would be the same bits; the question is the cost.
// Output: lane utilisation, wave instructions and iterations per policy.
//
// build: g++ -O2 -std=c++17 -Iinclude tools/trav_sim.cpp \
//          -Ltriangles-sdf-cpu-raytracing_amd/lib -lrtamd -Wl,-rpath,... -o /tmp/trav_sim
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtamd.h"

namespace {

struct Node {
  bool leaf;
  uint32_t n;          // children (inner) or index count (leaf)
  uint32_t start;      // leaf: first index position
  float box[48];       // Box8 SoA: mn.x[8] mn.y[8] mn.z[8] mx.x[8] mx.y[8] mx.z[8]
  uint32_t child[8];
};

bool g_split = false;  // leaves of more than 4 triangles as two iterations of one batch each
std::vector<Node> nodes;
std::vector<uint32_t> canon;
std::vector<float> vpos;
std::vector<uint32_t> idx, perm;

uint32_t parse(size_t &at) {
  const uint32_t me = (uint32_t)nodes.size();
  nodes.emplace_back();
  const uint32_t *r = canon.data() + 52 * at;
  ++at;
  Node nd{};
  nd.leaf = r[0] != 0;
  nd.n = r[1];
  nd.start = r[2];
  std::memcpy(nd.box, r + 4, 192);
  if (!nd.leaf)
    for (uint32_t c = 0; c < nd.n; ++c) nd.child[c] = parse(at);
  nodes[me] = nd;
  return me;
}

struct V3 {
  float x, y, z;
};
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

float slab(const float *b, int c, V3 o, V3 inv, float tn, float tf) {
  const float t1x = (b[c] - o.x) * inv.x, t2x = (b[24 + c] - o.x) * inv.x;
  const float t1y = (b[8 + c] - o.y) * inv.y, t2y = (b[32 + c] - o.y) * inv.y;
  const float t1z = (b[16 + c] - o.z) * inv.z, t2z = (b[40 + c] - o.z) * inv.z;
  auto mn = [](float a, float b2) { return a < b2 ? a : b2; };
  auto mx = [](float a, float b2) { return a > b2 ? a : b2; };
  float tMin = mx(mn(t1x, t2x), mx(mn(t1y, t2y), mn(t1z, t2z)));
  float tMax = mn(mx(t1x, t2x), mn(mx(t1y, t2y), mx(t1z, t2z)));
  tMin = mx(tMin, tn);
  tMax = mn(tMax, tf);
  return (tMax < 0.0f || tMin > tMax) ? -1.0f : tMin;
}

float tri(uint32_t slot, V3 o, V3 d) {
  const uint32_t *t = idx.data() + 3 * (size_t)perm[slot];
  V3 v[3];
  for (int k = 0; k < 3; ++k) {
    const float *p = vpos.data() + 4 * (size_t)t[k];
    v[k] = {p[0] / p[3], p[1] / p[3], p[2] / p[3]};
  }
  const V3 e1 = sub(v[1], v[0]), e2 = sub(v[2], v[0]);
  const V3 pv = cross(d, e2);
  const float det = dot(e1, pv);
  if (det < 1e-8f && det > -1e-8f) return INFINITY;
  const float inv = 1.0f / det;
  const V3 tv = sub(o, v[0]);
  const float u = dot(tv, pv) * inv;
  const V3 qv = cross(tv, e1);
  const float vv = dot(d, qv) * inv;
  if (u < 0.0f || u > 1.0f || vv < 0.0f || u + vv > 1.0f) return INFINITY;
  return dot(e2, qv) * inv;
}

// traverseNode recursion with the iteration trace: 'I' per inner node, 'L' per leaf
float trace(uint32_t ni, V3 o, V3 d, V3 inv, float tn, float tf, std::string &seq) {
  const Node &nd = nodes[ni];
  float best = INFINITY;
  if (nd.leaf) {
    if (nd.n / 3 > 4) {
      if (g_split) seq += "LL";
      else seq.push_back('M');
    } else {
      seq.push_back('L');
    }
    for (uint32_t k = 0; k < nd.n / 3; ++k) {
      const float t = tri(nd.start / 3 + k, o, d);
      if (t < best) best = t;
    }
    return best;
  }
  seq.push_back('I');
  float t[8];
  int id[8];
  for (int c = 0; c < 8; ++c) {
    t[c] = (uint32_t)c < nd.n ? slab(nd.box, c, o, inv, tn, tf) : -1.0f;
    id[c] = c;
  }
  const int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                          {0, 4}, {3, 7}, {1, 5}, {2, 6}, {1, 4}, {3, 6}, {2, 4}, {3, 5}, {3, 4}};
  for (auto &p : net)
    if (t[p[0]] > t[p[1]]) {
      std::swap(t[p[0]], t[p[1]]);
      std::swap(id[p[0]], id[p[1]]);
    }
  for (int i = 0; i < 8; ++i) {
    if (t[i] < 0.0f || (uint32_t)id[i] >= nd.n) continue;
    if (best < t[i]) break;
    const float r = trace(nd.child[id[i]], o, d, inv, tn, tf, seq);
    if (r < best) best = r;
  }
  return best;
}

double g_k = 1.0;  // P1: a side is skipped when the other has more than K times its lanes

struct Cost {
  double lane_instr = 0, wave_instr = 0, iters = 0;
};

// SIMT replay of one tile's sequences under a policy
void replay(const std::vector<std::string> &s, int policy, double cI, double cL, double cC, Cost &out) {
  std::vector<size_t> pos(s.size(), 0);
  for (;;) {
    int nI = 0, nL = 0, live = 0, nM = 0;
    for (size_t k = 0; k < s.size(); ++k) {
      if (pos[k] >= s[k].size()) continue;
      ++live;
      (s[k][pos[k]] == 'I' ? nI : nL)++;
      nM += s[k][pos[k]] == 'M';
    }
    if (!live) break;
    bool runI = nI > 0, runL = nL > 0;
    if (policy == 1 && runI && runL) {  // skip the side with K x fewer lanes
      if (nL * g_k < nI) runL = false;
      else if (nI * g_k < nL) runI = false;
    }
    if (policy == 2 && runI) runL = false;
    double w = cC;
    if (runI) w += cI;
    if (runL) w += nM ? cL : cL / 2;  // a second batch of 4 triangles when any lane's leaf has more
    out.wave_instr += w;
    out.iters += 1;
    // lanes doing useful work: the common part for every lane that advances
    int adv = 0;
    for (size_t k = 0; k < s.size(); ++k) {
      if (pos[k] >= s[k].size()) continue;
      const char c = s[k][pos[k]];
      if ((c == 'I' && runI) || (c != 'I' && runL)) {
        out.lane_instr += (c == 'I' ? cI : c == 'M' ? cL : cL / 2) + cC;
        ++pos[k];
        ++adv;
      }
    }
    (void)adv;
  }
}

}  // namespace

int main(int argc, char **argv) {
  const char *obj = argc > 1 ? argv[1] : "data/_unpacked/stanford-bunny.obj";
  const int W = argc > 2 ? std::atoi(argv[2]) : 1920, H = argc > 3 ? std::atoi(argv[3]) : 1080;
  const double cI = argc > 4 ? std::atof(argv[4]) : 250, cL = argc > 5 ? std::atof(argv[5]) : 360,
               cC = argc > 6 ? std::atof(argv[6]) : 40;
  g_k = argc > 7 ? std::atof(argv[7]) : 1.0;
  g_split = argc > 8 && std::atoi(argv[8]) != 0;
  int64_t nv = 0, ni = 0;
  if (rt_load_obj(obj, 1, nullptr, &nv, nullptr, &ni)) return std::printf("load: %s\n", rt_last_error()), 1;
  vpos.resize(4 * nv);
  idx.resize(ni);
  rt_load_obj(obj, 1, vpos.data(), &nv, idx.data(), &ni);
  rt_set_bvh_builder(RT_BVH_HOST);
  int64_t nn = 0;
  int32_t depth = 0;
  perm.resize(ni / 3);
  rt_bvh_export(vpos.data(), nv, idx.data(), ni, nullptr, &nn, nullptr, &depth);
  canon.resize(52 * nn);
  if (rt_bvh_export(vpos.data(), nv, idx.data(), ni, canon.data(), &nn, perm.data(), &depth))
    return std::printf("export: %s\n", rt_last_error()), 1;
  size_t at = 0;
  parse(at);
  std::printf("%zu nodes, depth %d, %lld tris\n", nodes.size(), depth, (long long)ni / 3);
  // orbit frame 0 of bench.py (pos = (0, 0.5, 2.5)), the kernel's eye rays
  const float pos[3] = {0.0f, 0.5f, 2.5f}, tgt[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  float vi[16], pi[16];
  rt_camera(pos, tgt, up, 45.0f, (float)W / (float)H, 0.01f, 100.0f, vi, pi);
  auto eye = [&](int x, int y) {
    const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    float p[4] = {2.0f * fx / (float)W - 1.0f, 2.0f * fy / (float)H - 1.0f, 0.0f, 1.0f}, q[4];
    for (int r = 0; r < 4; ++r) q[r] = pi[r] * p[0] + pi[4 + r] * p[1] + pi[8 + r] * p[2] + pi[12 + r] * p[3];
    const float w = q[3];
    V3 dd{q[0] / w, q[1] / w, q[2] / w};
    const float l = std::sqrt(dot(dd, dd));
    dd = {dd.x / l, dd.y / l, dd.z / l};
    return V3{vi[0] * dd.x + vi[4] * dd.y + vi[8] * dd.z, vi[1] * dd.x + vi[5] * dd.y + vi[9] * dd.z,
              vi[2] * dd.x + vi[6] * dd.y + vi[10] * dd.z};
  };
  Cost c[3];
  double both = 0, iters0 = 0, steps = 0;
  long tiles = 0, busy_tiles = 0, root_only = 0;
  for (int ty = 0; ty < H / 8; ++ty)
    for (int tx = 0; tx < W / 8; ++tx) {
      std::vector<std::string> seqs(64);
      bool any = false;
      for (int l = 0; l < 64; ++l) {
        const int x = tx * 8 + (l & 7), yo = ty * 8 + (l >> 3), y = H - yo - 1;
        const V3 d = eye(x, y);
        const V3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        trace(0, V3{pos[0], pos[1], pos[2]}, d, inv, 0.01f, 100.0f, seqs[l]);
        steps += seqs[l].size();
        any |= seqs[l].size() > 1;
      }
      ++tiles;
      if (!any) {  // (every ray ends at the root: one iteration of the root expansion)
        for (int p = 0; p < 3; ++p) replay(seqs, p, cI, cL, cC, c[p]);
        continue;
      }
      ++busy_tiles;
      for (int l = 0; l < 64; ++l) root_only += seqs[l].size() <= 1;
      for (int p = 0; p < 3; ++p) replay(seqs, p, cI, cL, cC, c[p]);
      // iterations of P0 that run both branches
      std::vector<size_t> pos2(64, 0);
      for (;;) {
        int nI = 0, nL = 0;
        for (int k = 0; k < 64; ++k)
          if (pos2[k] < seqs[k].size()) (seqs[k][pos2[k]] == 'I' ? nI : nL)++, ++pos2[k];
        if (!nI && !nL) break;
        iters0 += 1;
        both += (nI && nL);
      }
    }
  // P1 with lane refill (the ray pump): a wave streams the pixels of 2x1-tile
  // items in queue order (every item of a row of items, frame rows top to
  // bottom) and hands each finished lane the next pixel once >= R lanes are
  // free; stream length = one row of items per wave
  for (int R : {8, 16, 32}) {
    Cost cr;
    for (int ty = 0; ty < H / 8; ++ty) {
      std::vector<std::string> stream;
      for (int tx2 = 0; tx2 < W / 16; ++tx2)
        for (int half = 0; half < 2; ++half)
          for (int l = 0; l < 64; ++l) {
            const int x = (tx2 * 2 + half) * 8 + (l & 7), yo = ty * 8 + (l >> 3), y = H - yo - 1;
            const V3 d = eye(x, y);
            const V3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
            std::string sq;
            trace(0, V3{pos[0], pos[1], pos[2]}, d, inv, 0.01f, 100.0f, sq);
            stream.push_back(sq);
          }
      size_t next = 0;
      std::vector<std::string> lane(64);
      std::vector<size_t> at(64, 0);
      std::vector<bool> live(64, false);
      for (;;) {
        int dead = 0;
        for (int k = 0; k < 64; ++k) dead += !live[k];
        if (dead >= R || next == 0)
          for (int k = 0; k < 64 && next < stream.size(); ++k)
            if (!live[k]) { lane[k] = stream[next++]; at[k] = 0; live[k] = !lane[k].empty(); }
        int nI = 0, nL = 0, nlive = 0;
        for (int k = 0; k < 64; ++k)
          if (live[k]) { ++nlive; (lane[k][at[k]] == 'I' ? nI : nL)++; }
        if (!nlive) { if (next >= stream.size()) break; continue; }
        bool runI = nI > 0, runL = nL > 0;
        if (runI && runL) { if (nL * g_k < nI) runL = false; else if (nI * g_k < nL) runI = false; }
        int nM = 0;
        for (int k = 0; k < 64; ++k) nM += live[k] && lane[k][at[k]] == 'M';
        cr.wave_instr += cC + (runI ? cI : 0) + (runL ? (nM ? cL : cL / 2) : 0);
        cr.iters += 1;
        for (int k = 0; k < 64; ++k) {
          if (!live[k]) continue;
          const char c = lane[k][at[k]];
          if ((c == 'I' && runI) || (c != 'I' && runL)) {
            cr.lane_instr += (c == 'I' ? cI : c == 'M' ? cL : cL / 2) + cC;
            if (++at[k] >= lane[k].size()) live[k] = false;
          }
        }
      }
    }
    std::printf("P1 + refill at %2d free lanes: lane util %.3f  wave instr %.4g  iterations %.4g  (x%.3f instr vs P1 per tile; whole frame)\n",
                R, cr.lane_instr / (64.0 * cr.wave_instr), cr.wave_instr, cr.iters, cr.wave_instr / c[1].wave_instr);
  }
  std::printf("tiles %ld (%ld with any ray past the root), steps per ray %.3f\n", tiles, busy_tiles,
              steps / ((double)W * H));
  std::printf("rays of those tiles that end at the root: %.1f %%\n", 100.0 * root_only / (64.0 * busy_tiles));
  std::printf("P0 iterations running both branches: %.1f %%\n", 100.0 * both / iters0);
  const char *name[3] = {"P0 both branches (kernel)", "P1 minority side waits (K)", "P2 inner first"};
  for (int p = 0; p < 3; ++p)
    std::printf("%-28s lane util %.3f  wave instr %.4g  iterations %.4g  (x%.3f instr, x%.3f iters vs P0)\n",
                name[p], c[p].lane_instr / (64.0 * c[p].wave_instr), c[p].wave_instr, c[p].iters,
                c[p].wave_instr / c[0].wave_instr, c[p].iters / c[0].iters);
  return 0;
}
