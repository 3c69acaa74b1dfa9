// prune_probe.cpp -- dev probe (not product code): how much traversal work a
// GLOBAL-best prune of the BVH8 descent would save, and whether it changes
// any primary hit, on the bench's camera orbit.
//
// The reference prunes a child only against the best hit of its own recursion
// frame (triangles_raytracing.cpp:282-283). The variant additionally skips a
// child box whose entry t exceeds the best hit found anywhere so far by a
// margin (rel * |best| + abs), and only when that entry is unclamped (> tNear,
// so the negative-t quirk boxes around the origin are kept). Builds on the
// oracle's restatement (#included: same BVH, same float ops).
//
//   g++ -std=c++20 -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp -o /tmp/prune_probe tools/prune_probe.cpp
//   /tmp/prune_probe data/_unpacked/stanford-bunny.obj 1920 1080 [frames]
#include "../oracle/cpuref.cpp"

namespace probe {

struct Cost {
  long long n = 0;
};

// BVHBuilder::traverseNode with the extra global prune (margin < 0: off)
HitInfo trav(const BVHBuilder &B, size_t index, float3 o, float3 d, float tNear, float tFar, float &gbest,
             double rel, double abs_m, long long &cost) {
  const BVH8Node &node = B.nodes[index];
  HitInfo result;
  ++cost;
  if (!node.isLeaf) {
    float t[8] = {};
    float3 inv = 1.0f / d;
    float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
    intersect_box_8(node.boxes, oo, ii, tNear, tFar, t);
    int ch[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    sort8(t, ch);
    for (int i = 0; i < 8; ++i) {
      uint32_t c = (uint32_t)ch[i];
      if (c >= node.realCount || (t[i] < 0) || (result.hitten && result.t < t[i])) continue;
      if (rel >= 0 && t[i] > tNear && gbest < INF && (double)t[i] > (double)gbest + rel * std::fabs(gbest) + abs_m)
        continue;
      HitInfo cur = trav(B, node.offset + c, o, d, tNear, tFar, gbest, rel, abs_m, cost);
      if (cur.hitten && (!result.hitten || result.t > cur.t)) result = cur;
    }
  } else {
    uint32_t start = node.startIndex, end = start + node.count;
    uint32_t ntri = std::min((end - start) / 3, 8u);
    cost += ntri;
    for (uint32_t k = 0; k < ntri; ++k) {
      float4 v0 = B.mesh.vPos4f[B.mesh.indices[start + k * 3]];
      float4 v1 = B.mesh.vPos4f[B.mesh.indices[start + k * 3 + 1]];
      float4 v2 = B.mesh.vPos4f[B.mesh.indices[start + k * 3 + 2]];
      v0 = v0 / v0.w; v1 = v1 / v1.w; v2 = v2 / v2.w;
      TriHit h = triangle_intersection(o, d, to_float3(v0), to_float3(v1), to_float3(v2));
      if (h.hit && (!result.hitten || result.t > h.t)) {
        result.hitten = true;
        result.normal = h.n;
        result.t = h.t;
        result.prim = B.triId[start / 3 + k];
      }
      if (h.hit && h.t < gbest) gbest = h.t;
    }
  }
  return result;
}

}  // namespace probe

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s mesh.obj W H [frames] [subdiv]\n", argv[0]);
    return 2;
  }
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
  const int frames = argc > 4 ? std::atoi(argv[4]) : 8;
  Mesh m;
  if (!load_obj(argv[1], m)) return 1;
  load_and_scale(m);
  BVHBuilder B;
  B.perform(m);
  const double rels[] = {-1.0, 0.0, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2};
  const int NV = sizeof(rels) / sizeof(rels[0]);
  long long sum[NV] = {}, mx[NV] = {}, bad[NV] = {}, tile_max_sum[NV] = {}, tile_max_max[NV] = {};
  long long tiles = 0, hits = 0, mx_miss = 0, mx_hit = 0, heavy = 0, heavy_miss = 0;
  for (int f = 0; f < frames; ++f) {
    const int k = (f * 64) / frames;
    const float th = 2.0f * 3.14159265358979f * (float)k / 64.0f;
    const float pos[3] = {2.5f * std::sin(th), 0.5f, 2.5f * std::cos(th)}, tgt[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    float vi[16], pi[16];
    cpuref_camera(pos, tgt, up, 45.0f, (float)W / (float)H, 0.01f, 100.0f, vi, pi);
    float4x4 viewInv, projInv;
    std::memcpy(viewInv.m, vi, 64);
    std::memcpy(projInv.m, pi, 64);
    const float3 o(pos[0], pos[1], pos[2]);
    std::vector<int32_t> cost((size_t)NV * W * H);
#pragma omp parallel for schedule(dynamic) reduction(+ : sum[:NV], bad[:NV], hits, heavy, heavy_miss) reduction(max : mx[:NV], mx_miss, mx_hit)
    for (int yo = 0; yo < H; ++yo) {
      const int y = H - yo - 1;
      for (int x = 0; x < W; ++x) {
        float4 dir4 = EyeRayDir4f((float)x + 0.5f, (float)y + 0.5f, (float)W, (float)H, projInv);
        dir4.w = 0.0f;
        dir4 = mul(viewInv, dir4);
        const float3 d = to_float3(dir4);
        HitInfo ref;
        for (int v = 0; v < NV; ++v) {
          float g = INF;
          long long c = 0;
          HitInfo h = probe::trav(B, 0, o, d, 0.01f, 100.0f, g, rels[v], 0.0, c);
          if (v == 0) {
            ref = h;
            hits += h.hitten;
            (h.hitten ? mx_hit : mx_miss) = std::max(h.hitten ? mx_hit : mx_miss, c);
            if (c >= 64) { ++heavy; heavy_miss += !h.hitten; }
          } else if (h.hitten != ref.hitten || (h.hitten && (std::memcmp(&h.t, &ref.t, 4) != 0 ||
                                                             h.prim != ref.prim))) {
            ++bad[v];
          }
          sum[v] += c;
          mx[v] = std::max(mx[v], c);
          cost[((size_t)v * H + yo) * W + x] = (int32_t)c;
        }
      }
    }
    for (int ty = 0; ty < H; ty += 8)
      for (int tx = 0; tx < W; tx += 8) {
        ++tiles;
        for (int v = 0; v < NV; ++v) {
          long long tm = 0;
          for (int yy = ty; yy < std::min(H, ty + 8); ++yy)
            for (int xx = tx; xx < std::min(W, tx + 8); ++xx)
              tm = std::max<long long>(tm, cost[((size_t)v * H + yy) * W + xx]);
          tile_max_sum[v] += tm;
          tile_max_max[v] = std::max(tile_max_max[v], tm);
        }
      }
  }
  const double px = (double)frames * W * H;
  std::printf("%s %dx%d, %d orbit frames, %lld primary hits\n", argv[1], W, H, frames, hits);
  std::printf("reference: max cost of a hit ray %lld, of a miss ray %lld; rays with cost >= 64: %lld, of them "
              "misses %lld\n", mx_hit, mx_miss, heavy, heavy_miss);
  std::printf("%-10s %10s %8s %14s %12s %10s\n", "margin", "mean/px", "max/px", "mean tile max", "max tile", "mismatch");
  for (int v = 0; v < NV; ++v)
    std::printf("%-10s %10.3f %8lld %14.2f %12lld %10lld\n",
                v == 0 ? "reference" : (std::string("rel ") + std::to_string(rels[v]).substr(0, 8)).c_str(),
                sum[v] / px, mx[v], (double)tile_max_sum[v] / tiles, tile_max_max[v], bad[v]);
  return 0;
}
