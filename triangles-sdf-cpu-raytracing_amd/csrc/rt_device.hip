// rt_device.hip -- HIP kernels (gfx950) and the C ABI (include/rtamd.h).
//
// One thread per pixel; a 256-thread workgroup renders a 16x16 pixel block as
// four 8x8 wave tiles (coherent rays share BVH / octree nodes and grid
// voxels in L1/L2). Framebuffer stores are row-major, so a wave writes 8 rows
// x 32 B per buffer. Per-lane traversal stacks live in LDS, lane-interleaved.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rtamd.h"
#include "rt_error.h"
#include "rt_host.h"
#include "rt_layout.h"
#include "rt_math.h"
#include "rt_scenes.h"

using namespace rtd;

namespace rterr {
thread_local std::string g_err;
int set(int code, const std::string &msg) {
  g_err = msg;
  return code;
}
const char *get() { return g_err.c_str(); }
thread_local std::string g_noted;
thread_local hipError_t g_noted_err = hipSuccess;
hipError_t note(const char *call, hipError_t e) {
  if (e != hipSuccess) {
    g_noted = call;
    g_noted_err = e;
  }
  return e;
}
std::string take_stale() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return {};
  std::string m = std::string("stale HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) +
                  ") was pending from an earlier call: ";
  m += e == g_noted_err ? "librtamd's " + g_noted : std::string("a HIP call outside librtamd");
  g_noted.clear();
  g_noted_err = hipSuccess;
  return m;
}

namespace {
struct StreamInfo {
  int device;
  std::string label;
  const char *last;  // the last library call that queued work on it (static strings)
};
std::mutex g_stream_mu;
std::map<hipStream_t, StreamInfo> g_streams;

// errors HIP keeps for the context once raised (a faulting kernel or copy):
// every later call may report them, whichever work raised them
bool sticky(hipError_t e) {
  return e == hipErrorIllegalAddress || e == hipErrorLaunchFailure || e == hipErrorLaunchTimeOut ||
         e == hipErrorAssert || e == hipErrorIllegalState || e == hipErrorUnknown;
}
}  // namespace

void stream_add(hipStream_t s, int device, const std::string &label) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  g_streams[s] = StreamInfo{device, label, "(nothing queued yet)"};
}
void stream_remove(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  g_streams.erase(s);
}
void stream_mark(hipStream_t s, const char *what) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  auto it = g_streams.find(s);
  if (it != g_streams.end()) it->second.last = what;
}
hipError_t streams_sync() {
  std::vector<std::pair<hipStream_t, int>> all;
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    for (const auto &kv : g_streams) all.emplace_back(kv.first, kv.second.device);
  }
  int prev = 0;
  if (const hipError_t e = hipGetDevice(&prev)) return e;
  hipError_t first = hipSuccess;
  for (const auto &[s, dev] : all) {
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess && first == hipSuccess) first = e;
  }
  (void)hipSetDevice(prev);
  return first;
}
std::string stream_faults() {
  std::vector<std::pair<hipStream_t, StreamInfo>> all;
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    for (const auto &kv : g_streams) all.emplace_back(kv.first, kv.second);
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::string m;
  for (const auto &[s, info] : all) {
    if (hipSetDevice(info.device) != hipSuccess) continue;
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess || e == hipErrorNotReady) continue;
    m += (m.empty() ? "" : "; ") + info.label + " (device " + std::to_string(info.device) + ", last queued: " +
         info.last + "): " + hipGetErrorName(e);
  }
  (void)hipSetDevice(prev);
  (void)hipGetLastError();  // (the queries' errors are reported here, not left pending)
  return m.empty() ? std::string("; no librtamd stream reports an error (the fault came from work queued "
                                 "by this call itself or outside librtamd)")
                   : "; librtamd streams reporting errors: " + m;
}
std::string hip_fail(const char *expr, hipError_t e) {
  std::string m = std::string(expr) + ": " + hipGetErrorString(e);
  if (sticky(e)) m += stream_faults();
  return m;
}
}  // namespace rterr

// ------------------------------------------------ caller host memory (rtdma) --
namespace {
// Host ranges pinned through rt_host_pin (base -> bytes): rt_render writes a
// cleared frame's hits straight into such buffers, and rtdma DMAs them directly.
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pins;

// The process-wide bounce buffer of rtdma: two halves of kBounce bytes of
// pinned host memory (allocated on first use, kept for the process).
constexpr size_t kBounce = 8u << 20;
std::mutex g_bounce_mu;
char *g_bounce[2] = {nullptr, nullptr};

hipError_t bounce_ready() {
  for (char *&b : g_bounce)
    if (!b)
      if (const hipError_t e = hipHostMalloc((void **)&b, kBounce, hipHostMallocPortable)) {
        b = nullptr;
        return e;
      }
  return hipSuccess;
}
}  // namespace

namespace rtdma {
void *pinned_device_ptr(const void *p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  uintptr_t base = 0;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.upper_bound(a);
    if (it == g_pins.begin()) return nullptr;
    --it;
    if (a < it->first || a + bytes > it->first + it->second) return nullptr;
    base = it->first;
  }
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, (void *)base, 0) != hipSuccess || !d) {
    (void)hipGetLastError();  // (not mapped: take the staged path)
    return nullptr;
  }
  return (char *)d + (a - base);
}
bool pinned(const void *p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  auto it = g_pins.upper_bound(a);
  if (it == g_pins.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}
hipError_t h2d(void *d, const void *h, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (pinned(h, n)) {
    hipError_t e = hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
  }
  std::lock_guard<std::mutex> lk(g_bounce_mu);
  if (const hipError_t e = bounce_ready()) return e;
  // chunk k fills half k & 1 while the DMA of chunk k - 1 runs from the other
  for (size_t off = 0, k = 0; off < n; off += kBounce, ++k) {
    const size_t m = std::min(kBounce, n - off);
    if (k >= 2)
      if (const hipError_t e = hipStreamSynchronize(st)) return e;
    std::memcpy(g_bounce[k & 1], (const char *)h + off, m);
    if (const hipError_t e = hipMemcpyAsync((char *)d + off, g_bounce[k & 1], m, hipMemcpyHostToDevice, st)) {
      (void)hipStreamSynchronize(st);
      return e;
    }
  }
  return hipStreamSynchronize(st);
}
hipError_t d2h(void *h, const void *d, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (pinned(h, n)) {
    hipError_t e = hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
  }
  std::lock_guard<std::mutex> lk(g_bounce_mu);
  if (const hipError_t e = bounce_ready()) return e;
  // two chunks per round trip: both DMAs queued, then both copied out
  for (size_t off = 0; off < n; off += 2 * kBounce) {
    size_t m[2] = {0, 0};
    for (int k = 0; k < 2 && off + k * kBounce < n; ++k) {
      m[k] = std::min(kBounce, n - off - k * kBounce);
      if (const hipError_t e = hipMemcpyAsync(g_bounce[k], (const char *)d + off + k * kBounce, m[k],
                                              hipMemcpyDeviceToHost, st)) {
        (void)hipStreamSynchronize(st);
        return e;
      }
    }
    if (const hipError_t e = hipStreamSynchronize(st)) return e;
    for (int k = 0; k < 2; ++k)
      if (m[k]) std::memcpy((char *)h + off + k * kBounce, g_bounce[k], m[k]);
  }
  return hipSuccess;
}
}  // namespace rtdma

namespace {

inline int set_err(int code, const std::string &msg) { return rterr::set(code, msg); }

constexpr int kBlock = 256;  // 4 waves, 16x16 pixels
// Workgroup of the persistent multi-frame kernel (render_persist_kernel), in
// threads. Its waves are independent (each pulls its own items), so the block
// only sets the granularity at which a launch's resources are handed back:
// the next launch on the other stream gets a workgroup slot only when every
// wave of a finished workgroup has left. One wave per workgroup lets the next
// launch replace the draining one wave by wave (128 and
// 256, the block-dispatch size, are A/B settings).
#ifndef RT_PERSIST_BLOCK
#define RT_PERSIST_BLOCK 64
#endif
constexpr int kPBlock = RT_PERSIST_BLOCK;
static_assert(kPBlock % 64 == 0 && kPBlock >= 64 && kPBlock <= 1024, "persistent block: whole waves");
constexpr int kTile = 16;

struct FrameArgs {
  rt_render_params P;
  uint32_t *color;
  float *t;
  int32_t W, H;
  uint32_t flags;
  int32_t band_rows, rank, nranks, rows_local;
  const uint32_t *order;  // block -> tile schedule (NULL: blockIdx order)
  uint32_t *cost;         // per-tile cost of this frame (shader cycles, max over waves), or NULL
  // one-frame kernel: bounding box of the pixels a hit was stored to, as
  // (min x, -max x, min y, -max y) in buffer coordinates (four atomicMin
  // words, initialised to INT32_MAX), or NULL (rt_render's partial download).
  // With kFlagRowSpan in flags: per buffer row instead, the span of those
  // pixels as (min x, -max x), two such words per row (rt_render's zero-copy
  // cleared frames on pageable buffers: the host copies just these spans)
  int32_t *hit_box;
};

// ---------------------------------------------------------- scene adapters --
// kFields = LDS words per traversal frame (mesh: node, list|count, best t;
// octree: node, list|count; grid: none).
// occupancy floors (min_waves below), overridable for A/B builds
#ifndef RT_GRID_WAVES
#define RT_GRID_WAVES 1
#endif
#ifndef RT_OCT_WAVES
#define RT_OCT_WAVES 6
#endif
// mesh primary: a floor of 5 waves per SIMD (102 VGPRs). Built without the SLP
// vectorizer (Makefile) the persistent kernel takes 96 VGPRs and 36 B of
// scratch per lane at 5 waves, and is faster than at 4 (117 VGPRs, no
// scratch): bunny 8 x 2 0.0855 -> 0.0825, the 1.1 M-triangle stand-in 0.3314 ->
// 0.3149 ms/frame (profiles/r05/slp_ab.txt, two rounds). With SLP on, 5 waves
// were slower.
#ifndef RT_MESH_WAVES
#define RT_MESH_WAVES 5
#endif
// shading kernels (GENERAL, the reference's default mode): a floor of 4 waves
// per SIMD. The mesh's takes 135 VGPRs (3 waves) on its own; at 4 it gets 127
// and spills 12 B per lane, and is faster: bunny default mode 1080p, 8 frames
// x 2 / x 1 streams, 0.2267 -> 0.2068 / 0.2877 -> 0.2738 ms/frame (same box).
// 1 = the compiler's choice (A/B switch).
#ifndef RT_GENERAL_WAVES
#define RT_GENERAL_WAVES 4
#endif
struct MeshS {
  static constexpr int kFields = 3;
  static constexpr bool kCoop = true;  // primary rays: wave-cooperative tail (mesh_primary_wave)
  static constexpr int kMinWaves = RT_MESH_WAVES;
  static constexpr int kQueueGroup = 2;  // wave tiles per work-queue item (render_persist_kernel)
  static constexpr int kLdsNodes = RT_LDS_NODES;  // top-of-tree nodes per persistent block in LDS
  MeshDev d;
  // rays at or below which the wave hands its remaining rays to 8-lane groups
  // (wave-uniform; the persistent kernel raises it for a wave's last item)
  int coop_rays = kCoopRays;
  // traversal iterations after which a wave raises its priority (0: never;
  // the persistent kernel sets RT_HEAVY_PRIO, the one-frame kernel keeps 0)
  int prio_iters = 0;
  template <int B>
  __device__ __forceinline__ Hit primary(f3 o, f3 dir, float tn, float tf, bool active,
                                         uint32_t *stk) const {
    float t;
    uint32_t k;
    Hit h = miss_hit();
    if (mesh_primary_wave<B>(d, o, dir, tn, tf, active, stk, t, k, coop_rays, prio_iters) && active) {
      h.hit = true;
      h.t = t;
      h.n = tri_normal(d.tris, k);
      h.prim = (int64_t)d.tris[k].orig_id;
    }
    return h;
  }
  template <int B, class CT>
  __device__ __forceinline__ Hit intersect(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return mesh_intersect<B>(d, o, dir, tn, tf, st, cnt);
  }
  template <int B, class CT>
  __device__ __forceinline__ bool occluded(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return mesh_occluded<B>(d, o, dir, tn, tf, st, cnt);
  }
};
template <int kMode>
struct GridS {
  static constexpr int kFields = 1;  // no traversal stack (one unused LDS word per lane)
  static constexpr bool kCoop = false;
  static constexpr int kMinWaves = RT_GRID_WAVES;
  // block dispatch: a grid tile is too short for the queue's claims to pay
  // (256^3, 8 frames x 2 streams: 0.0506 ms/frame vs 0.0541 at 4 tiles per claim)
  static constexpr int kQueueGroup = 0;
  static constexpr int kLdsNodes = 0;
  GridDev d;
  template <int B, class CT>
  __device__ __forceinline__ Hit intersect(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return grid_intersect<kMode>(d, o, dir, tn, tf, cnt);
  }
  template <int B, class CT>
  __device__ __forceinline__ bool occluded(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return grid_occluded<kMode>(d, o, dir, tn, tf, cnt);
  }
};
// PACK: the traversal carries the node coordinates packed in one register
// (OctXYZ; trees of depth <= 8, i.e. up to 7 stack slots)
template <bool PACK>
struct OctS {
  static constexpr int kFields = kOctFields;
  static constexpr bool kCoop = false;
  static constexpr int kMinWaves = RT_OCT_WAVES;
  static constexpr int kQueueGroup = 2;
  static constexpr int kLdsNodes = 0;
  OctDev d;
  template <int B, class CT>
  __device__ __forceinline__ Hit intersect(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return oct_intersect<B, PACK>(d, o, dir, tn, tf, st, cnt);
  }
  template <int B, class CT>
  __device__ __forceinline__ bool occluded(f3 o, f3 dir, float tn, float tf,
                                           LdsStack<B, kFields> st, CT &cnt) const {
    return oct_occluded<B, PACK>(d, o, dir, tn, tf, st, cnt);
  }
};

// SceneUnion(scene, plane)::intersect (raytracing.hpp:87-93): both are
// intersected, the smaller t wins, ties go to the plane.
struct SurfHit {
  Hit h;
  float albedo;   // grey albedo: mesh/SDF 1.0, plane checker 0.0 / 1.0
  float refl;     // reflectiveness: plane 0.3, else 0
};
template <class S, int B, class CT>
__device__ __forceinline__ SurfHit union_intersect(const S &sc, const PlaneDev &pl, f3 o, f3 d,
                                                   float tn, float tf, LdsStack<B, S::kFields> st, CT &cnt) {
  cnt.add(C_RAYS, 1);
  SurfHit r{sc.template intersect<B>(o, d, tn, tf, st, cnt), 1.0f, 0.0f};
  if (pl.on) {
    float tp = kInf, ap = 1.0f;
    const bool ph = plane_hit(pl, o, d, tn, tf, tp, ap);
    if (!(r.h.t < (ph ? tp : kInf))) {
      if (ph) {
        r.h = Hit{true, tp, pl.n, -2};
        r.albedo = ap;
        r.refl = 0.3f;
      } else {
        r.h = miss_hit();
        r.albedo = 1.0f;
        r.refl = 0.0f;
      }
    }
  }
  return r;
}
// Shadow query: HitInfo::hitten of the union is the OR of both hitten flags.
template <class S, int B, class CT>
__device__ __forceinline__ bool union_occluded(const S &sc, const PlaneDev &pl, f3 o, f3 d, float tn,
                                               float tf, LdsStack<B, S::kFields> st, CT &cnt) {
  cnt.add(C_RAYS, 1);
  if (sc.template occluded<B>(o, d, tn, tf, st, cnt)) return true;
  if (pl.on) {
    float tp, ap;
    return plane_hit(pl, o, d, tn, tf, tp, ap);
  }
  return false;
}

// Renderer::intersectionColor (raytracing.cpp:13-65) for one ray; the one
// reflection bounce (maxDepth 2 -> 1) is expanded in place, no recursion.
template <class S, int B, class CT>
__device__ __forceinline__ f4 lambert_color(const S &sc, const PlaneDev &pl,
                                            const rt_render_params &P, f3 o, f3 d,
                                            const SurfHit &sh, f3 n, LdsStack<B, S::kFields> st, CT &cnt) {
  bool visible = true;
  const f3 point = o + sh.h.t * d;
  const f3 L{P.light_pos[0], P.light_pos[1], P.light_pos[2]};
  if (P.enable_shadows) {
    const f3 sd = normalize(L - point);
    visible = !union_occluded<S, B>(sc, pl, point + 0.3f * sd, sd, 0.01f, 100.0f, st, cnt);
  }
  const float a = sh.albedo;
  if (!visible) return f4{a * 0.1f, a * 0.1f, a * 0.1f, 1.0f};
  const f3 ld = normalize(point - L);
  const float lam = std_max(dot(-ld, n), 0.0f);  // Lambert (raytracing.cpp:8-11)
  const f3 c = f3{a * 0.1f, a * 0.1f, a * 0.1f} + lam * f3{a, a, a};
  return f4{std_min(c.x, 1.0f), std_min(c.y, 1.0f), std_min(c.z, 1.0f), 1.0f};
}

template <class S, int B, class CT>
__device__ __forceinline__ f4 shade_one(const S &sc, const PlaneDev &pl, const rt_render_params &P,
                                        f3 o, f3 d, float tFarEff, bool allow_refl, bool &hit,
                                        float &t_out, LdsStack<B, S::kFields> st, int64_t *prim, CT &cnt) {
  const SurfHit sh = union_intersect<S, B>(sc, pl, o, d, 0.01f, tFarEff, st, cnt);
  if (prim) *prim = sh.h.hit ? sh.h.prim : -1;
  if (!sh.h.hit) {
    hit = false;
    t_out = kInf;
    return f4{0.0f, 0.0f, 0.0f, 1.0f};
  }
  hit = true;
  t_out = sh.h.t;
  f3 n = sh.h.n;
  if (dot(n, d) > 0) n = n * -1.0f;
  f4 c;
  if (P.shading_mode == RT_SHADING_NORMAL) {
    c = f4{(n.x + 1.0f) / 2.0f, (n.y + 1.0f) / 2.0f, (n.z + 1.0f) / 2.0f, (1.0f + 1.0f) / 2.0f};
  } else if (P.shading_mode == RT_SHADING_COLOR) {
    c = f4{sh.albedo, sh.albedo, sh.albedo, 1.0f};
  } else {
    c = lambert_color<S, B>(sc, pl, P, o, d, sh, n, st, cnt);
    if (allow_refl && P.enable_reflections && sh.refl > 0.0f) {
      const float dn = dot(d, n);
      const f3 R = normalize(n * dn * (-2.0f) + d);  // LiteMath reflect(dir, normal)
      const f3 point = o + sh.h.t * d;
      // recursive call with maxDepth 1, tPrev = +inf (raytracing.cpp:51-61)
      const SurfHit rh = union_intersect<S, B>(sc, pl, point + 0.02f * R, R, 0.01f, 100.0f, st, cnt);
      f4 rc{0.0f, 0.0f, 0.0f, 1.0f};
      if (rh.h.hit) {
        f3 rn = rh.h.n;
        if (dot(rn, R) > 0) rn = rn * -1.0f;
        rc = lambert_color<S, B>(sc, pl, P, point + 0.02f * R, R, rh, rn, st, cnt);
      }
      const float r = sh.refl, k = 1.0f - sh.refl;
      c = f4{c.x * k + r * rc.x, c.y * k + r * rc.y, c.z * k + r * rc.z, c.w * k + r * rc.w};
    }
  }
  return c;
}

// Framebuffer stores. The frame (8 B/pixel, 16.6 MB at 1080p) is written once
// and never re-read by the kernel; plain stores keep every written line in the
// XCD's 4 MiB L2 and push scene data out. Agent-scope relaxed atomic stores
// lower to `global_store ... sc1`, which the MI355X L2 drops after writing.
// A peer's frame mapped over xGMI (RT_FLAG_TILE_NATURAL, the row-split p2p
// exchange) takes system-scope stores: they write through this GPU's L2 to the
// owner's memory whatever caching the IPC mapping got, so the kernel's
// completion (before the stream-ordered RCCL signal) covers them.
template <class T>
__device__ __forceinline__ void fb_store(T *p, T v, bool peer) {
  if (peer) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Peer frames (RT_FLAG_TILE_NATURAL, the row-split p2p exchange): a system-
// scope release after the wave's last peer store. The stores above are relaxed;
// the fence waits for them to complete and makes them visible at system scope
// before the wave ends, so the RCCL completion signal the host enqueues after
// this kernel on the same stream cannot overtake them over xGMI, whatever the
// end-of-kernel release of the dispatch covers. Once per wave (A/B switch
// RT_PEER_RELEASE=0 drops it).
#ifndef RT_PEER_RELEASE
#define RT_PEER_RELEASE 1
#endif
// (A frame in HOST memory -- rt_render's zero-copy cleared frames -- takes the
// device frame's stores: the dispatch's end-of-kernel system-scope release,
// before rt_render's stream synchronisation, makes them visible to the host.
// A per-wave system-scope fence there costs an L2 write-back per wave: the
// one-frame kernel's 32 k waves took the frame from 0.19 to ~0.38 ms.)
constexpr uint32_t kSysStoreFlags = RT_FLAG_TILE_NATURAL;
// Internal flag (never passed through the C ABI; fill_frame rejects it): the
// frame lives in host memory (rt_render's zero-copy cleared frames) and takes
// system-scope stores, which write through this GPU's L2, with no per-wave
// fence. Agent-scope stores leave the lines dirty in L2 for the end-of-kernel
// release to write back over PCIe after the last wave; RTAMD_HOST_STORES=agent
// keeps those (A/B switch).
constexpr uint32_t kFlagHostFrame = 1u << 30;
// Internal flag: FrameArgs::hit_box holds per-row spans (see FrameArgs).
constexpr uint32_t kFlagRowSpan = 1u << 29;
// Internal flag: the frame's eye rays take eye_ray_fast (fill_frame sets it
// when fast_eye_ok holds for its projection and size).
constexpr uint32_t kFlagFastEye = 1u << 28;
// Internal flag: a row-band tile's rows are stored at their own rows of a full
// W x H frame (as RT_FLAG_TILE_NATURAL) but with the frame's plain stores and
// no peer fence: rt_multi_render's zero-copy slots, whose frame is one host
// frame shared by every slot (the kernels' end-of-dispatch release before the
// host's stream synchronisation covers their stores, as for rt_render's).
constexpr uint32_t kFlagNatural = 1u << 27;
__device__ __forceinline__ void peer_release(uint32_t flags) {
#if RT_PEER_RELEASE
  if (flags & kSysStoreFlags) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#endif
}

__device__ __forceinline__ int image_row(int yl, const FrameArgs &fa) {
  if (fa.nranks <= 1) return yl;
  // unsigned (yl, band_rows > 0): no sign fix-ups around the division
  const uint32_t br = (uint32_t)fa.band_rows, k = (uint32_t)yl / br, r = (uint32_t)yl - k * br;
  return (int)((k * (uint32_t)fa.nranks + (uint32_t)fa.rank) * br + r);
}

// Renderer::draw (raytracing.cpp:67-102). GENERAL=false is the primary-ray
// path (Normal shading, no plane, no secondary rays) used by the headline
// benchmark; GENERAL=true runs intersectionColor in full.
// DIAG selects diagnostic variants of the same kernel (the timed kernels use 0):
//   1: accumulate the work counters (algorithmic-bytes model) into diag[C_NUM];
//   2: per-wave timestamps: diag[4*w .. 4*w+3] = start, end (s_memrealtime,
//      100 MHz), (sum << 32 | max) over lanes of work units, XCC_ID register;
//      w = linear block * 4 + wave.
template <int DIAG>
struct CntSel { using T = NoCnt; };
template <>
struct CntSel<1> { using T = LaneCnt; };
template <>
struct CntSel<2> { using T = LaneCnt; };

__device__ __forceinline__ void flush_counts(NoCnt &, unsigned long long *) {}
__device__ __forceinline__ void flush_counts(LaneCnt &c, unsigned long long *out) {
#pragma unroll
  for (int i = 0; i < C_NUM; ++i) {
    unsigned long long v = c.v[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(out + i, v);
  }
}

// Block -> tile map: plain 2-D dispatch (tiles dealt round-robin over the 8
// XCDs in blockIdx order). Measured and rejected: one contiguous band of tiles
// per XCD (GEMM-style XCD swizzle: the XCD owning the model's band becomes the
// tail; bunny 0.356 -> 0.378 ms, octree 4K default 1.72 -> 2.30 ms) and a
// centre-out order that dispatches the model tiles first (octree 4K primary
// 1.15 -> 1.29 ms: the heavy tiles then compete for the same CUs at once).

// Diagnostic switch (never in a shipping build): 1 drops the stores into host
// frames, 2 keeps only their colour stores, to time what the traversal costs
// without them
#ifndef RT_DIAG_HOST_NOSTORE
#define RT_DIAG_HOST_NOSTORE 0
#endif

// Host-frame pair flush (one-frame kernel, 16x16 tiles of 4 waves). The
// stores of a cleared frame in host memory (rt_render's and rt_multi_render's
// zero-copy frames) cross the host link, where their number, not their bytes,
// is what costs: an 8x8 wave tile's rows are 32-byte pieces, and the stores
// were 45-95 us of the one-frame kernel's ~0.19 ms (dropping only the t
// stores took ~3/4 of that, profiles/r06/dropin_host_store_cost.txt). The two
// waves side by side in a tile (one 16-pixel row band of 8 rows) therefore
// leave their pixels in LDS -- a miss as the cleared frame's words, which the
// host frame already holds -- and the second of the two to finish writes the
// band's 8 rows of colour and t as 64-byte pieces (one 16-byte store per
// lane), or nothing when neither wave stored a hit. Taken for whole bands
// inside the frame with 16-byte aligned rows (W % 4 == 0, aligned buffers);
// other bands store per pixel as before. RT_PAIR_FLUSH=0: off (A/B switch).
#ifndef RT_PAIR_FLUSH
#define RT_PAIR_FLUSH 1
#endif
constexpr int kPairWords = 2 * 8 * 16;  // per buffer: 2 bands x 8 rows x 16 pixels

// One pixel per lane of the wave's 8x8 tile: column xo, rank-local row yl.
// Returns true iff this lane stored a hit (its pixel differs from a cleared
// frame's or from tPrev).
// defer (host-frame pair flush, render_body): this lane's colour and t words
// go to defer[0] and defer[kPairWords] in LDS instead of the frame
template <class S, int SLOTS, bool GENERAL, int DIAG, int B = kBlock, class CT>
__device__ __forceinline__ bool render_pixels(const S &sc, const PlaneDev &pl, const FrameArgs &fa,
                                              CT &cnt, uint32_t *stk, int xo, int yl,
                                              uint32_t *defer = nullptr) {
  const bool active = xo < fa.W && yl < fa.rows_local;
  // wave-cooperative primary path: every lane of the wave takes part
  constexpr bool kWaveCoop = DIAG == 0 && !GENERAL && S::kCoop;
  if (DIAG == 0 && !kWaveCoop && !active) return false;
  if (active || kWaveCoop) {  // (the counting variant keeps every lane for its wave reduction)
    LdsStack<B, S::kFields> st{stk + threadIdx.x};
    const int yo = image_row(active ? yl : 0, fa);
    const int y = fa.H - yo - 1;  // loop row y is stored to image row H-y-1 (raytracing.cpp:82)
    const f3 o{fa.P.camera_pos[0], fa.P.camera_pos[1], fa.P.camera_pos[2]};
    f3 d;
    if (fa.flags & kFlagFastEye)
      d = eye_ray_fast(active ? xo : 0, y, fa.W, fa.H, fa.P.proj_inv, fa.P.view_inv);
    else
      d = eye_ray(active ? xo : 0, y, fa.W, fa.H, fa.P.proj_inv, fa.P.view_inv);
    // packed band layout (rank-local row yl) or, with RT_FLAG_TILE_NATURAL, the
    // full frame's own row (a peer's frame mapped over xGMI)
    const bool natural = (fa.flags & (kSysStoreFlags | kFlagNatural)) != 0;
    const bool sys = (fa.flags & (kSysStoreFlags | kFlagHostFrame)) != 0;
    const int yb = natural ? yo : yl;
    // 32-bit pixel index (check_params caps W*H at 2^31): one register live
    // across the traversal instead of two
    const uint32_t idx = active ? (uint32_t)yb * (uint32_t)fa.W + (uint32_t)xo : 0u;
    const bool clear = (fa.flags & RT_FLAG_CLEAR) != 0;
    const bool hits_only = (fa.flags & RT_FLAG_HITS_ONLY) != 0;
    const float tPrev = (clear || !active) ? kInf : fa.t[idx];
    const float tFarEff = std_min(100.0f, tPrev);  // std::min(tFar, tPrev)
    bool hit;
    float t;
    f4 c;
    if (!GENERAL) {
      cnt.add(C_RAYS, 1);
      Hit h;
      if constexpr (kWaveCoop)
        h = sc.template primary<B>(o, d, 0.01f, tFarEff, active, stk);
      else
        h = sc.template intersect<B>(o, d, 0.01f, tFarEff, st, cnt);
      hit = h.hit;
      t = h.t;
      f3 n = h.n;
      if (dot(n, d) > 0) n = n * -1.0f;
      c = f4{(n.x + 1.0f) / 2.0f, (n.y + 1.0f) / 2.0f, (n.z + 1.0f) / 2.0f, (1.0f + 1.0f) / 2.0f};
    } else {
      c = shade_one<S, B>(sc, pl, fa.P, o, d, tFarEff, true, hit, t, st, nullptr, cnt);
    }
    // the reference stores only when !isinf(tNew) (raytracing.cpp:91-94)
    const bool store = hit && !__builtin_isinf(t);
    if (defer) {
      // a cleared host frame's pixel, hit or not: the pair flush writes whole
      // rows (a miss's words are the cleared frame's own)
      defer[0] = store ? pack_rgba(c) : 0u;
      defer[kPairWords] = __float_as_uint(store ? t : kInf);
    } else if (RT_DIAG_HOST_NOSTORE == 1 && (fa.flags & kFlagHostFrame)) {
      // diagnostic build only: a host frame's stores dropped (wrong output)
    } else if (RT_DIAG_HOST_NOSTORE == 2 && (fa.flags & kFlagHostFrame)) {
      if (active && store) fb_store(fa.color + idx, pack_rgba(c), sys);  // (colour only)
    } else if (!active) {
      // helper lane of the cooperative path: no pixel of its own
    } else if (clear && !hits_only) {
      fb_store(fa.color + idx, store ? pack_rgba(c) : 0u, sys);
      fb_store(fa.t + idx, store ? t : kInf, sys);
    } else if (store) {
      fb_store(fa.color + idx, pack_rgba(c), sys);
      fb_store(fa.t + idx, t, sys);
    }
    return active && store;
  }
  return false;
}

// 16 bytes into a host frame, written through to memory at system scope (the
// 16-byte form of fb_store's system-scope relaxed store: global_store ... sc0 sc1)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void host_store16(uint32_t *p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

// hf: the pair-flush LDS (render_kernel; nullptr elsewhere): kPairWords colour
// words, kPairWords t words, then one arrival counter per band (zeroed by the
// kernel before any wave gets here)
template <class S, int SLOTS, bool GENERAL, int DIAG, int BT = kBlock>
__device__ __forceinline__ void render_body(const S &sc, const PlaneDev &pl, const FrameArgs &fa,
                                            unsigned long long *counters, uint32_t *stk,
                                            uint32_t *hf = nullptr) {
  typename CntSel<DIAG>::T cnt{};
  unsigned long long t_start = 0;
  if (DIAG == 2) t_start = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t bx = blockIdx.x, by = blockIdx.y;
  if (DIAG == 0 && fa.order) {  // cost-ordered schedule: this block renders tile order[b]
    const uint32_t tl = fa.order[blockIdx.y * gridDim.x + blockIdx.x];
    bx = tl % gridDim.x;
    by = tl / gridDim.x;
  }
  const uint64_t c0 = (DIAG == 0 && fa.cost) ? __builtin_amdgcn_s_memtime() : 0;
  const int xo = BT == 64 ? (int)bx * 8 + (lane & 7) : (int)bx * kTile + (wave & 1) * 8 + (lane & 7);
  const int yl = BT == 64 ? (int)by * 8 + (lane >> 3) : (int)by * kTile + (wave >> 1) * 8 + (lane >> 3);
  // host-frame pair flush: this wave's band of 8 rows x 16 pixels lies inside
  // the frame and its rows are 16-byte aligned (wave-uniform; the same for
  // both waves of the band)
  const int band = wave >> 1;
  const bool flush = RT_PAIR_FLUSH && DIAG == 0 && BT == kBlock && hf != nullptr &&
                     (fa.flags & kFlagHostFrame) && (fa.flags & RT_FLAG_CLEAR) && (fa.flags & RT_FLAG_HITS_ONLY) &&
                     (fa.W & 3) == 0 && (((uintptr_t)fa.color | (uintptr_t)fa.t) & 15u) == 0 &&
                     (int)bx * kTile + kTile <= fa.W && (int)by * kTile + band * 8 + 8 <= fa.rows_local;
  uint32_t *slot = flush ? hf + band * 128 + (lane >> 3) * 16 + (wave & 1) * 8 + (lane & 7) : nullptr;
  const bool stored = render_pixels<S, SLOTS, GENERAL, DIAG, BT>(sc, pl, fa, cnt, stk, xo, yl, slot);
  if (flush) {
    const uint32_t any = __ballot(stored) != 0 ? 1u : 0u;
    // this wave's LDS words are written before its arrival is counted, and the
    // band's second wave reads them only after counting its own
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(hf + 2 * kPairWords + band, 1u | (any << 16));
    old = __builtin_amdgcn_readfirstlane(old);
    if ((old & 0xFFFFu) == 1u && (any | (old >> 16)) != 0u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      // lanes 0-31 write the colour rows, 32-63 the t rows: row r, 4 pixels at 4 ch
      const int b = lane >> 5, r = (lane & 31) >> 2, ch = lane & 3;
      const u32x4 v = *reinterpret_cast<const u32x4 *>(hf + b * kPairWords + band * 128 + r * 16 + ch * 4);
      const int ylr = (int)by * kTile + band * 8 + r;
      const bool natural = (fa.flags & (kSysStoreFlags | kFlagNatural)) != 0;
      const uint32_t row = (uint32_t)(natural ? image_row(ylr, fa) : ylr);
      uint32_t *base = b ? reinterpret_cast<uint32_t *>(fa.t) : fa.color;
      host_store16(base + row * (uint32_t)fa.W + (uint32_t)bx * kTile + (uint32_t)ch * 4u, v);
    }
  }
  if constexpr (DIAG == 0) {
    if (fa.hit_box && !(fa.flags & kFlagRowSpan) && __ballot(stored)) {  // this wave's stored pixels into the frame's hit box
      int32_t v[4] = {stored ? xo : INT32_MAX, stored ? -xo : INT32_MAX, stored ? yl : INT32_MAX,
                      stored ? -yl : INT32_MAX};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const int32_t o = __shfl_xor(v[i], off, 64);
          v[i] = o < v[i] ? o : v[i];
        }
      // one lane, and only the words this wave improves: ~30 k waves' atomics
      // on one cache line would queue behind each other at the L2
      if (lane == __ffsll((unsigned long long)__ballot(1)) - 1)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (v[i] < __hip_atomic_load(fa.hit_box + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(fa.hit_box + i, v[i]);
    }
    if (fa.hit_box && (fa.flags & kFlagRowSpan) && __ballot(stored)) {  // per row of the tile: its stored pixels' span
      int32_t lo = stored ? xo : INT32_MAX, nhi = stored ? -xo : INT32_MAX;
#pragma unroll
      for (int off = 1; off < 8; off <<= 1) {  // the 8 lanes of one tile row
        const int32_t a = __shfl_xor(lo, off, 64), b = __shfl_xor(nhi, off, 64);
        lo = a < lo ? a : lo;
        nhi = b < nhi ? b : nhi;
      }
      if ((lane & 7) == 0 && lo != INT32_MAX) {
        int32_t *sp = fa.hit_box + 2 * yl;
        if (lo < __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(sp, lo);
        if (nhi < __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(sp + 1, nhi);
      }
    }
  }
  if constexpr (DIAG == 0) {
    if (fa.cost) {  // this wave's duration; the tile keeps its slowest wave's
      const uint64_t dt = __builtin_amdgcn_s_memtime() - c0;
      if (lane == __ffsll((unsigned long long)__ballot(1)) - 1)
        atomicMax(fa.cost + by * gridDim.x + bx, dt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)dt);
    }
  }
  if constexpr (DIAG == 1) flush_counts(cnt, counters);
  if constexpr (DIAG == 2) {
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    // this lane's sequential work units (node/leaf visits, tests, steps, sdf evals)
    uint32_t units = 0;
#pragma unroll
    for (int i = 0; i < C_RAYS; ++i) units += cnt.v[i];
    uint32_t mx = units, sm = units;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t om = __shfl_xor(mx, off, 64), os = __shfl_xor(sm, off, 64);
      mx = mx > om ? mx : om;
      sm += os;
    }
    // the 9th-largest lane's units: the work the wave does with more than 8 lanes busy
    uint32_t rest = units, u9 = 0;
    for (int r = 0; r < 9; ++r) {
      uint32_t m = rest;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const uint32_t om = __shfl_xor(m, off, 64);
        m = m > om ? m : om;
      }
      u9 = m;
      const uint64_t who = __ballot(rest == m);
      if ((threadIdx.x & 63) == (int)__builtin_ctzll(who)) rest = 0;
    }
    if ((threadIdx.x & 63) == 0) {
      const size_t w = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
      counters[4 * w] = t_start;
      counters[4 * w + 1] = t_end;
      counters[4 * w + 2] = ((unsigned long long)sm << 32) | mx;
      // HW_REG_XCC_ID (4 bits) | 9th-largest lane units << 8
      counters[4 * w + 3] = __builtin_amdgcn_s_getreg(0x1814) | ((unsigned long long)u9 << 8);
    }
  }
}

// Occupancy floor of the primary-ray kernels (waves per SIMD; 1 = the
// compiler's choice). The octree primary kernel is register-limited to 5 waves
// and gains ~5 % at 6 (a few spilled words outside the traversal loop); more
// (8) or the same on the grid (64 VGPRs, spills in the march) lose 5-25 %.
// Trees deeper than 7 slots are LDS-limited anyway.
template <class S, int SLOTS, bool GENERAL, int DIAG>
constexpr int min_waves() {
  return (DIAG != 0 || SLOTS > 7) ? 1 : GENERAL ? RT_GENERAL_WAVES : S::kMinWaves;
}

// Workgroup of the one-frame kernel (render_kernel, DIAG == 0): 64 = one 8x8
// wave tile per workgroup (the cost-ordered schedule then orders 8x8 tiles),
// 256 = 16x16 tiles of 4 waves (A/B switch). The counting and stamping
// variants (DIAG 1, 2) keep 16x16 tiles.
#ifndef RT_FRAME_BLOCK
#define RT_FRAME_BLOCK 256
#endif
constexpr int kFBlock = RT_FRAME_BLOCK;
constexpr int kFTile = kFBlock == 64 ? 8 : kTile;
static_assert(kFBlock == 64 || kFBlock == kBlock, "one-frame workgroup: one wave or the 16x16 tile");
template <int DIAG>
constexpr int frame_block() { return DIAG == 0 ? kFBlock : kBlock; }
template <int DIAG>
constexpr int frame_tile() { return DIAG == 0 ? kFTile : kTile; }

// one-frame kernel, mesh primary rays: wave priority after this many traversal
// iterations and the cooperative tail's ray threshold (A/B switches; the
// persistent kernel's are RT_HEAVY_PRIO and its own)
#ifndef RT_FRAME_PRIO
#define RT_FRAME_PRIO 0
#endif
#ifndef RT_FRAME_COOP
#define RT_FRAME_COOP RT_COOP_RAYS
#endif
template <class S, int SLOTS, bool GENERAL, int DIAG>
__global__ __launch_bounds__(frame_block<DIAG>()) __attribute__((amdgpu_waves_per_eu(min_waves<S, SLOTS, GENERAL, DIAG>())))
void render_kernel(S sc_arg, PlaneDev pl, FrameArgs fa,
                                                        unsigned long long *counters) {
  __shared__ uint32_t stk[SLOTS * S::kFields * frame_block<DIAG>()];
  constexpr bool kPair = RT_PAIR_FLUSH && DIAG == 0 && frame_block<DIAG>() == kBlock;
  __shared__ __attribute__((aligned(16))) uint32_t hf[kPair ? 2 * kPairWords + 4 : 4];
  S sc = sc_arg;
  if constexpr (S::kCoop && !GENERAL && DIAG == 0) {
    sc.prio_iters = RT_FRAME_PRIO;
    sc.coop_rays = RT_FRAME_COOP;
  }
  // (grid-uniform condition: every wave of the block passes the barrier or none)
  if (kPair && (fa.flags & kFlagHostFrame) && (fa.flags & RT_FLAG_CLEAR) && (fa.flags & RT_FLAG_HITS_ONLY)) {
    if (threadIdx.x < 2) hf[2 * kPairWords + threadIdx.x] = 0u;
    __syncthreads();
  }
  render_body<S, SLOTS, GENERAL, DIAG, frame_block<DIAG>()>(sc, pl, fa, counters, stk, kPair ? hf : nullptr);
  peer_release(fa.flags);
}

// Several frames in one launch: blockIdx.z selects the frame. The tiles of
// frame z+1 fill the CUs while frame z's last tiles (grazing rays at the
// silhouette, the per-frame tail) finish, so only the batch's last frame
// leaves a tail. The per-frame arguments travel in the kernarg segment
// (uniform blockIdx.z index: scalar loads).
// At most 16 frames per launch (3.7 KiB of kernel arguments): row-band ranks
// of a multi-GPU split render 1/N of each frame, so they take 16 frames per
// launch to keep a launch's bulk long against its tail (bench.py --group;
// rank compute at N = 8: 0.0170 -> 0.0133 ms/frame); whole frames stay at 8.
#ifndef RT_MAX_BATCH
#define RT_MAX_BATCH 16
#endif
constexpr int kMaxBatch = RT_MAX_BATCH;
struct FrameBatch {
  FrameArgs f[kMaxBatch];
};
// the whole batch travels in the kernarg segment next to the scene, plane and queue words
static_assert(sizeof(FrameBatch) + 256 <= 4096, "FrameBatch exceeds the 4 KiB kernel-argument budget");

// Workgroup of the multi-frame block dispatch (render_batch_kernel; grids and
// the small row bands of N >= 4 ranks): one 8x8 wave tile per workgroup, so a
// finished wave frees its slot for the next tile at once instead of waiting for
// the slowest wave of a 16x16 tile (256^3 grid 0.0542 -> 0.0512, bunny rank
// bands at N = 4 0.0305 -> 0.0269 ms/frame). 256 = the
// 16x16 tile of 4 waves (A/B switch).
#ifndef RT_BATCH_BLOCK
#define RT_BATCH_BLOCK 64
#endif
constexpr int kBBlock = RT_BATCH_BLOCK;
// Multi-frame block dispatch, block b -> tile b / n of frame b % n: the
// batch's frames advance together, so the last blocks dispatched are every
// frame's last rows instead of the whole last frame (256^3 grid one stream
// 0.0537 / 0.0523 -> 0.0510 / 0.0501 ms/frame, two streams ~1 %; row bands
// level). 0: frame after frame (A/B switch).
#ifndef RT_BATCH_INTERLEAVE
#define RT_BATCH_INTERLEAVE 1
#endif
constexpr int kBTile = kBBlock == 64 ? 8 : kTile;
static_assert(kBBlock == 64 || kBBlock == kBlock, "batch workgroup: one wave or the 16x16 tile");

template <class S, int SLOTS, bool GENERAL>
__global__ __launch_bounds__(kBBlock) __attribute__((amdgpu_waves_per_eu(min_waves<S, SLOTS, GENERAL, 0>())))
void render_batch_kernel(S sc, PlaneDev pl, FrameBatch fb) {
  __shared__ uint32_t stk[SLOTS * S::kFields * kBBlock];
  if constexpr (kBBlock == kBlock) {
    render_body<S, SLOTS, GENERAL, 0>(sc, pl, fb.f[blockIdx.z], nullptr, stk);
  } else {
    NoCnt cnt{};
    const int lane = threadIdx.x & 63;
#if RT_BATCH_INTERLEAVE
    const uint32_t n = gridDim.z, b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    // heavy-first tile order of row bands (fb.f[0].order, from the previous
    // launch's recorded tile costs on this stream; band_sched)
    const uint32_t f = b % n, tl = fb.f[0].order ? fb.f[0].order[b / n] : b / n;
    const uint32_t tx = tl % gridDim.x, ty = tl / gridDim.x;
#else
    const uint32_t f = blockIdx.z, tl = blockIdx.y * gridDim.x + blockIdx.x, tx = blockIdx.x, ty = blockIdx.y;
#endif
    const uint64_t c0 = fb.f[0].cost ? __builtin_amdgcn_s_memtime() : 0;
    render_pixels<S, SLOTS, GENERAL, 0, kBBlock>(sc, pl, fb.f[f], cnt, stk, (int)tx * 8 + (lane & 7),
                                                 (int)ty * 8 + (lane >> 3));
    if (fb.f[0].cost && lane == 0) {  // this tile's cost: the slowest of its frames' waves
      const uint64_t dc = __builtin_amdgcn_s_memtime() - c0;
      atomicMax(fb.f[0].cost + tl, (uint32_t)(dc < 0xFFFFFFFFull ? dc : 0xFFFFFFFFull));
    }
  }
  peer_release(fb.f[0].flags);
}

// Persistent form of render_batch_kernel: a grid of just the resident blocks;
// every wave pulls 8x8 pixel tiles (items) from a work queue until the batch
// is drained, so a wave whose tile finishes early takes the next one at once
// instead of waiting for the in-order workgroup dispatcher (which stalls
// behind a full SE while other SEs have free slots). The queue is sharded per
// XCD: item i belongs to head i % 8 (HW_REG_XCC_ID picks a wave's own head),
// a wave whose head is drained moves on to the other seven, so the batch
// completes whatever XCDs the grid lands on. The next item is claimed before
// the current one is traced (its atomic's latency hides under the traversal).
// The last wave out resets the heads for the next launch on the stream.
struct PersistQ {
  uint32_t *heads;   // 8 heads kHeadStride words apart; heads[8 * kHeadStride] = waves done
  uint32_t items;    // frames * per_frame
  uint32_t tiles_x, per_frame;  // items (groups of gx x gy wave tiles) per row / per frame
  uint32_t waves;    // waves in the grid
  uint32_t gx, gy;   // wave tiles (8x8 pixels) per item: 1x1, 2x1 or 2x2
  uint32_t stride;   // words between heads
  // item order of a head (render_persist_kernel): cpf == 0 interleaved (item
  // i on head i % 8); cpf > 0 banded: head h takes tile rows [h cpf, (h+1) cpf)
  // of the row-major items of every frame, frame after frame (nper = frames x
  // cpf slots, slots past per_frame are empty), so an XCD's L2 holds the part
  // of the scene its band of the image sees; a drained head steals as before
  uint32_t cpf, nper;
  // diagnostic builds (-DRT_PERSIST_STAMPS, tools/build_variant.sh; see
  // rtx_set_persist_stamps): per wave w = blockIdx.x * (kPBlock / 64) + wave, 8 x u64 =
  // start, end (s_memrealtime, 100 MHz), items traced | XCD << 32, end of its
  // last item, start of its last item, last item, longest item's duration, longest item
  unsigned long long *stamps;
};
// 4 KiB + 256 B apart: every head on its own memory channel's lines, so the
// memory-side atomics of different heads do not queue behind each other
// (RTAMD_QSTRIDE=<words> overrides it for A/B runs, at most kHeadStrideMax)
constexpr int kHeadStride = 1088;
constexpr int kHeadStrideMax = 4096;

__device__ __forceinline__ uint32_t q_claim(uint32_t *head) {
  uint32_t k = 0;
  if ((threadIdx.x & 63) == 0) k = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(k);
}

template <class S, int SLOTS, bool GENERAL>
__global__ __launch_bounds__(kPBlock) __attribute__((amdgpu_waves_per_eu(min_waves<S, SLOTS, GENERAL, 0>())))
void render_persist_kernel(S sc_arg, PlaneDev pl, FrameBatch fb, PersistQ q) {
  __shared__ uint32_t stk[SLOTS * S::kFields * kPBlock];
  S sc = sc_arg;
  if constexpr (S::kCoop && !GENERAL) sc.prio_iters = RT_HEAVY_PRIO;
  if constexpr (S::kLdsNodes > 0 && !GENERAL) {
    // the top BVH levels (the first inner nodes, BFS order) copied into this
    // block's LDS once per launch; every item's traversal reads them there
    constexpr int kQ = (int)(sizeof(rtl::GNode) / 16);
    __shared__ float4 lnodes[S::kLdsNodes * kQ];
    const uint32_t n = sc.d.n_inner < (uint32_t)S::kLdsNodes ? sc.d.n_inner : (uint32_t)S::kLdsNodes;
    const float4 *src = reinterpret_cast<const float4 *>(sc.d.nodes);
    for (uint32_t i = threadIdx.x; i < n * kQ; i += kPBlock) lnodes[i] = src[i];
    __syncthreads();
    sc.d.lnodes = reinterpret_cast<const rtl::GNode *>(lnodes);
    sc.d.n_lds = n;
  }
  const int lane = threadIdx.x & 63;
  const uint32_t xcc = __builtin_amdgcn_s_getreg(0x1814) & 7;  // HW_REG_XCC_ID: this wave's XCD
#ifdef RT_PERSIST_STAMPS
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_item = t_start, t_last = t_start, d_max = 0;
  uint32_t n_items = 0, last_item = 0, max_item = 0;
#endif
  uint32_t h = xcc;
  uint32_t k = q_claim(q.heads + h * q.stride);
  NoCnt cnt{};
  for (;;) {
    // slot k of head h -> item (frame f, row-major index r in the frame)
    uint32_t item, f, r;
    bool drained, empty = false;
    if (q.cpf == 0) {
      item = k * 8 + h;
      drained = item >= q.items;
      f = item / q.per_frame;
      r = item - f * q.per_frame;
    } else {
      drained = k >= q.nper;
      f = k / q.cpf;
      r = h * q.cpf + (k - f * q.cpf);
      empty = r >= q.per_frame;
      item = f * q.per_frame + r;
    }
    if (drained) {
      // head h drained: read all eight heads at once (lanes 0-7, one round
      // trip) and claim from a head that still has items, the first one after
      // this XCD's own; none left: done. A claim that loses the race to the
      // last item just comes back here.
      uint32_t v = 0xFFFFFFFFu;
      if (lane < 8) v = __hip_atomic_load(q.heads + lane * q.stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t cap = q.cpf ? q.nper : (q.items + 7u - (uint32_t)lane) / 8u;
      const uint64_t m = __ballot(lane < 8 && v < cap) & 0xFFull;
      if (m == 0) break;
      const uint32_t rot = (uint32_t)(((m >> (xcc + 1)) | (m << (7 - xcc))) & 0xFFull);  // bit i: head xcc+1+i
      h = (xcc + 1 + (uint32_t)__builtin_ctz(rot)) & 7u;
      k = q_claim(q.heads + h * q.stride);
      continue;
    }
    const uint32_t knext = q_claim(q.heads + h * q.stride);
    if (empty) {
      k = knext;
      continue;
    }
    const uint32_t ty = r / q.tiles_x, tx = r - ty * q.tiles_x;
#ifdef RT_PERSIST_STAMPS
    const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
#endif
    for (uint32_t j = 0; j < q.gy; ++j)
      for (uint32_t i = 0; i < q.gx; ++i) {
        // the frame index is made opaque per tile, so the frame's arguments
        // (two 4x4 matrices among them) are re-read from the kernarg segment by
        // each tile instead of being hoisted out of the tile loop and kept
        // live across the traversal
        uint32_t fo = f;
        asm volatile("" : "+s"(fo));
        render_pixels<S, SLOTS, GENERAL, 0, kPBlock>(sc, pl, fb.f[fo], cnt, stk, (int)((tx * q.gx + i) * 8) + (lane & 7),
                                            (int)((ty * q.gy + j) * 8) + (lane >> 3));
      }
#ifdef RT_PERSIST_STAMPS
    ++n_items;
    t_item = __builtin_amdgcn_s_memrealtime();
    t_last = t_begin;
    last_item = item;
    if (t_item - t_begin > d_max) {
      d_max = t_item - t_begin;
      max_item = item;
    }
#endif
    k = knext;
  }
#ifdef RT_PERSIST_STAMPS
  if (q.stamps && lane == 0) {
    const size_t w = (size_t)blockIdx.x * (kPBlock / 64) + (threadIdx.x >> 6);
    unsigned long long *o = q.stamps + 8 * w;
    o[0] = t_start;
    o[1] = __builtin_amdgcn_s_memrealtime();
    o[2] = n_items | ((unsigned long long)xcc << 32);
    o[3] = t_item;
    o[4] = t_last;
    o[5] = last_item;
    o[6] = d_max;
    o[7] = max_item;
  }
#endif
  peer_release(fb.f[0].flags);
  if (lane == 0) {
    uint32_t *done = q.heads + 8 * q.stride;
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == q.waves - 1) {
      // every wave has left its claim loop: no claim is in flight any more
      for (int i = 0; i < 8; ++i)
        __hip_atomic_store(q.heads + i * q.stride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- ray pump --
// render_pump_kernel: the persistent multi-frame kernel with wavefront
// active-ray compaction (north star: "ballot/prefix-sum active-ray compaction
// for the sphere-march and octree steps", replacing the 8-wide ISPC gangs of
// ray_pack.ispc:241-273 and the recursion of octree_raytracing.cpp:166-202).
// A wave does not own a fixed 8x8 tile: each lane owns ONE ray at a time, and
// the wave pulls pixels from a per-wave pixel stream (consecutive pixels of
// the work-queue items, 8x8 tiles in order, so a refill's rays are coherent).
// The traversal of every live lane runs until `refill_min` lanes have
// finished (__ballot of the lanes still in the loop); the wave then writes the
// finished lanes' pixels, hands each dead lane the next pixel of the stream
// (its rank in the dead-lane ballot, __mbcnt, is its offset in the stream) and
// resumes. Traversal state stays in the lane's registers and its own LDS stack
// column, so nothing moves. Once the queue is drained the remaining rays run
// to the end. Primary rays (Normal shading, no plane); every image is the
// same as render_kernel's, bit for bit.
struct PumpFrame {  // the per-frame arguments a lane needs, copied to LDS
  float o[3];
  float proj_inv[16];
  float view_inv[16];
  uint32_t *color;
  float *t;
};

// wave-uniform work-item stream over the sharded queue (render_persist_kernel's
// protocol): the ticket of the next item on head h is claimed one ahead
struct ItemStream {
  uint32_t h, k;
};
__device__ __forceinline__ uint32_t take_item(const PersistQ &q, ItemStream &s, uint32_t xcc, int lane) {
  for (;;) {
    const uint32_t item = s.k * 8 + s.h;
    if (item < q.items) {
      s.k = q_claim(q.heads + s.h * q.stride);
      return item;
    }
    uint32_t v = 0xFFFFFFFFu;
    if (lane < 8) v = __hip_atomic_load(q.heads + lane * q.stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t m = __ballot(lane < 8 && v < (q.items + 7u - (uint32_t)lane) / 8u) & 0xFFull;
    if (m == 0) return 0xFFFFFFFFu;
    const uint32_t rot = (uint32_t)(((m >> (xcc + 1)) | (m << (7 - xcc))) & 0xFFull);
    s.h = (xcc + 1 + (uint32_t)__builtin_ctz(rot)) & 7u;
    s.k = q_claim(q.heads + s.h * q.stride);
  }
}

struct OctP {
  using Ray = OctRay;
  static constexpr int kFields = kOctFields;
  static constexpr int kMinWaves = RT_OCT_WAVES;
  OctDev d;
  template <bool FAST>
  __device__ __forceinline__ int start(f3 o, f3 dir, f3 inv, float tf, Ray &R, float &t, f3 &n) const {
    NoCnt c;
    OctHitPt hp;
    const int s = oct_start<FAST>(d, o, dir, inv, 0.01f, tf, R, t, hp, c);
    if (s == RAY_HIT) n = oct_normal_at(d, hp, c);
    return s;
  }
  template <bool FAST>
  __device__ __forceinline__ int run(f3 o, f3 dir, f3 inv, float tf, LdsStack<kBlock, kOctFields> st, Ray &R, int limit,
                                     float &t, f3 &n) const {
    NoCnt c;
    OctHitPt hp;
    const int s = oct_run<kBlock, FAST, true, false>(d, o, dir, inv, 0.01f, tf, st, R, limit, t, hp, c);
    if (s == RAY_HIT) n = oct_normal_at(d, hp, c);
    return s;
  }
};

// the grid's sphere march on the pump (grid_start / grid_run): a lane's state
// is (t, p), so a refill costs an eye ray and a box entry
template <int kMode>
struct GridP {
  using Ray = GridRay;
  static constexpr int kFields = 1;  // no traversal stack (one unused LDS word per lane)
  static constexpr int kMinWaves = RT_GRID_WAVES;
  GridDev d;
  template <bool FAST>
  __device__ __forceinline__ int start(f3 o, f3 dir, f3 inv, float tf, Ray &R, float &, f3 &) const {
    return grid_start(o, dir, inv, 0.01f, tf, R);
  }
  template <bool FAST>
  __device__ __forceinline__ int run(f3 o, f3 dir, f3, float, LdsStack<kBlock, kFields>, Ray &R, int limit,
                                     float &t, f3 &n) const {
    NoCnt c;
    f3 hp;
    const int s = grid_run<kMode, true>(d, o, dir, R, limit, t, hp, c);
    if (s == RAY_HIT) n = grid_normal<kMode>(d, hp, c);
    return s;
  }
};

#ifndef RT_REFILL_MIN
#define RT_REFILL_MIN 16  // dead lanes that trigger a refill (RTAMD_REFILL overrides)
#endif

#ifndef RT_PUMP_WAVES
#define RT_PUMP_WAVES 0  // occupancy floor of the pump kernel: 0 = the scene's kMinWaves, 1 = the compiler's
#endif
template <class P, int SLOTS>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(SLOTS > 7 ? 1 : (RT_PUMP_WAVES ? RT_PUMP_WAVES : P::kMinWaves))))
void render_pump_kernel(P sc, FrameBatch fb, PersistQ q, int32_t nframes, int32_t refill_min) {
  __shared__ uint32_t stk[SLOTS * P::kFields * kBlock];
  __shared__ PumpFrame frames[kMaxBatch];
  if ((int)threadIdx.x < nframes) {
    const FrameArgs &fa = fb.f[threadIdx.x];
    PumpFrame &pf = frames[threadIdx.x];
    for (int i = 0; i < 3; ++i) pf.o[i] = fa.P.camera_pos[i];
    for (int i = 0; i < 16; ++i) {
      pf.proj_inv[i] = fa.P.proj_inv[i];
      pf.view_inv[i] = fa.P.view_inv[i];
    }
    pf.color = fa.color;
    pf.t = fa.t;
  }
  __syncthreads();
  const FrameArgs &F = fb.f[0];  // size, flags and tile are the same for every frame of a batch
  const int lane = threadIdx.x & 63;
  const uint32_t xcc = __builtin_amdgcn_s_getreg(0x1814) & 7;  // HW_REG_XCC_ID
  const bool clear = (F.flags & RT_FLAG_CLEAR) != 0, hits_only = (F.flags & RT_FLAG_HITS_ONLY) != 0;
  const bool peer = (F.flags & kSysStoreFlags) != 0;
  const uint32_t isz = 64u * q.gx * q.gy;  // pixels per item
  ItemStream is{xcc, q_claim(q.heads + xcc * q.stride)};
  uint32_t cur = take_item(q, is, xcc, lane), off = 0;
  LdsStack<kBlock, P::kFields> st{stk + threadIdx.x};
  typename P::Ray R;
  bool live = false, fast = true;
  uint32_t f = 0;
  uint32_t idx = 0;
  f3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f}, inv{kInf, kInf, 1.0f};
  float tfar = 100.0f;
  // Renderer::draw's store (raytracing.cpp:91-94) of a finished ray, Normal shading
  auto finish = [&](int status, float t, f3 n) {
    const bool hit = status == RAY_HIT;
    const bool store = hit && !__builtin_isinf(t);
    if (dot(n, d) > 0) n = n * -1.0f;
    const f4 c{(n.x + 1.0f) / 2.0f, (n.y + 1.0f) / 2.0f, (n.z + 1.0f) / 2.0f, (1.0f + 1.0f) / 2.0f};
    uint32_t *cp = frames[f].color + idx;
    float *tp = frames[f].t + idx;
    if (clear && !hits_only) {
      fb_store(cp, store ? pack_rgba(c) : 0u, peer);
      fb_store(tp, store ? t : kInf, peer);
    } else if (store) {
      fb_store(cp, pack_rgba(c), peer);
      fb_store(tp, t, peer);
    }
  };
  for (;;) {
    // refill: every dead lane takes the next pixel of the wave's stream
    while (cur != 0xFFFFFFFFu) {
      const uint64_t dead = __ballot(!live);
      const uint32_t ndead = (uint32_t)__popcll(dead);
      if ((int)ndead < refill_min) break;
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(dead >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)dead, 0u));
      const uint32_t nxt = (off + ndead >= isz) ? take_item(q, is, xcc, lane) : 0xFFFFFFFFu;
      // (frame, tile row, tile column) of the two items, wave-uniform (scalar divisions)
      const uint32_t fc = cur / q.per_frame, rc = cur - fc * q.per_frame;
      const uint32_t tyc = rc / q.tiles_x, txc = rc - tyc * q.tiles_x;
      uint32_t fn = 0, txn = 0, tyn = 0;
      if (nxt != 0xFFFFFFFFu) {
        fn = nxt / q.per_frame;
        const uint32_t rn = nxt - fn * q.per_frame;
        tyn = rn / q.tiles_x;
        txn = rn - tyn * q.tiles_x;
      }
      bool got = false;
      uint32_t p = 0, tx = 0, ty = 0;
      if (!live) {
        if (off + rank < isz) { got = true; p = off + rank; f = fc; tx = txc; ty = tyc; }
        else if (nxt != 0xFFFFFFFFu) { got = true; p = off + rank - isz; f = fn; tx = txn; ty = tyn; }
      }
      off += ndead;
      if (off >= isz) { cur = nxt; off -= isz; }
      if (got) {
        const uint32_t tile = p >> 6;
        const uint32_t ti = q.gx == 1 ? 0u : (tile & 1u), tj = q.gx == 1 ? tile : (tile >> 1);
        const int x = (int)((tx * q.gx + ti) * 8 + (p & 7u));
        const int yl = (int)((ty * q.gy + tj) * 8 + ((p >> 3) & 7u));
        if (x < F.W && yl < F.rows_local) {
          const int yo = image_row(yl, F);
          const PumpFrame &pf = frames[f];
          idx = (uint32_t)(peer ? yo : yl) * (uint32_t)F.W + (uint32_t)x;
          o = f3{pf.o[0], pf.o[1], pf.o[2]};
          d = eye_ray(x, F.H - yo - 1, F.W, F.H, pf.proj_inv, pf.view_inv);
          inv = f3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
          fast = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z);
          tfar = clear ? 100.0f : std_min(100.0f, pf.t[idx]);  // std::min(tFar, tPrev)
          float t = kInf;
          f3 n{0.0f, 1.0f, 0.0f};
          const int s = fast ? sc.template start<true>(o, d, inv, tfar, R, t, n)
                             : sc.template start<false>(o, d, inv, tfar, R, t, n);
          if (s == RAY_PENDING) live = true;
          else finish(s, t, n);
        }
      }
    }
    if (__ballot(live) == 0) {
      if (cur == 0xFFFFFFFFu) break;
      continue;
    }
    const int limit = cur == 0xFFFFFFFFu ? 0 : 64 - refill_min;
    float t = kInf;
    f3 n{0.0f, 1.0f, 0.0f};
    int s = RAY_PENDING;
    if (__ballot(live && !fast) == 0) {  // every live ray has finite 1/d: the fast slab form for all
      if (live) s = sc.template run<true>(o, d, inv, tfar, st, R, limit, t, n);
    } else {  // the exact ISPC form (the same bits for finite 1/d too)
      if (live) s = sc.template run<false>(o, d, inv, tfar, st, R, limit, t, n);
    }
    if (live && s != RAY_PENDING) {
      finish(s, t, n);
      live = false;
    }
  }
  peer_release(F.flags);
  if (lane == 0) {
    uint32_t *done = q.heads + 8 * q.stride;
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == q.waves - 1) {
      for (int i = 0; i < 8; ++i)
        __hip_atomic_store(q.heads + i * q.stride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <class S, int SLOTS>
__global__ __launch_bounds__(kBlock) void rays_kernel(S sc, PlaneDev pl, const float *o3,
                                                       const float *d3, int64_t n, float tn,
                                                       float tf, int32_t *hit, float *t,
                                                       float *nrm, int64_t *prim) {
  __shared__ uint32_t stk[SLOTS * S::kFields * kBlock];
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  LdsStack<kBlock, S::kFields> st{stk + threadIdx.x};
  const f3 o{o3[3 * i], o3[3 * i + 1], o3[3 * i + 2]};
  const f3 d{d3[3 * i], d3[3 * i + 1], d3[3 * i + 2]};
  NoCnt cnt;
  const SurfHit sh = union_intersect<S, kBlock>(sc, pl, o, d, tn, tf, st, cnt);
  hit[i] = sh.h.hit ? 1 : 0;
  t[i] = sh.h.t;
  nrm[3 * i] = sh.h.n.x;
  nrm[3 * i + 1] = sh.h.n.y;
  nrm[3 * i + 2] = sh.h.n.z;
  prim[i] = sh.h.hit ? sh.h.prim : -1;
}

// FrameBuffer::clear() (raytracing.hpp:16-19): 16 B per lane per buffer.
__global__ void clear_kernel(uint32_t *c, float *t, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    *reinterpret_cast<uint4 *>(c + i) = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<float4 *>(t + i) = make_float4(kInf, kInf, kInf, kInf);
  } else {
    for (int64_t j = i; j < n; ++j) {
      c[j] = 0u;
      t[j] = kInf;
    }
  }
}

// rt_render's hit box / row spans (n words) to their pinned, mapped host
// copy: system-scope stores, which the host reads after synchronising the
// stream (a kernel in stream order instead of a small DMA copy)
__global__ void box_out_kernel(const int32_t *d_box, int32_t *h_box, int n) {
  for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < n; i += (int)(gridDim.x * blockDim.x))
    __hip_atomic_store(h_box + i, d_box[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the staging frame's stored spans (the row spans of its last frame) cleared
// again, and the span words reset for the next frame: block y clears row y's
// span. A row without hits holds (INT32_MAX, INT32_MAX): it returns before
// any index is formed from them.
__global__ void clear_spans_kernel(uint32_t *c, float *t, int32_t *span, int32_t W) {
  const int32_t y = (int32_t)blockIdx.x, lo = span[2 * y], hi = -span[2 * y + 1];
  __syncthreads();  // (every thread has read the row's span)
  if (threadIdx.x == 0) {
    span[2 * y] = INT32_MAX;
    span[2 * y + 1] = INT32_MAX;
  }
  if (lo > hi || lo < 0 || hi >= W) return;
  for (int32_t x = lo + (int32_t)threadIdx.x; x <= hi; x += (int32_t)blockDim.x) {
    const size_t i = (size_t)y * (size_t)W + (size_t)x;
    c[i] = 0u;
    t[i] = kInf;
  }
}

// rtx_rcp_check: out[0] += floats checked, out[1] += mismatches, out[2] = bits
// of a mismatching x
// rtx_calib_read: a grid-stride pass, each element loaded once; the xor of
// everything is stored only if it equals a value a zeroed buffer never gives
// (the loads cannot be dropped, and no store lands)
__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }
template <class T>
__global__ __launch_bounds__(256) void calib_read_kernel(const T *__restrict__ p, int64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc ^= fold(p[i]);
  if (acc == 0x9E3779B9u) out[0] = acc;
}

__global__ void rcp_check_kernel(uint32_t base, unsigned long long *out) {
  const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(bits);
  const float ax = __builtin_fabsf(x);
  const bool in = ax >= 1e-8f && ax < 0x1p126f;
  const bool bad = in && __float_as_uint(1.0f / x) != __float_as_uint(rtm::rcp_rn(x));
  const unsigned long long nin = __popcll(__ballot(in)), nbad = __popcll(__ballot(bad));
  if ((threadIdx.x & 63) == 0) {
    if (nin) atomicAdd(out, nin);
    if (nbad) atomicAdd(out + 1, nbad);
  }
  if (bad) out[2] = bits;
}

// rtx_div_check: rtm::div_mk against the division. mode 0: 2 (x + 1/2) / W for
// every W in [1, 32768] and x < W (blockIdx.y = W - 1); mode 1: random pairs in
// the eye ray's ranges (|a| in [2^-72, 2^24] or +-0, |b| in [2^-20, 2^24],
// random signs and mantissas). out[0] += checked, out[1] += mismatches,
// out[2] = a mismatching pair (a's bits | b's bits << 32)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void div_check_kernel(int mode, uint64_t base, uint64_t seed, unsigned long long *out) {
  uint64_t n_in = 0, n_bad = 0, bad_ab = 0;
  if (mode == 0) {
    const int W = (int)blockIdx.y + 1;
    for (int x = (int)threadIdx.x; x < W; x += (int)blockDim.x) {
      const float a = 2.0f * ((float)x + 0.5f), b = (float)W;
      ++n_in;
      if (__float_as_uint(rtm::div_mk(a, b)) != __float_as_uint(a / b)) {
        ++n_bad;
        bad_ab = __float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32);
      }
    }
  } else {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t h = mix64(i ^ (seed << 40)), g = mix64(h);
    const uint32_t ea = 127 - 72 + (uint32_t)(g % 97), eb = 127 - 20 + (uint32_t)((g >> 16) % 45);
    uint32_t ua = ((uint32_t)h & 0x807FFFFFu) | (ea << 23);
    const uint32_t ub = ((uint32_t)(h >> 32) & 0x807FFFFFu) | (eb << 23);
    if (((g >> 32) & 63) == 0) ua &= 0x80000000u;  // +-0 numerators
    const float a = __uint_as_float(ua), b = __uint_as_float(ub);
    n_in = 1;
    if (__float_as_uint(rtm::div_mk(a, b)) != __float_as_uint(a / b)) {
      n_bad = 1;
      bad_ab = ua | ((uint64_t)ub << 32);
    }
  }
  if (n_in) atomicAdd(out, (unsigned long long)n_in);
  if (n_bad) {
    atomicAdd(out + 1, (unsigned long long)n_bad);
    out[2] = bad_ab;
  }
}

__global__ void untile_kernel(const uint32_t *pc, const float *pt, int64_t per_rank, uint32_t *c,
                              float *t, int W, int H, int band_rows, int nranks) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)W * H) return;
  const int yo = (int)(i / W), x = (int)(i - (int64_t)yo * W);
  const int b = yo / band_rows, r = b % nranks, k = b / nranks;
  const int64_t src = (int64_t)r * per_rank + ((int64_t)k * band_rows + (yo - b * band_rows)) * W + x;
  if (c) c[i] = pc[src];
  if (t) t[i] = pt[src];
}

// Block schedule for the next frame from this frame's per-tile costs:
// tiles in descending cost class (2 classes per octave of shader cycles), so
// the long-running tiles of a frame -- grazing rays at silhouettes, the tail
// that otherwise starts late and runs alone -- are dispatched first. Order
// within a class is arbitrary; the image does not depend on the order. Resets
// the costs for the next frame.
constexpr int kCostClasses = 66;
__device__ __forceinline__ uint32_t cost_class(uint32_t c) {
  if (c == 0) return 0;
  const uint32_t e = 32u - (uint32_t)__clz(c);
  return 2 * e + (e >= 2 ? (c >> (e - 2)) & 1u : 0u);
}
__global__ __launch_bounds__(1024) void order_kernel(uint32_t *cost, uint32_t *order, uint32_t n) {
  __shared__ uint32_t hist[kCostClasses];
  for (uint32_t i = threadIdx.x; i < kCostClasses; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[cost_class(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int b = kCostClasses - 1; b >= 0; --b) {
      const uint32_t h = hist[b];
      hist[b] = run;
      run += h;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    order[atomicAdd(&hist[cost_class(cost[i])], 1u)] = i;
    cost[i] = 0;
  }
}

// Diagnostic: the world-space primary ray of every pixel, as render_kernel
// computes it (image row yo, loop row y = H - yo - 1).
__global__ void eye_rays_kernel(rt_render_params P, int W, int H, float *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  const int yo = i / W, x = i - yo * W;
  const f3 d = eye_ray(x, H - yo - 1, W, H, P.proj_inv, P.view_inv);
  out[3 * i] = d.x;
  out[3 * i + 1] = d.y;
  out[3 * i + 2] = d.z;
}

// Diagnostic: the 8-lane group primitives of the cooperative tail on test
// vectors (one 8-lane group per vector of 8 keys): sort8 across lanes, the
// first-wins min, the OR reduction. Checked against the scalar forms in tests.
__global__ void grp_test_kernel(const float *keys, int n, float *st, uint32_t *sid, float *mt,
                                uint32_t *mk, uint32_t *orv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // blockDim = 64: 8 groups per wave
  const int g = i >> 3, k = i & 7;
  const bool ok = g < n;
  float t = ok ? keys[8 * g + k] : 0.0f;
  uint32_t id = (uint32_t)k;
  grp_sort8(t, id, k);
  float m = ok ? keys[8 * g + k] : 0.0f;
  uint32_t kk = (uint32_t)k;
  grp_min_first(m, kk, k);
  const uint32_t o = grp_or(1u << (3 * k), k);
  if (ok) {
    st[8 * g + k] = t;
    sid[8 * g + k] = id;
    if (k == 0) { mt[g] = m; mk[g] = kk; orv[g] = o; }
  }
}

}  // namespace

// ================================================================== C ABI ==
struct rt_scene {
  int kind = 0;
  int device = 0;
  int32_t maxd = 1;  // LDS stack frames the kernel is instantiated for
  // mesh
  rtl::GNode *d_nodes = nullptr;
  rtl::GTri *d_tris = nullptr;
  uint32_t root = rtl::kInvalidChild;
  float root_box[6] = {0, 0, 0, 0, 0, 0};
  int64_t host_nodes = 0, host_inner = 0;
  uint32_t n_inner = 0;  // inner nodes on the device (MeshDev::n_inner)
  float dmax2 = 0.0f;    // MeshDev::dmax2 (mesh_dmax2; 0: every ray takes the division)
  int32_t bvh_depth = 0;
  // grid
  float *d_vals = nullptr;
  uint32_t size[3] = {0, 0, 0};
  bool grid_bricked = false;  // device layout (rt_scenes.h GridDev): bricked, or the reference's linear
  // octree
  rtl::OctWord *d_child = nullptr;
  rtl::OctVals *d_ovals = nullptr;
  int32_t oct_depth = 0;
  PlaneDev plane{};
  int64_t dev_bytes = 0;
  // cached buffers for host-buffer entry points
  uint32_t *d_color = nullptr;
  float *d_t = nullptr;
  size_t fb_cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_host = nullptr;  // rt_render's pageable cleared frame: the spans are on the host
  hipStream_t xs[2] = {nullptr, nullptr};  // rt_render: colour / t copy streams (render on xs[0])
  hipEvent_t xev = nullptr;
  // rt_render: FrameArgs::hit_box of its frame (4 words) and a pinned,
  // mapped host copy (h_hit_box_dev: its device address, box_out_kernel)
  int32_t *d_hit_box = nullptr;
  int32_t *h_hit_box = nullptr;
  int32_t *h_hit_box_dev = nullptr;
  // the pageable zero-copy path: FrameArgs::row_span (2 words per row) and its
  // pinned, mapped host copy, for span_cap rows
  int32_t *d_row_span = nullptr;
  int32_t *h_row_span = nullptr;
  int32_t *h_row_span_dev = nullptr;
  int32_t span_cap = 0;
  // rt_render's staging frame for a cleared frame on pageable buffers: pinned
  // host memory the kernel stores its hits into (zero-copy), kept cleared
  uint32_t *stage_c = nullptr;
  float *stage_t = nullptr;
  size_t stage_cap = 0;
  int32_t stage_W = 0, stage_H = 0;
  bool stage_dirty = true;
  // cost-ordered block schedule (see launch_render), double-buffered: frame k
  // of the scene's one-frame kernel records its tiles' costs into d_cost[k & 1]
  // and dispatches in the order d_order[k & 1] that frame k - 2's costs gave;
  // frame k's own order is computed by order_kernel on the side stream
  // sched_os as soon as frame k is done (frame_ev), beside frame k + 1, and
  // ord_ev[k & 1] marks it done. sched_key[b] = the grid (gx << 16 | gy) whose
  // order d_order[b] holds (0: none). sched_on = false renders in plain
  // blockIdx order
  uint32_t *d_cost[2] = {nullptr, nullptr};
  uint32_t *d_order[2] = {nullptr, nullptr};
  uint32_t sched_key[2] = {0, 0};
  bool ord_rec[2] = {false, false};
  int sched_par = 0;
  uint32_t sched_cap = 0;
  bool sched_on = true;
  bool coop = true;  // mesh primary rays: cooperative tail (rtx_set_coop)
  hipStream_t last_stream = nullptr;   // stream of the previous frame (scheduled or not)
  hipStream_t sched_os = nullptr;      // side stream of the order kernels
  hipEvent_t ord_ev[2] = {nullptr, nullptr};
  hipEvent_t frame_ev = nullptr;
  bool pump_on = false;  // primary-ray batches on the ray pump (rtx_set_pump)
};

namespace {

// bricked sample count of a grid (rt_scenes.h GridDev)
uint64_t grid_bricked_samples(const uint32_t size[3]) {
  return (uint64_t)grid_bricks(size[0]) * grid_bricks(size[1]) * grid_bricks(size[2]) * 64u;
}

// device samples of a grid scene (s->grid_bricked picks the layout)
uint64_t grid_samples(const rt_scene *s) {
  return s->grid_bricked ? grid_bricked_samples(s->size) : (uint64_t)s->size[0] * s->size[1] * s->size[2];
}

// diagnostic (rtx_set_grid_force): bit 0 = grids created from now on take the
// bricked layout whatever their size, bit 1 = every grid launch takes the 64-bit
// address path (no buffer loads); tests reach each grid_mode branch with it
int g_grid_force = 0;

GridDev grid_dev(const rt_scene *s) {
  const uint64_t n = grid_samples(s);
  // buffer loads: 32-bit byte offsets and num_records, so only grids below
  // 4 GiB (a grid of exactly 2^32 bytes would put its last sample past a
  // saturated num_records) -- larger ones take the 64-bit address path
  const uint32_t bytes = 4 * n < (1ull << 32) ? (uint32_t)(4 * n) : 0u;
  if (!s->grid_bricked) return GridDev{s->d_vals, s->size[0], s->size[1], s->size[2], s->size[2],
                                       s->size[1] * s->size[2], bytes};
  const uint32_t ys = grid_bricks(s->size[2]) * 64u;
  return GridDev{s->d_vals, s->size[0], s->size[1], s->size[2], ys, grid_bricks(s->size[1]) * ys, bytes};
}

int grid_mode(const rt_scene *s, const GridDev &gd) {
  // buffer mode: 32-bit byte offsets and 24-bit stride multiplies (grid_mul)
  const bool buf = gd.bytes != 0 && gd.xs < (1u << 24) && gd.ys < (1u << 24) && !(g_grid_force & 2);
  return (buf ? kGridBuf : 0) | (s->grid_bricked ? kGridBricked : 0);
}

// reference x-major values -> 4x4x4 bricks; one thread per bricked sample
// (padding samples get 0 and are never read)
__global__ __launch_bounds__(256) void brick_kernel(const float *__restrict__ src, float *__restrict__ dst,
                                                    uint32_t sx, uint32_t sy, uint32_t sz, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t nby = grid_bricks(sy), nbz = grid_bricks(sz);
  const uint32_t l = (uint32_t)(i & 63u);
  const uint64_t b = i >> 6;
  const uint32_t bz = (uint32_t)(b % nbz), by = (uint32_t)((b / nbz) % nby), bx = (uint32_t)(b / nbz / nby);
  const uint32_t x = bx * 4 + (l >> 4), y = by * 4 + ((l >> 2) & 3u), z = bz * 4 + (l & 3u);
  dst[i] = (x < sx && y < sy && z < sz) ? src[((uint64_t)x * sy + y) * sz + z] : 0.0f;
}

MeshDev mesh_dev(const rt_scene *s) {
  MeshDev m{s->d_nodes, s->d_tris, s->root, {}, s->coop, s->n_inner, nullptr, 0, s->dmax2};
  for (int k = 0; k < 6; ++k) m.rbox[k] = s->root_box[k];
  return m;
}

// LDS frame slots per lane for a tree with `depth` inner levels: the top frame
// lives in registers, so depth-1 slots. Sized to the tree (not a worst case)
// so the stack does not cap occupancy: 4 slots x 12 B x 256 lanes = 12 KiB.
int pick_maxd(int depth, int32_t &maxd) {
  const int need = depth > 1 ? depth - 1 : 1;
  const int options[] = {4, 7, 15, 31};
  for (int m : options)
    if (need <= m) { maxd = m; return RT_OK; }
  return set_err(RT_E_INVALID, "tree deeper than 32 levels");
}

int ensure_events(rt_scene *s) {
  if (!s->ev0) HIP_TRY(hipEventCreate(&s->ev0));
  if (!s->ev1) HIP_TRY(hipEventCreate(&s->ev1));
  if (!s->ev_host) HIP_TRY(hipEventCreateWithFlags(&s->ev_host, hipEventDisableTiming));
  return RT_OK;
}

// rt_render's two copy/render streams (non-blocking: no implicit sync with
// the null stream) and the event that orders the uploads before the kernel
int ensure_copy_streams(rt_scene *s) {
  for (int k = 0; k < 2; ++k)
    if (!s->xs[k]) {
      HIP_TRY(hipStreamCreateWithFlags(&s->xs[k], hipStreamNonBlocking));
      char label[64];
      std::snprintf(label, sizeof label, "scene %p stream %s", (void *)s, k ? "t" : "render/colour");
      rterr::stream_add(s->xs[k], s->device, label);
    }
  if (!s->xev) HIP_TRY(hipEventCreateWithFlags(&s->xev, hipEventDisableTiming));
  if (!s->d_hit_box) HIP_TRY(hipMalloc(&s->d_hit_box, 4 * sizeof(int32_t)));
  if (!s->h_hit_box_dev) {  // (guarded on the device address: a failed lookup is retried next call)
    if (!s->h_hit_box) HIP_TRY(hipHostMalloc(&s->h_hit_box, 4 * sizeof(int32_t), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void **)&s->h_hit_box_dev, s->h_hit_box, 0));
  }
  return RT_OK;
}

int ensure_fb(rt_scene *s, size_t px) {
  if (px <= s->fb_cap) return RT_OK;
  if (s->d_color) HIP_NOTE(hipFree(s->d_color));
  if (s->d_t) HIP_NOTE(hipFree(s->d_t));
  s->d_color = nullptr;
  s->d_t = nullptr;
  s->fb_cap = 0;
  HIP_TRY(hipMalloc(&s->d_color, px * 4));
  HIP_TRY(hipMalloc(&s->d_t, px * 4));
  s->fb_cap = px;
  return RT_OK;
}

template <class S, int MAXD>
void launch_render_t(const S &sc, const PlaneDev &pl, const FrameArgs &fa, bool general,
                     hipStream_t stream, unsigned long long *counters, int diag) {
  const dim3 grid((fa.W + kTile - 1) / kTile, (fa.rows_local + kTile - 1) / kTile);
  const dim3 fgrid((fa.W + kFTile - 1) / kFTile, (fa.rows_local + kFTile - 1) / kFTile);
  if (diag == 1) {
    if (general)
      render_kernel<S, MAXD, true, 1><<<grid, kBlock, 0, stream>>>(sc, pl, fa, counters);
    else
      render_kernel<S, MAXD, false, 1><<<grid, kBlock, 0, stream>>>(sc, pl, fa, counters);
  } else if (diag == 2) {
    if (general)
      render_kernel<S, MAXD, true, 2><<<grid, kBlock, 0, stream>>>(sc, pl, fa, counters);
    else
      render_kernel<S, MAXD, false, 2><<<grid, kBlock, 0, stream>>>(sc, pl, fa, counters);
  } else {
    if (general)
      render_kernel<S, MAXD, true, 0><<<fgrid, kFBlock, 0, stream>>>(sc, pl, fa, nullptr);
    else
      render_kernel<S, MAXD, false, 0><<<fgrid, kFBlock, 0, stream>>>(sc, pl, fa, nullptr);
  }
}

// The pageable drop-in path's staging frame (render_cleared_zero_copy) freed;
// the caller has synchronised the streams that use it.
void stage_free(rt_scene *s) {
  for (void **q : {(void **)&s->stage_c, (void **)&s->stage_t}) {
    if (*q) {
      HIP_NOTE(hipHostFree(*q));
      *q = nullptr;
    }
  }
  s->stage_cap = 0;
}

// The scene's staging frame for px pixels: pinned, mapped host memory the
// runtime owns (hipHostMalloc), never handed back to the process heap, so no
// caller buffer can later land on pages this library registered and
// unregistered (aligned_alloc + hipHostRegister did that in round 5). Used by
// rt_render on pageable caller buffers: the zero-copy cleared frame stores its
// hits into it, and the other frames' uploads / downloads go through it (host
// copies on one side, DMA on the other). Its stream xs[0] is synchronised
// before a smaller frame is replaced.
int ensure_stage(rt_scene *s, size_t px) {
  if (px <= s->stage_cap) return RT_OK;
  if (s->xs[0]) HIP_TRY(hipStreamSynchronize(s->xs[0]));  // (the previous frame's work on the old frame)
  if (s->xs[1]) HIP_TRY(hipStreamSynchronize(s->xs[1]));
  stage_free(s);
  for (void **q : {(void **)&s->stage_c, (void **)&s->stage_t}) {
    if (const hipError_t e = hipHostMalloc(q, px * 4, hipHostMallocDefault)) {
      *q = nullptr;
      stage_free(s);
      return set_err(RT_E_DEVICE, std::string("staging frame: ") + hipGetErrorString(e));
    }
  }
  s->stage_cap = px;
  s->stage_dirty = true;
  return RT_OK;
}

// Cost-ordered schedule state for a frame of grid gx x gy blocks on `stream`.
// Two cost / order buffer pairs alternate (rt_scene::d_cost): a frame waits
// for the order kernel of two frames before (ord_ev of its parity: its order
// is ready and its cost buffer zeroed), renders in that order, and its own
// order kernel runs on the side stream after it, concurrently with the next
// frame -- so back-to-back one-frame launches never queue behind an order
// kernel (~8 us at 1080p), at the price of an order two frames old.
#ifndef RT_SCHED_FRESH
#define RT_SCHED_FRESH 1  // A/B switch: 0 always renders in the order two frames old
#endif
int schedule_begin(rt_scene *s, FrameArgs &fa, uint32_t gx, uint32_t gy, hipStream_t stream) {
  fa.order = nullptr;
  fa.cost = nullptr;
  // Frames of this scene arriving on alternating streams are frames in flight:
  // each one's tail is filled by the next frame's tiles. Such frames render in
  // blockIdx order and leave the schedule state alone.
  const bool same_stream = stream == s->last_stream;
  s->last_stream = stream;
  if (!s->sched_on || !same_stream) return RT_OK;
  const uint32_t nb = gx * gy;
  if (!s->sched_os) {
    HIP_TRY(hipStreamCreateWithFlags(&s->sched_os, hipStreamNonBlocking));
    char label[64];
    std::snprintf(label, sizeof label, "scene %p schedule stream", (void *)s);
    rterr::stream_add(s->sched_os, s->device, label);
    for (hipEvent_t &e : s->ord_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->frame_ev, hipEventDisableTiming));
  }
  if (nb > s->sched_cap) {
    HIP_TRY(hipStreamSynchronize(s->sched_os));  // (no order kernel still reads the old buffers)
    for (int b = 0; b < 2; ++b) {
      if (s->d_cost[b]) HIP_NOTE(hipFree(s->d_cost[b]));
      if (s->d_order[b]) HIP_NOTE(hipFree(s->d_order[b]));
      s->d_cost[b] = s->d_order[b] = nullptr;
      s->sched_key[b] = 0;
    }
    s->sched_cap = 0;
    for (int b = 0; b < 2; ++b) {
      HIP_TRY(hipMalloc(&s->d_cost[b], (size_t)nb * 4));
      HIP_TRY(hipMalloc(&s->d_order[b], (size_t)nb * 4));
      HIP_TRY(hipMemsetAsync(s->d_cost[b], 0, (size_t)nb * 4, stream));  // (in the frame's stream order)
    }
    s->sched_cap = nb;
  }
  const int p = s->sched_par;
  if (s->ord_rec[p]) {
    // usually long done (it ran beside the previous frame): then no
    // cross-stream barrier goes into the frame's stream
    const hipError_t q = hipEventQuery(s->ord_ev[p]);
    if (q == hipErrorNotReady) {
      HIP_TRY(hipStreamWaitEvent(stream, s->ord_ev[p], 0));
    } else if (q != hipSuccess) {
      HIP_TRY(q);
    }
  }
  const uint32_t key = (gx << 16) | gy;
  // The previous frame's order when its order kernel has already finished --
  // a frame issued after the host waited for the one before it (the drop-in's
  // Renderer::draw loop) -- else the one two frames old. The previous frame's
  // order buffer is rewritten only by the next frame's order kernel, which
  // runs after the next frame, so after this one.
  if (RT_SCHED_FRESH && s->ord_rec[p ^ 1] && s->sched_key[p ^ 1] == key &&
      hipEventQuery(s->ord_ev[p ^ 1]) == hipSuccess) {
    fa.order = s->d_order[p ^ 1];
  } else if (s->sched_key[p] == key) {
    fa.order = s->d_order[p];
  }
  fa.cost = s->d_cost[p];
  return RT_OK;
}

// the frame's order kernel on the side stream, after the frame
int schedule_end(rt_scene *s, const FrameArgs &fa, uint32_t gx, uint32_t gy, hipStream_t stream) {
  if (!fa.cost) return RT_OK;
  const int p = s->sched_par;
  HIP_TRY(hipEventRecord(s->frame_ev, stream));
  HIP_TRY(hipStreamWaitEvent(s->sched_os, s->frame_ev, 0));
  order_kernel<<<1, 1024, 0, s->sched_os>>>(s->d_cost[p], s->d_order[p], gx * gy);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(s->ord_ev[p], s->sched_os));
  s->ord_rec[p] = true;
  s->sched_key[p] = (gx << 16) | gy;
  s->sched_par = p ^ 1;
  return RT_OK;
}

int launch_render(rt_scene *s, const FrameArgs &fa_in, hipStream_t stream,
                  unsigned long long *counters = nullptr, int diag = 0, bool sched = true) {
  FrameArgs fa = fa_in;
  const bool general = s->plane.on || fa.P.shading_mode != RT_SHADING_NORMAL;
  const uint32_t gx = (fa.W + kFTile - 1) / kFTile, gy = (fa.rows_local + kFTile - 1) / kFTile;
  fa.order = nullptr;
  fa.cost = nullptr;
  if (diag == 0 && sched) {
    const int rc = schedule_begin(s, fa, gx, gy, stream);
    if (rc) return rc;
  }
  if (s->kind == RT_SCENE_MESH) {
    MeshS sc{mesh_dev(s)};
    switch (s->maxd) {
      case 4: launch_render_t<MeshS, 4>(sc, s->plane, fa, general, stream, counters, diag); break;
      case 7: launch_render_t<MeshS, 7>(sc, s->plane, fa, general, stream, counters, diag); break;
      case 15: launch_render_t<MeshS, 15>(sc, s->plane, fa, general, stream, counters, diag); break;
      default: launch_render_t<MeshS, 31>(sc, s->plane, fa, general, stream, counters, diag); break;
    }
  } else if (s->kind == RT_SCENE_GRID) {
    const GridDev gd = grid_dev(s);
    switch (grid_mode(s, gd)) {
      case kGridBuf | kGridBricked:
        launch_render_t<GridS<kGridBuf | kGridBricked>, 1>({gd}, s->plane, fa, general, stream, counters, diag);
        break;
      case kGridBricked: launch_render_t<GridS<kGridBricked>, 1>({gd}, s->plane, fa, general, stream, counters, diag); break;
      default: launch_render_t<GridS<kGridBuf>, 1>({gd}, s->plane, fa, general, stream, counters, diag); break;
    }
  } else if (s->kind == RT_SCENE_OCTREE) {
    const OctDev od{s->d_child, s->d_ovals};
    switch (s->maxd) {
      case 4: launch_render_t<OctS<true>, 4>(OctS<true>{od}, s->plane, fa, general, stream, counters, diag); break;
      case 7: launch_render_t<OctS<true>, 7>(OctS<true>{od}, s->plane, fa, general, stream, counters, diag); break;
      case 15: launch_render_t<OctS<false>, 15>(OctS<false>{od}, s->plane, fa, general, stream, counters, diag); break;
      default: launch_render_t<OctS<false>, 31>(OctS<false>{od}, s->plane, fa, general, stream, counters, diag); break;
    }
  } else {
    return set_err(RT_E_STATE, "scene has no geometry");
  }
  HIP_TRY(hipGetLastError());
  if (diag == 0 && sched) return schedule_end(s, fa, gx, gy, stream);
  return RT_OK;
}

// Work-queue heads of render_persist_kernel, one set per (device, stream):
// launches on one stream run in order, and each launch's last wave resets its
// heads, so consecutive launches on a stream reuse them; concurrent streams
// never share a set. The set is allocated and zeroed IN STREAM ORDER
// (hipMallocAsync + hipMemsetAsync on that stream): no device-wide sync, so a
// first launch on a new stream neither stalls the other streams nor breaks a
// graph capture. rt_stream_prepare() does it ahead of time (outside a timed
// region); rt_stream_release() frees the set, again in stream order.
constexpr size_t kQueueBytes = (8 * kHeadStrideMax + 16) * sizeof(uint32_t);
std::mutex g_queue_mu;
std::map<std::pair<int, hipStream_t>, uint32_t *> g_queues;

int stream_queue(hipStream_t stream, uint32_t **out) {
  *out = nullptr;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_queue_mu);
  auto it = g_queues.find({dev, stream});
  if (it != g_queues.end()) {
    *out = it->second;
    return RT_OK;
  }
  void *p = nullptr;
  HIP_TRY(hipMallocAsync(&p, kQueueBytes, stream));
  const hipError_t e = hipMemsetAsync(p, 0, kQueueBytes, stream);
  if (e != hipSuccess) {
    HIP_NOTE(hipFreeAsync(p, stream));
    return set_err(RT_E_DEVICE, std::string("work-queue init: ") + hipGetErrorString(e));
  }
  g_queues[{dev, stream}] = (uint32_t *)p;
  *out = (uint32_t *)p;
  return RT_OK;
}

// Heavy-first order of the block dispatch for row bands (a rank's 1/N of each
// frame at N > 1): with so little work per launch, a rank's time is its
// slowest tiles' chains (silhouette tiles) unless they start first. Each
// (device, stream) keeps the per-tile cost of its previous band launch (the
// slowest wave of each tile, any frame) and the order derived from it
// (order_kernel: half-octave cost classes, heaviest first); consecutive orbit
// frames keep their heavy tiles near the model's outline, so the last launch
// predicts the next. Output-neutral: only the dispatch order changes.
// Off by default: 8 ranks x 16 frames of bunny / the 1.1 M-triangle stand-in,
// two interleaved A/B rounds, came out level within the run-to-run spread
// (profiles/r05/band_order_ab.txt). RTAMD_BAND_ORDER=1 (or rtx_set_band_order)
// switches it on.
struct BandSched {
  uint32_t *cost = nullptr, *order = nullptr;
  uint32_t ntiles = 0;
  bool valid = false;
};
std::map<std::pair<int, hipStream_t>, BandSched> g_band_sched;  // (under g_queue_mu)

bool band_order_env() {
  const char *e = ab_env("RTAMD_BAND_ORDER");
  return e && e[0] == '1';
}
std::atomic<bool> g_band_order{band_order_env()};
bool band_order_enabled() { return g_band_order.load(std::memory_order_relaxed); }

int band_sched(hipStream_t stream, uint32_t ntiles, BandSched **out) {
  *out = nullptr;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_queue_mu);
  BandSched &b = g_band_sched[{dev, stream}];
  if (b.ntiles != ntiles) {  // new band geometry: fresh buffers in stream order, no order yet
    if (b.cost) HIP_NOTE(hipFreeAsync(b.cost, stream));
    if (b.order) HIP_NOTE(hipFreeAsync(b.order, stream));
    b = BandSched{};
    void *c = nullptr, *o = nullptr;
    HIP_TRY(hipMallocAsync(&c, (size_t)ntiles * 4, stream));
    HIP_TRY(hipMallocAsync(&o, (size_t)ntiles * 4, stream));
    HIP_TRY(hipMemsetAsync(c, 0, (size_t)ntiles * 4, stream));
    b.cost = (uint32_t *)c;
    b.order = (uint32_t *)o;
    b.ntiles = ntiles;
  }
  *out = &b;
  return RT_OK;
}

// diagnostic per-wave stamps of the persistent launches (rtx_set_persist_stamps)
unsigned long long *g_persist_stamps = nullptr;
int64_t g_persist_stamps_cap = 0;

// RTAMD_PERSIST=0 selects the one-block-per-16x16-tile dispatch (A/B switch).
bool persist_enabled() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_PERSIST");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Which row-band launches take the work queue. A rank's share of a frame is
// 1/N of the pixels; below about a million pixels per frame the queue's drain
// (a wave probes all 8 heads before it exits) and its launch-to-launch
// hand-over cost more than its balancing gains. Bunny 1080p, max over ranks, 8
// frames x 2 streams (ms/frame, queue vs blocks): N = 2 (1.04 M px) 0.0595 vs
// 0.0607, N = 4 0.0425 vs 0.0342, N = 8 0.0379 vs 0.0218. The 1.1 M-triangle
// stand-in at 4K (2.07 M px per rank at N = 4) took 3.18x at N = 4 on the block
// dispatch against 1.93x at N = 2 on the queue (profiles/r03/split_mesh_large.txt).
// RTAMD_BAND_PERSIST=<N> (ranks) or RTAMD_BAND_PERSIST_PX=<pixels> override the
// rule (A/B switches).
// (rtx_set_band_queue_px sets the pixel threshold at run time, for tests)
std::atomic<int64_t> g_band_queue_px{[] {
  const char *e = ab_env("RTAMD_BAND_PERSIST_PX");
  return e ? (int64_t)std::atoll(e) : (int64_t)1000000;
}()};
bool band_takes_queue(const FrameArgs &f) {
  if (f.nranks <= 1) return true;
  static const int max_ranks = [] {
    const char *e = ab_env("RTAMD_BAND_PERSIST");
    return e ? std::atoi(e) : -1;
  }();
  if (max_ranks >= 0) return f.nranks <= max_ranks;
  return (int64_t)f.rows_local * f.W >= g_band_queue_px.load(std::memory_order_relaxed);
}

// wave tiles per queue item (0: block dispatch); RTAMD_PERSIST_G=1|2|4 overrides
// the scene's default (A/B switch)
int persist_group(int dflt) {
  static const int g = [] {
    const char *e = ab_env("RTAMD_PERSIST_G");
    return e ? std::atoi(e) : 0;
  }();
  return (g == 1 || g == 2 || g == 4) ? g : dflt;
}

// Resident workgroups of a persistent kernel on the current device (cached per
// kernel instantiation and device).
template <class K>
int resident_blocks(K kernel, int &blocks, int &dev_cached, int block = kBlock) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (blocks == 0 || dev != dev_cached) {
    int per_cu = 0, cus = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0));
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // RTAMD_PERSIST_OVERSUB=k launches k x the resident workgroups (A/B
    // switch: extra waves start as resident ones leave and exit at once when
    // the queue is drained)
    static const int oversub = [] {
      const char *e = ab_env("RTAMD_PERSIST_OVERSUB");
      const int v = e ? std::atoi(e) : 1;
      return v >= 1 && v <= 8 ? v : 1;
    }();
    blocks = std::max(1, per_cu) * std::max(1, cus) * oversub;
    dev_cached = dev;
  }
  return RT_OK;
}

// Work queue of one multi-frame launch: items of `group` 8x8 wave tiles
// (1: 1x1, 2: 2x1, 4: 2x2) of n frames, the stream's head set; *grid = the
// launch's workgroups (the resident ones, fewer for a small batch).
int make_queue(const FrameBatch &fb, int n, int group, int blocks, hipStream_t stream, PersistQ &q,
               uint32_t &grid, int block = kBlock) {
  uint32_t *heads = nullptr;
  if (const int rc = stream_queue(stream, &heads)) return rc;
  q.heads = heads;
  static const uint32_t stride = [] {
    const char *e = ab_env("RTAMD_QSTRIDE");
    const int v = e ? std::atoi(e) : 0;
    return (uint32_t)((v >= 1 && v <= kHeadStrideMax) ? v : kHeadStride);
  }();
  q.stride = stride;
  q.gx = group >= 2 ? 2 : 1;
  q.gy = group >= 4 ? 2 : 1;
  q.tiles_x = (uint32_t)((fb.f[0].W + 8 * q.gx - 1) / (8 * q.gx));
  q.per_frame = q.tiles_x * (uint32_t)((fb.f[0].rows_local + 8 * q.gy - 1) / (8 * q.gy));
  q.items = q.per_frame * (uint32_t)n;
  // RTAMD_QMAP=band: banded item order per head (PersistQ::cpf)
  static const bool banded = [] {
    const char *e = ab_env("RTAMD_QMAP");
    return e && std::strcmp(e, "band") == 0;
  }();
  q.cpf = banded ? (q.per_frame + 7) / 8 : 0;
  q.nper = q.cpf * (uint32_t)n;
  const uint32_t wpb = (uint32_t)block / 64;  // waves per workgroup
  grid = std::min<uint32_t>((uint32_t)blocks, (q.items + wpb - 1) / wpb);
  q.waves = grid * wpb;
  q.stamps = (g_persist_stamps && (int64_t)q.waves <= g_persist_stamps_cap) ? g_persist_stamps : nullptr;
  return RT_OK;
}

template <class S, int MAXD, bool GENERAL>
int launch_persist_t(rt_scene *s, const S &sc, const PlaneDev &pl, const FrameBatch &fb, int n, int group,
                     hipStream_t stream) {
  static int blocks = 0, dev_cached = -1;
  if (const int rc = resident_blocks(render_persist_kernel<S, MAXD, GENERAL>, blocks, dev_cached, kPBlock)) return rc;
  PersistQ q;
  uint32_t grid = 0;
  if (const int rc = make_queue(fb, n, group, blocks, stream, q, grid, kPBlock)) return rc;
  render_persist_kernel<S, MAXD, GENERAL><<<grid, kPBlock, 0, stream>>>(sc, pl, fb, q);
  return RT_OK;
}

// The ray pump is measured slower than one tile per wave on every scene (DESIGN.md
// section 8: refills break the coherence of a wave's rays), so primary-ray batches
// take render_persist_kernel unless RTAMD_PUMP=1 or rtx_set_pump(scene, 1) asks
// for the pump; RTAMD_REFILL=<lanes> sets its refill threshold.
bool pump_env() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_PUMP");
    return e && e[0] == '1';
  }();
  return on;
}
std::atomic<int> g_refill{[] {
  const char *e = ab_env("RTAMD_REFILL");
  const int r = e ? std::atoi(e) : 0;
  return (r >= 1 && r <= 64) ? r : RT_REFILL_MIN;
}()};
int refill_min() { return g_refill.load(std::memory_order_relaxed); }

// scenes with a ray-pump adapter (primary-ray batches)
template <class S>
struct PumpOf {
  static constexpr bool kHas = false;
};
template <bool PK>
struct PumpOf<OctS<PK>> {
  static constexpr bool kHas = true;
  using P = OctP;
  static P make(const OctS<PK> &s) { return P{s.d}; }
};
template <int kMode>
struct PumpOf<GridS<kMode>> {
  static constexpr bool kHas = true;
  using P = GridP<kMode>;
  static P make(const GridS<kMode> &s) { return P{s.d}; }
};
// work-queue item of the pump for scenes that otherwise take the block
// dispatch (the grid): 2x2 wave tiles, so a wave's pixel stream claims once per
// 256 pixels
constexpr int kPumpGroup = 4;

template <class P, int MAXD>
int launch_pump_t(const P &sc, const FrameBatch &fb, int n, int group, hipStream_t stream) {
  static int blocks = 0, dev_cached = -1;
  if (const int rc = resident_blocks(render_pump_kernel<P, MAXD>, blocks, dev_cached)) return rc;
  PersistQ q;
  uint32_t grid = 0;
  if (const int rc = make_queue(fb, n, group, blocks, stream, q, grid)) return rc;
  render_pump_kernel<P, MAXD><<<grid, kBlock, 0, stream>>>(sc, fb, q, n, refill_min());
  return RT_OK;
}

template <class S, int MAXD>
int launch_batch_t(rt_scene *s, const S &sc, const PlaneDev &pl, const FrameBatch &fb, int n, bool general,
                   hipStream_t stream) {
  // Row-band tiles (a rank's share of a multi-GPU frame) with fewer than about
  // a million pixels take the block dispatch (band_takes_queue).
  const int group = persist_group(S::kQueueGroup);
  if constexpr (PumpOf<S>::kHas) {
    if (!general && (pump_env() || (s && s->pump_on)) && persist_enabled() && band_takes_queue(fb.f[0]))
      return launch_pump_t<typename PumpOf<S>::P, MAXD>(PumpOf<S>::make(sc), fb, n,
                                                        persist_group(S::kQueueGroup ? S::kQueueGroup : kPumpGroup),
                                                        stream);
  }
  if (persist_enabled() && group > 0 && band_takes_queue(fb.f[0])) {
    return general ? launch_persist_t<S, MAXD, true>(s, sc, pl, fb, n, group, stream)
                   : launch_persist_t<S, MAXD, false>(s, sc, pl, fb, n, group, stream);
  }
  const dim3 grid((fb.f[0].W + kBTile - 1) / kBTile, (fb.f[0].rows_local + kBTile - 1) / kBTile, n);
  BandSched *bs = nullptr;
  if (kBBlock == 64 && RT_BATCH_INTERLEAVE && fb.f[0].nranks > 1 && band_order_enabled()) {
    if (const int rc = band_sched(stream, grid.x * grid.y, &bs)) return rc;
  }
  const FrameBatch *fbp = &fb;
  FrameBatch fbo;
  if (bs) {
    fbo = fb;
    fbo.f[0].order = bs->valid ? bs->order : nullptr;
    fbo.f[0].cost = bs->cost;
    fbp = &fbo;
  }
  if (general)
    render_batch_kernel<S, MAXD, true><<<grid, kBBlock, 0, stream>>>(sc, pl, *fbp);
  else
    render_batch_kernel<S, MAXD, false><<<grid, kBBlock, 0, stream>>>(sc, pl, *fbp);
  if (bs) {  // this launch's tile costs -> the next launch's order (and the costs cleared)
    // one wave: it takes the first wave slot the other stream's launch frees
    // (a 1024-thread block would wait for a whole CU and hold this stream's
    // next launch behind it)
    order_kernel<<<1, 64, 0, stream>>>(bs->cost, bs->order, bs->ntiles);
    HIP_TRY(hipGetLastError());
    bs->valid = true;
  }
  return RT_OK;
}

// One launch for n <= kMaxBatch frames of equal size / tile (blockIdx order).
int launch_batch(rt_scene *s, FrameBatch &fb, int n, hipStream_t stream) {
  const bool general = s->plane.on || fb.f[0].P.shading_mode != RT_SHADING_NORMAL;
  for (int i = 0; i < n; ++i) {
    if (general != (s->plane.on || fb.f[i].P.shading_mode != RT_SHADING_NORMAL))
      return set_err(RT_E_INVALID, "frames of one batch must share the shading path");
    fb.f[i].order = nullptr;
    fb.f[i].cost = nullptr;
  }
  int rc = RT_OK;
  if (s->kind == RT_SCENE_MESH) {
    MeshS sc{mesh_dev(s)};
    switch (s->maxd) {
      case 4: rc = launch_batch_t<MeshS, 4>(s, sc, s->plane, fb, n, general, stream); break;
      case 7: rc = launch_batch_t<MeshS, 7>(s, sc, s->plane, fb, n, general, stream); break;
      case 15: rc = launch_batch_t<MeshS, 15>(s, sc, s->plane, fb, n, general, stream); break;
      default: rc = launch_batch_t<MeshS, 31>(s, sc, s->plane, fb, n, general, stream); break;
    }
  } else if (s->kind == RT_SCENE_GRID) {
    const GridDev gd = grid_dev(s);
    const int mode = grid_mode(s, gd);
    switch (mode) {
      case kGridBuf | kGridBricked:
        rc = launch_batch_t<GridS<kGridBuf | kGridBricked>, 1>(s, {gd}, s->plane, fb, n, general, stream);
        break;
      case kGridBricked: rc = launch_batch_t<GridS<kGridBricked>, 1>(s, {gd}, s->plane, fb, n, general, stream); break;
      default: rc = launch_batch_t<GridS<kGridBuf>, 1>(s, {gd}, s->plane, fb, n, general, stream); break;
    }
  } else if (s->kind == RT_SCENE_OCTREE) {
    const OctDev od{s->d_child, s->d_ovals};
    switch (s->maxd) {
      case 4: rc = launch_batch_t<OctS<true>, 4>(s, OctS<true>{od}, s->plane, fb, n, general, stream); break;
      case 7: rc = launch_batch_t<OctS<true>, 7>(s, OctS<true>{od}, s->plane, fb, n, general, stream); break;
      case 15: rc = launch_batch_t<OctS<false>, 15>(s, OctS<false>{od}, s->plane, fb, n, general, stream); break;
      default: rc = launch_batch_t<OctS<false>, 31>(s, OctS<false>{od}, s->plane, fb, n, general, stream); break;
    }
  } else {
    return set_err(RT_E_STATE, "scene has no geometry");
  }
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

int check_params(const rt_render_params *p, int32_t W, int32_t H) {
  if (!p) return set_err(RT_E_INVALID, "params is NULL");
  if (W <= 0 || H <= 0 || (int64_t)W * H > (int64_t)1 << 31) return set_err(RT_E_INVALID, "bad frame size");
  if (p->shading_mode < 0 || p->shading_mode > 2) return set_err(RT_E_INVALID, "bad shading mode");
  return RT_OK;
}

// Whether eye_ray_fast gives eye_ray's bits for every pixel of a W x H frame
// with this inverse projection: the operand ranges rtm::div_mk needs, bounded
// over the whole frame. Every entry zero or of magnitude in [2^-10, 2^10] (the
// z column, which meets z = 0, only finite), so a
// nonzero pos component (NDC steps >= 2^-24) is at least ~2^-60 and at most
// 3 x 2^10; |w| >= 2^-10 over [-1, 1]^2 (one sign); a component of pos whose
// constant term dominates keeps |p| >= 2^-20. Then pos / w, p and p / |p|
// stay in [2^-96, 2^44] (or are +-0). 2 fx / W: every W <= 32768 is checked.
// The reference's projection (perspectiveMatrix(45, W/H, 0.01, 100)) passes.
// RTAMD_FAST_EYE=0 keeps the divisions (A/B switch)
bool fast_eye_enabled() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_FAST_EYE");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool fast_eye_ok(const float *m, int32_t W, int32_t H) {
  if (W > 32768 || H > 32768) return false;
  for (int i = 0; i < 16; ++i) {
    const float a = std::fabs(m[i]);
    if (i >= 8 && i < 12) {  // the z column meets z = 0: any finite entry adds +-0
      if (!std::isfinite(m[i])) return false;
    } else if (!(m[i] == 0.0f || (a >= 0x1p-10f && a <= 0x1p10f))) {
      return false;
    }
  }
  const double wc = std::fabs((double)m[15]), wr = std::fabs((double)m[3]) + std::fabs((double)m[7]);
  if (!(wc - wr >= 0x1p-10)) return false;
  const double wmax = wc + wr;
  double lmin = 0.0;
  for (int i = 0; i < 3; ++i)
    lmin = std::max(lmin, (std::fabs((double)m[12 + i]) - std::fabs((double)m[i]) - std::fabs((double)m[4 + i])) / wmax);
  return lmin >= 0x1p-20;
}

int fill_frame(FrameArgs &fa, const rt_render_params *p, uint32_t *c, float *t, int32_t W, int32_t H,
               uint32_t flags, const rt_tile *tile) {
  fa.P = *p;
  fa.color = c;
  fa.t = t;
  fa.W = W;
  fa.H = H;
  fa.flags = flags;
  fa.band_rows = H;
  fa.rank = 0;
  fa.nranks = 1;
  fa.rows_local = H;
  fa.order = nullptr;
  fa.cost = nullptr;
  fa.hit_box = nullptr;
  if ((flags & RT_FLAG_HITS_ONLY) && !(flags & RT_FLAG_CLEAR))
    return set_err(RT_E_INVALID, "RT_FLAG_HITS_ONLY needs RT_FLAG_CLEAR (a cleared frame)");
  if (flags & ~(RT_FLAG_CLEAR | RT_FLAG_TILE_NATURAL | RT_FLAG_HITS_ONLY))
    return set_err(RT_E_INVALID, "unknown render flag");
  if (tile && tile->num_ranks > 1) {
    if (tile->band_rows <= 0 || tile->rank < 0 || tile->rank >= tile->num_ranks)
      return set_err(RT_E_INVALID, "bad tile");
    fa.band_rows = tile->band_rows;
    fa.rank = tile->rank;
    fa.nranks = tile->num_ranks;
    fa.rows_local = (int32_t)(rt_tile_pixels(W, H, tile) / W);
  }
  if (fast_eye_enabled() && fast_eye_ok(p->proj_inv, W, H)) fa.flags |= kFlagFastEye;
  return RT_OK;
}

template <class S, int MAXD>
void launch_rays_t(const S &sc, const PlaneDev &pl, const float *o, const float *d, int64_t n,
                   float tn, float tf, int32_t *hit, float *t, float *nrm, int64_t *prim) {
  const int64_t blocks = (n + kBlock - 1) / kBlock;
  rays_kernel<S, MAXD><<<(unsigned)blocks, kBlock>>>(sc, pl, o, d, n, tn, tf, hit, t, nrm, prim);
}

}  // namespace

namespace {
// BVH8 builder selection (rt_set_bvh_builder): both builders give the same tree
int g_bvh_mode = RT_BVH_AUTO;
constexpr int64_t kBvhDeviceMinTris = 32768;  // auto: the device builder from this many triangles

// which builder produced this thread's last tree (rtx_bvh_last_builder):
// 1 host, 2 device, 3 host after a failed device build (AUTO)
thread_local int t_bvh_last = 0;

int build_bvh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, rth::BVHGpu &b,
              unsigned want) {
  std::string err;
  int ndev = 0;
  const bool dev = g_bvh_mode == RT_BVH_DEVICE ||
                   (g_bvh_mode == RT_BVH_AUTO && nidx / 3 >= kBvhDeviceMinTris &&
                    hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0);
  bool fell_back = false;
  if (dev) {
    if (rth::build_bvh8_gpu(vpos4, nverts, idx, nidx, b, err, want)) {
      t_bvh_last = 2;
      return RT_OK;
    }
    if (err.rfind("GPU BVH builder bound", 0) == 0) return set_err(RT_E_DEVICE, err);
    const bool device_failure = err.rfind("GPU BVH build:", 0) == 0;
    if (!device_failure) return set_err(RT_E_INVALID, err);
    if (g_bvh_mode == RT_BVH_DEVICE) return set_err(RT_E_DEVICE, err);
    // AUTO: the host builder gives the identical tree, unless
    // the device is left in a sticky fault state: then every later call on it
    // fails too, so the failure is reported here instead of at the upload
    if (const hipError_t e = hipDeviceSynchronize(); e != hipSuccess)
      return set_err(RT_E_DEVICE, err + "; device unusable afterwards: " + hipGetErrorString(e));
    (void)hipGetLastError();  // the builder's failure was reported above: clear it
    std::fprintf(stderr, "rtamd: %s; building the BVH on the host instead\n", err.c_str());
    fell_back = true;
    err.clear();
  }
  if (!rth::build_bvh8(vpos4, nverts, idx, nidx, b, err, want)) return set_err(RT_E_INVALID, err);
  t_bvh_last = fell_back ? 3 : 1;
  return RT_OK;
}

int new_scene(rt_scene **out) {
  if (!out) return set_err(RT_E_INVALID, "out is NULL");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  rt_scene *s = new rt_scene();
  s->device = dev;
  s->plane.on = 0;
  s->plane.n = f3{0.0f, 1.0f, 0.0f};
  *out = s;
  return RT_OK;
}

// upload + `pad` zeroed trailing elements (kernels may read past the end).
template <class T>
int upload_padded(T **dst, const T *src, size_t n, size_t pad, int64_t &bytes) {
  HIP_TRY(hipMalloc(dst, (n + pad) * sizeof(T)));
  HIP_TRY(hipMemset(*dst, 0, (n + pad) * sizeof(T)));
  if (n) HIP_TRY(rtdma::h2d(*dst, src, n * sizeof(T), nullptr));
  bytes += (int64_t)((n + pad) * sizeof(T));
  return RT_OK;
}

template <class T>
int upload(T **dst, const T *src, size_t n, int64_t &bytes) {
  if (n == 0) n = 1;  // keep a valid pointer
  HIP_TRY(hipMalloc(dst, n * sizeof(T)));
  if (src) HIP_TRY(rtdma::h2d(*dst, src, n * sizeof(T), nullptr));
  bytes += (int64_t)(n * sizeof(T));
  return RT_OK;
}

}  // namespace

extern "C" {

const char *rt_last_error(void) { return rterr::get(); }
int rt_abi_version(void) { return RTAMD_ABI_VERSION; }

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int rt_set_device(int device) {
  HIP_TRY(hipSetDevice(device));
  return RT_OK;
}

int rt_load_obj(const char *path, int scale, float *vpos4, int64_t *nverts, uint32_t *idx,
                int64_t *nidx) {
  if (!path || !nverts || !nidx) return set_err(RT_E_INVALID, "NULL argument");
  rth::Mesh m;
  std::string err;
  if (!rth::load_obj(path, scale != 0, m, err)) return set_err(RT_E_IO, err);
  const int64_t nv = (int64_t)m.vpos4.size() / 4, ni = (int64_t)m.idx.size();
  if (vpos4 || idx) {
    if (*nverts < nv || *nidx < ni) return set_err(RT_E_INVALID, "buffers too small");
    if (vpos4) std::memcpy(vpos4, m.vpos4.data(), m.vpos4.size() * 4);
    if (idx) std::memcpy(idx, m.idx.data(), m.idx.size() * 4);
  }
  *nverts = nv;
  *nidx = ni;
  return RT_OK;
}

int rt_load_grid(const char *path, uint32_t size[3], float *values) {
  if (!path || !size) return set_err(RT_E_INVALID, "NULL argument");
  std::vector<float> v;
  uint32_t sz[3];
  std::string err;
  if (!rth::load_grid(path, sz, v, err)) return set_err(RT_E_IO, err);
  if (values) {
    if ((uint64_t)size[0] * size[1] * size[2] < v.size()) return set_err(RT_E_INVALID, "buffer too small");
    std::memcpy(values, v.data(), v.size() * 4);
  }
  size[0] = sz[0]; size[1] = sz[1]; size[2] = sz[2];
  return RT_OK;
}

int rt_load_octree(const char *path, int64_t *count, void *nodes36) {
  if (!path || !count) return set_err(RT_E_INVALID, "NULL argument");
  std::vector<uint8_t> v;
  std::string err;
  if (!rth::load_octree(path, v, err)) return set_err(RT_E_IO, err);
  const int64_t n = (int64_t)v.size() / 36;
  if (nodes36) {
    if (*count < n) return set_err(RT_E_INVALID, "buffer too small");
    std::memcpy(nodes36, v.data(), v.size());
  }
  *count = n;
  return RT_OK;
}

int rt_camera(const float pos[3], const float target[3], const float up[3], float fovy_deg,
              float aspect, float znear, float zfar, float view_inv[16], float proj_inv[16]) {
  if (!pos || !target || !up || !view_inv || !proj_inv) return set_err(RT_E_INVALID, "NULL argument");
  rth::camera_matrices(pos, target, up, fovy_deg, aspect, znear, zfar, view_inv, proj_inv);
  return RT_OK;
}

int rt_set_bvh_builder(int mode) {
  if (mode < RT_BVH_AUTO || mode > RT_BVH_DEVICE) return set_err(RT_E_INVALID, "bad BVH builder mode");
  g_bvh_mode = mode;
  return RT_OK;
}

int rt_bvh_export(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                  uint32_t *canon, int64_t *nnodes, uint32_t *perm_tri, int32_t *max_depth) {
  if (!vpos4 || !idx || !nnodes || nverts <= 0 || nidx <= 0) return set_err(RT_E_INVALID, "bad mesh");
  rth::BVHGpu b;
  const unsigned want = (canon ? rth::kBvhCanon : 0u) | (perm_tri ? rth::kBvhPerm : 0u);
  if (int rc = build_bvh(vpos4, nverts, idx, nidx, b, want)) return rc;
  const int64_t n = canon ? (int64_t)b.canon.size() / 52 : b.host_nodes;
  if (canon) {
    if (*nnodes < n) return set_err(RT_E_INVALID, "buffer too small");
    std::memcpy(canon, b.canon.data(), b.canon.size() * 4);
  }
  if (perm_tri) std::memcpy(perm_tri, b.perm_tri.data(), b.perm_tri.size() * 4);
  if (max_depth) *max_depth = b.max_depth;
  *nnodes = n;
  return RT_OK;
}

// max over triangle slots of |e1| |e2| (float bits: the values are >= 0, so
// their bit patterns order like them; NaN counts as +inf)
__global__ void tri_edge_bound_kernel(const rtl::GTri *__restrict__ tris, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  float m = 0.0f;
  if (i < n) {
    const float4 *q = reinterpret_cast<const float4 *>(tris + i);
    const float4 b = q[1], c = q[2];
    const float v = __builtin_sqrtf(b.x * b.x + b.y * b.y + b.z * b.z) *
                    __builtin_sqrtf(c.x * c.x + c.y * c.y + c.z * c.z);
    m = __builtin_isnan(v) ? kInf : v;
  }
  for (int off = 32; off > 0; off >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0 && m > 0.0f) atomicMax(out, __float_as_uint(m));
}

// MeshDev::dmax2 of a mesh scene: (2^124 / (2 M))^2, M = max |e1| |e2| over its
// triangles. A ray with dot(d, d) <= dmax2 has |d| <= 2^124 / (2 M) (up to a
// few ulps), and tri_t's float det = e1 . (d x e2) is at most sqrt(2) |e1|
// |e2| |d| (1 + 2^-24)^5 < 1.5 M |d| <= 0.75 x 2^124 in magnitude: inside the
// range where rtm::rcp_rn is the division. M = 0 (no triangle with both edges)
// leaves every direction; M = inf or NaN leaves none.
int mesh_dmax2(rt_scene *s, uint32_t n_tris) {
  s->dmax2 = 0.0f;
  if (n_tris == 0) return RT_OK;
  uint32_t *d = nullptr, h = 0;
  HIP_TRY(hipMalloc(&d, 4));
  hipError_t e = hipMemset(d, 0, 4);
  if (e == hipSuccess) {
    tri_edge_bound_kernel<<<(n_tris + 255) / 256, 256>>>(s->d_tris, n_tris, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("triangle edge bound: ") + hipGetErrorString(e));
  float M;
  std::memcpy(&M, &h, 4);
  if (M == 0.0f) {
    s->dmax2 = std::numeric_limits<float>::max();
  } else if (std::isfinite(M)) {
    const double r = std::ldexp(1.0, 124) / (2.0 * (double)M * (1.0 + 1e-6));
    const double r2 = r * r;
    s->dmax2 = r2 >= (double)std::numeric_limits<float>::max() ? std::numeric_limits<float>::max()
                                                                  : std::nextafter((float)r2, 0.0f);
  }
  return RT_OK;
}

int rt_scene_create_mesh(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                         rt_scene **out) {
  if (!vpos4 || !idx || nverts <= 0 || nidx <= 0) return set_err(RT_E_INVALID, "empty mesh");
  rth::BVHGpu b;
  if (int rc = build_bvh(vpos4, nverts, idx, nidx, b, rth::kBvhTris | rth::kBvhDeviceTris)) return rc;
  int32_t maxd = 8;
  int rc = pick_maxd(b.max_depth, maxd);
  if (rc) return rc;
  rt_scene *s;
  if ((rc = new_scene(&s))) return rc;
  s->kind = RT_SCENE_MESH;
  s->maxd = maxd;
  s->root = b.root_word;
  std::memcpy(s->root_box, b.root_box, sizeof(s->root_box));
  s->host_nodes = b.host_nodes;
  s->host_inner = b.host_inner;
  s->bvh_depth = b.max_depth;
  s->n_inner = (uint32_t)b.nodes.size();
  if (b.dev_tris.p) {  // the device builder left the triangles on the device (with the zero pad)
    s->dev_bytes += (int64_t)b.dev_tris.bytes;
    s->d_tris = static_cast<rtl::GTri *>(b.dev_tris.take());
  }
  if ((rc = upload(&s->d_nodes, b.nodes.data(), b.nodes.size(), s->dev_bytes)) ||
      (!s->d_tris && (rc = upload_padded(&s->d_tris, b.tris.data(), b.tris.size(), 8, s->dev_bytes))) ||
      (rc = mesh_dmax2(s, b.n_tris))) {
    rt_scene_destroy(s);
    return rc;
  }
  *out = s;
  return RT_OK;
}

int rt_scene_create_grid(const uint32_t size[3], const float *values, rt_scene **out) {
  if (!size || !values) return set_err(RT_E_INVALID, "NULL argument");
  const uint64_t n = (uint64_t)size[0] * size[1] * size[2];
  if (size[0] < 1 || size[1] < 1 || size[2] < 1 || n > (1ull << 32))
    return set_err(RT_E_INVALID, "bad grid size");
  rt_scene *s;
  int rc = new_scene(&s);
  if (rc) return rc;
  s->kind = RT_SCENE_GRID;
  s->size[0] = size[0]; s->size[1] = size[1]; s->size[2] = size[2];
  if ((uint64_t)n * 4 <= kGridLinearMaxBytes && !(g_grid_force & 1)) {  // fits one XCD's L2: the reference layout
    if ((rc = upload(&s->d_vals, values, (size_t)n, s->dev_bytes))) {
      rt_scene_destroy(s);
      return rc;
    }
    *out = s;
    return RT_OK;
  }
  const uint64_t nb = grid_bricked_samples(size);
  if (nb >= (1ull << 32)) {
    rt_scene_destroy(s);
    return set_err(RT_E_INVALID, "bad grid size");
  }
  s->grid_bricked = true;
  float *d_ref = nullptr;  // the reference array, staged for the device-side bricking
  if ((rc = upload(&d_ref, values, (size_t)n, s->dev_bytes)) ||
      (rc = upload(&s->d_vals, (const float *)nullptr, (size_t)nb, s->dev_bytes))) {
    if (d_ref) HIP_NOTE(hipFree(d_ref));
    rt_scene_destroy(s);
    return rc;
  }
  s->dev_bytes -= (int64_t)(n * sizeof(float));
  brick_kernel<<<(unsigned)((nb + 255) / 256), 256>>>(d_ref, s->d_vals, size[0], size[1], size[2], nb);
  const hipError_t e1 = hipGetLastError(), e2 = hipDeviceSynchronize(), e3 = hipFree(d_ref);
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
    rt_scene_destroy(s);
    return set_err(RT_E_DEVICE, std::string("grid bricking: ") +
                                    hipGetErrorString(e1 != hipSuccess ? e1 : e2 != hipSuccess ? e2 : e3));
  }
  *out = s;
  return RT_OK;
}

int rt_scene_create_octree(const void *nodes36, int64_t count, rt_scene **out) {
  if (!nodes36 || count <= 0) return set_err(RT_E_INVALID, "empty octree");
  rth::OctGpu g;
  std::string err;
  if (!rth::flatten_octree((const uint8_t *)nodes36, count, g, err)) return set_err(RT_E_INVALID, err);
  int32_t maxd = 8;
  int rc = pick_maxd(g.max_depth, maxd);
  if (rc) return rc;
  rt_scene *s;
  if ((rc = new_scene(&s))) return rc;
  s->kind = RT_SCENE_OCTREE;
  s->maxd = maxd;
  s->oct_depth = g.max_depth;
  if ((rc = upload(&s->d_child, g.child.data(), g.child.size(), s->dev_bytes)) ||
      (rc = upload(&s->d_ovals, g.vals.data(), g.vals.size(), s->dev_bytes))) {
    rt_scene_destroy(s);
    return rc;
  }
  *out = s;
  return RT_OK;
}

int rt_scene_replicate(const rt_scene *src, int device, rt_scene **out) {
  if (!src || !out) return set_err(RT_E_INVALID, "bad arguments");
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_err(RT_E_INVALID, "rt_scene_replicate: no such device");
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(device));
  rt_scene *s = new rt_scene();
  // the scene's description (kind, tree shape, plane, kernel instantiation)
  s->kind = src->kind;
  s->device = device;
  s->maxd = src->maxd;
  s->root = src->root;
  std::memcpy(s->root_box, src->root_box, sizeof s->root_box);
  s->host_nodes = src->host_nodes;
  s->host_inner = src->host_inner;
  s->n_inner = src->n_inner;
  s->dmax2 = src->dmax2;
  s->bvh_depth = src->bvh_depth;
  std::memcpy(s->size, src->size, sizeof s->size);
  s->grid_bricked = src->grid_bricked;
  s->oct_depth = src->oct_depth;
  s->plane = src->plane;
  s->dev_bytes = src->dev_bytes;
  s->sched_on = src->sched_on;
  s->coop = src->coop;
  s->pump_on = src->pump_on;
  // the device arrays, copied device to device (over xGMI between GPUs)
  void *const from[] = {src->d_nodes, src->d_tris, src->d_vals, src->d_child, src->d_ovals};
  void **to[] = {(void **)&s->d_nodes, (void **)&s->d_tris, (void **)&s->d_vals, (void **)&s->d_child,
                 (void **)&s->d_ovals};
  hipError_t e = hipSuccess;
  const char *step = "";
  for (int i = 0; i < 5 && e == hipSuccess; ++i) {
    if (!from[i]) continue;
    size_t bytes = 0;
    if ((e = hipMemPtrGetInfo(from[i], &bytes)) != hipSuccess) { step = "hipMemPtrGetInfo"; break; }
    if ((e = hipMalloc(to[i], bytes)) != hipSuccess) { step = "hipMalloc"; break; }
    if ((e = hipMemcpyPeer(*to[i], device, from[i], src->device, bytes)) != hipSuccess) step = "hipMemcpyPeer";
  }
  HIP_NOTE(hipSetDevice(prev));
  if (e != hipSuccess) {
    rt_scene_destroy(s);
    return set_err(RT_E_DEVICE, std::string("rt_scene_replicate: ") + step + ": " + hipGetErrorString(e));
  }
  *out = s;
  return RT_OK;
}

int rt_scene_device(const rt_scene *s) { return s ? s->device : RT_E_INVALID; }

int rt_scene_get_plane(const rt_scene *s, int *enabled, float normal[3], float *offset) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  if (enabled) *enabled = s->plane.on;
  if (normal) { normal[0] = s->plane.n.x; normal[1] = s->plane.n.y; normal[2] = s->plane.n.z; }
  if (offset) *offset = s->plane.off;
  return RT_OK;
}

int rt_scene_set_plane(rt_scene *s, int enabled, const float normal[3], float offset) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  PlaneDev &p = s->plane;
  p.on = enabled ? 1 : 0;
  if (!enabled) return RT_OK;
  if (!normal) return set_err(RT_E_INVALID, "normal is NULL");
  // Plane(normal, offset) + recalcBasis (raytracing.hpp:121-124, 169-179)
  const float n[3] = {normal[0], normal[1], normal[2]};
  const float a[3] = {std::fabs(n[0]), std::fabs(n[1]), std::fabs(n[2])};
  float b1[3];
  if (a[0] > a[1] && a[0] > a[2]) { b1[0] = n[1]; b1[1] = -n[0]; b1[2] = 0; }
  else { b1[0] = 0; b1[1] = n[2]; b1[2] = -n[1]; }
  auto nrm = [](float v[3]) {
    const float l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] = v[0] / l; v[1] = v[1] / l; v[2] = v[2] / l;
  };
  nrm(b1);
  float b2[3] = {b1[1] * n[2] - b1[2] * n[1], b1[2] * n[0] - b1[0] * n[2], b1[0] * n[1] - b1[1] * n[0]};
  nrm(b2);
  p.n = f3{n[0], n[1], n[2]};
  p.off = offset;
  p.b1 = f3{b1[0], b1[1], b1[2]};
  p.b2 = f3{b2[0], b2[1], b2[2]};
  return RT_OK;
}

int rt_scene_kind(const rt_scene *s) { return s ? s->kind : RT_E_INVALID; }
int64_t rt_scene_device_bytes(const rt_scene *s) { return s ? s->dev_bytes : 0; }

int rt_scene_bvh_stats(const rt_scene *s, int64_t *nodes, int64_t *inner, int32_t *max_depth) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  if (s->kind != RT_SCENE_MESH && s->kind != RT_SCENE_OCTREE) return set_err(RT_E_STATE, "not a tree scene");
  if (nodes) *nodes = s->host_nodes;
  if (inner) *inner = s->host_inner;
  if (max_depth) *max_depth = s->kind == RT_SCENE_MESH ? s->bvh_depth : s->oct_depth;
  return RT_OK;
}

int rt_scene_destroy(rt_scene *s) {
  if (!s) return RT_OK;
  int prev = 0;
  HIP_NOTE(hipGetDevice(&prev));
  HIP_NOTE(hipSetDevice(s->device));
  // the scene's own copy/render streams drain before anything they may still
  // read or write is freed (rt_render returns only after both, but a failed
  // call or a caller-stream launch may not have)
  for (hipStream_t x : s->xs)
    if (x) HIP_NOTE(hipStreamSynchronize(x));
  if (s->sched_os) HIP_NOTE(hipStreamSynchronize(s->sched_os));
  void *ptrs[] = {s->d_nodes, s->d_tris, s->d_vals, s->d_child, s->d_ovals, s->d_color, s->d_t,
                  s->d_cost[0], s->d_order[0], s->d_cost[1], s->d_order[1]};
  for (void *p : ptrs)
    if (p) HIP_NOTE(hipFree(p));
  for (hipEvent_t e : s->ord_ev)
    if (e) HIP_NOTE(hipEventDestroy(e));
  if (s->frame_ev) HIP_NOTE(hipEventDestroy(s->frame_ev));
  if (s->sched_os) {
    rterr::stream_remove(s->sched_os);
    HIP_NOTE(hipStreamDestroy(s->sched_os));
  }
  if (s->ev0) HIP_NOTE(hipEventDestroy(s->ev0));
  if (s->ev1) HIP_NOTE(hipEventDestroy(s->ev1));
  if (s->ev_host) HIP_NOTE(hipEventDestroy(s->ev_host));
  if (s->xev) HIP_NOTE(hipEventDestroy(s->xev));
  if (s->d_hit_box) HIP_NOTE(hipFree(s->d_hit_box));
  if (s->h_hit_box) HIP_NOTE(hipHostFree(s->h_hit_box));
  if (s->d_row_span) HIP_NOTE(hipFree(s->d_row_span));
  if (s->h_row_span) HIP_NOTE(hipHostFree(s->h_row_span));
  stage_free(s);
  for (hipStream_t x : s->xs)
    if (x) {
      rterr::stream_remove(x);
      HIP_NOTE(hipStreamDestroy(x));
    }
  HIP_NOTE(hipSetDevice(prev));
  delete s;
  return RT_OK;
}

int64_t rt_tile_pixels(int32_t W, int32_t H, const rt_tile *tile) {
  if (W <= 0 || H <= 0) return 0;
  if (!tile || tile->num_ranks <= 1) return (int64_t)W * H;
  if (tile->band_rows <= 0) return 0;
  int64_t rows = 0;
  const int32_t nb = (H + tile->band_rows - 1) / tile->band_rows;
  for (int32_t b = tile->rank; b < nb; b += tile->num_ranks)
    rows += std::min(tile->band_rows, H - b * tile->band_rows);
  return rows * W;
}

int rt_render_device(rt_scene *s, const rt_render_params *p, uint32_t *d_color, float *d_t, int32_t W,
                     int32_t H, uint32_t flags, const rt_tile *tile, void *stream) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  int rc = check_params(p, W, H);
  if (rc) return rc;
  if (!d_color || !d_t) return set_err(RT_E_INVALID, "NULL framebuffer");
  FrameArgs fa;
  if ((rc = fill_frame(fa, p, d_color, d_t, W, H, flags, tile))) return rc;
  if (fa.rows_local <= 0) return RT_OK;
  return launch_render(s, fa, (hipStream_t)stream);
}

int rt_render_device_frames(rt_scene *s, const rt_render_params *params, int32_t frames,
                            uint32_t *const *d_color, float *const *d_t, int32_t W, int32_t H,
                            uint32_t flags, const rt_tile *tile, void *stream) {
  if (!s || !params || !d_color || !d_t || frames < 0) return set_err(RT_E_INVALID, "bad arguments");
  if (frames == 1) return rt_render_device(s, params, d_color[0], d_t[0], W, H, flags, tile, stream);
  FrameBatch fb;
  for (int32_t f0 = 0; f0 < frames; f0 += kMaxBatch) {
    const int n = std::min<int32_t>(kMaxBatch, frames - f0);
    for (int i = 0; i < n; ++i) {
      int rc = check_params(params + f0 + i, W, H);
      if (rc) return rc;
      if (!d_color[f0 + i] || !d_t[f0 + i]) return set_err(RT_E_INVALID, "NULL framebuffer");
      if ((rc = fill_frame(fb.f[i], params + f0 + i, d_color[f0 + i], d_t[f0 + i], W, H, flags, tile)))
        return rc;
    }
    if (fb.f[0].rows_local <= 0) return RT_OK;
    const int rc = launch_batch(s, fb, n, (hipStream_t)stream);
    if (rc) return rc;
  }
  return RT_OK;
}

int rt_clear_device(uint32_t *d_color, float *d_t, int64_t n, void *stream) {
  if (!d_color || !d_t || n < 0) return set_err(RT_E_INVALID, "bad arguments");
  if (((uintptr_t)d_color | (uintptr_t)d_t) & 15) return set_err(RT_E_INVALID, "buffers must be 16-byte aligned");
  if (n == 0) return RT_OK;
  const int64_t lanes = (n + 3) / 4;
  clear_kernel<<<(unsigned)((lanes + 255) / 256), 256, 0, (hipStream_t)stream>>>(d_color, d_t, n);
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

int rt_stream_prepare(void *stream) {
  uint32_t *heads = nullptr;
  return stream_queue((hipStream_t)stream, &heads);
}

int rt_stream_release(void *stream) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  uint32_t *p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_queue_mu);
    auto b = g_band_sched.find({dev, (hipStream_t)stream});
    if (b != g_band_sched.end()) {  // the band order state (band_sched), freed in stream order too
      if (b->second.cost) HIP_NOTE(hipFreeAsync(b->second.cost, (hipStream_t)stream));
      if (b->second.order) HIP_NOTE(hipFreeAsync(b->second.order, (hipStream_t)stream));
      g_band_sched.erase(b);
    }
    auto it = g_queues.find({dev, (hipStream_t)stream});
    if (it == g_queues.end()) return RT_OK;
    p = it->second;
    g_queues.erase(it);
  }
  HIP_TRY(hipFreeAsync(p, (hipStream_t)stream));
  return RT_OK;
}

// Exchange slots: uncached device memory, so stores arriving from a peer GPU
// over xGMI are never shadowed by stale lines in this GPU's L2.
int rt_exchange_alloc(int64_t bytes, void **d_ptr) {
  if (!d_ptr || bytes <= 0) return set_err(RT_E_INVALID, "bad arguments");
  *d_ptr = nullptr;
  HIP_TRY(hipExtMallocWithFlags(d_ptr, (size_t)bytes, hipDeviceMallocUncached));
  return RT_OK;
}

int rt_exchange_free(void *d_ptr) {
  if (d_ptr) HIP_TRY(hipFree(d_ptr));
  return RT_OK;
}

int rt_ipc_get_handle(void *d_ptr, uint8_t handle[RT_IPC_HANDLE_BYTES]) {
  static_assert(sizeof(hipIpcMemHandle_t) == RT_IPC_HANDLE_BYTES, "IPC handle size");
  if (!d_ptr || !handle) return set_err(RT_E_INVALID, "bad arguments");
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, d_ptr));
  std::memcpy(handle, &h, sizeof h);
  return RT_OK;
}

int rt_ipc_open(const uint8_t handle[RT_IPC_HANDLE_BYTES], void **d_ptr) {
  if (!d_ptr || !handle) return set_err(RT_E_INVALID, "bad arguments");
  *d_ptr = nullptr;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  HIP_TRY(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
  return RT_OK;
}

int rt_ipc_close(void *d_ptr) {
  if (d_ptr) HIP_TRY(hipIpcCloseMemHandle(d_ptr));
  return RT_OK;
}

// rt_render's failure injection (rtx_render_inject_failure): the next n calls
// fail after their uploads were issued; g_render_drains counts the returns that
// waited for both copy streams (rtx_render_drain_count)
std::atomic<int> g_render_fault{0};
std::atomic<int64_t> g_render_drains{0};

namespace {

using rtdma::pinned_device_ptr;

// RTAMD_DROPIN_ZC=0: rt_render's cleared frames take the device frame + boxed
// download instead of the zero-copy path (A/B switch)
bool dropin_zero_copy() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_DROPIN_ZC");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool dropin_trace() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_DROPIN_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

// The pageable drop-in's staging spans reset by the host threads that copy
// them; RTAMD_HOST_CLEAR=0: by clear_spans_kernel instead (A/B switch).
bool host_clears_stage() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_HOST_CLEAR");
    return !(e && e[0] == '0');
  }();
  return on;
}

// System-scope stores into host frames (kFlagHostFrame); RTAMD_HOST_STORES=agent
// turns them off (A/B switch).
bool host_sys_stores() {
  static const bool on = [] {
    const char *e = ab_env("RTAMD_HOST_STORES");
    return !(e && std::strcmp(e, "agent") == 0);
  }();
  return on;
}

// rt_render of a cleared frame (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY: the app's
// frameBuf.clear() + draw, src/main.cpp:197,203): only hit pixels differ from
// the caller's buffers (raytracing.cpp:91-94), and the kernel stores exactly
// those -- into HOST memory (zero-copy), so no download follows the kernel:
//  * buffers pinned by rt_host_pin: the hits go straight into them;
//  * pageable buffers: into the scene's pinned staging frame, which is kept
//    cleared. The kernel records, per row, the span of the pixels it stored
//    (kFlagRowSpan); box_out_kernel moves the spans to mapped host memory, the
//    host copies just those spans to the caller's buffers (OpenMP rows) and
//    resets them in the staging frame as it goes (RTAMD_HOST_CLEAR=0: the
//    GPU does, clear_spans_kernel, in stream order before the next frame).
int render_cleared_zero_copy(rt_scene *s, FrameArgs fa, uint32_t *color, float *t, int32_t W, int32_t H,
                             float *ms) {
  const size_t px = (size_t)W * H;
  hipStream_t a = s->xs[0];
  rterr::stream_mark(a, "rt_render (zero-copy cleared frame)");
  // every return waits for stream a while it may still touch the caller's
  // buffers; the span-word reset (below) is the library's own and
  // is left running when the call returns
  struct Drain {
    hipStream_t a;
    bool on = true;
    ~Drain() {
      if (on && hipStreamSynchronize(a) == hipSuccess) g_render_drains.fetch_add(1);
    }
  } drain{a};
  void *dc = pinned_device_ptr(color, px * 4), *dt = pinned_device_ptr(t, px * 4);
  fa.flags |= RT_FLAG_HITS_ONLY | (host_sys_stores() ? kFlagHostFrame : 0u);
  fa.hit_box = nullptr;
  if (dc && dt) {
    fa.color = (uint32_t *)dc;
    fa.t = (float *)dt;
    if (g_render_fault.load() > 0) {
      g_render_fault.fetch_sub(1);
      return set_err(RT_E_DEVICE, "injected rt_render failure (rtx_render_inject_failure)");
    }
    HIP_TRY(hipEventRecord(s->ev0, a));
    // (the frame's tile-order kernel runs on the schedule's side stream: not waited for)
    if (int rc = launch_render(s, fa, a)) return rc;
    HIP_TRY(hipEventRecord(s->ev1, a));
    HIP_TRY(hipEventSynchronize(s->ev1));
    drain.on = false;
    if (ms) HIP_TRY(hipEventElapsedTime(ms, s->ev0, s->ev1));
    return RT_OK;
  }
  if (int rc = ensure_stage(s, px)) return rc;
  void *sc = nullptr, *st = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&sc, s->stage_c, 0));
  HIP_TRY(hipHostGetDevicePointer(&st, s->stage_t, 0));
  if (H > s->span_cap) {
    HIP_TRY(hipStreamSynchronize(a));  // (the previous frame's span clear reads d_row_span)
    if (s->d_row_span) HIP_NOTE(hipFree(s->d_row_span));
    if (s->h_row_span) HIP_NOTE(hipHostFree(s->h_row_span));
    s->d_row_span = s->h_row_span = s->h_row_span_dev = nullptr;
    s->span_cap = 0;
    HIP_TRY(hipMalloc(&s->d_row_span, (size_t)H * 2 * sizeof(int32_t)));
    HIP_TRY(hipHostMalloc(&s->h_row_span, (size_t)H * 2 * sizeof(int32_t), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void **)&s->h_row_span_dev, s->h_row_span, 0));
    s->span_cap = H;
    s->stage_dirty = true;  // (the spans of the frame in the staging frame are gone)
  }
  if (s->stage_dirty || s->stage_W != W || s->stage_H != H) {
    // (otherwise the previous frame's span reset left both the staging
    // frame and the span words reset)
    rth::clear_frame(s->stage_c, s->stage_t, (int64_t)px, 8);
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->d_row_span, 0x7FFFFFFF, (size_t)H * 2, a));
    s->stage_W = W;
    s->stage_H = H;
    s->stage_dirty = false;
  }
  fa.color = (uint32_t *)sc;
  fa.t = (float *)st;
  fa.hit_box = s->d_row_span;
  fa.flags |= kFlagRowSpan;
  if (g_render_fault.load() > 0) {
    g_render_fault.fetch_sub(1);
    return set_err(RT_E_DEVICE, "injected rt_render failure (rtx_render_inject_failure)");
  }
  const auto h0 = std::chrono::steady_clock::now();
  HIP_TRY(hipEventRecord(s->ev0, a));
  s->stage_dirty = true;  // until its spans are cleared again below
  if (int rc = launch_render(s, fa, a)) return rc;
  HIP_TRY(hipEventRecord(s->ev1, a));
  box_out_kernel<<<(unsigned)((2 * H + 255) / 256), 256, 0, a>>>(s->d_row_span, s->h_row_span_dev, 2 * H);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(s->ev_host, a));
  const auto h1 = std::chrono::steady_clock::now();
  HIP_TRY(hipEventSynchronize(s->ev_host));
  const auto h2 = std::chrono::steady_clock::now();
  if (ms) HIP_TRY(hipEventElapsedTime(ms, s->ev0, s->ev1));
  // the stored spans to the caller (host threads; every other pixel of the
  // caller's cleared frame already holds the staging frame's 0 / +inf); the
  // host resets the same spans of the staging frame as it goes (the GPU only
  // stores into it, from the next call on), and the span words are reset in
  // stream order before the next frame's kernel; the call does not wait for that
  const bool host_clear = host_clears_stage();
  rth::copy_spans(color, t, s->stage_c, s->stage_t, W, H, s->h_row_span, 0, host_clear);
  const auto h3 = std::chrono::steady_clock::now();
  drain.on = false;
  if (host_clear) {
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->d_row_span, 0x7FFFFFFF, (size_t)H * 2, a));
  } else {
    clear_spans_kernel<<<(unsigned)H, 256, 0, a>>>((uint32_t *)sc, (float *)st, s->d_row_span, W);
    HIP_TRY(hipGetLastError());
  }
  s->stage_dirty = false;
  if (dropin_trace()) {  // RTAMD_DROPIN_TRACE=1: host-side phases of this call (dev switch)
    const auto h4 = std::chrono::steady_clock::now();
    auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
    int64_t pxs = 0;
    for (int32_t y = 0; y < H; ++y)
      if (s->h_row_span[2 * y] <= -s->h_row_span[2 * y + 1]) pxs += -s->h_row_span[2 * y + 1] - s->h_row_span[2 * y] + 1;
    std::fprintf(stderr, "dropin: issue %.1f, wait %.1f, copy %.1f (%lld px), clear issue %.1f us; kernel %.1f us\n",
                 us(h0, h1), us(h1, h2), us(h2, h3), (long long)pxs, us(h3, h4), ms ? *ms * 1e3 : -1.0);
  }
  return RT_OK;
}

}  // namespace

int rt_render(rt_scene *s, const rt_render_params *p, uint32_t *color, float *t, int32_t W, int32_t H,
              uint32_t flags, float *ms) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  int rc = check_params(p, W, H);
  if (rc) return rc;
  if (!color || !t) return set_err(RT_E_INVALID, "NULL framebuffer");
  if (flags & RT_FLAG_TILE_NATURAL) return set_err(RT_E_INVALID, "rt_render renders whole frames (no tile)");
  // every argument is checked before the first copy is queued
  FrameArgs fa;
  if ((rc = fill_frame(fa, p, nullptr, nullptr, W, H, flags & ~RT_FLAG_HITS_ONLY, nullptr))) return rc;
  const size_t px = (size_t)W * H;
  if (flags == (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY) && dropin_zero_copy()) {
    if ((rc = ensure_events(s)) || (rc = ensure_copy_streams(s))) return rc;
    return render_cleared_zero_copy(s, fa, color, t, W, H, ms);
  }
  if ((rc = ensure_fb(s, px)) || (rc = ensure_events(s)) || (rc = ensure_copy_streams(s))) return rc;
  fa.color = s->d_color;
  fa.t = s->d_t;
  // The DMA engines only ever see pinned memory (rtdma):
  // buffers pinned by rt_host_pin are copied directly; pageable ones go through
  // the scene's staging frame, host threads copying between it and the caller's
  // buffers on the host side of each DMA (hc / ht: where the DMAs read / write).
  const bool direct = rtdma::pinned(color, px * 4) && rtdma::pinned(t, px * 4);
  if (!direct && (rc = ensure_stage(s, px))) return rc;
  uint32_t *hc = direct ? color : s->stage_c;
  float *ht = direct ? t : s->stage_t;
  // colour and t move on two streams (two DMA engines, concurrent). Once a copy
  // is queued, every return -- an error included -- first waits for both
  // streams, so the caller may unpin or free its buffers as soon as the call
  // returns.
  hipStream_t a = s->xs[0], b = s->xs[1];
  rterr::stream_mark(a, "rt_render (render + colour copies)");
  rterr::stream_mark(b, "rt_render (t copies)");
  struct Drain {
    hipStream_t a, b;
    ~Drain() {
      const hipError_t ea = hipStreamSynchronize(a), eb = hipStreamSynchronize(b);
      if (ea == hipSuccess && eb == hipSuccess) g_render_drains.fetch_add(1);
    }
  } drain{a, b};
  // Which pixels can differ from the caller's buffers after the frame:
  //  * RT_FLAG_CLEAR: every pixel (misses become 0 / +inf), so all are copied back;
  //  * RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY: the caller's buffers already hold a
  //    cleared frame (the app's frameBuf.clear() + draw, src/main.cpp:197,203),
  //    so only stored hits differ (raytracing.cpp:91-94);
  //  * no flag (tPrev frame): colour and t are written only on hit, so again
  //    only stored hits differ.
  // In the last two cases the kernel records the bounding box of its stored
  // pixels and only that box is copied back. The device frame is always
  // written whole (a cleared frame) or uploaded whole (tPrev), so the box
  // holds exactly the caller's values outside the hits.
  const bool boxed = !(flags & RT_FLAG_CLEAR) || (flags & RT_FLAG_HITS_ONLY);
  if (!direct) s->stage_dirty = true;  // (the zero-copy path's cleared staging frame is overwritten)
  if (!(flags & RT_FLAG_CLEAR)) {
    if (!direct) rth::copy_rect(hc, ht, color, t, W, 0, W - 1, 0, H - 1, 0);
    HIP_TRY(hipMemcpyAsync(s->d_color, hc, px * 4, hipMemcpyHostToDevice, a));
    HIP_TRY(hipMemcpyAsync(s->d_t, ht, px * 4, hipMemcpyHostToDevice, b));
    HIP_TRY(hipEventRecord(s->xev, b));
    HIP_TRY(hipStreamWaitEvent(a, s->xev, 0));
  }
  if (g_render_fault.load() > 0) {
    g_render_fault.fetch_sub(1);
    return set_err(RT_E_DEVICE, "injected rt_render failure (rtx_render_inject_failure)");
  }
  if (boxed) {
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)s->d_hit_box, 0x7FFFFFFF, 4, a));
    fa.hit_box = s->d_hit_box;
  }
  HIP_TRY(hipEventRecord(s->ev0, a));
  if ((rc = launch_render(s, fa, a))) return rc;
  HIP_TRY(hipEventRecord(s->ev1, a));
  int32_t x0 = 0, x1 = W - 1, y0 = 0, y1 = H - 1;  // the region copied back
  if (!boxed) {
    HIP_TRY(hipStreamWaitEvent(b, s->ev1, 0));
    HIP_TRY(hipMemcpyAsync(ht, s->d_t, px * 4, hipMemcpyDeviceToHost, b));
    HIP_TRY(hipMemcpyAsync(hc, s->d_color, px * 4, hipMemcpyDeviceToHost, a));
  } else {
    box_out_kernel<<<1, 64, 0, a>>>(s->d_hit_box, s->h_hit_box_dev, 4);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(a));
    x0 = s->h_hit_box[0], x1 = -s->h_hit_box[1], y0 = s->h_hit_box[2], y1 = -s->h_hit_box[3];
    if (x0 <= x1 && y0 <= y1) {  // else: no hit, nothing changed
      HIP_TRY(hipStreamWaitEvent(b, s->ev1, 0));
      const size_t off = (size_t)y0 * W + x0, rows = (size_t)(y1 - y0 + 1), w = (size_t)(x1 - x0 + 1);
      if (w * 2 > (size_t)W) {  // wide box: whole rows, one contiguous copy per buffer
        x0 = 0;
        x1 = W - 1;
        HIP_TRY(hipMemcpyAsync(ht + (size_t)y0 * W, s->d_t + (size_t)y0 * W, rows * W * 4, hipMemcpyDeviceToHost, b));
        HIP_TRY(hipMemcpyAsync(hc + (size_t)y0 * W, s->d_color + (size_t)y0 * W, rows * W * 4,
                               hipMemcpyDeviceToHost, a));
      } else {
        HIP_TRY(hipMemcpy2DAsync(ht + off, (size_t)W * 4, s->d_t + off, (size_t)W * 4, w * 4, rows,
                                 hipMemcpyDeviceToHost, b));
        HIP_TRY(hipMemcpy2DAsync(hc + off, (size_t)W * 4, s->d_color + off, (size_t)W * 4, w * 4, rows,
                                 hipMemcpyDeviceToHost, a));
      }
    }
  }
  HIP_TRY(hipStreamSynchronize(a));
  HIP_TRY(hipStreamSynchronize(b));
  if (!direct && x0 <= x1 && y0 <= y1) rth::copy_rect(color, t, hc, ht, W, x0, x1, y0, y1, 0);
  if (ms) HIP_TRY(hipEventElapsedTime(ms, s->ev0, s->ev1));
  return RT_OK;
}

// test hooks: fail the next n rt_render calls after their uploads; how many
// rt_render returns have waited for both copy streams
int rtx_render_inject_failure(int32_t n) {
  g_render_fault.store(n);
  return RT_OK;
}
int64_t rtx_render_drain_count(void) { return g_render_drains.load(); }

#ifndef RT_PIN_COARSE
#define RT_PIN_COARSE 1  // A/B switch: 0 registers caller ranges fine-grained (the HIP default)
#endif
int rt_host_pin(void *ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return set_err(RT_E_INVALID, "bad host range");
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.upper_bound((uintptr_t)ptr + (size_t)bytes - 1);
    if (it != g_pins.begin() && (--it)->first + it->second > (uintptr_t)ptr)
      return set_err(RT_E_INVALID, "rt_host_pin: the range overlaps a range pinned earlier and not unpinned "
                                   "(a buffer freed without rt_host_unpin?)");
  }
  // portable: mapped on every device (rt_multi_render's slots store into it).
  // Coarse-grained (RT_PIN_COARSE): the range is coherent with the host at
  // kernel and copy boundaries only -- which is all the library relies on: the
  // host reads or writes a pinned frame only after the stream that used it is
  // synchronised, and a dispatch's end-of-kernel release covers its stores --
  // so the GPU's stores into it are not snooped by the host's caches: the
  // zero-copy cleared frame's kernel (hits stored into the caller's pinned
  // buffers) ran 0.19-0.24 ms into a fine-grained registration against
  // ~0.18 into the library's own (coarse-grained) hipHostMalloc staging frame
  // (profiles/r06/pin_coarse_ab.txt)
  hipError_t e = hipHostRegister(ptr, (size_t)bytes,
                                 hipHostRegisterMapped | hipHostRegisterPortable | (RT_PIN_COARSE ? hipExtHostRegisterCoarseGrained : 0u));
  if (RT_PIN_COARSE && e == hipErrorInvalidValue) {  // (a runtime without the flag)
    (void)hipGetLastError();
    e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable);
  }
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    (void)hipGetLastError();
    return set_err(RT_E_INVALID, "rt_host_pin: the HIP runtime already holds a registration over this range "
                                 "(registered outside librtamd, or freed without unregistering)");
  }
  HIP_TRY(e);
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pins[(uintptr_t)ptr] = (size_t)bytes;
  return RT_OK;
}

int rt_host_unpin(void *ptr) {
  if (!ptr) return set_err(RT_E_INVALID, "NULL pointer");
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (!g_pins.erase((uintptr_t)ptr)) return set_err(RT_E_INVALID, "rt_host_unpin: not a range pinned by rt_host_pin");
  }
  // no library stream may still read or write the range when it is unregistered
  // (every entry point drains its streams before returning; a failed call or a
  // stream-ordered launch may not have)
  if (const hipError_t e = rterr::streams_sync())
    return set_err(RT_E_DEVICE, rterr::hip_fail("rt_host_unpin: draining the library's streams", e));
  HIP_TRY(hipHostUnregister(ptr));
  return RT_OK;
}

int rt_untile_device(const uint32_t *d_packed_color, const float *d_packed_t, int64_t per_rank_pixels,
                     uint32_t *d_color, float *d_t, int32_t W, int32_t H, const rt_tile *tile,
                     void *stream) {
  if (!tile || tile->num_ranks < 1 || tile->band_rows <= 0 || W <= 0 || H <= 0)
    return set_err(RT_E_INVALID, "bad tile");
  const int64_t n = (int64_t)W * H;
  untile_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      d_packed_color, d_packed_t, per_rank_pixels, d_color, d_t, W, H, tile->band_rows, tile->num_ranks);
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

int rt_intersect_rays(rt_scene *s, const float *o, const float *d, int64_t n, float tnear, float tfar,
                      int32_t *hit, float *t, float *normal, int64_t *prim) {
  if (!s || !o || !d || !hit || !t || !normal || !prim) return set_err(RT_E_INVALID, "NULL argument");
  if (n <= 0) return RT_OK;
  float *dO = nullptr, *dD = nullptr, *dT = nullptr, *dN = nullptr;
  int32_t *dH = nullptr;
  int64_t *dP = nullptr;
  auto cleanup = [&]() {
    void *ps[] = {dO, dD, dT, dN, dH, dP};
    for (void *q : ps)
      if (q) HIP_NOTE(hipFree(q));
  };
  hipError_t e = hipSuccess;
  do {
    if ((e = hipMalloc(&dO, n * 12)) || (e = hipMalloc(&dD, n * 12)) || (e = hipMalloc(&dT, n * 4)) ||
        (e = hipMalloc(&dN, n * 12)) || (e = hipMalloc(&dH, n * 4)) || (e = hipMalloc(&dP, n * 8)))
      break;
    if ((e = rtdma::h2d(dO, o, n * 12, nullptr)) || (e = rtdma::h2d(dD, d, n * 12, nullptr))) break;
    if (s->kind == RT_SCENE_MESH) {
      MeshS sc{mesh_dev(s)};
      switch (s->maxd) {
        case 4: launch_rays_t<MeshS, 4>(sc, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        case 7: launch_rays_t<MeshS, 7>(sc, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        case 15: launch_rays_t<MeshS, 15>(sc, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        default: launch_rays_t<MeshS, 31>(sc, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
      }
    } else if (s->kind == RT_SCENE_GRID) {
      const GridDev gd = grid_dev(s);
      switch (grid_mode(s, gd)) {
        case kGridBuf | kGridBricked:
          launch_rays_t<GridS<kGridBuf | kGridBricked>, 1>({gd}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP);
          break;
        case kGridBricked:
          launch_rays_t<GridS<kGridBricked>, 1>({gd}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP);
          break;
        default: launch_rays_t<GridS<kGridBuf>, 1>({gd}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
      }
    } else {
      const OctDev od{s->d_child, s->d_ovals};
      switch (s->maxd) {
        case 4: launch_rays_t<OctS<true>, 4>(OctS<true>{od}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        case 7: launch_rays_t<OctS<true>, 7>(OctS<true>{od}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        case 15: launch_rays_t<OctS<false>, 15>(OctS<false>{od}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
        default: launch_rays_t<OctS<false>, 31>(OctS<false>{od}, s->plane, dO, dD, n, tnear, tfar, dH, dT, dN, dP); break;
      }
    }
    if ((e = hipGetLastError())) break;
    if ((e = rtdma::d2h(hit, dH, n * 4, nullptr)) || (e = rtdma::d2h(t, dT, n * 4, nullptr)) ||
        (e = rtdma::d2h(normal, dN, n * 12, nullptr)) || (e = rtdma::d2h(prim, dP, n * 8, nullptr)))
      break;
  } while (0);
  cleanup();
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("rt_intersect_rays: ") + hipGetErrorString(e));
  return RT_OK;
}

int rt_count_work(rt_scene *s, const rt_render_params *params, int32_t frames, int32_t W, int32_t H,
                  uint32_t flags, const rt_tile *tile, int64_t counters[9]) {
  if (!s || !params || frames <= 0 || !counters) return set_err(RT_E_INVALID, "bad arguments");
  int rc = check_params(params, W, H);
  if (rc) return rc;
  const size_t px = (size_t)W * H;
  if ((rc = ensure_fb(s, px))) return rc;
  unsigned long long *d = nullptr;
  HIP_TRY(hipMalloc(&d, C_NUM * sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, C_NUM * sizeof(unsigned long long));
  if (e == hipSuccess) HIP_NOTE(hipMemset(s->d_t, 0x7f, px * 4));
  for (int32_t f = 0; f < frames && e == hipSuccess && rc == RT_OK; ++f) {
    FrameArgs fa;
    if (!(rc = check_params(params + f, W, H)) &&
        !(rc = fill_frame(fa, params + f, s->d_color, s->d_t, W, H, flags, tile)))
      rc = launch_render(s, fa, 0, d, 1);
  }
  unsigned long long h[C_NUM] = {};
  if (e == hipSuccess && rc == RT_OK) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (rc) return rc;
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("rt_count_work: ") + hipGetErrorString(e));
  for (int i = 0; i < C_NUM; ++i) counters[i] = (int64_t)h[i];
  return RT_OK;
}

// Diagnostic (not part of include/rtamd.h): per-wave timestamps of one frame.
// out: 4 x u64 per wave (see DIAG == 2); *nwaves in/out: capacity / written.
int rtx_wave_stamps(rt_scene *s, const rt_render_params *params, int32_t W, int32_t H, uint32_t flags,
                    uint64_t *out, int64_t *nwaves) {
  if (!s || !params || !out || !nwaves) return set_err(RT_E_INVALID, "bad arguments");
  int rc = check_params(params, W, H);
  if (rc) return rc;
  const int64_t nb = (int64_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
  const int64_t nw = nb * (kBlock / 64);
  if (*nwaves < nw) { *nwaves = nw; return set_err(RT_E_INVALID, "buffer too small"); }
  const size_t px = (size_t)W * H;
  if ((rc = ensure_fb(s, px))) return rc;
  unsigned long long *d = nullptr;
  HIP_TRY(hipMalloc(&d, nw * 4 * sizeof(unsigned long long)));
  FrameArgs fa;
  if (!(rc = fill_frame(fa, params, s->d_color, s->d_t, W, H, flags, nullptr)))
    rc = launch_render(s, fa, 0, d, 2);
  hipError_t e = rc ? hipSuccess : hipMemcpy(out, d, nw * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (rc) return rc;
  if (e != hipSuccess) return set_err(RT_E_DEVICE, hipGetErrorString(e));
  *nwaves = nw;
  return RT_OK;
}

// ---- orbit camera + image output (host-only; rt_host.cpp) ----------------
static_assert(sizeof(rt_camera_state) == sizeof(rth::CamState), "camera state layout");
#define CAM(c) (*reinterpret_cast<rth::CamState *>(c))
int rt_camera_init(const float pos[3], const float target[3], const float up[3], rt_camera_state *c) {
  if (!pos || !target || !up || !c) return set_err(RT_E_INVALID, "bad arguments");
  rth::cam_init(CAM(c), pos, target, up);
  return RT_OK;
}
int rt_camera_rotate(rt_camera_state *c, float dx, float dy) {
  if (!c) return set_err(RT_E_INVALID, "camera is NULL");
  rth::cam_rotate(CAM(c), dx, dy);
  return RT_OK;
}
int rt_camera_reset_position(rt_camera_state *c, const float pos[3]) {
  if (!c || !pos) return set_err(RT_E_INVALID, "bad arguments");
  rth::cam_reset_position(CAM(c), pos);
  return RT_OK;
}
int rt_camera_reset_target(rt_camera_state *c, const float target[3]) {
  if (!c || !target) return set_err(RT_E_INVALID, "bad arguments");
  rth::cam_reset_target(CAM(c), target);
  return RT_OK;
}
int rt_camera_set_lock_up(rt_camera_state *c, int on) {
  if (!c) return set_err(RT_E_INVALID, "camera is NULL");
  rth::cam_set_lock_up(CAM(c), on != 0);
  return RT_OK;
}
int rt_camera_zoom(rt_camera_state *c, float wheel) {
  if (!c) return set_err(RT_E_INVALID, "camera is NULL");
  rth::cam_zoom(CAM(c), wheel);
  return RT_OK;
}
int rt_camera_basis(const rt_camera_state *c, float up[3], float right[3], float forward[3]) {
  if (!c) return set_err(RT_E_INVALID, "camera is NULL");
  rth::cam_basis(*reinterpret_cast<const rth::CamState *>(c), up, right, forward);
  return RT_OK;
}
int rt_camera_view_inverse(const rt_camera_state *c, float view_inv[16]) {
  if (!c || !view_inv) return set_err(RT_E_INVALID, "bad arguments");
  rth::cam_view_inverse(*reinterpret_cast<const rth::CamState *>(c), view_inv);
  return RT_OK;
}
#undef CAM
int rt_write_png(const char *path, const uint32_t *color, int32_t W, int32_t H) {
  std::string err;
  if (!rth::write_png(path, color, W, H, err)) return set_err(RT_E_IO, err);
  return RT_OK;
}

int rt_save_obj(const char *path, const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx,
                const float *vnorm4, const float *vtex2) {
  std::string err;
  if (nverts < 0 || nidx < 0) return set_err(RT_E_INVALID, "bad counts");
  if (!rth::save_obj(path, vpos4, nverts, idx, nidx, vnorm4, vtex2, err))
    return set_err(err.rfind("cannot", 0) == 0 || err == "short write" ? RT_E_IO : RT_E_INVALID, err);
  return RT_OK;
}

// Diagnostic: primary ray directions as the render kernel computes them (host buffer [H][W][3]).
int rtx_eye_rays(const rt_render_params *p, int32_t W, int32_t H, float *out) {
  int rc = check_params(p, W, H);
  if (rc) return rc;
  float *d = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)W * H * 12));
  eye_rays_kernel<<<(W * H + 255) / 256, 256>>>(*p, W, H, d);
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, d, (size_t)W * H * 12, hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, hipGetErrorString(e));
  return RT_OK;
}

// Diagnostic: run the 8-lane group primitives on n vectors of 8 keys (host buffers).
int rtx_grp_test(const float *keys, int32_t n, float *st, uint32_t *sid, float *mt, uint32_t *mk,
                 uint32_t *orv) {
  if (n <= 0) return set_err(RT_E_INVALID, "n must be positive");
  float *dk = nullptr, *dst = nullptr, *dmt = nullptr;
  uint32_t *dsid = nullptr, *dmk = nullptr, *dor = nullptr;
  const size_t n8 = (size_t)n * 8;
  HIP_TRY(hipMalloc(&dk, n8 * 4));
  HIP_TRY(hipMalloc(&dst, n8 * 4));
  HIP_TRY(hipMalloc(&dsid, n8 * 4));
  HIP_TRY(hipMalloc(&dmt, (size_t)n * 4));
  HIP_TRY(hipMalloc(&dmk, (size_t)n * 4));
  HIP_TRY(hipMalloc(&dor, (size_t)n * 4));
  HIP_TRY(hipMemcpy(dk, keys, n8 * 4, hipMemcpyHostToDevice));
  grp_test_kernel<<<(unsigned)((n8 + 63) / 64), 64>>>(dk, n, dst, dsid, dmt, dmk, dor);
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(st, dst, n8 * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(sid, dsid, n8 * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(mt, dmt, (size_t)n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(mk, dmk, (size_t)n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(orv, dor, (size_t)n * 4, hipMemcpyDeviceToHost);
  for (void *q : {(void *)dk, (void *)dst, (void *)dsid, (void *)dmt, (void *)dmk, (void *)dor}) HIP_NOTE(hipFree(q));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, hipGetErrorString(e));
  return RT_OK;
}

// Row bands with at least this many pixels per frame take the work queue
// (band_takes_queue); < 0 restores the default threshold.
int rtx_set_band_queue_px(int64_t px) {
  g_band_queue_px.store(px < 0 ? (int64_t)1000000 : px);
  return RT_OK;
}

// The pageable drop-in's host copy (rth::copy_spans) on caller arrays, no GPU:
// span[2y] = first stored column of row y, span[2y+1] = -last (INT32_MAX,
// INT32_MAX: none); threads 0 = the library's default; clear_src != 0: the
// copied spans of the source reset to (0, +inf). Not part of include/rtamd.h.
int rtx_copy_spans(uint32_t *dc, float *dt, uint32_t *sc, float *st, int64_t W, int32_t H, const int32_t *span,
                   int32_t threads, int32_t clear_src) {
  if (!dc || !dt || !sc || !st || !span || W <= 0 || H <= 0) return set_err(RT_E_INVALID, "bad arguments");
  rth::copy_spans(dc, dt, sc, st, W, H, span, threads, clear_src != 0);
  return RT_OK;
}

// Exhaustive check of rtm::rcp_rn (rt_rcp.h, tri_t's reciprocal) on this
// device: every float x with 1e-8 <= |x| < 2^126 against the IEEE division
// 1 / x. *checked = floats in that range, *bad = mismatches, *first_bad = the
// bits of one mismatching x (0 if none). Not part of include/rtamd.h.
int rtx_rcp_check(uint64_t *checked, uint64_t *bad, uint32_t *first_bad) {
  if (!checked || !bad || !first_bad) return set_err(RT_E_INVALID, "NULL argument");
  unsigned long long *d = nullptr;
  HIP_TRY(hipMalloc(&d, 3 * sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, 3 * sizeof(unsigned long long));
  const uint32_t block = 256, chunk = 1u << 28;  // 2^28 bit patterns per launch
  for (uint64_t base = 0; e == hipSuccess && base < (1ull << 32); base += chunk) {
    rcp_check_kernel<<<chunk / block, block>>>((uint32_t)base, d);
    e = hipGetLastError();
  }
  unsigned long long h[3] = {0, 0, 0};
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("rcp check: ") + hipGetErrorString(e));
  *checked = h[0];
  *bad = h[1];
  *first_bad = (uint32_t)h[2];
  return RT_OK;
}

// Diagnostic (bench.py's PMC calibration, tools/prof_frames.py): one pass of
// calib_read_kernel over `bytes` of device memory, every byte loaded once
// (`width` = 4 or 16 bytes per lane, consecutive lanes on consecutive
// addresses), so the vector L1 misses every line exactly once and the
// dispatch's TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES counts give the bytes
// per L1->L2 read request and per L1 access on gfx950. Not part of rtamd.h.
int rtx_calib_read(int64_t bytes, int32_t width, uint32_t *sink) {
  if (bytes <= 0 || (width != 4 && width != 16) || bytes % 1024) return set_err(RT_E_INVALID, "bad arguments");
  void *d = nullptr;
  uint32_t *o = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)bytes));
  hipError_t e = hipMalloc(&o, 4);
  if (e == hipSuccess) e = hipMemset(d, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipMemset(o, 0, 4);
  if (e == hipSuccess) {
    const int64_t n = bytes / width;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    if (width == 16)
      calib_read_kernel<uint4><<<blocks, 256>>>((const uint4 *)d, n, o);
    else
      calib_read_kernel<uint32_t><<<blocks, 256>>>((const uint32_t *)d, n, o);
    e = hipGetLastError();
  }
  uint32_t h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (o) HIP_NOTE(hipFree(o));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("calib read: ") + hipGetErrorString(e));
  if (sink) *sink = h;
  return RT_OK;
}

// fast_eye_ok for tests (host only): 1 when a W x H frame with this inverse
// projection takes eye_ray_fast. Not part of include/rtamd.h.
int rtx_fast_eye_ok(const float *proj_inv, int32_t W, int32_t H) {
  return proj_inv && fast_eye_ok(proj_inv, W, H) ? 1 : 0;
}

// The checks behind rtm::div_mk on this device (div_check_kernel's modes; n:
// pairs for mode 1). out[0] = checked, out[1] = mismatches, out[2] = one
// mismatching pair's bits. Not part of include/rtamd.h.
int rtx_div_check(int32_t mode, uint64_t n, uint64_t seed, uint64_t out[3]) {
  if (!out || mode < 0 || mode > 1) return set_err(RT_E_INVALID, "bad arguments");
  unsigned long long *d = nullptr;
  HIP_TRY(hipMalloc(&d, 3 * sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, 3 * sizeof(unsigned long long));
  const uint32_t block = 256;
  if (e == hipSuccess && mode == 0) {
    div_check_kernel<<<dim3(1, 32768), block>>>(0, 0, seed, d);
    e = hipGetLastError();
  } else if (e == hipSuccess) {
    const uint64_t chunk = 1ull << 28;
    for (uint64_t b0 = 0; e == hipSuccess && b0 < n; b0 += chunk) {
      const uint64_t m = std::min(chunk, n - b0);
      div_check_kernel<<<(unsigned)((m + block - 1) / block), block>>>(mode, b0, seed, d);
      e = hipGetLastError();
    }
  }
  unsigned long long h[3] = {0, 0, 0};
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  HIP_NOTE(hipFree(d));
  if (e != hipSuccess) return set_err(RT_E_DEVICE, std::string("div check: ") + hipGetErrorString(e));
  for (int i = 0; i < 3; ++i) out[i] = h[i];
  return RT_OK;
}

// Heavy-first band order on (1) / off (0) from now on; < 0 restores the
// RTAMD_BAND_ORDER setting. Not part of include/rtamd.h.
int rtx_set_band_order(int on) {
  g_band_order.store(on < 0 ? band_order_env() : (on != 0));
  return RT_OK;
}

// Builder of this thread's last BVH: 1 host, 2 device, 3 host after a failed
// device build (AUTO mode falls back; see rtx_bvh_inject_failure)
int rtx_bvh_last_builder(void) { return t_bvh_last; }

// Diagnostic: persistent launches from now on write per-wave stamps (see
// PersistQ::stamps) into the device buffer d_buf of cap_waves x 8 u64
// (d_buf = NULL turns it off). Not part of include/rtamd.h.
int rtx_set_persist_stamps(void *d_buf, int64_t cap_waves) {
  g_persist_stamps = (unsigned long long *)d_buf;
  g_persist_stamps_cap = d_buf ? cap_waves : 0;
  return RT_OK;
}

// Diagnostic: force grid layouts / address paths (g_grid_force bits). Not part
// of include/rtamd.h.
int rtx_set_grid_force(int flags) {
  if (flags < 0 || flags > 3) return set_err(RT_E_INVALID, "grid force flags must be 0..3");
  g_grid_force = flags;
  return RT_OK;
}

// Diagnostic A/B switch: cooperative tail of the mesh primary path on (default) / off.
int rtx_set_coop(rt_scene *s, int on) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  s->coop = on != 0;
  return RT_OK;
}

// Diagnostic switch: primary-ray batches of this scene on the ray pump
// (render_pump_kernel) instead of one tile per wave (default off).

// the ray pump's refill threshold in lanes (1..64; other values: the default)
int rtx_set_refill(int32_t lanes) {
  g_refill.store((lanes >= 1 && lanes <= 64) ? lanes : RT_REFILL_MIN);
  return RT_OK;
}

int rtx_set_pump(rt_scene *s, int on) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  s->pump_on = on != 0;
  return RT_OK;
}

// Diagnostic A/B switch: cost-ordered block schedule on (default) / off.
int rtx_set_schedule(rt_scene *s, int on) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  s->sched_on = on != 0;
  s->sched_key[0] = s->sched_key[1] = 0;
  return RT_OK;
}

int rt_bench_frames(rt_scene *s, const rt_render_params *params, int32_t frames, int32_t W, int32_t H,
                    uint32_t flags, float *mean_ms, float *total_ms) {
  if (!s || !params || frames <= 0) return set_err(RT_E_INVALID, "bad arguments");
  int rc = check_params(params, W, H);
  if (rc) return rc;
  const size_t px = (size_t)W * H;
  if ((rc = ensure_fb(s, px)) || (rc = ensure_events(s))) return rc;
  HIP_TRY(hipMemset(s->d_t, 0x7f, px * 4));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipEventRecord(s->ev0, 0));
  for (int32_t f = 0; f < frames; ++f) {
    FrameArgs fa;
    if ((rc = check_params(params + f, W, H)) ||
        (rc = fill_frame(fa, params + f, s->d_color, s->d_t, W, H, flags, nullptr)) ||
        (rc = launch_render(s, fa, 0)))
      return rc;
  }
  HIP_TRY(hipEventRecord(s->ev1, 0));
  HIP_TRY(hipEventSynchronize(s->ev1));
  float ms = 0.0f;
  HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
  if (total_ms) *total_ms = ms;
  if (mean_ms) *mean_ms = ms / (float)frames;
  return RT_OK;
}

}  // extern "C"

// ------------------------------------------------ rt_multi_render internals --
namespace rti {
// One slot of rt_multi_render's zero-copy cleared frame (RT_FLAG_CLEAR |
// RT_FLAG_HITS_ONLY over a cleared host frame): the slot's bands of `tile` go
// through the one-frame kernel on `stream`, storing only their hits, at their
// own rows of the W x H host frame whose device addresses (on the scene's
// device) are dc / dt (kFlagNatural: one frame shared by every slot). With
// d_span != NULL the kernel records per LOCAL row (tile->rank's rows in
// increasing order) the span of the pixels it stored (kFlagRowSpan, 2 words per
// row, pre-set to INT32_MAX by the caller).
int render_band_host(rt_scene *s, const rt_render_params *p, uint32_t *dc, float *dt, int32_t W, int32_t H,
                     const rt_tile *tile, int32_t *d_span, hipStream_t stream) {
  if (!s) return set_err(RT_E_INVALID, "scene is NULL");
  if (int rc = check_params(p, W, H)) return rc;
  FrameArgs fa;
  if (int rc = fill_frame(fa, p, dc, dt, W, H, RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY, tile)) return rc;
  if (fa.rows_local <= 0) return RT_OK;
  fa.flags |= kFlagHostFrame | kFlagNatural | (d_span ? kFlagRowSpan : 0u);
  fa.hit_box = d_span;
  return launch_render(s, fa, stream);
}
}  // namespace rti
