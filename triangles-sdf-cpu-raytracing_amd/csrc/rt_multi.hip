// rt_multi.hip -- Renderer::draw over several GPUs of ONE process.
//
// The reference renders one frame per Renderer::draw call (src/main.cpp:
// 196-207) and splits it by image rows over OpenMP threads
// (src/raytracing.cpp:77-96). Here the rows go to GPUs: the scene is
// replicated on every device of the handle (rt_scene_replicate), the frame is
// cut into bands of band_rows rows, band b -> slot b mod n (rt_tile), each
// slot renders its bands PACKED on its own stream, and one gather per frame
// and buffer brings them to the root (slot 0), which de-interleaves them
// (rt_untile_device) into the frame. SURVEY.md 8(b): "the tile/row range for
// multi-GPU ... the call blocks until the gather completes"; 8(e): "single
// process, 8 devices, ncclCommInitAll", one ncclGather of the framebuffer
// bands to the root.
//
// The gather is RCCL's ncclGather over a communicator of all slots
// (ncclCommInitAll, one rank per slot, root = rank 0) when the devices are
// distinct; RCCL refuses a device twice in one communicator, so a device list
// with repeats (the one-GPU box runs {0, 0}) gathers with device-to-device
// copies instead (hipMemcpyPeerAsync on each slot's stream, the root waiting
// on each slot's event). Pixels are independent and every slot renders its
// bands with the single-device kernels, so an assembled frame is bitwise the
// single-device frame (tests/test_multi.py).
//
// Host buffers (rt_multi_render). The reference app's frame loop is
// frameBuf.clear(); draw() into host memory (src/main.cpp:196-207); that
// cleared frame (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY) takes no gather at all:
// every slot's kernel stores its bands' hits at their own rows straight into
// host memory, as rt_render's zero-copy path does on one device -- into the
// caller's buffers when rt_host_pin pinned them (portable: mapped on every
// device), else into the handle's pinned staging frame (kept cleared), whose
// per-row spans of stored pixels the host then copies to the caller. The other
// flags keep the device gather and move the caller's frame through the staging
// frame on pageable buffers: the DMA only ever sees pinned memory (DESIGN.md
// section 0e).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtamd.h"
#include "rt_error.h"
#include "rt_host.h"

namespace {

constexpr int32_t kChunk = 16;  // frames per slot launch (rt_render_device_frames' batch)

#define NCCL_TRY(expr)                                                                      \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess)                                                                  \
      return rterr::set(RT_E_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(r_));   \
  } while (0)

// restores the calling thread's HIP device on every return
struct DeviceGuard {
  int prev = 0;
  DeviceGuard() { HIP_NOTE(hipGetDevice(&prev)); }
  ~DeviceGuard() { HIP_NOTE(hipSetDevice(prev)); }
};

}  // namespace

struct rt_multi {
  rt_scene *root = nullptr;  // the caller's scene on dev[0] (not owned)
  int32_t n = 0, band_rows = 8;
  std::vector<int> dev;
  std::vector<rt_scene *> scene;  // per slot; [0] = root, the others owned replicas
  std::vector<hipStream_t> st;    // per slot, on its device
  std::vector<hipEvent_t> done;   // per slot: its bands have left for the root
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // root: first launch .. assembled frame
  hipEvent_t rc_free = nullptr;  // root: the last untile has read the receive buffers (peer copies wait)
  bool rccl = false;
  std::vector<ncclComm_t> comm;  // per slot (RCCL exchange)
  // buffers for frames of W x H, up to fcap frames per chunk
  int32_t W = 0, H = 0, fcap = 0;
  int64_t cap = 0;  // packed pixels of the slot with the most rows
  std::vector<uint32_t *> pc;  // per slot: fcap * cap
  std::vector<float *> pt;
  uint32_t *rc = nullptr;  // root: fcap * n * cap (slot i of frame f at (f * n + i) * cap)
  float *rt = nullptr;
  uint32_t *fc = nullptr;  // root: one assembled frame for the host path
  float *ft = nullptr;
  // host frames: the staging frame for pageable caller buffers (pinned, mapped
  // on every device; kept cleared between zero-copy cleared frames while
  // hs_dirty is false) and its address on each slot's device
  uint32_t *hs_c = nullptr;
  float *hs_t = nullptr;
  size_t hs_cap = 0;
  bool hs_dirty = true;
  std::vector<uint32_t *> hs_c_dev;
  std::vector<float *> hs_t_dev;
  // zero-copy cleared frames on the staging frame: per slot, the span of
  // stored pixels of each of its rows (2 words per local row, INT32_MAX when
  // none) on its device and in pinned host memory; span_rows = rows per slot
  std::vector<int32_t *> d_span, h_span;
  int32_t span_rows = 0;
  std::vector<int32_t> merged;  // the spans by image row
};

namespace {

rt_tile tile_of(const rt_multi *m, int32_t i) { return rt_tile{m->band_rows, i, m->n, 0}; }

void free_buffers(rt_multi *m) {
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_NOTE(hipSetDevice(m->dev[i]));
    if (m->st[i]) HIP_NOTE(hipStreamSynchronize(m->st[i]));
  }
  for (int32_t i = 0; i < (int32_t)m->pc.size(); ++i) {
    HIP_NOTE(hipSetDevice(m->dev[i]));
    if (m->pc[i]) HIP_NOTE(hipFree(m->pc[i]));
    if (m->pt[i]) HIP_NOTE(hipFree(m->pt[i]));
  }
  m->pc.assign(m->n, nullptr);
  m->pt.assign(m->n, nullptr);
  HIP_NOTE(hipSetDevice(m->dev[0]));
  for (void *p : {(void *)m->rc, (void *)m->rt, (void *)m->fc, (void *)m->ft})
    if (p) HIP_NOTE(hipFree(p));
  m->rc = m->fc = nullptr;
  m->rt = m->ft = nullptr;
  m->W = m->H = m->fcap = 0;
  m->cap = 0;
}

void free_host(rt_multi *m) {
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_NOTE(hipSetDevice(m->dev[i]));
    if (m->st[i]) HIP_NOTE(hipStreamSynchronize(m->st[i]));
  }
  for (int32_t i = 0; i < (int32_t)m->d_span.size(); ++i) {
    HIP_NOTE(hipSetDevice(m->dev[i]));
    if (m->d_span[i]) HIP_NOTE(hipFree(m->d_span[i]));
    if (m->h_span[i]) HIP_NOTE(hipHostFree(m->h_span[i]));
  }
  m->d_span.assign(m->n, nullptr);
  m->h_span.assign(m->n, nullptr);
  m->span_rows = 0;
  if (m->hs_c) HIP_NOTE(hipHostFree(m->hs_c));
  if (m->hs_t) HIP_NOTE(hipHostFree(m->hs_t));
  m->hs_c = nullptr;
  m->hs_t = nullptr;
  m->hs_cap = 0;
  m->hs_c_dev.assign(m->n, nullptr);
  m->hs_t_dev.assign(m->n, nullptr);
}

// the staging frame for px pixels (every slot stream is drained first when it grows)
int ensure_host_stage(rt_multi *m, size_t px) {
  if (px <= m->hs_cap) return RT_OK;
  free_host(m);
  const unsigned fl = hipHostMallocPortable | hipHostMallocMapped;
  HIP_TRY(hipHostMalloc((void **)&m->hs_c, px * 4, fl));
  HIP_TRY(hipHostMalloc((void **)&m->hs_t, px * 4, fl));
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    HIP_TRY(hipHostGetDevicePointer((void **)&m->hs_c_dev[i], m->hs_c, 0));
    HIP_TRY(hipHostGetDevicePointer((void **)&m->hs_t_dev[i], m->hs_t, 0));
  }
  m->hs_cap = px;
  m->hs_dirty = true;
  return RT_OK;
}

// per-slot span buffers for `rows` rows per slot, set to INT32_MAX (no span)
int ensure_spans(rt_multi *m, int32_t rows) {
  if (rows <= m->span_rows) return RT_OK;
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    HIP_TRY(hipStreamSynchronize(m->st[i]));
    if (m->d_span[i]) HIP_NOTE(hipFree(m->d_span[i]));
    if (m->h_span[i]) HIP_NOTE(hipHostFree(m->h_span[i]));
    m->d_span[i] = m->h_span[i] = nullptr;
  }
  m->span_rows = 0;
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    HIP_TRY(hipMalloc((void **)&m->d_span[i], (size_t)rows * 8));
    // in the slot's stream order: a plain hipMemsetD32 goes to the null stream,
    // which the slot's non-blocking stream does not wait for (the first
    // frame's kernel then met uninitialised span words: lost spans at 4K)
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)m->d_span[i], 0x7FFFFFFF, (size_t)rows * 2, m->st[i]));
    HIP_TRY(hipHostMalloc((void **)&m->h_span[i], (size_t)rows * 8, hipHostMallocDefault));
  }
  m->span_rows = rows;
  return RT_OK;
}

// buffers for `frames` frames (one chunk at most) of W x H
int ensure(rt_multi *m, int32_t W, int32_t H, int32_t frames, bool host_frame) {
  frames = std::min(frames, kChunk);
  if (W != m->W || H != m->H || frames > m->fcap || (host_frame && !m->fc)) {
    const bool want_host = host_frame || m->fc;
    free_buffers(m);
    int64_t cap = 0;
    for (int32_t i = 0; i < m->n; ++i) {
      const rt_tile tl = tile_of(m, i);
      cap = std::max(cap, rt_tile_pixels(W, H, &tl));
    }
    if (cap <= 0) return rterr::set(RT_E_INVALID, "rt_multi: empty frame");
    const int32_t fcap = std::max(frames, 1);
    for (int32_t i = 0; i < m->n; ++i) {
      HIP_TRY(hipSetDevice(m->dev[i]));
      HIP_TRY(hipMalloc(&m->pc[i], (size_t)fcap * cap * 4));
      HIP_TRY(hipMalloc(&m->pt[i], (size_t)fcap * cap * 4));
    }
    HIP_TRY(hipSetDevice(m->dev[0]));
    HIP_TRY(hipMalloc(&m->rc, (size_t)fcap * m->n * cap * 4));
    HIP_TRY(hipMalloc(&m->rt, (size_t)fcap * m->n * cap * 4));
    if (want_host) {
      HIP_TRY(hipMalloc(&m->fc, (size_t)W * H * 4));
      HIP_TRY(hipMalloc(&m->ft, (size_t)W * H * 4));
    }
    m->W = W;
    m->H = H;
    m->fcap = fcap;
    m->cap = cap;
  }
  return RT_OK;
}

// the root scene's plane on every replica (the caller may change it between frames)
int sync_planes(rt_multi *m) {
  int on = 0;
  float nrm[3], off = 0.0f;
  if (int rc = rt_scene_get_plane(m->root, &on, nrm, &off)) return rc;
  for (int32_t i = 1; i < m->n; ++i)
    if (int rc = rt_scene_set_plane(m->scene[i], on, nrm, off)) return rc;
  return RT_OK;
}

// Bring frames [0, k) of every slot's packed buffers to the root's receive
// buffers: one ncclGather per frame and buffer (one RCCL group), or peer
// copies. On return st[0] is ordered after every slot's contribution.
int exchange(rt_multi *m, int32_t k) {
  const int32_t n = m->n;
  const size_t cap = (size_t)m->cap;
  if (m->rccl) {
    NCCL_TRY(ncclGroupStart());
    for (int32_t f = 0; f < k; ++f)
      for (int32_t i = 0; i < n; ++i) {
        uint32_t *rc = i == 0 ? m->rc + (size_t)f * n * cap : nullptr;
        float *rt = i == 0 ? m->rt + (size_t)f * n * cap : nullptr;
        ncclResult_t r = ncclGather(m->pc[i] + f * cap, rc, cap, ncclUint32, 0, m->comm[i], m->st[i]);
        if (r == ncclSuccess) r = ncclGather(m->pt[i] + f * cap, rt, cap, ncclFloat32, 0, m->comm[i], m->st[i]);
        if (r != ncclSuccess) {
          (void)ncclGroupEnd();
          return rterr::set(RT_E_DEVICE, std::string("rt_multi: ncclGather: ") + ncclGetErrorString(r));
        }
      }
    NCCL_TRY(ncclGroupEnd());
    return RT_OK;
  }
  // peer copies: slot 0 rendered straight into the root's receive slots; the
  // other slots write them only after the root's previous untile read them
  for (int32_t i = 1; i < n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    HIP_TRY(hipStreamWaitEvent(m->st[i], m->rc_free, 0));
    for (int32_t f = 0; f < k; ++f) {
      const size_t at = ((size_t)f * n + i) * cap;
      HIP_TRY(hipMemcpyPeerAsync(m->rc + at, m->dev[0], m->pc[i] + f * cap, m->dev[i], cap * 4, m->st[i]));
      HIP_TRY(hipMemcpyPeerAsync(m->rt + at, m->dev[0], m->pt[i] + f * cap, m->dev[i], cap * 4, m->st[i]));
    }
    HIP_TRY(hipEventRecord(m->done[i], m->st[i]));
  }
  HIP_TRY(hipSetDevice(m->dev[0]));
  for (int32_t i = 1; i < n; ++i) HIP_TRY(hipStreamWaitEvent(m->st[0], m->done[i], 0));
  return RT_OK;
}

// slot i's packed output of frame f of the current chunk
uint32_t *slot_color(rt_multi *m, int32_t i, int32_t f) {
  return (!m->rccl && i == 0) ? m->rc + (size_t)f * m->n * m->cap : m->pc[i] + (size_t)f * m->cap;
}
float *slot_t(rt_multi *m, int32_t i, int32_t f) {
  return (!m->rccl && i == 0) ? m->rt + (size_t)f * m->n * m->cap : m->pt[i] + (size_t)f * m->cap;
}

// Render frames params[0..k) on every slot (the slots first wait for ev0 when
// `wait`), exchange, and untile frame f into out_c[f] / out_t[f] on the
// root's stream st[0]. Chunks of one call need no wait between them: a slot's
// next render follows its previous send on its own stream, and the root's
// next gather follows its previous untile on st[0].
int render_chunk(rt_multi *m, const rt_render_params *params, int32_t k, uint32_t *const *out_c,
                 float *const *out_t, uint32_t flags, bool wait) {
  uint32_t *cp[kChunk];
  float *tp[kChunk];
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    if (i > 0 && wait) HIP_TRY(hipStreamWaitEvent(m->st[i], m->ev0, 0));
    for (int32_t f = 0; f < k; ++f) {
      cp[f] = slot_color(m, i, f);
      tp[f] = slot_t(m, i, f);
    }
    const rt_tile tl = tile_of(m, i);
    if (int rc = rt_render_device_frames(m->scene[i], params, k, cp, tp, m->W, m->H, flags, &tl, m->st[i])) return rc;
  }
  if (int rc = exchange(m, k)) return rc;
  HIP_TRY(hipSetDevice(m->dev[0]));
  const rt_tile all = tile_of(m, 0);
  for (int32_t f = 0; f < k; ++f)
    if (int rc = rt_untile_device(m->rc + (size_t)f * m->n * m->cap, m->rt + (size_t)f * m->n * m->cap, m->cap,
                                  out_c[f], out_t[f], m->W, m->H, &all, m->st[0]))
      return rc;
  HIP_TRY(hipEventRecord(m->rc_free, m->st[0]));
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(rt_scene *scene, const int32_t *devices, int32_t n, int32_t band_rows, rt_multi **out) {
  if (!scene || !devices || n < 1 || !out) return rterr::set(RT_E_INVALID, "rt_multi_create: bad arguments");
  *out = nullptr;
  if (n > 64) return rterr::set(RT_E_INVALID, "rt_multi_create: at most 64 slots");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  for (int32_t i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= ndev)
      return rterr::set(RT_E_INVALID, "rt_multi_create: device " + std::to_string(devices[i]) + " not visible (" +
                                          std::to_string(ndev) + " devices)");
  if (rt_scene_device(scene) != devices[0])
    return rterr::set(RT_E_INVALID, "rt_multi_create: the scene must live on devices[0]");
  DeviceGuard guard;
  rt_multi *m = new rt_multi();
  m->root = scene;
  m->n = n;
  m->band_rows = band_rows > 0 ? band_rows : 8;
  m->dev.assign(devices, devices + n);
  m->scene.assign(n, nullptr);
  m->st.assign(n, nullptr);
  m->done.assign(n, nullptr);
  m->pc.assign(n, nullptr);
  m->pt.assign(n, nullptr);
  m->hs_c_dev.assign(n, nullptr);
  m->hs_t_dev.assign(n, nullptr);
  m->d_span.assign(n, nullptr);
  m->h_span.assign(n, nullptr);
  m->scene[0] = scene;
  std::vector<int> sorted(m->dev);
  std::sort(sorted.begin(), sorted.end());
  m->rccl = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  int rc = RT_OK;
  for (int32_t i = 0; i < n && rc == RT_OK; ++i) {
    if (i > 0) rc = rt_scene_replicate(scene, m->dev[i], &m->scene[i]);
    if (rc != RT_OK) break;
    hipError_t e = hipSetDevice(m->dev[i]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->st[i], hipStreamNonBlocking);
    if (e == hipSuccess) rterr::stream_add(m->st[i], m->dev[i], "rt_multi slot " + std::to_string(i));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->done[i], hipEventDisableTiming);
    if (e == hipSuccess && i > 0 && m->dev[i] != m->dev[0]) {
      // peer copies and RCCL's transport between the slot and the root
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, m->dev[i], m->dev[0]) == hipSuccess && can) {
        const hipError_t pe = hipDeviceEnablePeerAccess(m->dev[0], 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) e = pe;
        (void)hipGetLastError();  // (already enabled is not an error here)
      }
    }
    if (e != hipSuccess) rc = rterr::set(RT_E_DEVICE, std::string("rt_multi_create: slot setup: ") + hipGetErrorString(e));
  }
  if (rc == RT_OK) {
    hipError_t e = hipSetDevice(m->dev[0]);
    if (e == hipSuccess) e = hipEventCreate(&m->ev0);
    if (e == hipSuccess) e = hipEventCreate(&m->ev1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->rc_free, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(m->rc_free, m->st[0]);
    if (e != hipSuccess) rc = rterr::set(RT_E_DEVICE, std::string("rt_multi_create: events: ") + hipGetErrorString(e));
  }
  if (rc == RT_OK && m->rccl) {
    m->comm.assign(n, nullptr);
    const ncclResult_t r = ncclCommInitAll(m->comm.data(), n, m->dev.data());
    if (r != ncclSuccess) {
      m->comm.clear();
      rc = rterr::set(RT_E_DEVICE, std::string("rt_multi_create: ncclCommInitAll: ") + ncclGetErrorString(r));
    }
  }
  if (rc != RT_OK) {
    rt_multi_destroy(m);
    return rc;
  }
  *out = m;
  return RT_OK;
}

int rt_multi_info(const rt_multi *m, int32_t *n, int32_t *exchange, int32_t *band_rows) {
  if (!m) return rterr::set(RT_E_INVALID, "rt_multi is NULL");
  if (n) *n = m->n;
  if (exchange) *exchange = m->rccl ? RT_MULTI_RCCL : RT_MULTI_PEER_COPY;
  if (band_rows) *band_rows = m->band_rows;
  return RT_OK;
}

int rt_multi_render(rt_multi *m, const rt_render_params *p, uint32_t *color, float *t, int32_t W, int32_t H,
                    uint32_t flags, float *ms) {
  if (!m || !p || !color || !t) return rterr::set(RT_E_INVALID, "rt_multi_render: bad arguments");
  if (W <= 0 || H <= 0 || (int64_t)W * H > 0x7FFFFFFFll) return rterr::set(RT_E_INVALID, "rt_multi_render: bad size");
  if (flags & ~(RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY))
    return rterr::set(RT_E_INVALID, "rt_multi_render: flags are 0, RT_FLAG_CLEAR or RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY");
  if ((flags & RT_FLAG_HITS_ONLY) && !(flags & RT_FLAG_CLEAR))
    return rterr::set(RT_E_INVALID, "rt_multi_render: RT_FLAG_HITS_ONLY needs RT_FLAG_CLEAR");
  DeviceGuard guard;
  if (int rc = sync_planes(m)) return rc;
  const size_t px = (size_t)W * H;
  for (int32_t i = 0; i < m->n; ++i) rterr::stream_mark(m->st[i], "rt_multi_render");
  // once anything is queued every return waits for all slot streams, so the
  // caller's buffers are never read or written after the call returns
  struct Drain {
    rt_multi *m;
    ~Drain() {
      for (int32_t i = 0; i < m->n; ++i) {
        HIP_NOTE(hipSetDevice(m->dev[i]));
        HIP_NOTE(hipStreamSynchronize(m->st[i]));
      }
    }
  } drain{m};
  // pinned caller buffers (rt_host_pin) are used directly; pageable ones go
  // through the staging frame
  bool direct = rtdma::pinned(color, px * 4) && rtdma::pinned(t, px * 4);
  if (flags == (RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY)) {
    // the cleared frame, zero-copy: each slot stores its hits at their own
    // rows of the host frame, no gather, no download
    std::vector<uint32_t *> dc(m->n, nullptr);
    std::vector<float *> dt(m->n, nullptr);
    for (int32_t i = 0; i < m->n && direct; ++i) {
      HIP_TRY(hipSetDevice(m->dev[i]));
      dc[i] = (uint32_t *)rtdma::pinned_device_ptr(color, px * 4);
      dt[i] = (float *)rtdma::pinned_device_ptr(t, px * 4);
      direct = dc[i] && dt[i];
    }
    int32_t rows = 0;
    if (!direct) {
      if (int rc = ensure_host_stage(m, px)) return rc;
      for (int32_t i = 0; i < m->n; ++i) {
        const rt_tile tl = tile_of(m, i);
        rows = std::max(rows, (int32_t)(rt_tile_pixels(W, H, &tl) / W));
      }
      if (int rc = ensure_spans(m, rows)) return rc;
      if (m->hs_dirty) {  // (a cleared frame stays cleared: the host resets each copied span)
        rth::clear_frame(m->hs_c, m->hs_t, (int64_t)px, 8);
        m->hs_dirty = false;
      }
      for (int32_t i = 0; i < m->n; ++i) {
        dc[i] = m->hs_c_dev[i];
        dt[i] = m->hs_t_dev[i];
      }
    }
    HIP_TRY(hipSetDevice(m->dev[0]));
    HIP_TRY(hipEventRecord(m->ev0, m->st[0]));
    if (!direct) m->hs_dirty = true;  // until the spans are copied and reset below
    for (int32_t i = 0; i < m->n; ++i) {
      HIP_TRY(hipSetDevice(m->dev[i]));
      if (i > 0) HIP_TRY(hipStreamWaitEvent(m->st[i], m->ev0, 0));
      const rt_tile tl = tile_of(m, i);
      if (int rc = rti::render_band_host(m->scene[i], p, dc[i], dt[i], W, H, &tl, direct ? nullptr : m->d_span[i],
                                         m->st[i]))
        return rc;
      if (!direct) {
        const size_t r = (size_t)(rt_tile_pixels(W, H, &tl) / W);
        HIP_TRY(hipMemcpyAsync(m->h_span[i], m->d_span[i], r * 8, hipMemcpyDeviceToHost, m->st[i]));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)m->d_span[i], 0x7FFFFFFF, r * 2, m->st[i]));
      }
      if (i > 0) HIP_TRY(hipEventRecord(m->done[i], m->st[i]));
    }
    HIP_TRY(hipSetDevice(m->dev[0]));
    for (int32_t i = 1; i < m->n; ++i) HIP_TRY(hipStreamWaitEvent(m->st[0], m->done[i], 0));
    HIP_TRY(hipEventRecord(m->ev1, m->st[0]));
    for (int32_t i = 0; i < m->n; ++i) {
      HIP_TRY(hipSetDevice(m->dev[i]));
      HIP_TRY(hipStreamSynchronize(m->st[i]));
    }
    if (!direct) {
      // the slots' spans by image row (slot i's local row yl is image row
      // (yl / band_rows * n + i) * band_rows + yl % band_rows), then the stored
      // spans to the caller, reset in the staging frame as they are copied
      m->merged.assign((size_t)H * 2, 0x7FFFFFFF);
      const int32_t br = m->band_rows;
      for (int32_t i = 0; i < m->n; ++i) {
        const rt_tile tl = tile_of(m, i);
        const int32_t r = (int32_t)(rt_tile_pixels(W, H, &tl) / W);
        for (int32_t yl = 0; yl < r; ++yl) {
          const int32_t yo = m->n == 1 ? yl : (yl / br * m->n + i) * br + yl % br;
          m->merged[2 * (size_t)yo] = m->h_span[i][2 * yl];
          m->merged[2 * (size_t)yo + 1] = m->h_span[i][2 * yl + 1];
        }
      }
      rth::copy_spans(color, t, m->hs_c, m->hs_t, W, H, m->merged.data(), 0, true);
      m->hs_dirty = false;
    }
    if (ms) HIP_TRY(hipEventElapsedTime(ms, m->ev0, m->ev1));
    return RT_OK;
  }
  if (int rc = ensure(m, W, H, 1, true)) return rc;
  if (!direct) {
    if (int rc = ensure_host_stage(m, px)) return rc;
    m->hs_dirty = true;
  }
  uint32_t *hc = direct ? color : m->hs_c;  // where the DMAs read / write on the host
  float *ht = direct ? t : m->hs_t;
  HIP_TRY(hipSetDevice(m->dev[0]));
  HIP_TRY(hipEventRecord(m->ev0, m->st[0]));
  const bool clear = (flags & RT_FLAG_CLEAR) != 0;
  if (!clear) {
    // tPrev frame (Renderer::draw over the caller's buffers, raytracing.cpp:
    // 89-94): every slot's packed buffers start as the caller's values of its
    // bands -- its full bands as one strided 2-D copy, a short last band apart
    if (!direct) rth::copy_rect(hc, ht, color, t, W, 0, W - 1, 0, H - 1, 0);
    const size_t row = (size_t)W * 4;
    const int32_t nb = (H + m->band_rows - 1) / m->band_rows;
    for (int32_t i = 0; i < m->n; ++i) {
      HIP_TRY(hipSetDevice(m->dev[i]));
      uint32_t *dc = slot_color(m, i, 0);
      float *dt = slot_t(m, i, 0);
      int32_t full = 0;  // this slot's bands of band_rows rows (all but possibly the frame's last band)
      for (int32_t b = i; b < nb; b += m->n)
        if ((int64_t)(b + 1) * m->band_rows <= H) ++full;
      const size_t band = row * m->band_rows, pitch = band * m->n;
      if (full > 0) {
        HIP_TRY(hipMemcpy2DAsync(dc, band, (const char *)hc + (size_t)i * band, pitch, band, full,
                                 hipMemcpyHostToDevice, m->st[i]));
        HIP_TRY(hipMemcpy2DAsync(dt, band, (const char *)ht + (size_t)i * band, pitch, band, full,
                                 hipMemcpyHostToDevice, m->st[i]));
      }
      const int32_t last = nb - 1;
      if (last % m->n == i && (int64_t)(last + 1) * m->band_rows > H) {  // the short last band is this slot's
        const size_t rows = (size_t)(H - last * m->band_rows);
        HIP_TRY(hipMemcpyAsync((char *)dc + full * band, (const char *)hc + (size_t)last * band, rows * row,
                               hipMemcpyHostToDevice, m->st[i]));
        HIP_TRY(hipMemcpyAsync((char *)dt + full * band, (const char *)ht + (size_t)last * band, rows * row,
                               hipMemcpyHostToDevice, m->st[i]));
      }
    }
  }
  uint32_t *oc[1] = {m->fc};
  float *ot[1] = {m->ft};
  if (int rc = render_chunk(m, p, 1, oc, ot, clear ? RT_FLAG_CLEAR : 0u, true)) return rc;
  HIP_TRY(hipSetDevice(m->dev[0]));
  HIP_TRY(hipEventRecord(m->ev1, m->st[0]));
  HIP_TRY(hipMemcpyAsync(hc, m->fc, px * 4, hipMemcpyDeviceToHost, m->st[0]));
  HIP_TRY(hipMemcpyAsync(ht, m->ft, px * 4, hipMemcpyDeviceToHost, m->st[0]));
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_TRY(hipSetDevice(m->dev[i]));
    HIP_TRY(hipStreamSynchronize(m->st[i]));
  }
  if (!direct) rth::copy_rect(color, t, hc, ht, W, 0, W - 1, 0, H - 1, 0);
  if (ms) HIP_TRY(hipEventElapsedTime(ms, m->ev0, m->ev1));
  return RT_OK;
}

int rt_multi_render_device_frames(rt_multi *m, const rt_render_params *params, int32_t frames,
                                  uint32_t *const *d_color, float *const *d_t, int32_t W, int32_t H,
                                  uint32_t flags, void *stream) {
  if (!m || !params || !d_color || !d_t || frames < 0) return rterr::set(RT_E_INVALID, "rt_multi_render_device_frames: bad arguments");
  if (!(flags & RT_FLAG_CLEAR) || (flags & ~(RT_FLAG_CLEAR | RT_FLAG_HITS_ONLY)))
    return rterr::set(RT_E_INVALID, "rt_multi_render_device_frames: flags must be RT_FLAG_CLEAR");
  if (W <= 0 || H <= 0 || (int64_t)W * H > 0x7FFFFFFFll) return rterr::set(RT_E_INVALID, "rt_multi: bad size");
  if (frames == 0) return RT_OK;
  DeviceGuard guard;
  if (int rc = sync_planes(m)) return rc;
  if (int rc = ensure(m, W, H, frames, false)) return rc;
  hipStream_t cs = (hipStream_t)stream;
  // the slots start after the caller's queued work
  HIP_TRY(hipSetDevice(m->dev[0]));
  HIP_TRY(hipEventRecord(m->ev0, cs));
  HIP_TRY(hipStreamWaitEvent(m->st[0], m->ev0, 0));
  for (int32_t f0 = 0; f0 < frames; f0 += kChunk) {
    const int32_t k = std::min(kChunk, frames - f0);
    if (int rc = render_chunk(m, params + f0, k, d_color + f0, d_t + f0, RT_FLAG_CLEAR, f0 == 0)) return rc;
  }
  // the caller's stream waits for the assembled frames
  HIP_TRY(hipSetDevice(m->dev[0]));
  HIP_TRY(hipEventRecord(m->ev1, m->st[0]));
  HIP_TRY(hipStreamWaitEvent(cs, m->ev1, 0));
  return RT_OK;
}

int rt_multi_rccl_version(int32_t *version) {
  if (!version) return rterr::set(RT_E_INVALID, "rt_multi_rccl_version: NULL argument");
  int v = 0;
  NCCL_TRY(ncclGetVersion(&v));
  *version = v;
  return RT_OK;
}

int rt_multi_destroy(rt_multi *m) {
  if (!m) return RT_OK;
  DeviceGuard guard;
  free_buffers(m);
  free_host(m);
  for (ncclComm_t c : m->comm)
    if (c) (void)ncclCommDestroy(c);
  for (int32_t i = 0; i < m->n; ++i) {
    HIP_NOTE(hipSetDevice(m->dev[i]));
    if (m->st[i]) {
      rterr::stream_remove(m->st[i]);
      HIP_NOTE(hipStreamDestroy(m->st[i]));
    }
    if (m->done[i]) HIP_NOTE(hipEventDestroy(m->done[i]));
    if (i > 0 && m->scene[i]) rt_scene_destroy(m->scene[i]);
  }
  HIP_NOTE(hipSetDevice(m->dev[0]));
  if (m->ev0) HIP_NOTE(hipEventDestroy(m->ev0));
  if (m->ev1) HIP_NOTE(hipEventDestroy(m->ev1));
  if (m->rc_free) HIP_NOTE(hipEventDestroy(m->rc_free));
  delete m;
  return RT_OK;
}

}  // extern "C"
