// rt_error.h -- the library's error slot behind rt_last_error() (one per host
// thread), the HIP error check used by every C entry point, the registry of the
// library's own HIP streams and the copies between the device and caller host
// memory (rtdma).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace rterr {
int set(int code, const std::string &msg);  // stores msg, returns code
const char *get();
// A HIP call whose failure librtamd does not return (destroy paths, best-effort
// cleanup) goes through HIP_NOTE: its name and error are remembered (per host
// thread), because HIP keeps the failure as the thread's pending last error,
// and a later hipGetLastError() -- or a synchronous call that reports it --
// would otherwise blame whatever call comes next.
hipError_t note(const char *call, hipError_t e);
// The pending HIP last error of this thread, read and cleared: "" when none,
// else a message naming the librtamd call that raised it (or "outside
// librtamd": torch, the caller). Entry points call it before their first
// copy, so a stale error is reported as such and not as the copy's failure.
std::string take_stale();

// Streams the library creates (scene copy/render streams, rt_multi slots, the
// SDF query stream), each with a label and the last library call that queued
// work on it (stream_mark). rt_host_unpin drains them all before it
// unregisters a range, and a sticky device error (a kernel or DMA fault, which
// HIP reports on whatever call comes next) is attributed: the message lists the
// library streams whose hipStreamQuery reports an error and what was last
// queued on each.
void stream_add(hipStream_t s, int device, const std::string &label);
void stream_remove(hipStream_t s);
void stream_mark(hipStream_t s, const char *what);
hipError_t streams_sync();     // every registered stream on its device; the first failure
std::string stream_faults();   // "" or "; library streams reporting errors: ..."
// The message of a failed HIP call: "expr: error", plus stream_faults() when
// the error is a sticky device fault.
std::string hip_fail(const char *expr, hipError_t e);
}  // namespace rterr

// Copies between device memory and CALLER host memory. The runtime's DMA only
// ever sees pinned memory: host ranges the caller pinned with rt_host_pin are
// copied directly, any other (pageable) host memory goes through a
// process-wide pinned bounce buffer (hipHostMalloc), with a host memcpy on one
// side of the DMA. Both return when the host range may be reused (they
// synchronise `st`). DESIGN.md section 0e: the round-5 GPU-suite stop was a
// runtime DMA from a caller's pageable buffer.
namespace rtdma {
// the device address of host range [p, p + bytes) when it lies inside one range
// pinned by rt_host_pin (on the current device), else nullptr
void *pinned_device_ptr(const void *p, size_t bytes);
bool pinned(const void *p, size_t bytes);
hipError_t h2d(void *d, const void *h, size_t n, hipStream_t st);
hipError_t d2h(void *h, const void *d, size_t n, hipStream_t st);
}  // namespace rtdma

struct rt_scene;
struct rt_render_params;
struct rt_tile;
namespace rti {  // librtamd-internal entry points shared between its translation units
int render_band_host(rt_scene *s, const rt_render_params *p, uint32_t *dc, float *dt, int32_t W, int32_t H,
                     const rt_tile *tile, int32_t *d_span, hipStream_t stream);
}  // namespace rti

#define HIP_NOTE(expr) ((void)rterr::note(#expr, (expr)))

#define HIP_TRY(expr)                                                   \
  do {                                                                  \
    hipError_t e_ = (expr);                                             \
    if (e_ != hipSuccess) return rterr::set(RT_E_DEVICE, rterr::hip_fail(#expr, e_)); \
  } while (0)
