// rt_error.h -- the library's error slot behind rt_last_error() (one per host
// thread) and the HIP error check used by every C entry point.
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
}  // namespace rterr

#define HIP_NOTE(expr) ((void)rterr::note(#expr, (expr)))

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return rterr::set(RT_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));  \
  } while (0)
