// rt_error.h -- the library's error slot behind rt_last_error() (one per host
// thread) and the HIP error check used by every C entry point.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace rterr {
int set(int code, const std::string &msg);  // stores msg, returns code
const char *get();
}  // namespace rterr

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return rterr::set(RT_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));  \
  } while (0)
