// rt_rcp.h -- the reciprocal of the triangle test, correctly rounded without
// the IEEE division sequence (two v_div_scale, v_rcp, five fma, v_div_fmas,
// v_div_fixup per triangle). v_rcp_f32 is within 1 ulp of 1/x; one
// Newton-Raphson step with fused operations, r + r (1 - x r), then lands on
// the correctly rounded 1/x -- checked for EVERY float x with
// 1e-8 <= |x| < 2^126 against the division on the GPU (rtx_rcp_check,
// tests/test_gpu_parity.py::test_fast_reciprocal_exhaustive). tri_t uses it in
// that range only: below it the triangle is a miss whatever the value, above
// it (and for inf / NaN) it takes the division.
#pragma once
#include <hip/hip_runtime.h>

namespace rtm {

__device__ __forceinline__ float rcp_rn(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(r, e, r);
}

// a / b correctly rounded for operands in the ranges the caller guarantees:
// y = rcp_rn(b) (b in its checked range), q = a y, the remainder a - b q
// exact by one fma, then the correction q + rem y (Markstein), which rounds
// to the quotient when a, q and the remainder stay normal: here
// |a| in [2^-102, 2^100] or a = +-0 (whose q = a y already carries the
// quotient's sign), |q| in [2^-100, 2^100]. Checked on the GPU: every
// 2 (x + 1/2) / W with x < W <= 32768 and 2^32 random pairs in the eye ray's
// ranges (rtx_div_check, tests/test_gpu_parity.py::test_fast_eye_division).
__device__ __forceinline__ float div_mk(float a, float b) {
  const float y = rcp_rn(b);
  const float q = a * y;
  const float rem = __builtin_fmaf(-b, q, a);
  const float q1 = __builtin_fmaf(rem, y, q);
  return a == 0.0f ? q : q1;
}

}  // namespace rtm
