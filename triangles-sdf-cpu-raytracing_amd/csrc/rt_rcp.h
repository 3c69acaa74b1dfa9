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

// 1 / x for any x: rcp_rn inside its checked range, the division outside it
// (a lane outside sends the wave through the division branch; per-ray setup
// code only, never inside a traversal loop)
__device__ __forceinline__ float rcp_any(float x) {
  const float ax = __builtin_fabsf(x);
  const bool in = ax >= 1e-8f && ax < 0x1p126f;
  float r = rcp_rn(x);
  if (__ballot(!in)) {
    if (!in) r = 1.0f / x;
  }
  return r;
}

// a / b correctly rounded: q = a y with y = rcp_rn(b) the correctly rounded
// reciprocal, the remainder a - b q exact by one fma, then q + rem y (the
// Markstein correction, exact for any a, b whose operands and quotient stay
// clear of overflow and the subnormal range). Used where those hold: b in
// rcp_rn's range, |a| and |q| in [2^-100, 2^100] (or a = +-0, whose quotient
// a y already carries the right sign); every other case takes the division.
// Checked on the GPU against the division: exhaustively for the eye ray's
// 2 (x + 1/2) / W (every x < W <= 32768), and on 2^32 random operand pairs
// (rtx_div_check, tests/test_gpu_parity.py::test_fast_division).
__device__ __forceinline__ float div_rn(float a, float b) {
  const float y = rcp_rn(b);
  const float q = a * y;
  const float rem = __builtin_fmaf(-b, q, a);
  const float q1 = __builtin_fmaf(rem, y, q);
  const float ab = __builtin_fabsf(b), aa = __builtin_fabsf(a), aq = __builtin_fabsf(q);
  const bool zero = a == 0.0f;
  const bool ok = ab >= 1e-8f && ab < 0x1p126f &&
                  (zero || (aa >= 0x1p-100f && aa <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f));
  float r = zero ? q : q1;
  if (__ballot(!ok)) {
    if (!ok) r = a / b;
  }
  return r;
}

}  // namespace rtm
