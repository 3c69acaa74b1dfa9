// rt_math.h -- device math with the reference's exact operation order.
//
// Compiled with -ffp-contract=off (no a*b+c fusion: the reference's default
// -O0 build never contracts). hipcc's default f32 division and
// sqrt are correctly rounded (v_div_scale/fmas/fixup; v_sqrt + correction),
// like the x86 divss/sqrtss the reference runs on.
//
// Two min/max flavours, kept distinct because they differ on NaN operands:
//   std_min/std_max : std::min/std::max and LiteMath float3 min/max
//                     (std::min(a,b) = b<a ? b : a; std::max(a,b) = a<b ? b : a)
//   isp_min/isp_max : ISPC stdlib min/max on x86 (MINPS/MAXPS operand order:
//                     a<b ? a : b, a>b ? a : b), used by ray_pack.ispc.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_rcp.h"

namespace rtd {

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ f3 operator/(f3 a, f3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float len(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return a / len(a); }

__device__ __forceinline__ float std_min(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float std_max(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float isp_min(float a, float b) { return (a < b) ? a : b; }
__device__ __forceinline__ float isp_max(float a, float b) { return (a > b) ? a : b; }
__device__ __forceinline__ f3 vstd_min(f3 a, f3 b) { return {std_min(a.x, b.x), std_min(a.y, b.y), std_min(a.z, b.z)}; }
__device__ __forceinline__ f3 vstd_max(f3 a, f3 b) { return {std_max(a.x, b.x), std_max(a.y, b.y), std_max(a.z, b.z)}; }

constexpr float kInf = __builtin_huge_valf();

// intersect_box_8 for ONE box (ray_pack.ispc:241-273): -1 on miss, else the
// entry distance max(tMin, tNear).
__device__ __forceinline__ float slab_ispc(float bx0, float by0, float bz0, float bx1, float by1,
                                           float bz1, f3 o, f3 inv, float tNear, float tFar) {
  const float t1x = (bx0 - o.x) * inv.x, t1y = (by0 - o.y) * inv.y, t1z = (bz0 - o.z) * inv.z;
  const float t2x = (bx1 - o.x) * inv.x, t2y = (by1 - o.y) * inv.y, t2z = (bz1 - o.z) * inv.z;
  const float mnx = isp_min(t1x, t2x), mny = isp_min(t1y, t2y), mnz = isp_min(t1z, t2z);
  const float mxx = isp_max(t1x, t2x), mxy = isp_max(t1y, t2y), mxz = isp_max(t1z, t2z);
  float tMin = isp_max(mnx, isp_max(mny, mnz));
  float tMax = isp_min(mxx, isp_min(mxy, mxz));
  tMin = isp_max(tMin, tNear);
  tMax = isp_min(tMax, tFar);
  return (tMax < 0.0f || tMin > tMax) ? -1.0f : tMin;
}

// slab_ispc when no operand can be NaN (every 1/d component finite, hence
// nonzero; box bounds finite or +inf): ISPC's MINPS/MAXPS forms then equal
// IEEE min/max (signed zeros aside, and a zero entry distance is only ever
// compared, never used arithmetically), and min/max are associative, so the
// hardware's 2- and 3-operand v_min/v_max give the same bits in fewer ops.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float slab_fast(float bx0, float by0, float bz0, float bx1, float by1,
                                           float bz1, f3 o, f3 inv, float tNear, float tFar) {
  // (lo, hi) pairs through the packed-math unit: the same IEEE sub and mul per element
  const v2f tx = (v2f{bx0, bx1} - v2f{o.x, o.x}) * v2f{inv.x, inv.x};
  const v2f ty = (v2f{by0, by1} - v2f{o.y, o.y}) * v2f{inv.y, inv.y};
  const v2f tz = (v2f{bz0, bz1} - v2f{o.z, o.z}) * v2f{inv.z, inv.z};
  const float t1x = tx.x, t2x = tx.y, t1y = ty.x, t2y = ty.y, t1z = tz.x, t2z = tz.y;
  const float tMin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x, t2x), __builtin_fminf(t1y, t2y)),
                                     __builtin_fmaxf(__builtin_fminf(t1z, t2z), tNear));
  const float tMax = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x, t2x), __builtin_fmaxf(t1y, t2y)),
                                     __builtin_fminf(__builtin_fmaxf(t1z, t2z), tFar));
  return (tMax < 0.0f || tMin > tMax) ? -1.0f : tMin;
}
template <bool FAST>
__device__ __forceinline__ float slab(float bx0, float by0, float bz0, float bx1, float by1, float bz1,
                                      f3 o, f3 inv, float tNear, float tFar) {
  return FAST ? slab_fast(bx0, by0, bz0, bx1, by1, bz1, o, inv, tNear, tFar)
              : slab_ispc(bx0, by0, bz0, bx1, by1, bz1, o, inv, tNear, tFar);
}

// LiteMath BBox3f::Intersection restatement:
// t1 = max(tmin, max3(min(lo,hi))), t2 = min(tmax, min3(max(lo,hi))), std semantics.
__device__ __forceinline__ void bbox_intersection(f3 bmin, f3 bmax, f3 o, f3 inv, float tmin,
                                                  float tmax, float &t1, float &t2) {
  const f3 lo = (bmin - o) * inv, hi = (bmax - o) * inv;
  const f3 mn = vstd_min(lo, hi), mx = vstd_max(lo, hi);
  t1 = std_max(tmin, std_max(mn.x, std_max(mn.y, mn.z)));
  t2 = std_min(tmax, std_min(mx.x, std_min(mx.y, mx.z)));
}

// bbox_intersection for a ray whose 1/d components are all finite and tmin > 0
// (every caller passes tNear = 0.01): no slab operand can be NaN, so std's
// min/max equal IEEE min/max up to the sign of a zero result; t1 >= tmin > 0
// is never zero, and a zero t2 only ever meets the t1 > t2 test. The
// hardware's v_min3/v_max3 then give the same bits in 6 instructions instead
// of 12 compare + select pairs.
__device__ __forceinline__ void bbox_intersection_fast(f3 bmin, f3 bmax, f3 o, f3 inv, float tmin,
                                                       float tmax, float &t1, float &t2) {
  const f3 lo = (bmin - o) * inv, hi = (bmax - o) * inv;
  t1 = __builtin_fmaxf(tmin, __builtin_fmaxf(__builtin_fminf(lo.x, hi.x),
                                             __builtin_fmaxf(__builtin_fminf(lo.y, hi.y), __builtin_fminf(lo.z, hi.z))));
  t2 = __builtin_fminf(tmax, __builtin_fminf(__builtin_fmaxf(lo.x, hi.x),
                                             __builtin_fminf(__builtin_fmaxf(lo.y, hi.y), __builtin_fmaxf(lo.z, hi.z))));
}
template <bool FAST>
__device__ __forceinline__ void bbox_isect(f3 bmin, f3 bmax, f3 o, f3 inv, float tmin, float tmax, float &t1,
                                           float &t2) {
  if constexpr (FAST)
    bbox_intersection_fast(bmin, bmax, o, inv, tmin, tmax, t1, t2);
  else
    bbox_intersection(bmin, bmax, o, inv, tmin, tmax, t1, t2);
}

// max / min of two non-NaN floats as the bare instruction. fmaxf / fminf
// lower to the same v_max_f32 / v_min_f32 but, in the kernels' IEEE mode, with
// a canonicalising v_max_f32 x, x in front of every operand the compiler cannot
// prove canonical (results of selects, kernel arguments); for non-NaN operands
// the value is the same.
__device__ __forceinline__ float vmax_f32(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmin_f32(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// std::min(std::max(x, lo), hi) for a finite (non-NaN) x and lo < hi, as one
// v_med3_f32 (the two forms differ only in the sign of a zero result, which
// callers never feed into arithmetic)
__device__ __forceinline__ float clamp_med3(float x, float lo, float hi) {
  return __builtin_amdgcn_fmed3f(x, lo, hi);
}

// 19-comparator network of sort8 (raytracing.hpp:188-213): swap iff t[a] > t[b].
#define RTD_CSWAP(a, b)                                   \
  {                                                       \
    const bool s_ = t[a] > t[b];                          \
    const float ta_ = t[a], tb_ = t[b];                   \
    const uint32_t ia_ = id[a], ib_ = id[b];              \
    t[a] = s_ ? tb_ : ta_;                                \
    t[b] = s_ ? ta_ : tb_;                                \
    id[a] = s_ ? ib_ : ia_;                               \
    id[b] = s_ ? ia_ : ib_;                               \
  }
__device__ __forceinline__ void sort8(float t[8], uint32_t id[8]) {
  RTD_CSWAP(0, 1); RTD_CSWAP(2, 3); RTD_CSWAP(4, 5); RTD_CSWAP(6, 7);
  RTD_CSWAP(0, 2); RTD_CSWAP(1, 3); RTD_CSWAP(4, 6); RTD_CSWAP(5, 7);
  RTD_CSWAP(1, 2); RTD_CSWAP(5, 6); RTD_CSWAP(0, 4); RTD_CSWAP(3, 7);
  RTD_CSWAP(1, 5); RTD_CSWAP(2, 6); RTD_CSWAP(1, 4); RTD_CSWAP(3, 6);
  RTD_CSWAP(2, 4); RTD_CSWAP(3, 5); RTD_CSWAP(3, 4);
}
#undef RTD_CSWAP

// Column-major 4x4 (LiteMath m_col): M(r,c) = m[c*4+r]; mul as LiteMath
// (row r: M(r,0)*v.x + M(r,1)*v.y + M(r,2)*v.z + M(r,3)*v.w, left to right).
struct f4 {
  float x, y, z, w;
};
__device__ __forceinline__ f4 mat_mul(const float *m, f4 v) {
  f4 r;
  r.x = m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * v.w;
  r.y = m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * v.w;
  r.z = m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * v.w;
  r.w = m[3] * v.x + m[7] * v.y + m[11] * v.z + m[15] * v.w;
  return r;
}

// Renderer::draw ray generation (raytracing.cpp:83-88) with LiteMath
// EyeRayDir4f restated: pos=(2x/w-1, 2y/h-1, 0, 1); pos=P*pos;
// pos/=pos.w; dir=normalize(pos.xyz); world dir = (viewInv*(dir,0)).xyz.
__device__ __forceinline__ f3 eye_ray(int x, int y, int W, int H, const float *projInv,
                                      const float *viewInv) {
  const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
  f4 pos{2.0f * fx / (float)W - 1.0f, 2.0f * fy / (float)H - 1.0f, 0.0f, 1.0f};
  pos = mat_mul(projInv, pos);
  const float w = pos.w;
  pos = f4{pos.x / w, pos.y / w, pos.z / w, pos.w / w};
  const f3 d = normalize(f3{pos.x, pos.y, pos.z});
  const f4 r = mat_mul(viewInv, f4{d.x, d.y, d.z, 0.0f});
  return f3{r.x, r.y, r.z};
}

// eye_ray with its divisions as rtm::div_mk (the same bits), for frames whose
// projection keeps every operand in div_mk's range (fast_eye_ok on the host,
// kFlagFastEye): 2 fx / W and 2 fy / H (W, H <= 32768), pos / w and p / |p|.
__device__ __forceinline__ f3 eye_ray_fast(int x, int y, int W, int H, const float *projInv,
                                           const float *viewInv) {
  const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
  f4 pos{rtm::div_mk(2.0f * fx, (float)W) - 1.0f, rtm::div_mk(2.0f * fy, (float)H) - 1.0f, 0.0f, 1.0f};
  pos = mat_mul(projInv, pos);
  const float w = pos.w;
  const f3 p{rtm::div_mk(pos.x, w), rtm::div_mk(pos.y, w), rtm::div_mk(pos.z, w)};
  const float l = len(p);
  const f3 d{rtm::div_mk(p.x, l), rtm::div_mk(p.y, l), rtm::div_mk(p.z, l)};
  const f4 r = mat_mul(viewInv, f4{d.x, d.y, d.z, 0.0f});
  return f3{r.x, r.y, r.z};
}

// LiteMath color_pack_rgba: (uint)(c*255) per channel, R in the low byte.
__device__ __forceinline__ uint32_t pack_rgba(f4 c) {
  const uint32_t r = (uint32_t)(c.x * 255.0f), g = (uint32_t)(c.y * 255.0f);
  const uint32_t b = (uint32_t)(c.z * 255.0f), a = (uint32_t)(c.w * 255.0f);
  return (a << 24) | (b << 16) | (g << 8) | r;
}

}  // namespace rtd
