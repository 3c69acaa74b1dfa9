// ============================================================================
// oracle/cpuref.cpp -- CPU RESTATEMENT OF THE REFERENCE HOT PATH (TEST INFRA)
// ============================================================================
// This file is TEST INFRASTRUCTURE. It is the parity checker ("oracle") for the
// MI355X renderer in triangles-sdf-cpu-raytracing_amd/. Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
// only as the checker / CPU baseline -- never as the thing measured or shipped.
//
// It restates, op for op, the reference's per-pixel hot path:
//   iMacsimus/Triangles-SDF-CPU-RayTracing @ 2025-07-04 (/root/reference)
//   - Renderer::draw / intersectionColor      src/raytracing.cpp:8-102
//   - Plane, SceneUnion, sort8, bbox helpers  src/raytracing.hpp:22-213
//   - BVH8 SAH builder + traversal            src/triangles_raytracing.cpp:12-335
//   - ISPC micro-kernels (scalar restatement) src/ray_pack.ispc:132-165,220-310
//   - SDF grid sphere tracer + loader         src/grid_raytracing.cpp:1-134
//   - SDF octree tracer + loader              src/octree_raytracing.cpp:1-208
//   - Camera / Quaternion (view matrix)       src/camera.{hpp,cpp}, src/quaternion.hpp
//   - OBJ loading (tinyobj semantics) + loadAndScale  src/core/mesh.cpp:178-287,
//                                                      src/main.cpp:326-343
//
// Pinning (see DESIGN.md "Oracle"): the reference cannot be built in this
// image (LiteMath submodule empty, ISPC absent), so there is no oracle/_ref.
// The LiteMath functions it calls are restated with the formulas recorded in
// SURVEY.md section 8(c); those formulas reproduce the golden frame hashes that
// the survey obtained from the reference's own unmodified translation units
// (checked by tests/test_oracle.py). LiteMath/ISPC semantics themselves stay
// unpinned beyond that.
//
// Numerics: compile with -ffp-contract=off (reference default build is -O0,
// which never contracts). ISPC min/max follow x86 MINPS/MAXPS
// operand semantics (a<b?a:b / a>b?a:b); LiteMath/std min/max use std::min/max.
// ============================================================================
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <unordered_map>
#include <utility>
#include <array>
#include <map>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace ref {

static const float INF = std::numeric_limits<float>::infinity();

// Work counters for the algorithmic-bytes model of SURVEY.md 8(d) (oracle
// bookkeeping only; they do not influence any result).
struct Counters {
  long long bvh_inner = 0, bvh_leaf = 0, bvh_tri = 0;   // traverseNode calls / triangle tests
  long long grid_sdf = 0;                               // SDFGrid::sdf(float3) evaluations
  long long oct_node = 0, oct_leaf = 0, oct_step = 0, oct_normal = 0;
  long long rays = 0;                                   // scene.intersect calls
};
static thread_local Counters tl_cnt;

// ---------------------------------------------------------------- L0 math --
// LiteMath restatement (SURVEY 8(c) "Shim formulas").
struct float3 {
  float x, y, z;
  float3() : x(0), y(0), z(0) {}
  explicit float3(float v) : x(v), y(v), z(v) {}
  float3(float a, float b, float c) : x(a), y(b), z(c) {}
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
struct float4 {
  float x, y, z, w;
  float4() : x(0), y(0), z(0), w(0) {}
  float4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
};
static inline float3 operator+(float3 a, float3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline float3 operator-(float3 a, float3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline float3 operator*(float3 a, float3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline float3 operator/(float3 a, float3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
static inline float3 operator*(float3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline float3 operator*(float s, float3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline float3 operator/(float3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline float3 operator+(float3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
static inline float3 operator/(float s, float3 a) { return {s / a.x, s / a.y, s / a.z}; }
static inline float3 operator-(float3 a) { return {-a.x, -a.y, -a.z}; }
static inline float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float length(float3 a) { return std::sqrt(dot(a, a)); }
static inline float3 normalize(float3 a) { return a / length(a); }
static inline float3 cross(float3 a, float3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline float3 vmin(float3 a, float3 b) {
  return {std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)};
}
static inline float3 vmax(float3 a, float3 b) {
  return {std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)};
}
static inline float3 vfloor(float3 a) { return {std::floor(a.x), std::floor(a.y), std::floor(a.z)}; }
static inline float3 vceil(float3 a) { return {std::ceil(a.x), std::ceil(a.y), std::ceil(a.z)}; }
static inline float4 operator*(float4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
static inline float4 operator*(float s, float4 a) { return {s * a.x, s * a.y, s * a.z, s * a.w}; }
static inline float4 operator+(float4 a, float4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
static inline float4 operator+(float4 a, float s) { return {a.x + s, a.y + s, a.z + s, a.w + s}; }
static inline float4 operator/(float4 a, float s) { return {a.x / s, a.y / s, a.z / s, a.w / s}; }
static inline float4 to_float4(float3 v, float w) { return {v.x, v.y, v.z, w}; }
static inline float3 to_float3(float4 v) { return {v.x, v.y, v.z}; }

// column-major float4x4, M(r,c) = m_col[c][r].
struct float4x4 {
  float m[4][4];  // m[c][r]
  float4x4() { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) m[c][r] = (r == c) ? 1.f : 0.f; }
  float &operator()(int r, int c) { return m[c][r]; }
  float operator()(int r, int c) const { return m[c][r]; }
};
static inline float4 mul(const float4x4 &M, float4 v) {
  float4 r;
  r.x = M(0, 0) * v.x + M(0, 1) * v.y + M(0, 2) * v.z + M(0, 3) * v.w;
  r.y = M(1, 0) * v.x + M(1, 1) * v.y + M(1, 2) * v.z + M(1, 3) * v.w;
  r.z = M(2, 0) * v.x + M(2, 1) * v.y + M(2, 2) * v.z + M(2, 3) * v.w;
  r.w = M(3, 0) * v.x + M(3, 1) * v.y + M(3, 2) * v.z + M(3, 3) * v.w;
  return r;
}
// gluLookAt: z = normalize(eye-center); x = cross(up,z); y = cross(z,x).
static float4x4 lookAt(float3 eye, float3 center, float3 up) {
  float3 z = normalize(eye - center);
  float3 x = normalize(cross(up, z));
  float3 y = normalize(cross(z, x));
  float4x4 M;
  M(0, 0) = x.x; M(0, 1) = x.y; M(0, 2) = x.z; M(0, 3) = -dot(x, eye);
  M(1, 0) = y.x; M(1, 1) = y.y; M(1, 2) = y.z; M(1, 3) = -dot(y, eye);
  M(2, 0) = z.x; M(2, 1) = z.y; M(2, 2) = z.z; M(2, 3) = -dot(z, eye);
  M(3, 0) = 0;   M(3, 1) = 0;   M(3, 2) = 0;   M(3, 3) = 1;
  return M;
}
static float4x4 perspectiveMatrix(float fovy, float aspect, float zNear, float zFar) {
  const float ymax = zNear * std::tan(fovy * 3.14159265358979323846f / 360.0f);
  const float xmax = ymax * aspect;
  float4x4 M;
  for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) M.m[c][r] = 0.f;
  M.m[0][0] = 2.0f * zNear / (2.0f * xmax);
  M.m[1][1] = 2.0f * zNear / (2.0f * ymax);
  M.m[2][2] = (-zFar - zNear) / (zFar - zNear);
  M.m[2][3] = -1.0f;
  M.m[3][2] = -2.0f * zFar * zNear / (zFar - zNear);
  return M;
}
// Double-precision Gauss-Jordan with partial pivoting, cast to float.
static float4x4 inverse4x4(const float4x4 &A) {
  double a[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) { a[r][c] = A(r, c); a[r][c + 4] = (r == c) ? 1.0 : 0.0; }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r) if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
    if (p != c) for (int k = 0; k < 8; ++k) std::swap(a[p][k], a[c][k]);
    double piv = a[c][c];
    for (int k = 0; k < 8; ++k) a[c][k] /= piv;
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      double f = a[r][c];
      if (f == 0.0) continue;
      for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
    }
  }
  float4x4 R;
  for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) R(r, c) = (float)a[r][c + 4];
  return R;
}
// EyeRayDir4f(x,y,w,h,P): pos=(2x/w-1, 2y/h-1, 0, 1); pos=P*pos; pos/=pos.w; (normalize(xyz),0).
static inline float4 EyeRayDir4f(float x, float y, float w, float h, const float4x4 &projInv) {
  float4 pos(2.0f * x / w - 1.0f, 2.0f * y / h - 1.0f, 0.0f, 1.0f);
  pos = mul(projInv, pos);
  pos = pos / pos.w;
  float3 d = normalize(to_float3(pos));
  return {d.x, d.y, d.z, 0.0f};
}
static inline uint32_t color_pack_rgba(float4 c) {
  uint32_t r = (uint32_t)(c.x * 255.0f), g = (uint32_t)(c.y * 255.0f);
  uint32_t b = (uint32_t)(c.z * 255.0f), a = (uint32_t)(c.w * 255.0f);
  return (a << 24) | (b << 16) | (g << 8) | r;
}
struct BBox3f {
  float3 boxMin, boxMax;
  // BBox3f::Intersection: {max(tmin,max3(min(lo,hi))), min(tmax,min3(max(lo,hi)))}
  void Intersection(float3 o, float3 inv, float tmin, float tmax, float &t1, float &t2) const {
    float3 lo = (boxMin - o) * inv, hi = (boxMax - o) * inv;
    float3 mn = vmin(lo, hi), mx = vmax(lo, hi);
    t1 = std::max(tmin, std::max(mn.x, std::max(mn.y, mn.z)));
    t2 = std::min(tmax, std::min(mx.x, std::min(mx.y, mx.z)));
  }
};

// Quaternion / Camera -- src/quaternion.hpp:8-70, src/camera.cpp:1-72
struct Quat { float x, y, z, w; };
static inline Quat qmul(Quat a, Quat b) {  // quaternion.hpp:40-45
  return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
          a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
          a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w,
          a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
static inline float3 rotateVector(float3 v, Quat q) {  // quaternion.hpp:47-52
  Quat p{v.x, v.y, v.z, 0.0f};
  Quat c{-q.x, -q.y, -q.z, q.w};
  Quat r = qmul(qmul(q, p), c);
  return {r.x, r.y, r.z};
}
struct Camera {
  float3 pos, target;
  Quat q{0, 0, 0, 1};
  // Camera(pos, target, up) -> updateOrientation(up)  camera.cpp:36-62
  Camera(float3 p, float3 t, float3 up) : pos(p), target(t) {
    float4x4 m = lookAt(pos, target, up);
    float tr;
    if (m(2, 2) < 0) {
      if (m(0, 0) > m(1, 1)) {
        tr = 1 + m(0, 0) - m(1, 1) - m(2, 2);
        q = {tr, m(0, 1) + m(1, 0), m(2, 0) + m(0, 2), m(1, 2) - m(2, 1)};
      } else {
        tr = 1 - m(0, 0) + m(1, 1) - m(2, 2);
        q = {m(0, 1) + m(1, 0), tr, m(1, 2) + m(2, 1), m(2, 0) - m(0, 2)};
      }
    } else {
      if (m(0, 0) < -m(1, 1)) {
        tr = 1 - m(0, 0) - m(1, 1) + m(2, 2);
        q = {m(2, 0) + m(0, 2), m(1, 2) + m(2, 1), tr, m(0, 1) - m(1, 0)};
      } else {
        tr = 1 + m(0, 0) + m(1, 1) + m(2, 2);
        q = {m(1, 2) - m(2, 1), m(2, 0) - m(0, 2), m(0, 1) - m(1, 0), tr};
      }
    }
    // camera.cpp:61: normalize(m_orientation) -- result discarded, q stays un-normalized.
  }
  float3 up() const { return normalize(rotateVector({0.0f, 1.0f, 0.0f}, q)); }  // camera.hpp:29-31
  float3 right() const { return normalize(rotateVector({1.0f, 0.0f, 0.0f}, q)); }  // camera.hpp:32-34
  float3 forward() const { return normalize(target - pos); }                      // camera.hpp:35-37
  float4x4 lookAtMatrix() const { return lookAt(pos, target, up()); }          // camera.hpp:24-26
  // ---- the viewer's interaction (camera.cpp:5-72, camera.hpp:39-47) ----
  float sens = 0.01f;
  bool lockUp = false;
  float3 lockedUp{0.0f, 0.0f, 0.0f};
  Camera() = default;
  void updateOrientation(float3 up_) {  // camera.cpp:36-62
    Camera c(pos, target, up_);
    q = c.q;
  }
  static Quat angleAxis(float angle, float3 axis) {  // quaternion.hpp:54-70
    float3 n = normalize(axis);
    float half = angle * 0.5f;
    Quat r;
    r.w = std::cos(half);
    r.x = n.x * std::sin(half);
    r.y = n.y * std::sin(half);
    r.z = n.z * std::sin(half);
    return r;
  }
  void rotate(float dx, float dy) {  // camera.cpp:5-20
    float pitch = dy * sens, yaw = dx * sens;
    Quat qYaw = angleAxis(yaw, up());
    Quat qPitch = angleAxis(pitch, right());
    Quat m = qmul(qmul(qPitch, qYaw), q);
    float n = std::sqrt(m.x * m.x + m.y * m.y + m.z * m.z + m.w * m.w);  // Quaternion::normalized
    q = {m.x / n, m.y / n, m.z / n, m.w / n};
    // updateVectors (camera.cpp:22-28)
    float3 f = normalize(rotateVector({0.0f, 0.0f, -1.0f}, q));
    float distance = length(target - pos);
    pos = target - f * distance;
    if (lockUp) updateOrientation(lockedUp);
  }
  void resetPosition(float3 p) { float3 u = up(); pos = p; updateOrientation(u); }    // camera.cpp:64-67
  void resetTarget(float3 t) { float3 u = up(); target = t; updateOrientation(u); }   // camera.cpp:69-72
  void setLockUp(bool to) {                                                           // camera.hpp:39-44
    if (!lockUp && to) lockedUp = up();
    lockUp = to;
  }
  void zoom(float wheel) {  // main.cpp:281-288
    float distance = length(target - pos);
    float r = wheel * distance / 25.0f;
    resetPosition(pos + forward() * r);
  }
};

// ------------------------------------------------------------ HitInfo etc --
// raytracing.hpp:67-73
struct HitInfo {
  bool hitten = false;
  float t = INF;
  float3 normal{0.0f, 1.0f, 0.0f};
  float3 albedo{1.0f, 1.0f, 1.0f};
  float reflectiveness = 0.0f;
  // oracle-only bookkeeping (not in the reference struct): primitive id of the hit
  //   mesh: original triangle index (OBJ face order); grid: linear c0 cell; octree: leaf node.
  int64_t prim = -1;
};

struct IScene {
  virtual HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const = 0;
  virtual ~IScene() {}
};

// sort8: raytracing.hpp:188-213 (19-comparator network, swap iff t[x] > t[y])
static inline void sort8(float t[8], int ch[8]) {
#define RSWAP(a, b) if (t[a] > t[b]) { std::swap(t[a], t[b]); std::swap(ch[a], ch[b]); }
  RSWAP(0, 1); RSWAP(2, 3); RSWAP(4, 5); RSWAP(6, 7);
  RSWAP(0, 2); RSWAP(1, 3); RSWAP(4, 6); RSWAP(5, 7);
  RSWAP(1, 2); RSWAP(5, 6); RSWAP(0, 4); RSWAP(3, 7);
  RSWAP(1, 5); RSWAP(2, 6); RSWAP(1, 4); RSWAP(3, 6);
  RSWAP(2, 4); RSWAP(3, 5); RSWAP(3, 4);
#undef RSWAP
}

// ---------------------------------------------------- ISPC micro-kernels --
// ISPC stdlib min/max on x86 targets lower to MINPS/MAXPS: min(a,b) = a<b?a:b.
static inline float imin(float a, float b) { return a < b ? a : b; }
static inline float imax(float a, float b) { return a > b ? a : b; }
struct Box8 { float xMin[8], yMin[8], zMin[8], xMax[8], yMax[8], zMax[8]; };
// ray_pack.ispc:241-273
static void intersect_box_8(const Box8 &b, const float o[3], const float inv[3], float tNear,
                            float tFar, float res[8]) {
  for (int i = 0; i < 8; ++i) {
    float t1x = (b.xMin[i] - o[0]) * inv[0], t1y = (b.yMin[i] - o[1]) * inv[1],
          t1z = (b.zMin[i] - o[2]) * inv[2];
    float t2x = (b.xMax[i] - o[0]) * inv[0], t2y = (b.yMax[i] - o[1]) * inv[1],
          t2z = (b.zMax[i] - o[2]) * inv[2];
    float mnx = imin(t1x, t2x), mny = imin(t1y, t2y), mnz = imin(t1z, t2z);
    float mxx = imax(t1x, t2x), mxy = imax(t1y, t2y), mxz = imax(t1z, t2z);
    float tMin = imax(mnx, imax(mny, mnz));
    float tMax = imin(mxx, imin(mxy, mxz));
    tMin = imax(tMin, tNear);
    tMax = imin(tMax, tFar);
    res[i] = (tMax < 0 || tMin > tMax) ? -1.0f : tMin;
  }
}
// ray_pack.ispc:220-239
static void divide_box_8(float3 bmin, float3 bmax, Box8 &r) {
  float3 center = (bmin + bmax) / 2.0f;
  float3 diff = center - bmin;
  for (int id = 0; id < 8; ++id) {
    int x = id >> 2, y = (id & 3) >> 1, z = id & 1;
    r.xMin[id] = x == 0 ? bmin.x : center.x;
    r.yMin[id] = y == 0 ? bmin.y : center.y;
    r.zMin[id] = z == 0 ? bmin.z : center.z;
    r.xMax[id] = r.xMin[id] + diff.x;
    r.yMax[id] = r.yMin[id] + diff.y;
    r.zMax[id] = r.zMin[id] + diff.z;
  }
}
// ray_pack.ispc:132-165 (uniform ray, varying triangle)
struct TriHit { bool hit; float t; float3 n; };
static inline TriHit triangle_intersection(float3 orig, float3 dir, float3 v0, float3 v1, float3 v2) {
  TriHit r;
  r.hit = false;
  r.t = -1.0f;
  float3 e1 = v1 - v0, e2 = v2 - v0;
  r.n = normalize(cross(e1, e2));
  float3 pvec = cross(dir, e2);
  float det = dot(e1, pvec);
  if (det < 1e-8f && det > -1e-8f) return r;
  float inv_det = 1 / det;
  float3 tvec = orig - v0;
  float u = dot(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return r;
  float3 qvec = cross(tvec, e1);
  float v = dot(dir, qvec) * inv_det;
  if (v < 0.0f || u + v > 1.0f) return r;
  r.t = dot(e2, qvec) * inv_det;
  r.hit = true;
  return r;
}

// ----------------------------------------------------------------- Plane --
// raytracing.hpp:119-186
struct Plane final : IScene {
  float3 n; float off; float3 b1, b2;
  Plane(float3 normal, float offset) : n(normal), off(offset) {
    float3 a{std::fabs(n.x), std::fabs(n.y), std::fabs(n.z)};
    if (a.x > a.y && a.x > a.z) b1 = normalize(float3(n.y, -n.x, 0));
    else b1 = normalize(float3(0, n.z, -n.y));
    b2 = normalize(cross(b1, n));
  }
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const override {
    HitInfo res;
    float div = dot(d, n);
    if (std::fabs(div) < 1e-8f) return res;
    float t = (off - dot(o, n)) / div;
    if (t < tNear || t > tFar) return res;
    float3 p = o + t * d;
    int x = (int)std::ceil(dot(p, b1));
    int y = (int)std::ceil(dot(p, b2));
    float3 c = (x + y) % 2 == 0 ? float3(0.0f) : float3(1.0f);
    res.hitten = true; res.t = t; res.normal = n; res.albedo = c; res.reflectiveness = 0.3f;
    res.prim = -2;
    return res;
  }
};
// raytracing.hpp:83-97 -- ties go to the second scene
struct SceneUnion final : IScene {
  const IScene *a, *b;
  SceneUnion(const IScene *x, const IScene *y) : a(x), b(y) {}
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const override {
    HitInfo h1 = a->intersect(o, d, tNear, tFar);
    HitInfo h2 = b->intersect(o, d, tNear, tFar);
    return (h1.t < h2.t) ? h1 : h2;
  }
};

// ------------------------------------------------------------- Mesh/BVH --
struct Mesh { std::vector<float4> vPos4f; std::vector<uint32_t> indices; };

static inline BBox3f empty_box() {
  BBox3f b; b.boxMin = float3(INF); b.boxMax = -b.boxMin; return b;
}
// raytracing.hpp:22-27
static inline BBox3f update_box(BBox3f box, float4 v) {
  v = v / v.w;
  box.boxMin = vmin(box.boxMin, to_float3(v));
  box.boxMax = vmax(box.boxMax, to_float3(v));
  return box;
}
static inline float surfaceArea(BBox3f b) {  // raytracing.hpp:62-65
  float3 d = b.boxMax - b.boxMin;
  return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
}

struct BVH8Node {                 // triangles_raytracing.hpp:10-36
  Box8 boxes;                     // child boxes (slots >= realCount: +inf, always miss)
  uint32_t realCount = 0, offset = 0;
  uint32_t startIndex = 0, count = 0;
  bool isLeaf = false;
};

struct Triple { uint32_t i[3]; };

struct BVHBuilder final : IScene {
  static constexpr float EMPTY_NODE_TRAVERSE_COST = 0.2f;  // triangles_raytracing.cpp:12
  struct Div { bool isDivided = false; size_t dividerId = (size_t)-1; float sah = INF; };
  std::vector<BVH8Node> nodes;
  std::vector<BBox3f> leftBoxes, rightBoxes;
  std::vector<uint32_t> indicesY, indicesZ;
  Mesh mesh;
  std::vector<uint32_t> triId;  // oracle bookkeeping: original triangle index per triple slot
  std::vector<uint32_t> triIdY, triIdZ;

  BBox3f triBox(const uint32_t *ids) const {  // raytracing.hpp:51-60
    BBox3f b = empty_box();
    b = update_box(b, mesh.vPos4f[ids[0]]);
    b = update_box(b, mesh.vPos4f[ids[1]]);
    b = update_box(b, mesh.vPos4f[ids[2]]);
    return b;
  }
  // triangles_raytracing.cpp:30-117. The triple sort is std::sort (the reference's
  // std::sort(par_unseq) resolves to serial std::sort without TBB).
  // Triples carry their original triangle id through the sort as a 4th word; the
  // comparator reads only the vertex indices so the permutation is unchanged.
  Div tryDivide(std::vector<uint32_t> &idx, std::vector<uint32_t> &tid, size_t start, size_t end, int axis) {
    struct T4 { uint32_t i[3]; uint32_t id; };
    size_t n = (end - start) / 3;
    std::vector<T4> tmp(n);
    for (size_t k = 0; k < n; ++k) {
      tmp[k] = {{idx[start + 3 * k], idx[start + 3 * k + 1], idx[start + 3 * k + 2]}, tid[start / 3 + k]};
    }
    auto comp = [&](const T4 &a, const T4 &b) {
      BBox3f b1 = triBox(a.i), b2 = triBox(b.i);
      return b1.boxMax[axis] < b2.boxMax[axis];
    };
    std::sort(tmp.begin(), tmp.end(), comp);
    for (size_t k = 0; k < n; ++k) {
      idx[start + 3 * k] = tmp[k].i[0]; idx[start + 3 * k + 1] = tmp[k].i[1];
      idx[start + 3 * k + 2] = tmp[k].i[2]; tid[start / 3 + k] = tmp[k].id;
    }
    for (size_t boxID = start / 3; boxID != end / 3; ++boxID) {
      BBox3f &box = leftBoxes[boxID];
      if (boxID == start / 3) box = empty_box(); else box = leftBoxes[boxID - 1];
      box = update_box(box, mesh.vPos4f[idx[boxID * 3]]);
      box = update_box(box, mesh.vPos4f[idx[boxID * 3 + 1]]);
      box = update_box(box, mesh.vPos4f[idx[boxID * 3 + 2]]);
    }
    for (size_t rev = start / 3; rev != end / 3; ++rev) {
      size_t boxID = end / 3 - rev + start / 3 - 1;
      BBox3f &box = rightBoxes[boxID];
      if (rev == start / 3) box = empty_box(); else box = rightBoxes[boxID + 1];
      box = update_box(box, mesh.vPos4f[idx[boxID * 3]]);
      box = update_box(box, mesh.vPos4f[idx[boxID * 3 + 1]]);
      box = update_box(box, mesh.vPos4f[idx[boxID * 3 + 2]]);
    }
    Div res;
    res.sah = static_cast<float>(end - start) / 3.0f;
    float parentSA = surfaceArea(leftBoxes[end / 3 - 1]);
    for (size_t div = start + 3; div < end; div += 3) {
      BBox3f lb = leftBoxes[div / 3 - 1], rb = rightBoxes[div / 3];
      float lc = static_cast<float>(div - start) / 3.0f;
      float rc = static_cast<float>(end - start) / 3.0f - lc;
      float cur = EMPTY_NODE_TRAVERSE_COST + surfaceArea(lb) / parentSA * lc + surfaceArea(rb) / parentSA * rc;
      if (cur < res.sah) { res.sah = cur; res.dividerId = div; res.isDivided = true; }
    }
    // align to 8 triangles: triangles_raytracing.cpp:100-114
    if (res.isDivided && (res.dividerId - start) % 24 != 0) {
      size_t d1 = (res.dividerId - 1) / 24 * 24;
      size_t d2 = ((res.dividerId - 1) / 24 + 1) * 24;
      size_t nearest = (res.dividerId - d1 <= d2 - res.dividerId) ? d1 : d2;
      size_t other = d1 + d2 - nearest;
      if (start < nearest && nearest < end) res.dividerId = nearest;
      else if (start < other && other < end) res.dividerId = other;
    }
    return res;
  }
  // triangles_raytracing.cpp:119-153
  Div tryDivide(size_t start, size_t end) {
    if (end - start <= 8 * 3) return Div{};
    std::copy(mesh.indices.begin() + start, mesh.indices.begin() + end, indicesY.begin() + start);
    std::copy(mesh.indices.begin() + start, mesh.indices.begin() + end, indicesZ.begin() + start);
    std::copy(triId.begin() + start / 3, triId.begin() + end / 3, triIdY.begin() + start / 3);
    std::copy(triId.begin() + start / 3, triId.begin() + end / 3, triIdZ.begin() + start / 3);
    std::vector<uint32_t> &tidY = triIdY, &tidZ = triIdZ;
    float curSAH = static_cast<float>(end - start) / 3.0f;
    Div dx = tryDivide(mesh.indices, triId, start, end, 0);
    Div dy = tryDivide(indicesY, tidY, start, end, 1);
    Div dz = tryDivide(indicesZ, tidZ, start, end, 2);
    float minSAH = std::min({curSAH, dx.sah, dy.sah, dz.sah});
    if (dx.sah == minSAH) return dx;
    if (dy.sah == minSAH) {
      std::copy(indicesY.begin() + start, indicesY.begin() + end, mesh.indices.begin() + start);
      std::copy(tidY.begin() + start / 3, tidY.begin() + end / 3, triId.begin() + start / 3);
      return dy;
    }
    if (dz.sah == minSAH) {
      std::copy(indicesZ.begin() + start, indicesZ.begin() + end, mesh.indices.begin() + start);
      std::copy(tidZ.begin() + start / 3, tidZ.begin() + end / 3, triId.begin() + start / 3);
      return dz;
    }
    return Div{};
  }
  // triangles_raytracing.cpp:155-225 (ChipQueue BFS of up to 7 dividers)
  void createNode(size_t offset, size_t start, size_t end) {
    BVH8Node node;
    size_t dividers[20] = {};
    size_t nd = 0;
    std::pair<size_t, size_t> q[40];
    int qf = 0, qr = -1, qc = 0;
    auto enq = [&](std::pair<size_t, size_t> v) { if (qc == 40) return; qr = (qr + 1) % 40; q[qr] = v; qc++; };
    enq({start, end});
    while (qc != 0) {
      auto cur = q[qf]; qf = (qf + 1) % 40; qc--;
      if (nd == 7) break;
      Div r = tryDivide(cur.first, cur.second);
      if (r.isDivided) {
        dividers[nd++] = r.dividerId;
        enq({cur.first, r.dividerId});
        enq({r.dividerId, cur.second});
      }
    }
    if (nd == 0) {
      if (end - start > 24) {
        dividers[nd++] = ((start / 3 + end / 3) / 2) * 3;
      } else {
        node.isLeaf = true;
        node.startIndex = (uint32_t)start;
        node.count = (uint32_t)(end - start);
        nodes[offset] = node;
        return;
      }
    }
    nd = std::min(nd, (size_t)7);
    node.isLeaf = false;
    node.realCount = (uint32_t)(nd + 1);
    std::sort(dividers, dividers + nd);
    for (int c = 0; c < 8; ++c) {
      node.boxes.xMin[c] = node.boxes.yMin[c] = node.boxes.zMin[c] = INF;
      node.boxes.xMax[c] = node.boxes.yMax[c] = node.boxes.zMax[c] = INF;
    }
    for (size_t c = 0; c < nd + 1; ++c) {
      size_t lo = (c == 0) ? start : dividers[c - 1];
      size_t hi = (c == nd) ? end : dividers[c];
      BBox3f b = empty_box();
      for (size_t id = lo; id < hi; ++id) b = update_box(b, mesh.vPos4f[mesh.indices[id]]);
      node.boxes.xMin[c] = b.boxMin.x; node.boxes.yMin[c] = b.boxMin.y; node.boxes.zMin[c] = b.boxMin.z;
      node.boxes.xMax[c] = b.boxMax.x; node.boxes.yMax[c] = b.boxMax.y; node.boxes.zMax[c] = b.boxMax.z;
    }
    node.offset = (uint32_t)nodes.size();
    for (size_t c = 0; c < nd + 1; ++c) nodes.emplace_back();
    nodes[offset] = node;
    for (size_t c = 0; c < nd + 1; ++c) {
      size_t lo = (c == 0) ? start : dividers[c - 1];
      size_t hi = (c == nd) ? end : dividers[c];
      createNode(node.offset + c, lo, hi);
    }
  }
  // triangles_raytracing.cpp:227-258
  void perform(Mesh m) {
    mesh = std::move(m);
    size_t ntri = mesh.indices.size() / 3;
    leftBoxes.assign(ntri, BBox3f{});
    rightBoxes.assign(ntri, BBox3f{});
    indicesY.assign(mesh.indices.size(), 0);
    indicesZ.assign(mesh.indices.size(), 0);
    triId.resize(ntri);
    for (size_t i = 0; i < ntri; ++i) triId[i] = (uint32_t)i;
    triIdY.assign(ntri, 0);
    triIdZ.assign(ntri, 0);
    nodes.assign(1, BVH8Node{});
    nodes.reserve(ntri * 2 + 1);
    createNode(0, 0, mesh.indices.size());
    leftBoxes.clear(); rightBoxes.clear(); indicesY.clear(); indicesZ.clear();
    leftBoxes.shrink_to_fit(); rightBoxes.shrink_to_fit(); indicesY.shrink_to_fit(); indicesZ.shrink_to_fit();
  }
  // triangles_raytracing.cpp:266-335
  HitInfo traverseNode(size_t index, float3 o, float3 d, float tNear, float tFar) const {
    const BVH8Node &node = nodes[index];
    HitInfo result;
    if (!node.isLeaf) tl_cnt.bvh_inner++; else tl_cnt.bvh_leaf++;
    if (!node.isLeaf) {
      float t[8] = {};
      float3 inv = 1.0f / d;  // triangles_raytracing.cpp:273
      float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
      intersect_box_8(node.boxes, oo, ii, tNear, tFar, t);
      int ch[8] = {0, 1, 2, 3, 4, 5, 6, 7};
      sort8(t, ch);
      for (int i = 0; i < 8; ++i) {
        uint32_t c = (uint32_t)ch[i];
        if (c >= node.realCount || (t[i] < 0) || (result.hitten && result.t < t[i])) continue;
        HitInfo cur = traverseNode(node.offset + c, o, d, tNear, tFar);
        if (cur.hitten && (!result.hitten || result.t > cur.t)) result = cur;
      }
    } else {
      uint32_t start = node.startIndex, end = start + node.count;
      uint32_t ntri = std::min((end - start) / 3, 8u);
      tl_cnt.bvh_tri += ntri;
      for (uint32_t k = 0; k < ntri; ++k) {
        float4 v0 = mesh.vPos4f[mesh.indices[start + k * 3]];
        float4 v1 = mesh.vPos4f[mesh.indices[start + k * 3 + 1]];
        float4 v2 = mesh.vPos4f[mesh.indices[start + k * 3 + 2]];
        v0 = v0 / v0.w; v1 = v1 / v1.w; v2 = v2 / v2.w;
        TriHit h = triangle_intersection(o, d, to_float3(v0), to_float3(v1), to_float3(v2));
        if (h.hit && (!result.hitten || result.t > h.t)) {
          result.hitten = true;
          result.normal = h.n;
          result.t = h.t;
          result.prim = triId[start / 3 + k];
        }
      }
    }
    return result;
  }
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const override {
    return traverseNode(0, o, d, tNear, tFar);
  }
};

// -------------------------------------------------------------- SDF grid --
struct SDFGrid final : IScene {  // grid_raytracing.hpp:10-21
  uint32_t sx = 0, sy = 0, sz = 0;
  std::vector<float> values;
  float at(uint32_t x, uint32_t y, uint32_t z) const { return values[(x * sy + y) * sz + z]; }
  // grid_raytracing.cpp:7-62
  float sdf(float3 p, int64_t *cell = nullptr) const {
    tl_cnt.grid_sdf++;
    p = (p + 1.0f) / 2.0f;
    p = p * float3((float)(sx - 1), (float)(sy - 1), (float)(sz - 1));
    float3 c0f = vfloor(p), c1f = vceil(p);
    uint32_t c0x = (uint32_t)c0f.x, c0y = (uint32_t)c0f.y, c0z = (uint32_t)c0f.z;
    uint32_t c1x = (uint32_t)c1f.x, c1y = (uint32_t)c1f.y, c1z = (uint32_t)c1f.z;
    float3 a = p - c0f, b = c1f - p;  // a = p_c0f, b = c1f_p
    if (c1x == c0x) { a.x = 1.0f; b.x = 0.0f; }
    if (c1y == c0y) { a.y = 1.0f; b.y = 0.0f; }
    if (c1z == c0z) { a.z = 1.0f; b.z = 0.0f; }
    float p0 = at(c0x, c0y, c0z), p1 = at(c0x, c0y, c1z), p2 = at(c0x, c1y, c0z), p3 = at(c0x, c1y, c1z);
    float p4 = at(c1x, c0y, c0z), p5 = at(c1x, c0y, c1z), p6 = at(c1x, c1y, c0z), p7 = at(c1x, c1y, c1z);
    float res = 0.0f;
    res += p0 * b.x * b.y * b.z;
    res += p1 * b.x * b.y * a.z;
    res += p2 * b.x * a.y * b.z;
    res += p3 * b.x * a.y * a.z;
    res += p4 * a.x * b.y * b.z;
    res += p5 * a.x * b.y * a.z;
    res += p6 * a.x * a.y * b.z;
    res += p7 * a.x * a.y * a.z;
    if (cell) *cell = (int64_t)((c0x * sy + c0y) * sz + c0z);
    return res;
  }
  float3 normal(float3 p) const {  // grid_raytracing.cpp:64-89
    const float E = 1e-3f;
    float xl = (p.x - E >= -1.0f) ? p.x - E : p.x, xr = (p.x + E <= 1.0f) ? p.x + E : p.x;
    float yl = (p.y - E >= -1.0f) ? p.y - E : p.y, yr = (p.y + E <= 1.0f) ? p.y + E : p.y;
    float zl = (p.z - E >= -1.0f) ? p.z - E : p.z, zr = (p.z + E <= 1.0f) ? p.z + E : p.z;
    float dx = sdf(float3(xr, p.y, p.z)) - sdf(float3(xl, p.y, p.z));
    float dy = sdf(float3(p.x, yr, p.z)) - sdf(float3(p.x, yl, p.z));
    float dz = sdf(float3(p.x, p.y, zr)) - sdf(float3(p.x, p.y, zl));
    return normalize(float3(dx, dy, dz));
  }
  // grid_raytracing.cpp:93-125
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const override {
    HitInfo res;
    BBox3f box{float3(-1.0f), float3(1.0f)};
    float t1, t2;
    box.Intersection(o, 1.0f / d, tNear, tFar, t1, t2);
    if (t1 > t2) return res;
    float t = t1;
    float3 p = o + t * d;
    p = vmax(p, float3(-1.0f));
    p = vmin(p, float3(1.0f));
    while (p.x <= 1.0f && p.y <= 1.0f && p.z <= 1.0f && p.x >= -1.0f && p.y >= -1.0f && p.z >= -1.0f) {
      int64_t cell;
      float s = sdf(p, &cell);
      if (s < 1e-3f) {
        res.hitten = true;
        res.t = t + s;
        res.normal = normal(p);
        res.prim = cell;
        break;
      }
      t += s;
      p = o + t * d;
    }
    return res;
  }
};

// ------------------------------------------------------------ SDF octree --
struct OctNode { float values[8]; uint32_t childrenOffset; };  // octree_raytracing.hpp:8-18
static_assert(sizeof(OctNode) == 36, "octree node must be 36 bytes");

struct SDFOctree final : IScene {
  std::vector<OctNode> nodes;
  static bool isEmpty(const OctNode &n) {  // octree_raytracing.hpp:12-17
    bool all10 = true, all0 = true;
    for (int i = 0; i < 8; ++i) { all10 = all10 && (n.values[i] > 10.0f); all0 = all0 && (n.values[i] == 0.0f); }
    return all10 || all0;
  }
  // octree_raytracing.cpp:18-57
  float nodeSDF(size_t id, const BBox3f &box, float3 p) const {
    tl_cnt.oct_step++;
    p = (p - box.boxMin) / (box.boxMax - box.boxMin);
    p = vmin(vmax(p, float3(0.0000001f)), float3(0.9999999f));
    float3 c0f = vfloor(p), c1f = vceil(p);
    uint32_t c0x = (uint32_t)c0f.x, c0y = (uint32_t)c0f.y, c0z = (uint32_t)c0f.z;
    uint32_t c1x = (uint32_t)c1f.x, c1y = (uint32_t)c1f.y, c1z = (uint32_t)c1f.z;
    float3 a = p - c0f, b = c1f - p;
    const float *v = nodes[id].values;
    auto V = [&](uint32_t x, uint32_t y, uint32_t z) { return v[(x << 2) + (y << 1) + z]; };
    float p0 = V(c0x, c0y, c0z), p1 = V(c0x, c0y, c1z), p2 = V(c0x, c1y, c0z), p3 = V(c0x, c1y, c1z);
    float p4 = V(c1x, c0y, c0z), p5 = V(c1x, c0y, c1z), p6 = V(c1x, c1y, c0z), p7 = V(c1x, c1y, c1z);
    float res = 0.0f;
    res += p0 * b.x * b.y * b.z;
    res += p1 * b.x * b.y * a.z;
    res += p2 * b.x * a.y * b.z;
    res += p3 * b.x * a.y * a.z;
    res += p4 * a.x * b.y * b.z;
    res += p5 * a.x * b.y * a.z;
    res += p6 * a.x * a.y * b.z;
    res += p7 * a.x * a.y * a.z;
    return res;
  }
  // octree_raytracing.cpp:60-118
  float3 nodeNormal(size_t id, const BBox3f &box, float3 p) const {
    tl_cnt.oct_normal++;
    p = (p - box.boxMin) / (box.boxMax - box.boxMin);
    p = vmin(vmax(p, float3(0.0000001f)), float3(0.9999999f));
    float3 c0f = vfloor(p), c1f = vceil(p);
    uint32_t c0x = (uint32_t)c0f.x, c0y = (uint32_t)c0f.y, c0z = (uint32_t)c0f.z;
    uint32_t c1x = (uint32_t)c1f.x, c1y = (uint32_t)c1f.y, c1z = (uint32_t)c1f.z;
    float3 a = p - c0f, b = c1f - p;
    float3 da(1.0f), db(-1.0f);
    const float *v = nodes[id].values;
    auto V = [&](uint32_t x, uint32_t y, uint32_t z) { return v[(x << 2) + (y << 1) + z]; };
    float p0 = V(c0x, c0y, c0z), p1 = V(c0x, c0y, c1z), p2 = V(c0x, c1y, c0z), p3 = V(c0x, c1y, c1z);
    float p4 = V(c1x, c0y, c0z), p5 = V(c1x, c0y, c1z), p6 = V(c1x, c1y, c0z), p7 = V(c1x, c1y, c1z);
    float dfdx = p0 * db.x * b.y * b.z + p1 * db.x * b.y * a.z + p2 * db.x * a.y * b.z +
                 p3 * db.x * a.y * a.z + p4 * da.x * b.y * b.z + p5 * da.x * b.y * a.z +
                 p6 * da.x * a.y * b.z + p7 * da.x * a.y * a.z;
    float dfdy = p0 * b.x * db.y * b.z + p1 * b.x * db.y * a.z + p2 * b.x * da.y * b.z +
                 p3 * b.x * da.y * a.z + p4 * a.x * db.y * b.z + p5 * a.x * db.y * a.z +
                 p6 * a.x * da.y * b.z + p7 * a.x * da.y * a.z;
    float dfdz = p0 * b.x * b.y * db.z + p1 * b.x * b.y * da.z + p2 * b.x * a.y * db.z +
                 p3 * b.x * a.y * da.z + p4 * a.x * b.y * db.z + p5 * a.x * b.y * da.z +
                 p6 * a.x * a.y * db.z + p7 * a.x * a.y * da.z;
    return normalize(float3(dfdx, dfdy, dfdz));
  }
  // octree_raytracing.cpp:122-164
  HitInfo intersectLeaf(size_t id, const BBox3f &box, float3 o, float3 d, float tNear, float tFar) const {
    HitInfo res;
    tl_cnt.oct_leaf++;
    const OctNode &n = nodes[id];
    if (isEmpty(n)) return res;
    bool allAbove = true;
    for (int i = 0; i < 8; ++i) allAbove = allAbove && (n.values[i] >= 1e-4f);
    if (allAbove) return res;
    float t1, t2;
    box.Intersection(o, 1.0f / d, tNear, tFar, t1, t2);
    if (t1 > t2) return res;
    float t = t1;
    float3 p = o + t * d;
    p = vmax(p, box.boxMin);
    p = vmin(p, box.boxMax);
    while (p.x <= box.boxMax.x && p.y <= box.boxMax.y && p.z <= box.boxMax.z &&
           p.x >= box.boxMin.x && p.y >= box.boxMin.y && p.z >= box.boxMin.z) {
      float s = nodeSDF(id, box, p);
      if (s < 1e-4f) {
        res.hitten = true;
        res.t = t + s;
        res.normal = nodeNormal(id, box, p);
        res.prim = (int64_t)id;
        break;
      }
      t += s;
      p = o + t * d;
    }
    return res;
  }
  // octree_raytracing.cpp:166-202
  HitInfo intersectNode(size_t id, float3 o, float3 d, float tNear, float tFar, const BBox3f &box) const {
    const OctNode &node = nodes[id];
    tl_cnt.oct_node++;
    if (node.childrenOffset == 0) return intersectLeaf(id, box, o, d, tNear, tFar);
    Box8 b8;
    divide_box_8(box.boxMin, box.boxMax, b8);
    float ts[8] = {};
    float oo[3] = {o.x, o.y, o.z}, ii[3] = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    intersect_box_8(b8, oo, ii, tNear, tFar, ts);
    int ch[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    sort8(ts, ch);
    HitInfo result;
    for (int i = 0; i < 8; ++i) {
      int c = ch[i];
      float t = ts[i];
      if (t > 0 && (!result.hitten || result.t > t)) {
        BBox3f cb;
        cb.boxMin = float3(b8.xMin[c], b8.yMin[c], b8.zMin[c]);
        cb.boxMax = float3(b8.xMax[c], b8.yMax[c], b8.zMax[c]);
        HitInfo h = intersectNode(node.childrenOffset + c, o, d, tNear, tFar, cb);
        if (h.hitten) { result = h; break; }
      }
    }
    return result;
  }
  HitInfo intersect(float3 o, float3 d, float tNear, float tFar) const override {
    BBox3f root{float3(-1.0f), float3(1.0f)};
    return intersectNode(0, o, d, tNear, tFar, root);
  }
};

// -------------------------------------------------------------- Renderer --
enum ShadingMode { Normal = 0, Lambert = 1, Color = 2 };  // raytracing.hpp:99
struct Renderer {
  float3 lightPos{2, 2, 2};
  bool enableShadows = true, enableReflections = true;
  int shadingMode = Lambert;
  mutable long long raysTraced = 0;

  static float3 LambertF(float3 L, float3 n, float3 a) {  // raytracing.cpp:8-11
    return std::max(dot(-L, n), 0.0f) * a;
  }
  // raytracing.cpp:13-65
  std::pair<float4, float> color(const IScene &scene, float3 o, float3 d, float tNear, float tFar,
                                 float tPrev, int maxDepth, int64_t *prim) const {
    tl_cnt.rays++;
    HitInfo hit = scene.intersect(o, d, tNear, std::min(tFar, tPrev));
    if (prim) *prim = hit.hitten ? hit.prim : -1;
    if (!hit.hitten) return {float4(0.0f, 0.0f, 0.0f, 1.0f), INF};
    if (dot(hit.normal, d) > 0) hit.normal = hit.normal * -1.0f;
    float4 c;
    if (shadingMode == Normal) {
      c = to_float4(hit.normal, 1.0f);
      c = (c + 1.0f) / 2.0f;
    } else if (shadingMode == Color) {
      c = to_float4(hit.albedo, 1.0f);
    } else {
      bool visible = true;
      float3 point = o + hit.t * d;
      if (enableShadows) {
        float3 sd = normalize(lightPos - point);
        tl_cnt.rays++;
        HitInfo sh = scene.intersect(point + 0.3f * sd, sd, 0.01f, 100.0f);
        visible = !sh.hitten;
      }
      if (!visible) {
        c = to_float4(hit.albedo * 0.1f, 1.0f);
      } else {
        c = to_float4(vmin(hit.albedo * 0.1f + LambertF(normalize(point - lightPos), hit.normal, hit.albedo),
                           float3(1.0f)), 1.0f);
      }
      if (enableReflections && maxDepth > 1 && hit.reflectiveness > 0.0f) {
        float dn = dot(d, hit.normal);
        float3 refl = hit.normal * dn * (-2.0f) + d;  // LiteMath reflect(dir, normal)
        float3 R = normalize(refl);
        float4 rc = color(scene, point + 0.02f * R, R, 0.01f, 100.0f, INF, maxDepth - 1, nullptr).first;
        c = c * (1.0f - hit.reflectiveness) + hit.reflectiveness * rc;
      }
    }
    return {c, hit.t};
  }
};

}  // namespace ref

// ============================================================================
// Loaders (host-side inputs; not timed)
// ============================================================================
namespace ref {
// tinyobj semantics for the subset the shipped OBJs use (v / vt / vn / f; all
// faces triangles): float via (float)strtod, vertex dedup by
// the (v, vn, vt) index tuple in first-use order (core/mesh.cpp:212-268).
static int fix_index(long idx, size_t n) {
  if (idx > 0) return (int)(idx - 1);
  if (idx == 0) return -1;
  return (int)((long)n + idx);
}
static bool load_obj(const char *path, Mesh &out) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  std::vector<float> V;
  size_t nvn = 0, nvt = 0;
  struct Key { int v, n, t; };
  struct KH { size_t operator()(const Key &k) const { return ((size_t)(uint32_t)k.v * 73856093u) ^ ((size_t)(uint32_t)k.n * 19349663u) ^ ((size_t)(uint32_t)k.t * 83492791u); } };
  struct KE { bool operator()(const Key &a, const Key &b) const { return a.v == b.v && a.n == b.n && a.t == b.t; } };
  std::unordered_map<Key, uint32_t, KH, KE> uniq;
  std::vector<Key> faceKeys;
  char line[4096];
  while (std::fgets(line, sizeof(line), f)) {
    char *p = line;
    while (*p == ' ' || *p == '\t') ++p;
    if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
      char *e;
      p += 2;
      float x = (float)std::strtod(p, &e); p = e;
      float y = (float)std::strtod(p, &e); p = e;
      float z = (float)std::strtod(p, &e);
      V.push_back(x); V.push_back(y); V.push_back(z);
    } else if (p[0] == 'v' && p[1] == 'n' && (p[2] == ' ' || p[2] == '\t')) {
      ++nvn;
    } else if (p[0] == 'v' && p[1] == 't' && (p[2] == ' ' || p[2] == '\t')) {
      ++nvt;
    } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
      p += 2;
      std::vector<Key> poly;
      while (*p) {
        while (*p == ' ' || *p == '\t') ++p;
        if (*p == '\0' || *p == '\n' || *p == '\r') break;
        Key k{-1, -1, -1};
        char *e;
        long vi = std::strtol(p, &e, 10); p = e;
        k.v = fix_index(vi, V.size() / 3);
        if (*p == '/') {
          ++p;
          if (*p != '/') { long ti = std::strtol(p, &e, 10); p = e; k.t = fix_index(ti, nvt); }
          if (*p == '/') { ++p; long ni = std::strtol(p, &e, 10); p = e; k.n = fix_index(ni, nvn); }
        }
        while (*p && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') ++p;
        poly.push_back(k);
      }
      for (size_t i = 2; i < poly.size(); ++i) {  // fan (all shipped faces are triangles)
        faceKeys.push_back(poly[0]); faceKeys.push_back(poly[i - 1]); faceKeys.push_back(poly[i]);
      }
    }
  }
  std::fclose(f);
  out.vPos4f.clear(); out.indices.clear();
  for (const Key &k : faceKeys) {
    auto it = uniq.find(k);
    uint32_t id;
    if (it != uniq.end()) id = it->second;
    else {
      id = (uint32_t)out.vPos4f.size();
      uniq.emplace(k, id);
      out.vPos4f.push_back(float4(V[3 * k.v], V[3 * k.v + 1], V[3 * k.v + 2], 1.0f));
    }
    out.indices.push_back(id);
  }
  return !out.indices.empty();
}
// main.cpp:326-343 loadAndScale
static void load_and_scale(Mesh &m) {
  BBox3f b = empty_box();
  for (auto &v : m.vPos4f) b = update_box(b, v);
  float3 center = (b.boxMin + b.boxMax) / 2.0f;
  float scale = length(b.boxMax - center);
  for (auto &v : m.vPos4f) {
    float w = v.w;
    v = v / w;
    float3 s = to_float3(v);
    s = s - center;
    s = s / scale;
    v = to_float4(s, 1.0f);
    v = v * w;
  }
}
}  // namespace ref

// ============================================================================
// C API for tests / bench (ctypes). All buffers are host memory.
// ============================================================================
using namespace ref;

struct RefScene {
  int kind = 0;  // 1 mesh, 2 grid, 3 octree
  BVHBuilder bvh;
  SDFGrid grid;
  SDFOctree oct;
  bool planeOn = false;
  Plane plane{float3(0, 1, 0), -1.0f};
  const IScene *base() const {
    return kind == 1 ? (const IScene *)&bvh : kind == 2 ? (const IScene *)&grid : (const IScene *)&oct;
  }
};

// Mirrors rt_render_params in include/rtamd.h (same field order / sizes).
struct RefParams {
  float camera_pos[3];
  float view_inv[16];   // column-major
  float proj_inv[16];   // column-major
  float light_pos[3];
  int32_t shading_mode;
  int32_t enable_shadows;
  int32_t enable_reflections;
  int32_t reserved;
};

static Counters g_cnt;


// ---------------------------------------------------------------------------
// Mesh -> signed distance. The reference has no SDF
// generator; this is the definition the GPU construction
// (triangles-sdf-cpu-raytracing_amd/csrc/rt_sdfgen.hip) must reproduce bit for
// bit, stated by BRUTE FORCE (every triangle, original order, strictly smaller
// d^2 wins, so ties keep the lowest triangle id):
//   closest point + Voronoi region: Ericson, Real-Time Collision Detection
//   5.1.5 (ClosestPtPointTriangle), regions 0..2 vertex a,b,c, 3 ab, 4 ac,
//   5 bc, 6 face; sign: angle-weighted pseudonormal (Baerentzen & Aanaes)
//   of that feature, over vertices welded by exact position bits, accumulated
//   in double in triangle order; negative iff dot(p - q, N) < 0.
// Parity of this definition is "unpinned" against the reference (it has no
// such function); it pins the GPU generator only.
namespace sdfref {
struct Feat { float3 q; int f; };
static Feat closest(float3 p, float3 a, float3 b, float3 c) {
  float3 ab = b - a, ac = c - a, ap = p - a;
  float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.0f && d2 <= 0.0f) return {a, 0};
  float3 bp = p - b;
  float d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.0f && d4 <= d3) return {b, 1};
  float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0f && d1 >= 0.0f && d3 <= 0.0f) { float v = d1 / (d1 - d3); return {a + ab * v, 3}; }
  float3 cp = p - c;
  float d5 = dot(ab, cp), d6 = dot(ac, cp);
  if (d6 >= 0.0f && d5 <= d6) return {c, 2};
  float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0f && d2 >= 0.0f && d6 <= 0.0f) { float w = d2 / (d2 - d6); return {a + ac * w, 4}; }
  float va = d3 * d6 - d5 * d4;
  if (va <= 0.0f && (d4 - d3) >= 0.0f && (d5 - d6) >= 0.0f) {
    float w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    return {b + (c - b) * w, 5};
  }
  float denom = 1.0f / (va + vb + vc);
  float v = vb * denom, w = vc * denom;
  return {a + ab * v + ac * w, 6};
}
struct Mesh {
  std::vector<float3> tv;   // 3 per triangle
  std::vector<float3> pn;   // 7 per triangle
};
static void prepare(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, Mesh &m) {
  const size_t ntri = (size_t)nidx / 3;
  std::vector<float3> P((size_t)nverts);
  for (int64_t v = 0; v < nverts; ++v)
    P[(size_t)v] = float3(vpos4[4 * v] / vpos4[4 * v + 3], vpos4[4 * v + 1] / vpos4[4 * v + 3],
                          vpos4[4 * v + 2] / vpos4[4 * v + 3]);
  std::map<std::array<uint32_t, 3>, uint32_t> wm;
  std::vector<uint32_t> weld((size_t)nverts);
  for (int64_t v = 0; v < nverts; ++v) {
    std::array<uint32_t, 3> k;
    std::memcpy(k.data(), (const void *)&P[(size_t)v], 12);
    auto it = wm.find(k);
    if (it == wm.end()) it = wm.emplace(k, (uint32_t)wm.size()).first;
    weld[(size_t)v] = it->second;
  }
  std::vector<std::array<double, 3>> va(wm.size(), {0.0, 0.0, 0.0});
  std::map<std::pair<uint32_t, uint32_t>, std::array<double, 3>> ea;
  std::vector<float3> fn(ntri);
  auto ek = [&](uint32_t a, uint32_t b) {
    return std::make_pair(std::min(weld[a], weld[b]), std::max(weld[a], weld[b]));
  };
  for (size_t t = 0; t < ntri; ++t) {
    const uint32_t *vi = idx + 3 * t;
    float3 a = P[vi[0]], b = P[vi[1]], c = P[vi[2]];
    float3 n = cross(b - a, c - a);
    float l = std::sqrt(dot(n, n));
    float3 nf = l > 0.0f ? float3(n.x / l, n.y / l, n.z / l) : float3(0.0f);
    fn[t] = nf;
    const float3 corner[3] = {a, b, c};
    for (int k = 0; k < 3; ++k) {
      float3 o = corner[k], u = corner[(k + 1) % 3], w = corner[(k + 2) % 3];
      double u0 = (double)u.x - o.x, u1 = (double)u.y - o.y, u2 = (double)u.z - o.z;
      double w0 = (double)w.x - o.x, w1 = (double)w.y - o.y, w2 = (double)w.z - o.z;
      double lu = std::sqrt(u0 * u0 + u1 * u1 + u2 * u2), lw = std::sqrt(w0 * w0 + w1 * w1 + w2 * w2);
      double ang = 0.0;
      if (lu > 0.0 && lw > 0.0) ang = std::acos(std::min(1.0, std::max(-1.0, (u0 * w0 + u1 * w1 + u2 * w2) / (lu * lw))));
      auto &acc = va[weld[vi[k]]];
      acc[0] += ang * nf.x; acc[1] += ang * nf.y; acc[2] += ang * nf.z;
    }
    for (auto key : {ek(vi[0], vi[1]), ek(vi[0], vi[2]), ek(vi[1], vi[2])}) {
      auto &e = ea[key];
      e[0] += nf.x; e[1] += nf.y; e[2] += nf.z;
    }
  }
  m.tv.resize(ntri * 3);
  m.pn.resize(ntri * 7);
  for (size_t t = 0; t < ntri; ++t) {
    const uint32_t *vi = idx + 3 * t;
    for (int k = 0; k < 3; ++k) {
      m.tv[3 * t + k] = P[vi[k]];
      const auto &acc = va[weld[vi[k]]];
      m.pn[7 * t + k] = float3((float)acc[0], (float)acc[1], (float)acc[2]);
    }
    const std::pair<uint32_t, uint32_t> keys[3] = {ek(vi[0], vi[1]), ek(vi[0], vi[2]), ek(vi[1], vi[2])};
    for (int k = 0; k < 3; ++k) {
      const auto &e = ea.at(keys[k]);
      m.pn[7 * t + 3 + k] = float3((float)e[0], (float)e[1], (float)e[2]);
    }
    m.pn[7 * t + 6] = fn[t];
  }
}
static float query(const Mesh &m, float3 p) {
  float best = INFINITY;
  size_t bt = 0;
  Feat bf{float3(0.0f), 0};
  for (size_t t = 0; t < m.tv.size() / 3; ++t) {
    Feat f = closest(p, m.tv[3 * t], m.tv[3 * t + 1], m.tv[3 * t + 2]);
    float3 e = p - f.q;
    float d2 = dot(e, e);
    if (d2 < best) { best = d2; bt = t; bf = f; }
  }
  if (!(best < INFINITY)) return INFINITY;
  float3 e = p - bf.q, N = m.pn[7 * bt + (size_t)bf.f];
  float s = e.x * N.x + e.y * N.y + e.z * N.z;
  float d = std::sqrt(best);
  return s < 0.0f ? -d : d;
}
}  // namespace sdfref

extern "C" {

// Work counters accumulated by cpuref_render since the last reset:
// out[0..8] = bvh_inner, bvh_leaf, bvh_tri, grid_sdf, oct_node, oct_leaf,
//             oct_step, oct_normal, rays.
void cpuref_counters(int reset, int64_t *out) {
  if (out) {
    out[0] = g_cnt.bvh_inner; out[1] = g_cnt.bvh_leaf; out[2] = g_cnt.bvh_tri; out[3] = g_cnt.grid_sdf;
    out[4] = g_cnt.oct_node; out[5] = g_cnt.oct_leaf; out[6] = g_cnt.oct_step; out[7] = g_cnt.oct_normal;
    out[8] = g_cnt.rays;
  }
  if (reset) g_cnt = Counters();
}

void *cpuref_load_obj(const char *path, int scale, int64_t *nverts, int64_t *nidx) {
  Mesh *m = new Mesh();
  if (!load_obj(path, *m)) { delete m; return nullptr; }
  if (scale) load_and_scale(*m);
  *nverts = (int64_t)m->vPos4f.size();
  *nidx = (int64_t)m->indices.size();
  return m;
}
void cpuref_mesh_copy(void *h, float *vpos4, uint32_t *idx) {
  Mesh *m = (Mesh *)h;
  std::memcpy(vpos4, m->vPos4f.data(), m->vPos4f.size() * 16);
  std::memcpy(idx, m->indices.data(), m->indices.size() * 4);
}
void cpuref_mesh_free(void *h) { delete (Mesh *)h; }

void *cpuref_scene_mesh(const float *vpos4, int64_t nv, const uint32_t *idx, int64_t ni) {
  RefScene *s = new RefScene();
  s->kind = 1;
  Mesh m;
  m.vPos4f.resize(nv);
  std::memcpy((void *)m.vPos4f.data(), vpos4, nv * 16);
  m.indices.assign(idx, idx + ni);
  s->bvh.perform(std::move(m));
  return s;
}
void *cpuref_scene_grid(uint32_t sx, uint32_t sy, uint32_t sz, const float *values) {
  RefScene *s = new RefScene();
  s->kind = 2;
  s->grid.sx = sx; s->grid.sy = sy; s->grid.sz = sz;
  s->grid.values.assign(values, values + (size_t)sx * sy * sz);
  return s;
}
void *cpuref_scene_octree(const void *nodes36, int64_t n) {
  RefScene *s = new RefScene();
  s->kind = 3;
  s->oct.nodes.resize(n);
  std::memcpy((void *)s->oct.nodes.data(), nodes36, n * 36);
  return s;
}
void cpuref_scene_set_plane(void *h, int enabled, const float *normal, float offset) {
  RefScene *s = (RefScene *)h;
  s->planeOn = enabled != 0;
  s->plane = Plane(float3(normal[0], normal[1], normal[2]), offset);
}
void cpuref_scene_free(void *h) { delete (RefScene *)h; }

int64_t cpuref_bvh_node_count(void *h) { return (int64_t)((RefScene *)h)->bvh.nodes.size(); }
// Export the BVH in canonical pre-order DFS (node ids renumbered) so trees built
// with different offset layouts compare equal iff topology, leaf ranges and
// boxes match. Record = 52 x uint32: isLeaf, realCount|count, startIndex, 0,
// then the Box8 (48 floats as bits; zero for leaves).
int64_t cpuref_bvh_export(void *h, uint32_t *out, int64_t cap) {
  const BVHBuilder &b = ((RefScene *)h)->bvh;
  int64_t n = 0;
  struct Rec { static void go(const BVHBuilder &bb, uint32_t id, uint32_t *o, int64_t cap, int64_t &n) {
    const BVH8Node &nd = bb.nodes[id];
    if (n < cap) {
      uint32_t *r = o + n * 52;
      r[0] = nd.isLeaf; r[1] = nd.isLeaf ? nd.count : nd.realCount; r[2] = nd.isLeaf ? nd.startIndex : 0; r[3] = 0;
      if (!nd.isLeaf) std::memcpy(r + 4, &nd.boxes, 192); else std::memset(r + 4, 0, 192);
    }
    ++n;
    if (!nd.isLeaf) for (uint32_t c = 0; c < nd.realCount; ++c) go(bb, nd.offset + c, o, cap, n);
  } };
  Rec::go(b, 0, out, cap, n);
  return n;
}
void cpuref_bvh_indices(void *h, uint32_t *idx, uint32_t *tri_ids) {
  const BVHBuilder &b = ((RefScene *)h)->bvh;
  std::memcpy(idx, b.mesh.indices.data(), b.mesh.indices.size() * 4);
  if (tri_ids) std::memcpy(tri_ids, b.triId.data(), b.triId.size() * 4);
}

// Camera: view matrix inverse = inverse4x4(Camera(pos,target,up).lookAtMatrix()),
// projInv = inverse4x4(perspectiveMatrix(fovy, W/H, near, far))  (main.cpp:198-201)
void cpuref_camera(const float *pos, const float *target, const float *up, float fovy, float aspect,
                   float znear, float zfar, float *view_inv, float *proj_inv) {
  Camera cam(float3(pos[0], pos[1], pos[2]), float3(target[0], target[1], target[2]), float3(up[0], up[1], up[2]));
  float4x4 vi = inverse4x4(cam.lookAtMatrix());
  float4x4 pi = inverse4x4(perspectiveMatrix(fovy, aspect, znear, zfar));
  std::memcpy(view_inv, vi.m, 64);
  std::memcpy(proj_inv, pi.m, 64);
}

// Renderer::draw (raytracing.cpp:67-102). color/t are read-modify-write host
// buffers (t is tPrev; both are written only on hit). prim (optional) receives
// the primary hit primitive id (-1 miss, -2 plane). Rows [row0,row1) of the
// OUTPUT image are rendered. Returns the pixel-loop time in ms.
double cpuref_render(void *h, const RefParams *P, uint32_t *color, float *tbuf, int64_t *prim,
                     int W, int H, int row0, int row1, int nthreads, int64_t *rays) {
  RefScene *s = (RefScene *)h;
  const IScene *base = s->base();
  SceneUnion uni(base, &s->plane);
  const IScene &scene = s->planeOn ? (const IScene &)uni : *base;
  Renderer R;
  R.lightPos = float3(P->light_pos[0], P->light_pos[1], P->light_pos[2]);
  R.enableShadows = P->enable_shadows != 0;
  R.enableReflections = P->enable_reflections != 0;
  R.shadingMode = P->shading_mode;
  float4x4 viewInv, projInv;
  std::memcpy(viewInv.m, P->view_inv, 64);
  std::memcpy(projInv.m, P->proj_inv, 64);
  float3 rayPos(P->camera_pos[0], P->camera_pos[1], P->camera_pos[2]);
  if (row1 > H) row1 = H;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  auto b = std::chrono::high_resolution_clock::now();
#pragma omp parallel
  {
  tl_cnt = Counters();
#pragma omp for schedule(dynamic)
  for (int yo = row0; yo < row1; ++yo) {
    int y = H - yo - 1;  // loop row y stores to image row H-y-1 (raytracing.cpp:82)
    for (int x = 0; x < W; ++x) {
      size_t xy = (size_t)yo * W + x;
      float4 dir4 = EyeRayDir4f((float)x + 0.5f, (float)y + 0.5f, (float)W, (float)H, projInv);
      dir4.w = 0.0f;
      dir4 = mul(viewInv, dir4);
      float3 dir = to_float3(dir4);
      int64_t pr = -1;
      auto res = R.color(scene, rayPos, dir, 0.01f, 100.0f, tbuf[xy], 2, prim ? &pr : nullptr);
      if (prim) prim[xy] = pr;
      if (!std::isinf(res.second)) {
        tbuf[xy] = res.second;
        color[xy] = color_pack_rgba(res.first);
      }
    }
  }
#pragma omp critical(cpuref_counters)
  {
    g_cnt.bvh_inner += tl_cnt.bvh_inner; g_cnt.bvh_leaf += tl_cnt.bvh_leaf; g_cnt.bvh_tri += tl_cnt.bvh_tri;
    g_cnt.grid_sdf += tl_cnt.grid_sdf; g_cnt.oct_node += tl_cnt.oct_node; g_cnt.oct_leaf += tl_cnt.oct_leaf;
    g_cnt.oct_step += tl_cnt.oct_step; g_cnt.oct_normal += tl_cnt.oct_normal; g_cnt.rays += tl_cnt.rays;
  }
  }
  auto e = std::chrono::high_resolution_clock::now();
  (void)rays;
  return std::chrono::duration<double, std::milli>(e - b).count();
}

// Per-pixel work of the primary ray (oracle bookkeeping for performance
// analysis): cost[y*W+x] = bvh_inner + bvh_leaf + bvh_tri + grid_sdf +
// oct_node + oct_leaf + oct_step for that pixel's primary intersection.
void cpuref_pixel_cost(void *h, const RefParams *P, int W, int H, int32_t *cost) {
  RefScene *s = (RefScene *)h;
  const IScene *base = s->base();
  float4x4 viewInv, projInv;
  std::memcpy(viewInv.m, P->view_inv, 64);
  std::memcpy(projInv.m, P->proj_inv, 64);
  float3 rayPos(P->camera_pos[0], P->camera_pos[1], P->camera_pos[2]);
#pragma omp parallel for schedule(dynamic)
  for (int yo = 0; yo < H; ++yo) {
    int y = H - yo - 1;
    for (int x = 0; x < W; ++x) {
      float4 dir4 = EyeRayDir4f((float)x + 0.5f, (float)y + 0.5f, (float)W, (float)H, projInv);
      dir4.w = 0.0f;
      dir4 = mul(viewInv, dir4);
      Counters before = tl_cnt;
      base->intersect(rayPos, to_float3(dir4), 0.01f, 100.0f);
      const Counters &a = tl_cnt;
      cost[(size_t)yo * W + x] = (int32_t)((a.bvh_inner - before.bvh_inner) + (a.bvh_leaf - before.bvh_leaf) +
                                           (a.bvh_tri - before.bvh_tri) + (a.grid_sdf - before.grid_sdf) +
                                           (a.oct_node - before.oct_node) + (a.oct_leaf - before.oct_leaf) +
                                           (a.oct_step - before.oct_step));
    }
  }
}

// Primary rays of a frame (origin shared): dirs[(y*W+x)*3..] in image layout.
void cpuref_primary_rays(const RefParams *P, int W, int H, float *dirs) {
  float4x4 viewInv, projInv;
  std::memcpy(viewInv.m, P->view_inv, 64);
  std::memcpy(projInv.m, P->proj_inv, 64);
  for (int yo = 0; yo < H; ++yo) {
    int y = H - yo - 1;
    for (int x = 0; x < W; ++x) {
      float4 d4 = EyeRayDir4f((float)x + 0.5f, (float)y + 0.5f, (float)W, (float)H, projInv);
      d4.w = 0.0f;
      d4 = mul(viewInv, d4);
      size_t i = ((size_t)yo * W + x) * 3;
      dirs[i] = d4.x; dirs[i + 1] = d4.y; dirs[i + 2] = d4.z;
    }
  }
}

// Ray-level entry: intersect arbitrary rays against the scene (union with plane
// if enabled). hit[i] in {0,1}; t, normal as in HitInfo; prim id as documented.
void cpuref_intersect_rays(void *h, const float *o, const float *d, int64_t n, float tNear, float tFar,
                           int32_t *hit, float *t, float *nrm, int64_t *prim) {
  RefScene *s = (RefScene *)h;
  const IScene *base = s->base();
  SceneUnion uni(base, &s->plane);
  const IScene &scene = s->planeOn ? (const IScene &)uni : *base;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < n; ++i) {
    HitInfo hi = scene.intersect(float3(o[3 * i], o[3 * i + 1], o[3 * i + 2]),
                                 float3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), tNear, tFar);
    hit[i] = hi.hitten;
    t[i] = hi.t;
    nrm[3 * i] = hi.normal.x; nrm[3 * i + 1] = hi.normal.y; nrm[3 * i + 2] = hi.normal.z;
    if (prim) prim[i] = hi.hitten ? hi.prim : -1;
  }
}

// Word-wise FNV-1a-64 over a colour buffer (SURVEY 8(c) golden-hash definition).
uint64_t cpuref_fnv1a64(const uint32_t *c, int64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (int64_t i = 0; i < n; ++i) h = (h ^ (uint64_t)c[i]) * 1099511628211ull;
  return h;
}


// Signed distance at n points (brute force; OpenMP over points).
int cpuref_sdf_points(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, const float *p3,
                      int64_t n, float *out, int nthreads) {
  if (nidx <= 0 || nidx % 3) return -1;
  sdfref::Mesh m;
  sdfref::prepare(vpos4, nverts, idx, nidx, m);
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : 1)
  for (int64_t i = 0; i < n; ++i) out[i] = sdfref::query(m, float3(p3[3 * i], p3[3 * i + 1], p3[3 * i + 2]));
  return 0;
}


// Orbit camera (camera.cpp) over a state of 18 floats laid out as
// rt_camera_state: position[3] target[3] q[4] sensitivity lock_up(int) locked[3].
static Camera cam_from(const float *st) {
  Camera c;
  c.pos = float3(st[0], st[1], st[2]);
  c.target = float3(st[3], st[4], st[5]);
  c.q = {st[6], st[7], st[8], st[9]};
  c.sens = st[10];
  int32_t lk;
  std::memcpy(&lk, st + 11, 4);
  c.lockUp = lk != 0;
  c.lockedUp = float3(st[12], st[13], st[14]);
  return c;
}
static void cam_to(const Camera &c, float *st) {
  st[0] = c.pos.x; st[1] = c.pos.y; st[2] = c.pos.z;
  st[3] = c.target.x; st[4] = c.target.y; st[5] = c.target.z;
  st[6] = c.q.x; st[7] = c.q.y; st[8] = c.q.z; st[9] = c.q.w;
  st[10] = c.sens;
  int32_t lk = c.lockUp ? 1 : 0;
  std::memcpy(st + 11, &lk, 4);
  st[12] = c.lockedUp.x; st[13] = c.lockedUp.y; st[14] = c.lockedUp.z;
}
// op: 0 init(a=pos, b=target, c3=up) 1 rotate(x, y) 2 resetPosition(a) 3 resetTarget(a)
//     4 setLockUp(x != 0) 5 zoom(x); view_inv (16 floats) returned after the op.
void cpuref_cam_op(float *st, int op, const float *a, const float *b, const float *c3, float x, float y,
                   float *view_inv) {
  Camera c;
  if (op == 0) {
    c = Camera(float3(a[0], a[1], a[2]), float3(b[0], b[1], b[2]), float3(c3[0], c3[1], c3[2]));
  } else {
    c = cam_from(st);
    if (op == 1) c.rotate(x, y);
    else if (op == 2) c.resetPosition(float3(a[0], a[1], a[2]));
    else if (op == 3) c.resetTarget(float3(a[0], a[1], a[2]));
    else if (op == 4) c.setLockUp(x != 0.0f);
    else if (op == 5) c.zoom(x);
  }
  cam_to(c, st);
  if (view_inv) {
    float4x4 vi = inverse4x4(c.lookAtMatrix());
    std::memcpy(view_inv, vi.m, 64);
  }
}
}  // extern "C"
