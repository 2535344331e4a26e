// kd_softdist.hpp -- the soft mask's per-pair distance type and probability
// (dibr_soft_mask_cuda.cu:100-163), bit-identical to the reference; host-compilable.
//
// Measured and not kept (C3, round 2): an fp32 variant that replaced the nine double quotients
// per pair by n * v_rcp_f32(float(D)) with rigorous error bounds and exact fallbacks (bit-identical,
// 16.5 M adversarial pairs on the CPU and the GPU suite): the fused forward went 169 -> 171 us and
// one view 64 -> 70 us.  The reference sequence is ~310 instructions per pair, the double
// divisions ~80 of them at the fp32 rate; the filter's bookkeeping cost more than it saved.
#pragma once

#include <math.h>
#include <string.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#ifndef __forceinline__
#define __forceinline__ inline
#endif
#endif

namespace kd {

#define KD_SOFT_EPS 1e-7  // dibr_soft_mask_cuda.cu:23 (a double literal)

__host__ __device__ __forceinline__ float kexp(float x) { return expf(x); }
__host__ __device__ __forceinline__ double kexp(double x) { return exp(x); }

// 1 / d (d > 0 finite) to within ~1 ulp: the hardware reciprocal refined by two Newton steps
// (the host build starts from an fp32 quotient, a coarser seed than v_rcp_f64).
__host__ __device__ __forceinline__ double rcp_nr(double d) {
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rcp(d);
#else
  double r = (double)(1.0f / (float)d);
#endif
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

// float(n / d) exactly as the reference rounds it -- the IEEE double quotient rounded to float --
// from r ~ 1 / d: q = n r is within a few double ulps of n / d, so it rounds to the same float
// unless n / d lies that close to a float rounding midpoint (its 29 bits below float precision
// within 32 of 0x10000000) or outside the normal float range; those (about 1 in 2^23) take the
// IEEE double division.  n may be any double (NaN / inf take the division).
__host__ __device__ __forceinline__ float quo_f(double n, double d, double r) {
  const double q = n * r;
#ifdef __HIP_DEVICE_COMPILE__
  const unsigned long long b = (unsigned long long)__double_as_longlong(q);
#else
  unsigned long long b;
  memcpy(&b, &q, sizeof b);
#endif
  const unsigned lo = (unsigned)b & 0x1fffffffu;
  // 2^-120 <= |q| < 2^120 <=> its biased exponent lies in [1023 - 120, 1023 + 120) (zero, NaN,
  // inf and subnormals fall outside), one unsigned compare
  const unsigned ex = (unsigned)(b >> 52) & 0x7ffu;
  const bool safe = (lo - (0x10000000u - 32u)) > 64u && ex - (1023u - 120u) < 240u;
  float res = (float)q;
  if (__builtin_expect(!safe, 0)) {
#ifdef __HIP_DEVICE_COMPILE__
    asm volatile("" ::: "memory");  // keep the division on this rare branch (no speculation)
#endif
    res = (float)(n / d);
  }
  return res;
}

// One edge of the reference (dibr_soft_mask_cuda.cu:103-140): squared perpendicular distance or
// the 4 M^2 sentinel when the foot lies outside the segment.
template <typename T>
__host__ __device__ __forceinline__ T soft_edge_ref(T x0, T y0, T x1, T y1, T x2, T y2, float M) {
  const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
  const T up = A * x0 + Bc * y0 + C;
  const T down = A * A + Bc * Bc;
  T x3 = Bc * Bc * x0 - A * Bc * y0 - A * C;
  T y3 = A * A * y0 - A * Bc * x0 - Bc * C;
  x3 = (T)((double)x3 / ((double)down + KD_SOFT_EPS));
  y3 = (T)((double)y3 / ((double)down + KD_SOFT_EPS));
  const T direct = (x3 - x1) * (x3 - x2) + (y3 - y1) * (y3 - y2);
  if (direct > (T)0) return (T)(4.0f * M * M);
  return (T)((double)(up * up) / ((double)down + KD_SOFT_EPS));
}

// The same edge in fp32 with one reciprocal for its three quotients (quo_f): bit-identical.
__host__ __device__ __forceinline__ float soft_edge_fast(float x0, float y0, float x1, float y1,
                                                         float x2, float y2, float M) {
  const float A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
  const float up = A * x0 + Bc * y0 + C;
  const float down = A * A + Bc * Bc;
  float x3 = Bc * Bc * x0 - A * Bc * y0 - A * C;
  float y3 = A * A * y0 - A * Bc * x0 - Bc * C;
  const double d = (double)down + KD_SOFT_EPS;
  const double r = rcp_nr(d);
  x3 = quo_f((double)x3, d, r);
  y3 = quo_f((double)y3, d, r);
  const float direct = (x3 - x1) * (x3 - x2) + (y3 - y1) * (y3 - y2);
  if (direct > 0.f) return 4.0f * M * M;
  return quo_f((double)(up * up), d, r);
}

// dibr_soft_mask_cuda.cu:100-163: squared distance type (0..5) and probability of one face
// (FAST: the fp32 edges of soft_edge_fast; the same bits).
template <typename T, bool FAST = false>
__host__ __device__ __forceinline__ void soft_face_dist_ref(T x0, T y0, const T v[6], float M,
                                                            float sigmainv, int &edgeid,
                                                            T &prob) {
  T pdis[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3;
    if constexpr (FAST)
      pdis[i] = soft_edge_fast(x0, y0, v[i * 2], v[i * 2 + 1], v[j * 2], v[j * 2 + 1], M);
    else
      pdis[i] = soft_edge_ref<T>(x0, y0, v[i * 2], v[i * 2 + 1], v[j * 2], v[j * 2 + 1], M);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T x1 = v[i * 2], y1 = v[i * 2 + 1];
    pdis[i + 3] = (x0 - x1) * (x0 - x1) + (y0 - y1) * (y0 - y1);
  }
  edgeid = 0;
  T d = pdis[0];
#pragma unroll
  for (int i = 1; i < 6; ++i)
    if (d > pdis[i]) {
      d = pdis[i];
      edgeid = i;
    }
  const T z = (T)sigmainv * d / (T)M / (T)M;
  prob = kexp(-z);
}

}  // namespace kd
