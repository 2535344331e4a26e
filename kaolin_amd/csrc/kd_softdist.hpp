// kd_softdist.hpp -- the soft mask's per-pair distance type and probability
// (dibr_soft_mask_cuda.cu:100-163), bit-identical to the reference, with a cheap exact filter for
// fp32.  Host-compilable (g++) so tools/softdist_check.cpp can compare the two on the CPU.
//
// The reference evaluates, for each of the three edges of a face, the foot of the perpendicular
// from the pixel centre (x3, y3: two divisions in double, rounded to float), the "foot outside the
// segment" test `direct > 0` and the squared perpendicular distance (a third double division),
// then the first minimum over the 3 edge and 3 vertex distances: nine double divisions per pair,
// most of them for values that cannot be the minimum and signs that are not in doubt.
//
// soft_face_dist_fast replaces each double quotient n / D by n * rcp(float(D)) with a rigorous
// error bound, and only falls back to the reference's exact double division where the bound
// leaves the outcome open:
//   * x3, y3 approximations carry relative error <= 2^-21 against the exact quotient (float(D):
//     2^-24, v_rcp_f32: <= 2 ulp, the product: 2^-24); the reference's x3 is that quotient
//     rounded twice (double, then float), <= 2^-23.9 away.  The sign of `direct` is taken from
//     the approximation when it clears a bound on every difference between the two evaluations
//     (4x margin); otherwise x3, y3 and `direct` are evaluated exactly as the reference does.
//   * edge distances likewise (relative 2^-20 with margin); vertex distances and the 4 M^2
//     sentinel are exact.  The first-minimum is decided from the intervals when one candidate
//     is strictly below every other's lower bound; otherwise every candidate is made exact and
//     the reference's first-min scan runs over them in index order.
//   * the chosen edge distance is then computed exactly (one double division).
// Non-finite inputs, or any non-finite intermediate, take the reference path for the whole pair.
// Results (distance type and probability) are bit-identical by construction; checked on the CPU
// over adversarial inputs (tools/softdist_check.cpp) and by the GPU parity suite.
#pragma once

#include <math.h>

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

#ifdef KD_SOFTDIST_STATS  // tools/softdist_check.cpp: how often each exact fallback runs
extern long long g_sd_direct, g_sd_tie, g_sd_ref;
#define KD_SD_COUNT(x) (++(x))
#else
#define KD_SD_COUNT(x) ((void)0)
#endif

#define KD_SOFT_EPS 1e-7  // dibr_soft_mask_cuda.cu:23 (a double literal)

__host__ __device__ __forceinline__ float kexp(float x) { return expf(x); }
__host__ __device__ __forceinline__ double kexp(double x) { return exp(x); }

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

// dibr_soft_mask_cuda.cu:100-163: squared distance type (0..5) and probability of one face.
template <typename T>
__host__ __device__ __forceinline__ void soft_face_dist_ref(T x0, T y0, const T v[6], float M,
                                                            float sigmainv, int &edgeid,
                                                            T &prob) {
  T pdis[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3;
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

// fp32 with the exact filter (file comment).  Rcp: float -> float approximate reciprocal with
// relative error <= 2^-22 (v_rcp_f32 on the device).
template <typename Rcp>
__host__ __device__ __forceinline__ void soft_face_dist_fast(float x0, float y0, const float v[6],
                                                             float M, float sigmainv,
                                                             int &edgeid, float &prob, Rcp rcp) {
  constexpr float kRelQ = 0x1p-20f;  // quotient approximations vs the reference (2x margin)
  constexpr float kRelP = 0x1p-21f;  // float rounding of the products / sums of `direct`
  constexpr float kTiny = 0x1p-100f; // absolute floor (underflow of the approximations)
  float pd[6], err[6];
  float uu[3];
  double D[3];
  bool finite = true;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3;
    const float x1 = v[i * 2], y1 = v[i * 2 + 1], x2 = v[j * 2], y2 = v[j * 2 + 1];
    const float A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const float up = A * x0 + Bc * y0 + C;
    const float down = A * A + Bc * Bc;
    const float x3n = Bc * Bc * x0 - A * Bc * y0 - A * C;
    const float y3n = A * A * y0 - A * Bc * x0 - Bc * C;
    D[i] = (double)down + KD_SOFT_EPS;
    uu[i] = up * up;
    const float r = rcp((float)D[i]);
    const float x3a = x3n * r, y3a = y3n * r;
    const float a1 = x3a - x1, a2 = x3a - x2, b1 = y3a - y1, b2 = y3a - y2;
    const float pa = a1 * a2, pb = b1 * b2;
    const float da = pa + pb;
    const float ex = fabsf(x3a) * kRelQ + kTiny, ey = fabsf(y3a) * kRelQ + kTiny;
    const float bnd = 4.f * (ex * (fabsf(a1) + fabsf(a2) + ex) + ey * (fabsf(b1) + fabsf(b2) + ey) +
                             kRelP * (fabsf(pa) + fabsf(pb)) + kTiny);
    bool outside;
    if (fabsf(da) > bnd) {  // false for NaN / inf: the exact evaluation decides
      outside = da > 0.f;
    } else {
      KD_SD_COUNT(g_sd_direct);
      float x3 = (float)((double)x3n / D[i]);
      float y3 = (float)((double)y3n / D[i]);
      const float direct = (x3 - x1) * (x3 - x2) + (y3 - y1) * (y3 - y2);
      outside = direct > 0.f;
      finite = finite && !isnan(direct);
    }
    if (outside) {
      pd[i] = 4.0f * M * M;
      err[i] = 0.f;
    } else {
      pd[i] = uu[i] * r;
      err[i] = pd[i] * kRelQ + kTiny;
    }
    // a subnormal (or flushed) reciprocal loses the relative bound: reference path
    finite = finite && r >= 0x1p-125f && isfinite(pd[i]) && isfinite(err[i]) && isfinite(bnd) &&
             isfinite(x3n) && isfinite(y3n) && isfinite(uu[i]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float x1 = v[i * 2], y1 = v[i * 2 + 1];
    pd[i + 3] = (x0 - x1) * (x0 - x1) + (y0 - y1) * (y0 - y1);
    err[i + 3] = 0.f;
    finite = finite && isfinite(pd[i + 3]);
  }
  if (!finite) {
    KD_SD_COUNT(g_sd_ref);
    soft_face_dist_ref<float>(x0, y0, v, M, sigmainv, edgeid, prob);
    return;
  }
  // first minimum from the intervals [pd - err, pd + err]
  float mhi = pd[0] + err[0];
  int imin = 0;
#pragma unroll
  for (int i = 1; i < 6; ++i)
    if (pd[i] + err[i] < mhi) {
      mhi = pd[i] + err[i];
      imin = i;
    }
  int ncand = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) ncand += (pd[i] - err[i] <= mhi) ? 1 : 0;
  float d;
  if (ncand == 1) {
    edgeid = imin;
    d = pd[imin];
    if (err[imin] != 0.f) d = (float)((double)uu[imin] / D[imin]);
  } else {
    // near-tie: exact values of the candidates, the reference's first-min scan over them
    KD_SD_COUNT(g_sd_tie);
    edgeid = -1;
    d = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      if (!(pd[i] - err[i] <= mhi)) continue;
      float e = pd[i];
      if (err[i] != 0.f) e = (float)((double)uu[i] / D[i]);  // edges only (i < 3)
      if (edgeid < 0 || d > e) {
        d = e;
        edgeid = i;
      }
    }
  }
  const float z = sigmainv * d / M / M;
  prob = kexp(-z);
}

}  // namespace kd
