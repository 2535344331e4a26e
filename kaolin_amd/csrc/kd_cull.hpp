// kd_cull.hpp -- edge-culling coefficients of one face for the fp32 pair raster
// (kd_raster_pairs.hpp pass A); host-compilable (tools/cull_check.cpp verifies the rule on the CPU).
//
// With the reference's fp32 centres x0, y0 and the scaled corners, w0 is computed as
// fl(fl(bex*cey) - fl(bey*cex)) over rounded edges bex = fl(bx - x0), ... (rasterization_cuda.cu
// :131-139); its exact counterpart is affine,
//   W0 = A0 + B0 x0 + C0 y0,  A0 = bx cy - by cx,  B0 = by - cy,  C0 = cx - bx  (cyclic for 1, 2).
// Every rounding there is relative to its own result (IEEE), and a pixel reaches the test only if
// its centre passed the face's tight box test (xmin <= x0 < xmax, ymin <= y0 < ymax), so every
// edge component is bounded by the box: |bx - x0| <= Wb = xmax - xmin, |cy - y0| <= Hb.  Hence
//   |w_i - W_i| <= 4.02u (|P1| + |P2|) <= 8.04u Wb Hb < tau = 2^-20 Wb Hb   (u = 2^-24)
// -- the face's own extent, not its distance from the origin (round 2 bounded the edge components
// by E = max|corner| + |M| only, which left every sliver and edge-on face unculled: twice the area
// of a pole-fan sliver at C3 is ~14 units^2 against 6 tau = 18.5 there); tau takes the smaller of
// the two bounds.  The three W_i sum to
// N = A0 + A1 + A2 (twice the signed area) at every pixel; the computed sum
// fl(fl(w0 + w1) + w2) is within 3 tau + 1.25 tau of N, so when |N| > 6 tau it has the sign s of
// N, and adding copysign(eps, .) keeps that sign: a pixel with s W_i < -2 tau has s w_i < -tau,
// so w_i / norm < 0 and the reference rejects it (rasterization_cuda.cu:145; |eps| <= 2^20 tau
// (fp64: 2^500 tau) keeps |norm| finite and below 2^126 tau, so the quotient is a normal number,
// never -0) -- culling it
// cannot change the result.  Keep iff s W_i >= -2 tau is, for s B_i > 0 (< 0), x0 >= (<=) X*(y0);
// in pixel units relative to the face's own span (column span.x0, row span.y0),
//   p*(y0) = P0 + P1 (y0 - y0ref),  y0ref = centre of row span.y0,
// and the raster keeps columns >= ceil(max_lo - 1/64) and <= floor(min_hi + 1/64).  The 1/64 px
// slack covers the fp32 evaluation there (|P0| <= 2^14, |P1 d| <= 2^13 over the span's rows, a
// handful of roundings of at most 2^-10 each), the centre rounding (u W / 2 <= 2^-10 for
// W <= 2^15) and the double-precision coefficients (terms bounded by 2^40 px: < 2^-12); the
// double N carries its own rounding margin (2^-48 E^2) in the |N| test.  Edges outside these
// bounds, degenerate or non-finite faces and non-positive pixel steps cull nothing (slots stay
// -inf / +inf).
// fp64 data (T = double): the reference evaluates the same expressions in double from the fp32
// centres, so the same derivation holds with u = 2^-53: tau = 2^-49 Wb Hb (> 8.04 u Wb Hb), and
// the corners' products are no longer exact in double -- their rounding (2^-52 E^2 at most) is
// inside the 2^-48 E^2 margin of the |N| test and, through the 2^40 px bound, the 1/64 px slack.
// out: {lo0 P0, lo0 P1, lo1 P0, lo1 P1, hi0 P0, hi0 P1, hi1 P0, hi1 P1}
#pragma once

#include <math.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace kd {

template <typename T>
__host__ __device__ inline void raster_cull_coefs_at(const T v[6], float M, int H, int W,
                                                     int span_x0, int span_y0, int span_y1,
                                                     float eps, float out[8]) {
  constexpr double kTauScale = sizeof(T) == 8 ? 0x1p-49 : 0x1p-20;  // > 8.04 u
  // (scalar slots, constant indices into out[]: a dynamically indexed out[] is a scratch array)
  float lo0p0 = -INFINITY, lo0p1 = 0.f, lo1p0 = -INFINITY, lo1p1 = 0.f;
  float hi0p0 = INFINITY, hi0p1 = 0.f, hi1p0 = INFINITY, hi1p1 = 0.f;
  auto emit = [&]() {
    out[0] = lo0p0;
    out[1] = lo0p1;
    out[2] = lo1p0;
    out[3] = lo1p1;
    out[4] = hi0p0;
    out[5] = hi0p1;
    out[6] = hi1p0;
    out[7] = hi1p1;
  };
  const double ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
  const double vm = fmax(fmax(fmax(fabs(ax), fabs(ay)), fmax(fabs(bx), fabs(by))),
                         fmax(fabs(cx), fabs(cy)));
  const float sxf = M / (float)W, syf = M / (float)H;
  if (!(vm < 0x1p59) || !(sxf > 0.f) || !(syf > 0.f) || W > 32768 || H > 32768) return emit();
  const double E = vm + 1.001 * fabs((double)M);
  // the box extents (corner differences in double; rounded up)
  const double Wb = (fmax(fmax(ax, bx), cx) - fmin(fmin(ax, bx), cx)) * (1.0 + 0x1p-50);
  const double Hb = (fmax(fmax(ay, by), cy) - fmin(fmin(ay, by), cy)) * (1.0 + 0x1p-50);
  // both bounds hold (|bex| <= E as well); the smaller one culls more (+ a floor below fp32
  // subnormal products)
  const double tau = kTauScale * fmin(Wb * Hb, E * E) + 0x1p-140;
  const double A[3] = {bx * cy - by * cx, cx * ay - cy * ax, ax * by - ay * bx};
  const double Bc[3] = {by - cy, cy - ay, ay - by};
  const double Cc[3] = {cx - bx, ax - cx, bx - ax};
  const double N = A[0] + A[1] + A[2];
  // |eps| keeps |norm| finite and the quotient a normal number (|w_i| > tau): fp32 |norm| <=
  // 2^126 tau, fp64 far wider
  constexpr double kEpsScale = sizeof(T) == 8 ? 0x1p500 : 0x1p20;
  if (!(fabs(N) > 6.0 * tau + 0x1p-48 * E * E) || !(fabs((double)eps) <= kEpsScale * tau))
    return emit();
  const double s = N > 0.0 ? 1.0 : -1.0;
  const double sx = sxf, sy = syf;
  const double y0ref = (double)(M / (float)H * (float)(H - 2 * span_y0 - 1));  // px_cy
  const double drows = 2.0 * sy * (double)(span_y1 - span_y0 + 1);  // >= |y0 - y0ref| on the span
  bool has_lo = false, has_hi = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double sB = s * Bc[i];
    if (sB == 0.0) continue;
    const double inv = 1.0 / (2.0 * sB * sx);
    const double P1 = -s * Cc[i] * inv;
    const double t = -2.0 * tau - s * (A[i] + Cc[i] * y0ref);
    if (!(fabs(P1) * drows <= 0x1p13) ||
        !((fabs(A[i]) + fabs(Cc[i] * y0ref) + 2.0 * tau) * fabs(inv) <= 0x1p40))
      continue;
    double P0 = t * inv + 0.5 * (double)(W - 1) - (double)span_x0;
    P0 = fmin(fmax(P0, -0x1p14), 0x1p14);
    // the exact signs of the B_i cannot all agree (B0 + B1 + B2 = 0): at most two per side
    if (sB > 0.0) {
      if (has_lo) {
        lo1p0 = (float)P0;
        lo1p1 = (float)P1;
      } else {
        lo0p0 = (float)P0;
        lo0p1 = (float)P1;
      }
      has_lo = true;
    } else {
      if (has_hi) {
        hi1p0 = (float)P0;
        hi1p1 = (float)P1;
      } else {
        hi0p0 = (float)P0;
        hi0p1 = (float)P1;
      }
      has_hi = true;
    }
  }
  emit();
}

}  // namespace kd
