// CPU check that the soft mask's fp32 edge distance with one reciprocal per edge
// (kd_softdist.hpp soft_edge_fast / quo_f) is bit-identical to the reference sequence
// (soft_edge_ref<float>: three IEEE double quotients rounded to float) -- on random edges at
// pixel centres over the scales the path sees, on near-degenerate edges, and on quotients placed
// at float rounding midpoints.  Build: g++ -O2 -ffp-contract=off tools/softdist_check.cpp
#include <cstdio>
#include <cstdint>
#include <random>

#include "../kaolin_amd/csrc/kd_softdist.hpp"

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  long bad = 0, fallback = 0;
  // 1. quotients at and around float midpoints, random magnitudes
  for (long i = 0; i < n; ++i) {
    const double d = std::ldexp(1.0 + 0.5 * (u(g) + 1.0), (int)(g() % 60) - 30);
    float f = (float)std::ldexp(1.0 + 0.5 * (u(g) + 1.0), (int)(g() % 80) - 40);
    if (g() & 1) f = -f;
    // n such that n / d sits near the midpoint above f (a few double ulps either way)
    const double mid = (double)f + 0.5 * ((double)std::nextafter(f, 2.f * f) - (double)f);
    double num = mid * d;
    for (int k = (int)(g() % 64) - 32; k != 0; k += (k > 0 ? -1 : 1))
      num = std::nextafter(num, k > 0 ? INFINITY : -INFINITY);
    const double r = kd::rcp_nr(d);
    const float a = kd::quo_f(num, d, r), b = (float)(num / d);
    if (memcmp(&a, &b, 4)) ++bad;
  }
  printf("midpoint quotients: %ld mismatches of %ld\n", bad, n);
  // 2. random edges / pixel centres at the path's scales (multiplier 1000, NDC in [-1.5, 1.5])
  long bad2 = 0;
  for (long i = 0; i < n; ++i) {
    const float M = 1000.f;
    const float s = (float)std::ldexp(1.0, -(int)(g() % 12));  // edge lengths from 1e3 down
    const float x1 = (float)(1500.0 * u(g)), y1 = (float)(1500.0 * u(g));
    float x2 = x1 + (float)(s * 1000.0 * u(g)), y2 = y1 + (float)(s * 1000.0 * u(g));
    if ((g() & 15) == 0) { x2 = x1; }  // vertical / degenerate edges
    if ((g() & 31) == 0) { y2 = y1; x2 = x1; }
    const int W = 512;
    const float x0 = M / (float)W * (float)(2 * (int)(g() % W) + 1 - W);
    const float y0 = M / (float)W * (float)(W - 2 * (int)(g() % W) - 1);
    const float a = kd::soft_edge_fast(x0, y0, x1, y1, x2, y2, M);
    const float b = kd::soft_edge_ref<float>(x0, y0, x1, y1, x2, y2, M);
    if (memcmp(&a, &b, 4)) {
      if (bad2 < 5) printf("edge mismatch %a %a vs %a\n", (double)a, (double)b, (double)x1);
      ++bad2;
    }
  }
  printf("edges: %ld mismatches of %ld\n", bad2, n);
  (void)fallback;
  return bad || bad2 ? 1 : 0;
}
