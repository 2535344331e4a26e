// CPU check of kd_softdist.hpp: soft_face_dist_fast (exact filter over approximate reciprocals)
// against the reference arithmetic soft_face_dist_ref, bit for bit (distance type and
// probability), on realistic and adversarial pairs.  The device's v_rcp_f32 (<= 1 ulp) is
// emulated by a correctly rounded reciprocal perturbed by up to +-2 ulp at random.
//   g++ -O2 -std=c++17 -ffp-contract=off -I kaolin_amd/csrc tools/softdist_check.cpp -o /tmp/sdc
//   /tmp/sdc [millions of pairs per family]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#define KD_SOFTDIST_STATS
#include "kd_softdist.hpp"

namespace kd {
long long g_sd_direct = 0, g_sd_tie = 0, g_sd_ref = 0;
}

static std::mt19937_64 rng(12345);
static float uni(float a, float b) { return std::uniform_real_distribution<float>(a, b)(rng); }

struct NoisyRcp {
  float operator()(float x) const {
    float r = 1.0f / x;
    const int k = (int)(rng() % 5) - 2;  // -2..2 ulp
    for (int i = 0; i < k; ++i) r = nextafterf(r, INFINITY);
    for (int i = 0; i < -k; ++i) r = nextafterf(r, -INFINITY);
    return r;
  }
};

static uint32_t bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

static long long n_checked = 0, n_bad = 0;

static void check(float x0, float y0, const float v[6], float M, float sig) {
  int e0, e1;
  float p0, p1;
  kd::soft_face_dist_ref<float>(x0, y0, v, M, sig, e0, p0);
  kd::soft_face_dist_fast(x0, y0, v, M, sig, e1, p1, NoisyRcp());
  ++n_checked;
  const bool same = e0 == e1 && (bits(p0) == bits(p1) || (std::isnan(p0) && std::isnan(p1)));
  if (!same && n_bad++ < 20)
    printf("MISMATCH x0=%a y0=%a v=(%a %a %a %a %a %a) M=%a: ref (%d, %a) fast (%d, %a)\n", x0,
           y0, v[0], v[1], v[2], v[3], v[4], v[5], M, e0, p0, e1, p1);
}

static float centre(float M, int n, int i) { return M / (float)n * (float)(2 * i + 1 - n); }

int main(int argc, char **argv) {
  const long long n = (argc > 1 ? atoll(argv[1]) : 2) * 1000000ll;
  const float Ms[] = {1000.f, 1.f, 100.f, 1e-3f, 1e5f};
  // 1. realistic: pixel centres of a 512 grid, small triangles around (in M-scaled units)
  for (long long it = 0; it < n; ++it) {
    const float M = Ms[it % 5];
    const int W = 512;
    const float x0 = centre(M, W, (int)(rng() % W)), y0 = centre(M, W, (int)(rng() % W));
    const float s = M / W * uni(0.5f, 30.f);
    float v[6];
    for (int k = 0; k < 3; ++k) {
      v[2 * k] = x0 + uni(-s, s);
      v[2 * k + 1] = y0 + uni(-s, s);
    }
    check(x0, y0, v, M, 7000.f);
  }
  printf("realistic: %lld pairs, exact direct %lld, near-tie %lld, reference path %lld\n",
         n_checked, kd::g_sd_direct, kd::g_sd_tie, kd::g_sd_ref);
  // 2. feet near / at the vertices: pixel on the normal through a vertex (direct ~ 0)
  for (long long it = 0; it < n; ++it) {
    const float M = Ms[it % 5];
    const float s = M * uni(0.001f, 0.05f);
    float v[6];
    const float cx = uni(-M, M), cy = uni(-M, M);
    for (int k = 0; k < 6; ++k) v[k] = (k & 1 ? cy : cx) + uni(-s, s);
    const int e = (int)(rng() % 3), j = (e + 1) % 3;
    const float ex = v[2 * j] - v[2 * e], ey = v[2 * j + 1] - v[2 * e + 1];
    const int at = (rng() & 1) ? e : j;
    const float t = uni(-2.f, 2.f) * (float)pow(2.0, -(double)(rng() % 30));
    const float x0 = v[2 * at] - ey * t + ex * uni(-1e-6f, 1e-6f);
    const float y0 = v[2 * at + 1] + ex * t + ey * uni(-1e-6f, 1e-6f);
    check(x0, y0, v, M, 7000.f);
  }
  // 3. near-ties: pixel on an angle bisector (two edges equidistant), or vertex vs edge
  for (long long it = 0; it < n; ++it) {
    const float M = Ms[it % 5];
    const float s = M * uni(0.001f, 0.05f);
    float v[6];
    for (int k = 0; k < 6; ++k) v[k] = uni(-s, s);
    const int a = (int)(rng() % 3), b = (a + 1) % 3, c = (a + 2) % 3;
    // direction bisecting the angle at vertex a
    float ux = v[2 * b] - v[2 * a], uy = v[2 * b + 1] - v[2 * a + 1];
    float wx = v[2 * c] - v[2 * a], wy = v[2 * c + 1] - v[2 * a + 1];
    const float lu = sqrtf(ux * ux + uy * uy), lw = sqrtf(wx * wx + wy * wy);
    if (!(lu > 0.f && lw > 0.f)) continue;
    const float dx = ux / lu + wx / lw, dy = uy / lu + wy / lw;
    const float t = (rng() & 1) ? uni(-3.f, 3.f) : uni(-1e-3f, 1e-3f);
    const float x0 = v[2 * a] + dx * t * s, y0 = v[2 * a + 1] + dy * t * s;
    check(x0, y0, v, M, 7000.f);
    // and exactly on a corner / on an edge line
    check(v[2 * a], v[2 * a + 1], v, M, 7000.f);
    check(v[2 * a] + ux * 0.5f, v[2 * a + 1] + uy * 0.5f, v, M, 7000.f);
  }
  // 4. degenerate faces (repeated corners, collinear), integer grids (exact ties)
  for (long long it = 0; it < n / 4; ++it) {
    const float M = Ms[it % 5];
    float v[6];
    const int mode = (int)(rng() % 3);
    for (int k = 0; k < 6; ++k) v[k] = (float)((int)(rng() % 9) - 4) * (M / 64.f);
    if (mode == 1) {
      v[2] = v[0];
      v[3] = v[1];
    } else if (mode == 2) {
      v[4] = 2.f * v[2] - v[0];
      v[5] = 2.f * v[3] - v[1];
    }
    const float x0 = (float)((int)(rng() % 17) - 8) * (M / 128.f);
    const float y0 = (float)((int)(rng() % 17) - 8) * (M / 128.f);
    check(x0, y0, v, M, 7000.f);
  }
  // 5. extreme magnitudes and non-finite corners
  const float mags[] = {1e-30f, 1e-20f, 1e-10f, 1e10f, 1e15f, 1e18f, 1e19f, 1e20f};
  for (long long it = 0; it < n / 4; ++it) {
    const float m = mags[it % 8];
    float v[6];
    for (int k = 0; k < 6; ++k) v[k] = uni(-m, m);
    if (it % 97 == 0) v[rng() % 6] = NAN;
    if (it % 101 == 0) v[rng() % 6] = INFINITY;
    check(uni(-m, m), uni(-m, m), v, 1000.f, 7000.f);
  }
  printf("checked %lld pairs, %lld mismatches\n", n_checked, n_bad);
  return n_bad ? 1 : 0;
}
