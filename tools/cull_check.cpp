// CPU check of the fp32 raster's edge culling (kd_cull.hpp raster_cull_coefs_at, applied as the
// pass A of kd_raster_pairs.hpp applies it): no pixel that the reference's per-face test accepts
// (rasterization_cuda.cu:115-148: half-open box, edge functions over rounded edges, eps-normalised
// norm, w_i / norm >= 0) may be culled.  Random faces of every shape the path sees -- regular,
// pole-fan slivers, edge-on slivers, tiny, large, far from the origin -- at random image sizes and
// multipliers.  Prints the culled fraction of box candidates and the violations (must be 0).
// Build: g++ -O2 -ffp-contract=off -std=c++17 tools/cull_check.cpp -o /tmp/cull_check
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../kaolin_amd/csrc/kd_cull.hpp"

static float px_cx(float M, int W, int w) { return M / (float)W * (float)(2 * w + 1 - W); }
static float px_cy(float M, int H, int h) { return M / (float)H * (float)(H - 2 * h - 1); }
static float fmed3(float x, float lo, float hi) { return std::min(std::max(x, lo), hi); }

// the reference test for one pixel whose centre passed the box test (T = the data type; the
// centres are fp32, widened)
template <typename T>
static bool ref_accepts(float x0f, float y0f, const T v[6], float eps) {
  const T x0 = x0f, y0 = y0f;
  const T ax = v[0] - x0, ay = v[1] - y0, bx = v[2] - x0, by = v[3] - y0;
  const T cx = v[4] - x0, cy = v[5] - y0;
  T w0 = bx * cy - by * cx;
  T w1 = cx * ay - cy * ax;
  T w2 = ax * by - ay * bx;
  T norm = w0 + w1 + w2;
  norm = (T)((double)norm + std::copysign((double)eps, (double)norm));
  w0 /= norm;
  w1 /= norm;
  w2 /= norm;
  return !(w0 < 0 || w1 < 0 || w2 < 0);
}

template <typename T>
static int run(long nf, long seed) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  long cand = 0, culled = 0, bad = 0, acc = 0;
  long kc[6] = {0}, kcul[6] = {0}, kacc[6] = {0};
  for (long f = 0; f < nf; ++f) {
    const int W = 8 + (int)(g() % 600), H = 8 + (int)(g() % 600);
    const float M = (g() % 4) ? 1000.f : (float)std::ldexp(1.0, (int)(g() % 30) - 10);
    const float eps = (g() % 8) ? 1e-8f : (float)std::ldexp(1.0, (int)(g() % 80) - 60);
    // a centre in or near the image (NDC), a shape
    const double cxn = 2.4 * u(g) - 1.2, cyn = 2.4 * u(g) - 1.2;
    const double px = 2.0 / W, py = 2.0 / H;  // one pixel in NDC
    double p[6];
    const int kind = (int)(g() % 6);
    if (kind == 0) {  // regular, a few pixels
      const double s = px * (0.3 + 8 * u(g));
      for (int k = 0; k < 3; ++k) {
        p[2 * k] = cxn + s * (2 * u(g) - 1);
        p[2 * k + 1] = cyn + s * (2 * u(g) - 1);
      }
    } else if (kind == 1) {  // pole-fan sliver: apex + two close points on a ring
      const double r = px * (1 + 10 * u(g)), a = 6.283185307 * u(g), da = 0.03 * u(g) + 1e-4;
      p[0] = cxn;
      p[1] = cyn;
      p[2] = cxn + r * std::cos(a);
      p[3] = cyn + r * std::sin(a) * (px / py);
      p[4] = cxn + r * std::cos(a + da);
      p[5] = cyn + r * std::sin(a + da) * (px / py);
    } else if (kind == 2) {  // edge-on sliver: long thin triangle
      const double L = px * (2 + 20 * u(g)), a = 6.283185307 * u(g), t = px * 0.05 * u(g);
      p[0] = cxn;
      p[1] = cyn;
      p[2] = cxn + L * std::cos(a);
      p[3] = cyn + L * std::sin(a);
      p[4] = cxn + 0.5 * L * std::cos(a) - t * std::sin(a);
      p[5] = cyn + 0.5 * L * std::sin(a) + t * std::cos(a);
    } else if (kind == 3) {  // tiny
      const double s = px * std::ldexp(1.0, -(int)(g() % 20));
      for (int k = 0; k < 3; ++k) {
        p[2 * k] = cxn + s * (2 * u(g) - 1);
        p[2 * k + 1] = cyn + s * (2 * u(g) - 1);
      }
    } else if (kind == 4) {  // large
      const double s = 0.05 + 0.5 * u(g);
      for (int k = 0; k < 3; ++k) {
        p[2 * k] = cxn + s * (2 * u(g) - 1);
        p[2 * k + 1] = cyn + s * (2 * u(g) - 1);
      }
    } else {  // vertices exactly on pixel centres (ties on the edges)
      for (int k = 0; k < 3; ++k) {
        const int ix = (int)(g() % W), iy = (int)(g() % H);
        p[2 * k] = px_cx(1.f, W, std::min(ix + (int)(g() % 3), W - 1));
        p[2 * k + 1] = px_cy(1.f, H, iy);
      }
    }
    T v[6];
    for (int k = 0; k < 6; ++k) v[k] = (T)p[k] * (T)M;  // fvi * M (in the data type)
    const T xmin = std::min({v[0], v[2], v[4]}), xmax = std::max({v[0], v[2], v[4]});
    const T ymin = std::min({v[1], v[3], v[5]}), ymax = std::max({v[1], v[3], v[5]});
    // exact span of the half-open box test
    int x0s = W, x1s = -1, y0s = H, y1s = -1;
    for (int x = 0; x < W; ++x) {
      const T c = px_cx(M, W, x);
      if (!(c < xmin) && !(c >= xmax)) { x0s = std::min(x0s, x); x1s = std::max(x1s, x); }
    }
    for (int y = 0; y < H; ++y) {
      const T c = px_cy(M, H, y);
      if (!(c < ymin) && !(c >= ymax)) { y0s = std::min(y0s, y); y1s = std::max(y1s, y); }
    }
    if (x0s > x1s || y0s > y1s) continue;
    float cc[8];
    kd::raster_cull_coefs_at<T>(v, M, H, W, x0s, y0s, y1s, eps, cc);
    for (int y = y0s; y <= y1s; ++y) {
      const int WY0 = y & ~7, r = y - WY0;
      const float ysub = px_cy(M, H, WY0);
      const float d = (px_cy(M, H, WY0 + r) - ysub) + (ysub - px_cy(M, H, y0s));
      for (int x = x0s; x <= x1s; ++x) {
        const int WX0 = x & ~7;
        const float xo = (float)(WX0 - x0s);
        const float l0 = cc[0] - xo, l2 = cc[2] - xo, h0 = cc[4] - xo, h2 = cc[6] - xo;
        const float plo = std::max(std::fma(cc[1], d, l0), std::fma(cc[3], d, l2)) - 1.f / 64.f;
        const float phi = std::min(std::fma(cc[5], d, h0), std::fma(cc[7], d, h2)) + 1.f / 64.f;
        const int rx0 = std::max(x0s - WX0, 0), rx1 = std::min(x1s - WX0, 7);
        const int xs = std::max((int)std::ceil(fmed3(plo, -1.f, 9.f)), rx0);
        const int xe = std::min((int)std::floor(fmed3(phi, -1.f, 9.f)), rx1);
        const bool keep = xs <= x - WX0 && x - WX0 <= xe;
        const bool a = ref_accepts<T>(px_cx(M, W, x), px_cy(M, H, y), v, eps);
        ++cand;
        acc += a;
        culled += !keep;
        ++kc[kind];
        kacc[kind] += a;
        kcul[kind] += !keep;
        if (a && !keep) {
          if (++bad <= 10)
            printf("VIOLATION face %ld kind %d pixel (%d,%d) W %d H %d M %g eps %g\n", f, kind, x,
                   y, W, H, (double)M, (double)eps);
        }
      }
    }
  }
  const char *kn[6] = {"regular", "fan sliver", "edge-on sliver", "tiny", "large", "on centres"};
  for (int k = 0; k < 6; ++k)
    printf("  %-15s candidates %11ld accepted %5.1f%% culled %5.1f%% (of the rejects %5.1f%%)\n",
           kn[k], kc[k], 100.0 * kacc[k] / std::max(kc[k], 1L), 100.0 * kcul[k] / std::max(kc[k], 1L),
           100.0 * kcul[k] / std::max(kc[k] - kacc[k], 1L));
  printf("%s: faces %ld, box candidates %ld, accepted %ld, culled %ld (%.1f%%), violations %ld\n", sizeof(T) == 8 ? "f64" : "f32", nf,
         cand, acc, culled, 100.0 * culled / std::max(cand, 1L), bad);
  return bad != 0;
}

int main(int argc, char **argv) {
  const long nf = argc > 1 ? atol(argv[1]) : 200000;
  const long seed = argc > 2 ? atol(argv[2]) : 7;
  const bool f64 = argc > 3 && argv[3][0] == 'd';
  return f64 ? run<double>(nf, seed) : run<float>(nf, seed);
}
