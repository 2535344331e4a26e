// kd_raster.hip -- rasterize forward / backward for gfx950.
//
// Forward (replaces packed_rasterize_forward_cuda_kernel, rasterization_cuda.cu:43-192):
//   one 256-thread workgroup per 16x16 pixel tile, one wave per 8x8 sub-tile (kd_tile.hpp).
//   The workgroup walks its coarse bin (ascending face order), keeps the faces whose exact pixel
//   span touches the tile and stages their corners and depths in LDS (SoA).  Each wave keeps the
//   spans of the faces touching its 8x8 sub-tile in registers; every lane (pixel) walks them in
//   order (readlane broadcast), and for the faces whose box holds its centre runs the
//   reference's exact test with LDS broadcast reads: the same sequence of faces the reference
//   visits, minus faces whose box misses the pixel, so face_idx / weights / features are
//   bit-identical.
// Backward (replaces rasterize_backward_cuda_kernel, rasterization_cuda.cu:238-402):
//   kd_raster_bwd_tile    -- one workgroup per 16x16 tile; a pixel's terms (6 corner terms summed
//                            over the features, 3*D feature terms) are summed per face in an LDS
//                            hash table, then flushed with one float atomic per (tile, face, term).
//                            Accepts any face_idx (the reference op's contract).
//   kd_raster_bwd_atomic  -- the same per pixel for wide features (D > 8).
#include "../../include/kaolin_dibr.h"
#include "kd_binning.hpp"
#include "kd_capi.hpp"
#include "kd_raster.hpp"
#include "kd_raster_bwd.hpp"
#include "kd_raster_pairs.hpp"
#include "kd_tile.hpp"

#include <type_traits>

namespace kd {


template <typename T>
__global__ __launch_bounds__(kBlock) void kd_raster_fwd(RasterFwdArgs<T> a) {
  __shared__ TileLists L;
  __shared__ T s_geo[9][kCap];  // ax ay bx by cx cy (scaled), az bz cz

  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W;
  int b, tl, nbin;
  tile_of_block(a.bb, H, W, b, tl, nbin, fs.dbg);
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  TileGeom t = tile_geom(H, W, tl);
  t.nbin = nbin;
  const T x0 = (T)px_cx(fs.M, W, t.px);
  const T y0 = (T)px_cy(fs.M, H, t.py);

  T max_z0 = (T)-INFINITY;
  int best = -1;
  T bw0 = 0., bw1 = 0., bw2 = 0.;

  auto stage = [&](int k, int64_t fi) {
    T v[6];
    load_corners(fs, fi, v);
#pragma unroll
    for (int q = 0; q < 6; ++q) s_geo[q][k] = v[q];
    const T *zz = a.fvz + fi * a.fvz_fs;
    s_geo[6][k] = zz[0];
    s_geo[7][k] = zz[a.fvz_cs];
    s_geo[8][k] = zz[2 * a.fvz_cs];
  };
  auto round = [&](int nsub, int) {
    if (nsub == 0 || ablate(fs.dbg, 1)) return;
    const SubSpans ss = load_subspans(L, nsub);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c * kWave >= nsub) break;
      const int nj = min(kWave, nsub - c * kWave);
      for (int l = 0; l < nj; ++l) {  // the sub-list in ascending face order
        PSpan sp;
        sp.lo = (uint32_t)__builtin_amdgcn_readlane((int)ss.s[c].lo, l);
        sp.hi = (uint32_t)__builtin_amdgcn_readlane((int)ss.s[c].hi, l);
        if (!t.inimg || !pspan_has(sp, t.px, t.py)) continue;  // :115, exact on spans
        const int k = __builtin_amdgcn_readlane(ss.k[c], l);
        T w0, w1, w2, z0;
        if (!raster_face_test<T>(x0, y0, s_geo[0][k], s_geo[1][k], s_geo[2][k], s_geo[3][k],
                                 s_geo[4][k], s_geo[5][k], s_geo[6][k], s_geo[7][k],
                                 s_geo[8][k], a.eps, w0, w1, w2, z0))
          continue;
        if (z0 <= max_z0) continue;  // :162, strict: ties keep the lower index
        max_z0 = z0;
        best = L.f[k];
        bw0 = w0;
        bw1 = w1;
        bw2 = w2;
      }
    }
  };
  tile_rounds(L, a.bb, (int)(hi - lo), b, lo, t, stage, round, fs.dbg);

  if (!t.inimg) return;
  const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
  a.face_idx[p] = best;
  T *wo = a.weights + p * 3;
  T *io = a.interp + p * a.D;
  if (best >= 0) {
    wo[0] = bw0;
    wo[1] = bw1;
    wo[2] = bw2;
    const T *r = a.feat + (lo + best) * 3 * a.D;
    for (int d = 0; d < a.D; ++d)
      io[d] = bw0 * r[d] + bw1 * r[a.D + d] + bw2 * r[2 * a.D + d];
  } else {
    wo[0] = 0.;
    wo[1] = 0.;
    wo[2] = 0.;
    for (int d = 0; d < a.D; ++d) io[d] = 0.;
  }
}


template <typename T>
__global__ __launch_bounds__(kBlock, sizeof(T) == 8 ? 4 : 6) void kd_raster_fwd_pairs(
    RasterFwdArgs<T> a) {
  TileClock clk(a.fs.tbuf, 0);
  __shared__ RasterPairsLDS<T> S;
  if (ablate(a.fs.dbg, 16384)) return;  // diagnostics: dispatch cost only
  int b, tl, nbin;
  tile_of_block(a.bb, a.fs.H, a.fs.W, b, tl, nbin, a.fs.dbg);
  raster_pairs_tile<T>(a, b, tl, nbin, S);
}

// General per-pixel form for wide features (D > 8): one thread per pixel, float atomics.
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_raster_bwd_atomic(
    int B, int H, int W, int64_t F, int D, const T *__restrict__ grad, const int64_t *face_idx,
    const T *__restrict__ weights, const T *__restrict__ fvi, const T *__restrict__ feat,
    float eps, T *grad_fvi, T *grad_feat) {
  const int64_t P = (int64_t)H * W;
  const int64_t total = (int64_t)B * P;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * kBlock) {
    const int64_t fi = face_idx[p];
    if (fi < 0 || fi >= F) continue;
    const int64_t b = p / P;
    const int64_t tf = b * F + fi;
    const T wts[3] = {weights[p * 3], weights[p * 3 + 1], weights[p * 3 + 2]};
    const T *g = grad + p * D;
    if (grad_feat)
      for (int ii = 0; ii < 3; ++ii)
        for (int d = 0; d < D; ++d) atomicAdd(grad_feat + tf * 3 * D + ii * D + d, g[d] * wts[ii]);
    const T *v = fvi + tf * 6;
    const T *c = feat + tf * 3 * D;
    // same terms as raster_bwd_pixel, features streamed one at a time
    const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
    const T x0 = wts[0] * ax + wts[1] * bx + wts[2] * cx;
    const T y0 = wts[0] * ay + wts[1] * by + wts[2] * cy;
    const T m = bx - ax, pp = by - ay, n = cx - ax, q = cy - ay, s = x0 - ax, t = y0 - ay;
    const T k1 = s * q - n * t, k2 = m * t - s * pp;
    T k3 = m * q - n * pp;
    k3 = (T)((double)k3 + copysign((double)eps, (double)k3));
    const T zero = (T)0;
    const T dw1dm = zero * k3 - q * k1, dw1dn = -t * k3 - (-pp) * k1;
    const T dw1dp = zero * k3 - (-n) * k1, dw1dq = s * k3 - m * k1;
    const T dw1ds = q * k3 - zero * k1, dw1dt = -n * k3 - zero * k1;
    const T dw2dm = t * k3 - q * k2, dw2dn = zero * k3 - (-pp) * k2;
    const T dw2dp = -s * k3 - (-n) * k2, dw2dq = zero * k3 - m * k2;
    const T dw2ds = -pp * k3 - zero * k2, dw2dt = m * k3 - zero * k2;
    const T dw1[6] = {-(dw1dm + dw1dn + dw1ds), -(dw1dp + dw1dq + dw1dt), dw1dm, dw1dp, dw1dn,
                      dw1dq};
    const T dw2[6] = {-(dw2dm + dw2dn + dw2ds), -(dw2dp + dw2dq + dw2dt), dw2dm, dw2dp, dw2dn,
                      dw2dq};
    T gv[6] = {0, 0, 0, 0, 0, 0};
    for (int d = 0; d < D; ++d) {
      const T c0 = c[d], c1 = c[D + d], c2 = c[2 * D + d];
      const T dldI = g[d] / (k3 * k3);
#pragma unroll
      for (int j = 0; j < 6; ++j) gv[j] += dldI * ((c1 - c0) * dw1[j] + (c2 - c0) * dw2[j]);
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) atomicAdd(grad_fvi + tf * 6 + j, gv[j]);
  }
}

template <typename T, int DMAX>
__global__ __launch_bounds__(kBlock) void kd_raster_bwd_tile(RasterBwdArgs<T> ra) {
  raster_bwd_tile_body<T, DMAX>(ra, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y,
                                gridDim.x);
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
// the pair pipeline with edge culling (fp32 and fp64; debug flag 8: the lane-per-pixel kernel)
template <typename T>
bool raster_uses_cull() {
  return !(KD_DIAG != 0 && (debug_flags() & 8) != 0);
}

template <typename T>
int raster_launch(RasterFwdArgs<T> &a, hipStream_t stream) {
  const FaceSet<T> &fs = a.fs;
  a.fs.dbg = debug_flags();
  a.fs.tbuf = debug_tile_buffer();
  const int ntiles = ((fs.W + kTile - 1) / kTile) * ((fs.H + kTile - 1) / kTile);
  {
    ProfScope prof(K_RASTER_FWD, stream);
    if (a.bb.cull)
      hipLaunchKernelGGL(kd_raster_fwd_pairs<T>, dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
    else if constexpr (KD_DIAG)  // (diagnostic flag 8: the lane-per-pixel kernel)
      hipLaunchKernelGGL(kd_raster_fwd<T>, dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "raster fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int raster_forward(const FaceSet<T> &fs, int64_t max_per_view, const T *fvz, const T *feat,
                   int D, float eps, T *interp, int64_t *face_idx, T *weights, void *ws,
                   size_t ws_bytes, hipStream_t stream) {
  const size_t need = bin_workspace_bytes(fs.B, fs.H, fs.W, fs.N, max_per_view);
  if (ws_bytes < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  if (fs.B == 0 || fs.H == 0 || fs.W == 0) return KD_OK;
  size_t off = 0;
  BinBuffers bb = bin_carve(ws, off, fs.B, fs.H, fs.W, fs.N, max_per_view);
  if (!raster_uses_cull<T>()) bb.cull = nullptr;
  bb.cull_eps = eps;
  hipError_t e = bin_faces<T>(fs, bb, stream);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "binning: %s", hipGetErrorString(e));
  RasterFwdArgs<T> a{fs, bb, fvz, 3, 1, feat, D, eps, interp, face_idx, weights};
  return raster_launch<T>(a, stream);
}

// The tile kernel only (gfvi / gfeat must hold zeros or partial sums to add to).
template <typename T>
int raster_backward_launch(int B, int H, int W, int64_t F, int D, const T *grad,
                           const int64_t *fidx, const T *weights, const T *fvi, const T *feat,
                           float eps, T *gfvi, T *gfeat, hipStream_t stream) {
  const int64_t nf = (int64_t)B * F;
  const int64_t total = (int64_t)B * H * W;
  if (total > 0 && nf > 0) {
    const int ntiles = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    const RasterBwdArgs<T> ra{B,   H,    W,   F,    D,     grad, fidx,
                              weights, fvi, feat, eps, gfvi, gfeat, debug_flags()};
    if (D <= 3) {  // 6 + 3 D <= 15 terms: 16 KB of LDS terms, 8 workgroups per CU
      ProfScope prof(K_RASTER_BWD_TILE, stream);
      hipLaunchKernelGGL((kd_raster_bwd_tile<T, 3>), dim3(ntiles, B), dim3(kBlock), 0, stream,
                         ra);
    } else if (D <= 4) {
      ProfScope prof(K_RASTER_BWD_TILE, stream);
      hipLaunchKernelGGL((kd_raster_bwd_tile<T, 4>), dim3(ntiles, B), dim3(kBlock), 0, stream,
                         ra);
    } else if (D <= 8) {
      ProfScope prof(K_RASTER_BWD_TILE, stream);
      hipLaunchKernelGGL((kd_raster_bwd_tile<T, 8>), dim3(ntiles, B), dim3(kBlock), 0, stream,
                         ra);
    } else {
      const int64_t blocks = (total + kBlock - 1) / kBlock;
      ProfScope prof(K_RASTER_BWD_ATOMIC, stream);
      hipLaunchKernelGGL(kd_raster_bwd_atomic<T>,
                         dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(kBlock), 0,
                         stream, B, H, W, F, D, grad, fidx, weights, fvi, feat, eps, gfvi, gfeat);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "raster bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int raster_backward(int B, int H, int W, int64_t F, int D, const T *grad, const int64_t *fidx,
                    const T *weights, const T *fvi, const T *feat, float eps, T *gfvi, T *gfeat,
                    hipStream_t stream) {
  const int64_t nf = (int64_t)B * F;
  if (nf > 0) {
    const int rc = zero_buffers<T>(gfvi, nf * 6, gfeat, gfeat ? nf * 3 * D : 0, stream);
    if (rc != KD_OK) return rc;
  }
  return raster_backward_launch<T>(B, H, W, F, D, grad, fidx, weights, fvi, feat, eps, gfvi,
                                   gfeat, stream);
}

template bool raster_uses_cull<float>();
template bool raster_uses_cull<double>();
template int raster_launch<float>(RasterFwdArgs<float> &, hipStream_t);
template int raster_launch<double>(RasterFwdArgs<double> &, hipStream_t);
template int raster_backward_launch<float>(int, int, int, int64_t, int, const float *,
                                           const int64_t *, const float *, const float *,
                                           const float *, float, float *, float *, hipStream_t);
template int raster_backward_launch<double>(int, int, int, int64_t, int, const double *,
                                            const int64_t *, const double *, const double *,
                                            const double *, float, double *, double *,
                                            hipStream_t);

}  // namespace kd

// ==============================================================================================
// C ABI
// ==============================================================================================
using namespace kd;

template <typename T>
static int packed_fwd(int B, int H, int W, int64_t Fp, int D, const T *fvz, const T *fvi,
                      const T *bboxes, const T *feat, const int64_t *first_idx, float M, float eps,
                      T *interp, int64_t *face_idx, T *weights, void *ws, size_t ws_bytes,
                      void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && Fp >= 0 && D >= 0, "negative size");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG(Fp < (1ll << 31), "too many faces");
  KD_CHECK_ARG(first_idx || B == 0, "first_idx is NULL");
  FaceSet<T> fs{};
  fs.B = B;
  fs.H = H;
  fs.W = W;
  fs.N = Fp;
  fs.F = 0;
  fs.first_idx = first_idx;
  fs.fvi = fvi;
  fs.scale = (T)1;
  fs.bbox = bboxes;
  fs.M = M;
  return raster_forward<T>(fs, Fp, fvz, feat, D, eps, interp, face_idx, weights, ws, ws_bytes,
                           (hipStream_t)stream);
}

template <typename T>
static int batched_fwd(int B, int H, int W, int64_t F, int D, const T *fvz, const T *fvi,
                       const T *feat, const uint8_t *valid, double M, float eps, T *interp,
                       int64_t *face_idx, T *weights, void *ws, size_t ws_bytes, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  FaceSet<T> fs{};
  fs.B = B;
  fs.H = H;
  fs.W = W;
  fs.N = (int64_t)B * F;
  fs.F = F;
  fs.fvi = fvi;
  fs.scale = (T)M;
  fs.valid = valid;
  fs.M = (float)M;
  return raster_forward<T>(fs, F, fvz, feat, D, eps, interp, face_idx, weights, ws, ws_bytes,
                           (hipStream_t)stream);
}

extern "C" {

int kd_packed_rasterize_forward_f32(int B, int H, int W, int64_t Fp, int D, const float *fvz,
                                    const float *fvi, const float *bboxes, const float *feat,
                                    const int64_t *first_idx, float M, float eps, float *interp,
                                    int64_t *face_idx, float *weights, void *ws, size_t wsb,
                                    void *stream) {
  return packed_fwd<float>(B, H, W, Fp, D, fvz, fvi, bboxes, feat, first_idx, M, eps, interp,
                           face_idx, weights, ws, wsb, stream);
}
int kd_packed_rasterize_forward_f64(int B, int H, int W, int64_t Fp, int D, const double *fvz,
                                    const double *fvi, const double *bboxes, const double *feat,
                                    const int64_t *first_idx, float M, float eps, double *interp,
                                    int64_t *face_idx, double *weights, void *ws, size_t wsb,
                                    void *stream) {
  return packed_fwd<double>(B, H, W, Fp, D, fvz, fvi, bboxes, feat, first_idx, M, eps, interp,
                            face_idx, weights, ws, wsb, stream);
}

int kd_rasterize_forward_f32(int B, int H, int W, int64_t F, int D, const float *fvz,
                             const float *fvi, const float *feat, const uint8_t *valid, double M,
                             float eps, float *interp, int64_t *face_idx, float *weights,
                             void *ws, size_t wsb, void *stream) {
  return batched_fwd<float>(B, H, W, F, D, fvz, fvi, feat, valid, M, eps, interp, face_idx,
                            weights, ws, wsb, stream);
}
int kd_rasterize_forward_f64(int B, int H, int W, int64_t F, int D, const double *fvz,
                             const double *fvi, const double *feat, const uint8_t *valid,
                             double M, float eps, double *interp, int64_t *face_idx,
                             double *weights, void *ws, size_t wsb, void *stream) {
  return batched_fwd<double>(B, H, W, F, D, fvz, fvi, feat, valid, M, eps, interp, face_idx,
                             weights, ws, wsb, stream);
}

int kd_rasterize_backward_f32(int B, int H, int W, int64_t F, int D, const float *grad,
                              const int64_t *fidx, const float *weights, const float *fvi,
                              const float *feat, float eps, float *gfvi, float *gfeat,
                              void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  return raster_backward<float>(B, H, W, F, D, grad, fidx, weights, fvi, feat, eps, gfvi, gfeat,
                                (hipStream_t)stream);
}
int kd_rasterize_backward_f64(int B, int H, int W, int64_t F, int D, const double *grad,
                              const int64_t *fidx, const double *weights, const double *fvi,
                              const double *feat, float eps, double *gfvi, double *gfeat,
                              void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  return raster_backward<double>(B, H, W, F, D, grad, fidx, weights, fvi, feat, eps, gfvi, gfeat,
                                 (hipStream_t)stream);
}

}  // extern "C"
