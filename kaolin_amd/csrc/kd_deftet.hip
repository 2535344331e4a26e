// kd_deftet.hip -- deftet_sparse_render (kaolin/render/mesh/deftet.py:269-417,
// deftet_cuda.cu:31-453): every intersection of a pixel's ray with the mesh, in
// depth order, up to knum per pixel.
//
// Reference per pixel (arbitrary image coordinates, not a grid): walk ALL faces in index order;
// a face counts when the pixel is in its half-open box, its three eps-normalised barycentric
// weights are >= 0 and the interpolated depth is in [min_depth, max_depth); the first knum such
// faces (by index) are kept, then sorted by depth, descending (deftet.py:300-303), and the features
// interpolated with w2 = 1 - (w0 + w1) (:304-313).  Its kernel gives each pixel 32 lanes that test
// 32 faces per step and scans every face of the mesh.
//
// Here:
//   kd_dt_chunks  the union box of each 64-face chunk of each view (faces whose box has a NaN
//                 never pass the box test and are left out).
//   kd_dt_fwd     one wave per pixel.  Lane c tests chunk c's union box (a face box holding the
//                 pixel implies the union box does), the wave walks the passing chunks in order,
//                 lane l tests face 64 * chunk + l with the reference arithmetic, and the hits are
//                 appended in face order (ballot + mbcnt) to the wave's LDS list.  The walk stops
//                 at knum hits (later faces can no longer enter).  The list is then ranked by
//                 depth, descending, ties by face order (a stable order; the reference's
//                 torch.argsort is not stable, so tied depths are the one place it is unpinned),
//                 and each slot writes its face index, weights (w0, w1, 1 - (w0 + w1)) and
//                 interpolated features; empty slots get -1 / 0.
//   backward      the rasterize backward (kd_raster.hip, the same per-sample math:
//                 deftet_cuda.cu:238-402 == rasterization_cuda.cu:238-402) over the (pixel, slot)
//                 samples laid out as a P x knum image.
// The eps of the box-normalisation is the reference's float parameter (copysignf of it), also for
// fp64 data.
#include "kd_capi.hpp"
#include "kd_common.hpp"
#include "kd_raster.hpp"
#include "kd_tile.hpp"

namespace kd {

template <typename T>
struct DtBox {
  T x0, y0, x1, y1;
};

template <typename T>
__global__ __launch_bounds__(kWave) void kd_dt_chunks(int64_t F, int64_t nchunk, const T *fvi,
                                                      DtBox<T> *box) {
  const int b = blockIdx.y;
  const int64_t c = blockIdx.x;
  const int64_t f = c * kWave + threadIdx.x;
  const T inf = (T)INFINITY;
  T x0 = inf, y0 = inf, x1 = -inf, y1 = -inf;
  if (f < F) {
    const T *v = fvi + ((int64_t)b * F + f) * 6;
    const T mx = nmin3(v[0], v[2], v[4]), my = nmin3(v[1], v[3], v[5]);
    const T Mx = nmax3(v[0], v[2], v[4]), My = nmax3(v[1], v[3], v[5]);
    if (!(isnan(mx) || isnan(my) || isnan(Mx) || isnan(My))) {
      x0 = mx;
      y0 = my;
      x1 = Mx;
      y1 = My;
    }
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    x0 = fmin(x0, __shfl_xor(x0, s));
    y0 = fmin(y0, __shfl_xor(y0, s));
    x1 = fmax(x1, __shfl_xor(x1, s));
    y1 = fmax(y1, __shfl_xor(y1, s));
  }
  if (threadIdx.x == 0) box[(int64_t)b * nchunk + c] = DtBox<T>{x0, y0, x1, y1};
}

template <typename T>
struct DtArgs {
  int B;
  int64_t P, F, nchunk;
  int K, D;
  float eps;
  const T *px;      // (B, P, 2)
  const T *range;   // (B, P, 2): min, max depth
  const T *fvz;     // (B, F, 3)
  const T *fvi;     // (B, F, 3, 2)
  const T *feat;    // (B, F, 3, D)
  const DtBox<T> *box;
  T *interp;        // (B, P, K, D)
  int64_t *face_idx;  // (B, P, K)
  T *weights;       // (B, P, K, 3)
};

constexpr int kDtWaves = 4;  // pixels per workgroup

// per-wave LDS list of (depth, face, w0, w1), knum entries
template <typename T>
__device__ __forceinline__ void dt_carve(char *base, int K, T *&dep, T *&w0, T *&w1, int *&fid) {
  dep = (T *)base;
  w0 = dep + K;
  w1 = w0 + K;
  fid = (int *)(w1 + K);
}

template <typename T>
__host__ __device__ inline size_t dt_wave_lds(int K) {
  return (size_t)K * (3 * sizeof(T) + sizeof(int));
}

template <typename T>
__global__ __launch_bounds__(kWave *kDtWaves) void kd_dt_fwd(DtArgs<T> a) {
  extern __shared__ __align__(16) char dt_lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int K = a.K;
  T *dep, *lw0, *lw1;
  int *fid;
  dt_carve<T>(dt_lds + (size_t)w * dt_wave_lds<T>(K), K, dep, lw0, lw1, fid);
  const int b = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * kDtWaves + w;
  if (p >= a.P) return;  // whole wave
  const int64_t pp = (int64_t)b * a.P + p;
  const T x0 = a.px[2 * pp], y0 = a.px[2 * pp + 1];
  const T dmin = a.range[2 * pp], dmax = a.range[2 * pp + 1];
  const DtBox<T> *box = a.box + (int64_t)b * a.nchunk;
  const T *fvi = a.fvi + (int64_t)b * a.F * 6;
  const T *fvz = a.fvz + (int64_t)b * a.F * 3;
  const T eps = (T)a.eps;
  int num = 0;
  for (int64_t g0 = 0; g0 < a.nchunk && num < K; g0 += kWave) {
    bool in = false;
    if (g0 + lane < a.nchunk) {
      const DtBox<T> u = box[g0 + lane];
      in = x0 >= u.x0 && x0 < u.x1 && y0 >= u.y0 && y0 < u.y1;
    }
    for (uint64_t cm = __ballot(in); cm && num < K; cm &= cm - 1ull) {
      const int64_t f = (g0 + __builtin_ctzll(cm)) * kWave + lane;
      bool hit = false;
      T w0 = 0, w1 = 0, depth = 0;
      if (f < a.F) {
        const T *v = fvi + f * 6;
        const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
        // deftet_cuda.cu:114-126: half-open box of min / max corners
        const T xmin = nmin3(ax, bx, cx), xmax = nmax3(ax, bx, cx);
        const T ymin = nmin3(ay, by, cy), ymax = nmax3(ay, by, cy);
        if (x0 >= xmin && x0 < xmax && y0 >= ymin && y0 < ymax) {
          // :128-147, same operation order
          const T aex = ax - x0, aey = ay - y0, bex = bx - x0, bey = by - y0;
          const T cex = cx - x0, cey = cy - y0;
          const T _w0 = bex * cey - bey * cex;
          const T _w1 = cex * aey - cey * aex;
          const T _w2 = aex * bey - aey * bex;
          const T norm = _w0 + _w1 + _w2;
          const T ne = (T)copysignf((float)eps, (float)norm);
          w0 = _w0 / (norm + ne);
          w1 = _w1 / (norm + ne);
          const T w2 = _w2 / (norm + ne);
          if (w0 >= (T)0 && w1 >= (T)0 && w2 >= (T)0) {
            const T *z = fvz + f * 3;
            depth = w0 * z[0] + w1 * z[1] + w2 * z[2];  // :156
            hit = depth < dmax && depth >= dmin;        // :158
          }
        }
      }
      const uint64_t hm = __ballot(hit);
      if (hit) {
        const int at = num + (int)__builtin_amdgcn_mbcnt_hi(
                                 (uint32_t)(hm >> 32),
                                 __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
        if (at < K) {
          dep[at] = depth;
          lw0[at] = w0;
          lw1[at] = w1;
          fid[at] = (int)f;
        }
      }
      num += __popcll(hm);
    }
  }
  const int n = num < K ? num : K;
  wave_lds_sync();
  // rank: depth descending, then list (= face) order
  const int D = a.D;
  const int64_t row = pp * K;
  const T *feat = a.feat + (int64_t)b * a.F * 3 * D;
  for (int i = lane; i < n; i += kWave) {
    const T di = dep[i];
    int r = 0;
    for (int j = 0; j < n; ++j) {
      const T dj = dep[j];
      r += (dj > di || (dj == di && j < i)) ? 1 : 0;
    }
    const T w0 = lw0[i], w1 = lw1[i];
    const T w2 = (T)1 - (w0 + w1);  // deftet.py:304
    const int f = fid[i];
    const int64_t o = row + r;
    a.face_idx[o] = f;
    a.weights[3 * o] = w0;
    a.weights[3 * o + 1] = w1;
    a.weights[3 * o + 2] = w2;
    const T *c = feat + (int64_t)f * 3 * D;
    T *out = a.interp + o * D;
    for (int d = 0; d < D; ++d)  // :312-313, the sum over the 3 corners in order
      out[d] = w0 * c[d] + w1 * c[D + d] + w2 * c[2 * D + d];
  }
  for (int s = n + lane; s < K; s += kWave) {
    const int64_t o = row + s;
    a.face_idx[o] = -1;
    a.weights[3 * o] = (T)0;
    a.weights[3 * o + 1] = (T)0;
    a.weights[3 * o + 2] = (T)0;
    for (int d = 0; d < D; ++d) a.interp[o * D + d] = (T)0;
  }
}

template <typename T>
static size_t dt_workspace(int B, int64_t F) {
  return sizeof(DtBox<T>) * (size_t)B * (size_t)((F + kWave - 1) / kWave);
}

template <typename T>
static int dt_forward(int B, int64_t P, int64_t F, int K, int D, const T *px, const T *range,
                      const T *fvz, const T *fvi, const T *feat, float eps, T *interp,
                      int64_t *face_idx, T *weights, void *ws, size_t wsb, hipStream_t stream) {
  KD_CHECK_ARG(B >= 0 && B <= 65535 && P >= 0 && F >= 0 && D >= 0, "deftet: bad sizes");
  KD_CHECK_ARG(K >= 1, "deftet: knum must be >= 1");
  KD_CHECK_ARG(F < (1ll << 31), "deftet: too many faces");
  const size_t lds = dt_wave_lds<T>(K) * kDtWaves;
  KD_CHECK_ARG(lds <= 160 * 1024, "deftet: knum too large for the LDS list (fp32 <= 2560, "
                                  "fp64 <= 1462)");
  const size_t need = dt_workspace<T>(B, F);
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  if (B == 0 || P == 0) return KD_OK;
  const int64_t nchunk = (F + kWave - 1) / kWave;
  DtBox<T> *box = (DtBox<T> *)ws;
  if (nchunk > 0) {
    ProfScope prof(K_DT_CHUNKS, stream);
    hipLaunchKernelGGL(kd_dt_chunks<T>, dim3((unsigned)nchunk, B), dim3(kWave), 0, stream, F,
                       nchunk, fvi, box);
  }
  DtArgs<T> a{B, P, F, nchunk, K, D, eps, px, range, fvz, fvi, feat, box, interp, face_idx,
              weights};
  const int64_t gx = (P + kDtWaves - 1) / kDtWaves;
  KD_CHECK_ARG(gx < (1ll << 31), "deftet: too many pixels");
  {
    ProfScope prof(K_DT_FWD, stream);
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void *)kd_dt_fwd<T>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kd_dt_fwd<T>, dim3((unsigned)gx, B), dim3(kWave * kDtWaves), lds, stream,
                       a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "deftet fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
static int dt_backward(int B, int64_t P, int64_t F, int K, int D, const T *grad,
                       const int64_t *face_idx, const T *weights, const T *fvi, const T *feat,
                       float eps, T *gfvi, T *gfeat, hipStream_t stream) {
  KD_CHECK_ARG(B >= 0 && P >= 0 && F >= 0 && D >= 0 && K >= 1, "deftet: bad sizes");
  KD_CHECK_ARG(P < (1ll << 31), "deftet: too many pixels");
  KD_CHECK_ARG(gfvi, "deftet: grad_face_vertices_image is NULL");
  const int64_t nf = (int64_t)B * F;
  int rc = zero_buffers<T>(gfvi, nf * 6, gfeat, gfeat ? nf * 3 * D : 0, stream);
  if (rc != KD_OK || B == 0 || P == 0) return rc;
  // (pixel, slot) samples as a P x K image: deftet_cuda.cu:238-402 is rasterization_cuda.cu's math
  return raster_backward_launch<T>(B, (int)P, K, F, D, grad, face_idx, weights, fvi, feat, eps,
                                   gfvi, gfeat, stream);
}

}  // namespace kd

using namespace kd;

extern "C" {

size_t kd_deftet_workspace_size(int B, int64_t F, int double_precision) {
  if (B < 0 || F < 0) return 0;
  return double_precision ? dt_workspace<double>(B, F) : dt_workspace<float>(B, F);
}

int kd_deftet_sparse_render_forward_f32(int B, int64_t P, int64_t F, int knum, int D,
                                        const float *pixel_coords, const float *render_ranges,
                                        const float *fvz, const float *fvi, const float *feat,
                                        float eps, float *interp, int64_t *face_idx,
                                        float *weights, void *ws, size_t wsb, void *stream) {
  return dt_forward<float>(B, P, F, knum, D, pixel_coords, render_ranges, fvz, fvi, feat, eps,
                           interp, face_idx, weights, ws, wsb, (hipStream_t)stream);
}
int kd_deftet_sparse_render_forward_f64(int B, int64_t P, int64_t F, int knum, int D,
                                        const double *pixel_coords,
                                        const double *render_ranges, const double *fvz,
                                        const double *fvi, const double *feat, float eps,
                                        double *interp, int64_t *face_idx, double *weights,
                                        void *ws, size_t wsb, void *stream) {
  return dt_forward<double>(B, P, F, knum, D, pixel_coords, render_ranges, fvz, fvi, feat, eps,
                            interp, face_idx, weights, ws, wsb, (hipStream_t)stream);
}
int kd_deftet_sparse_render_backward_f32(int B, int64_t P, int64_t F, int knum, int D,
                                         const float *grad_interp, const int64_t *face_idx,
                                         const float *weights, const float *fvi,
                                         const float *feat, float eps, float *grad_fvi,
                                         float *grad_feat, void *stream) {
  return dt_backward<float>(B, P, F, knum, D, grad_interp, face_idx, weights, fvi, feat, eps,
                            grad_fvi, grad_feat, (hipStream_t)stream);
}
int kd_deftet_sparse_render_backward_f64(int B, int64_t P, int64_t F, int knum, int D,
                                         const double *grad_interp, const int64_t *face_idx,
                                         const double *weights, const double *fvi,
                                         const double *feat, float eps, double *grad_fvi,
                                         double *grad_feat, void *stream) {
  return dt_backward<double>(B, P, F, knum, D, grad_interp, face_idx, weights, fvi, feat, eps,
                             grad_fvi, grad_feat, (hipStream_t)stream);
}

}  // extern "C"
