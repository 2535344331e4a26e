// kd_metrics.hip -- mask_iou (kaolin/metrics/render.py:18-40), the silhouette loss of the DIB-R
// training step (examples/tutorial/ian_dibr.py:264-265), forward and backward.
//
// Reference:  mul = l * r;  add = l + r;  U_b = sum(mul);  D_b = sum(add - mul)
//             loss = 1 - mean_b(U_b / (D_b + 1e-10))
// Forward: one pass over both masks.  Workgroup (chunk, view) reduces its chunk (16-byte loads,
// fp64 accumulators, fixed order: deterministic) into a partial; a one-workgroup finisher sums
// the partials of each view in order, writes the per-view (U_b, D_b) the backward needs and the
// scalar loss.  Everything is read and written on the device: no host synchronisation.
// Backward (torch autograd of the same expression):
//   g_i = -g / B,  gu = g_i / (D + e),  gd = -g_i * U / ((D + e) * (D + e))
//   dL/dl = (gu - gd) * r + gd,   dL/dr = (gu - gd) * l + gd
// one elementwise pass that reads both masks and writes both gradients.  The incoming gradient g
// is a device scalar (what autograd hands over), read by every workgroup.
// HBM: forward 2 * sizeof(T) per pixel, backward 4 * sizeof(T) per pixel.
#include "kd_capi.hpp"
#include "kd_common.hpp"

namespace kd {

constexpr int kIouIters = 2;  // 16-byte loads per thread per chunk

template <typename T>
struct Vec16 {
  static constexpr int n = 16 / sizeof(T);
};

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) x += __shfl_xor(x, s);
  return x;
}

template <typename T>
__device__ __forceinline__ void iou_terms(T l, T r, double &u, double &d) {
  const T mul = l * r;               // render.py:35
  const T add = l + r;               // :36
  u += (double)mul;                  // :37
  d += (double)(add - mul);          // :38
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kBlock) void kd_iou_partial(int64_t P, int64_t chunk,
                                                         const T *__restrict__ lhs,
                                                         const T *__restrict__ rhs,
                                                         double2 *__restrict__ part) {
  const int b = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = min(c0 + chunk, P);
  const T *l = lhs + (int64_t)b * P, *r = rhs + (int64_t)b * P;
  double u = 0.0, d = 0.0;
  if (VEC) {  // P % n == 0 and 16-byte aligned rows; chunk is a multiple of n
    constexpr int n = Vec16<T>::n;
    using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
    for (int64_t i = c0 + (int64_t)threadIdx.x * n; i < c1; i += (int64_t)kBlock * n) {
      const V lv = *(const V *)(l + i), rv = *(const V *)(r + i);
      const T *la = (const T *)&lv, *ra = (const T *)&rv;
#pragma unroll
      for (int k = 0; k < n; ++k) iou_terms<T>(la[k], ra[k], u, d);
    }
  } else {
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlock) iou_terms<T>(l[i], r[i], u, d);
  }
  u = wave_sum(u);
  d = wave_sum(d);
  __shared__ double s_u[kBlock / kWave], s_d[kBlock / kWave];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_u[w] = u;
    s_d[w] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[(int64_t)b * gridDim.x + blockIdx.x] =
        make_double2(s_u[0] + s_u[1] + s_u[2] + s_u[3], s_d[0] + s_d[1] + s_d[2] + s_d[3]);
}

// One workgroup: per view (one wave each, in turn) the ordered sum of its partials, then the loss.
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_iou_finish(int B, int nchunk,
                                                        const double2 *__restrict__ part,
                                                        T *__restrict__ stats, T *__restrict__ loss,
                                                        T *__restrict__ iou_out) {
  extern __shared__ double s_iou[];  // [B]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int b = w; b < B; b += kBlock / kWave) {
    double u = 0.0, d = 0.0;
    for (int c = lane; c < nchunk; c += kWave) {
      const double2 p = part[(int64_t)b * nchunk + c];
      u += p.x;
      d += p.y;
    }
    u = wave_sum(u);
    d = wave_sum(d);
    if (lane == 0) {
      const T U = (T)u, D = (T)d;
      const T iou = U / (D + (T)1e-10);  // render.py:39
      stats[2 * b] = U;
      stats[2 * b + 1] = D;
      if (iou_out) iou_out[b] = iou;
      s_iou[b] = (double)iou;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    T s = (T)0;
    for (int b = 0; b < B; ++b) s += (T)s_iou[b];
    *loss = (T)1.0 - s / (T)B;  // :40
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kBlock) void kd_iou_bwd(int64_t P, const T *__restrict__ lhs,
                                                     const T *__restrict__ rhs,
                                                     const T *__restrict__ stats,
                                                     const T *__restrict__ grad, int B,
                                                     T *__restrict__ gl, T *__restrict__ gr) {
  const int b = blockIdx.y;
  const T g = *grad;
  const T gi = -(g / (T)B);                       // mean and 1 - x
  const T U = stats[2 * b], Dp = stats[2 * b + 1] + (T)1e-10;
  const T gu = gi / Dp;                           // DivBackward: grad / other
  const T gd = -gi * U / (Dp * Dp);               //              -grad * self / other^2
  const T gm = gu - gd;                           // mul feeds U (+) and D (-)
  const int64_t off = (int64_t)b * P;
  if (VEC) {
    constexpr int n = Vec16<T>::n;
    using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
    for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * n; i < P;
         i += (int64_t)gridDim.x * kBlock * n) {
      const V lv = *(const V *)(lhs + off + i), rv = *(const V *)(rhs + off + i);
      V ol, orr;
      const T *la = (const T *)&lv, *ra = (const T *)&rv;
      T *oa = (T *)&ol, *ob = (T *)&orr;
#pragma unroll
      for (int k = 0; k < n; ++k) {
        oa[k] = gm * ra[k] + gd;
        ob[k] = gm * la[k] + gd;
      }
      if (gl) *(V *)(gl + off + i) = ol;
      if (gr) *(V *)(gr + off + i) = orr;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P;
         i += (int64_t)gridDim.x * kBlock) {
      const T l = lhs[off + i], r = rhs[off + i];
      if (gl) gl[off + i] = gm * r + gd;
      if (gr) gr[off + i] = gm * l + gd;
    }
  }
}

static bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// chunking of one view's P pixels: >= ~2048 workgroups over the batch where the size allows
static int64_t iou_chunk(int B, int64_t P, int n) {
  int64_t chunk = (int64_t)kBlock * n * kIouIters;
  const int64_t want = 2048 / (B > 0 ? B : 1);
  while (chunk > (int64_t)kBlock * n && (P + chunk - 1) / chunk < want) chunk >>= 1;
  while ((P + chunk - 1) / chunk > 65535) chunk <<= 1;
  return chunk;
}

size_t iou_workspace_bytes(int B, int64_t P, int esize) {
  if (B <= 0 || P <= 0) return 0;
  const int64_t nchunk = (P + iou_chunk(B, P, 16 / esize) - 1) / iou_chunk(B, P, 16 / esize);
  return sizeof(double2) * (size_t)B * (size_t)nchunk;
}

// The loss from per-view (U_b, D_b) partials accumulated elsewhere (the fused DIB-R forward:
// acc[b][nparts] in fp64): the same finisher as mask_iou's.
template <typename T>
int iou_finish_launch(int B, int nparts, const double *acc, T *stats, T *loss,
                      hipStream_t stream) {
  hipLaunchKernelGGL(kd_iou_finish<T>, dim3(1), dim3(kBlock), sizeof(double) * B, stream, B,
                     nparts, (const double2 *)acc, stats, loss, (T *)nullptr);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "mask_iou: %s", hipGetErrorString(e));
  return KD_OK;
}
template int iou_finish_launch<float>(int, int, const double *, float *, float *, hipStream_t);
template int iou_finish_launch<double>(int, int, const double *, double *, double *,
                                       hipStream_t);

template <typename T>
static int iou_forward(int B, int64_t P, const T *lhs, const T *rhs, T *loss, T *stats, T *iou,
                       void *ws, size_t wsb, hipStream_t stream) {
  KD_CHECK_ARG(B >= 1 && B <= 65535 && P >= 0, "mask_iou: need 1 <= batch <= 65535, pixels >= 0");
  KD_CHECK_ARG(loss && stats, "mask_iou: loss / stats are NULL");
  KD_CHECK_ARG(P == 0 || (lhs && rhs), "mask_iou: NULL mask");
  const size_t need = iou_workspace_bytes(B, P, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  constexpr int n = Vec16<T>::n;
  const int64_t chunk = iou_chunk(B, P, n);
  const int nchunk = P > 0 ? (int)((P + chunk - 1) / chunk) : 0;
  const bool vec = P % n == 0 && aligned16(lhs) && aligned16(rhs);
  double2 *part = (double2 *)ws;
  if (nchunk > 0) {
    ProfScope prof(K_IOU_FWD, stream);
    const dim3 grid((unsigned)nchunk, (unsigned)B);
    if (vec)
      hipLaunchKernelGGL((kd_iou_partial<T, true>), grid, dim3(kBlock), 0, stream, P, chunk, lhs,
                         rhs, part);
    else
      hipLaunchKernelGGL((kd_iou_partial<T, false>), grid, dim3(kBlock), 0, stream, P, chunk, lhs,
                         rhs, part);
  }
  hipLaunchKernelGGL(kd_iou_finish<T>, dim3(1), dim3(kBlock), sizeof(double) * B, stream, B,
                     nchunk, part, stats, loss, iou);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "mask_iou: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
static int iou_backward(int B, int64_t P, const T *lhs, const T *rhs, const T *stats,
                        const T *grad, T *gl, T *gr, hipStream_t stream) {
  KD_CHECK_ARG(B >= 1 && B <= 65535 && P >= 0, "mask_iou: need 1 <= batch <= 65535, pixels >= 0");
  KD_CHECK_ARG(stats && grad, "mask_iou: stats / grad_loss are NULL");
  if (P == 0 || (!gl && !gr)) return KD_OK;
  constexpr int n = Vec16<T>::n;
  const bool vec = P % n == 0 && aligned16(lhs) && aligned16(rhs) && (!gl || aligned16(gl)) &&
                   (!gr || aligned16(gr));
  const int64_t per = (int64_t)kBlock * (vec ? n : 1) * kIouIters;
  int64_t gx = (P + per - 1) / per;
  gx = gx > 65535 ? 65535 : gx;
  {
    ProfScope prof(K_IOU_BWD, stream);
    const dim3 grid((unsigned)gx, (unsigned)B);
    if (vec)
      hipLaunchKernelGGL((kd_iou_bwd<T, true>), grid, dim3(kBlock), 0, stream, P, lhs, rhs, stats,
                         grad, B, gl, gr);
    else
      hipLaunchKernelGGL((kd_iou_bwd<T, false>), grid, dim3(kBlock), 0, stream, P, lhs, rhs,
                         stats, grad, B, gl, gr);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "mask_iou bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

extern "C" {

size_t kd_mask_iou_workspace_size(int B, int64_t pixels, int double_precision) {
  return iou_workspace_bytes(B, pixels, double_precision ? 8 : 4);
}

int kd_mask_iou_forward_f32(int B, int64_t pixels, const float *lhs, const float *rhs,
                            float *loss, float *stats, float *iou, void *ws, size_t wsb,
                            void *stream) {
  return iou_forward<float>(B, pixels, lhs, rhs, loss, stats, iou, ws, wsb, (hipStream_t)stream);
}
int kd_mask_iou_forward_f64(int B, int64_t pixels, const double *lhs, const double *rhs,
                            double *loss, double *stats, double *iou, void *ws, size_t wsb,
                            void *stream) {
  return iou_forward<double>(B, pixels, lhs, rhs, loss, stats, iou, ws, wsb, (hipStream_t)stream);
}
int kd_mask_iou_backward_f32(int B, int64_t pixels, const float *lhs, const float *rhs,
                             const float *stats, const float *grad_loss, float *grad_lhs,
                             float *grad_rhs, void *stream) {
  return iou_backward<float>(B, pixels, lhs, rhs, stats, grad_loss, grad_lhs, grad_rhs,
                             (hipStream_t)stream);
}
int kd_mask_iou_backward_f64(int B, int64_t pixels, const double *lhs, const double *rhs,
                             const double *stats, const double *grad_loss, double *grad_lhs,
                             double *grad_rhs, void *stream) {
  return iou_backward<double>(B, pixels, lhs, rhs, stats, grad_loss, grad_lhs, grad_rhs,
                              (hipStream_t)stream);
}

}  // extern "C"
