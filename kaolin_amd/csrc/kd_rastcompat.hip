// kd_rastcompat.hip -- the nvdiffrast_fwd data path (kaolin/render/mesh/rasterization.py:145-241,
// SURVEY.md §8 f4): an external forward's `rast` buffer turned into what our rasterize backward
// consumes, plus the attribute interpolation.
//
// `rast` (B, H, W, 4) is nvdiffrast's wire format: (u, v, z/w, triangle_id + 1), 0 = empty.  The
// reference then runs, per pixel (:206-216):
//   interp    = nvdiff.interpolate(features, rast, tri)   -- u * a0 + v * a1 + (1 - u - v) * a2
//                                                            of the triangle's corner features
//   face_idx  = rast[..., 3].long() - 1
//   weights   = cat(rast[..., :2], 1 - sum(rast[..., :2]))
// and hands (face_idx, weights) to rasterize_backward_cuda.  One thread per pixel does all three
// here (tri = arange, so triangle t's corners are face t's three feature rows).  The third
// barycentric is 1 - (u + v), the reference's weights expression, for both the interpolation and
// the saved weights.  A triangle id outside [0, F] is treated as empty (nvdiffrast never emits
// one).  HBM: 4 * sizeof(T) in, (D + 3) * sizeof(T) + 8 out per pixel, plus the covered pixels'
// feature rows.
#include "kd_capi.hpp"
#include "kd_common.hpp"

namespace kd {

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_rast_interp(int64_t P, int64_t HW, int64_t F, int D,
                                                         const T *__restrict__ rast,
                                                         const T *__restrict__ feat,
                                                         T *__restrict__ interp,
                                                         int64_t *__restrict__ face_idx,
                                                         T *__restrict__ weights) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= P) return;
  T u, v, id;
  if (sizeof(T) == 4 && ((uintptr_t)rast & 15) == 0) {  // (the pixel's 16-byte row, one load)
    const float4 r = reinterpret_cast<const float4 *>(rast)[p];
    u = r.x;
    v = r.y;
    id = r.w;
  } else {
    u = rast[4 * p];
    v = rast[4 * p + 1];
    id = rast[4 * p + 3];
  }
  const T w2 = (T)1 - (u + v);  // rasterization.py:213-216
  store3(weights + 3 * p, u, v, w2);
  // .long() truncates toward zero; ids are exact integers in nvdiffrast's buffer
  const int64_t f = (id >= (T)1 && id <= (T)F) ? (int64_t)id - 1 : -1;
  face_idx[p] = f;
  T *out = interp + p * D;
  if (f < 0) {
    if (D == 2)
      store2(out, (T)0, (T)0);
    else
      for (int d = 0; d < D; ++d) out[d] = (T)0;
    return;
  }
  // (the launcher keeps P < 2^31: a 32-bit division)
  const int64_t b = (int64_t)((uint32_t)p / (uint32_t)HW);
  const T *a = feat + ((b * F + f) * 3) * (int64_t)D;
  if (D == 2)
    store2(out, u * a[0] + v * a[2] + w2 * a[4], u * a[1] + v * a[3] + w2 * a[5]);
  else
    for (int d = 0; d < D; ++d) out[d] = u * a[d] + v * a[D + d] + w2 * a[2 * D + d];
}

template <typename T>
static int rast_interp(int B, int H, int W, int64_t F, int D, const T *rast, const T *feat,
                       T *interp, int64_t *face_idx, T *weights, hipStream_t stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  KD_CHECK_ARG(F < (1ll << 24), "triangle ids above 2^24 are not exact in a float rast buffer");
  const int64_t P = (int64_t)B * H * W;
  if (P == 0) return KD_OK;
  KD_CHECK_ARG(P < (1ll << 31), "rasterize_from_rast: more than 2^31 pixels");
  KD_CHECK_ARG(rast && face_idx && weights && (D == 0 || (interp && feat)), "NULL buffer");
  {
    ProfScope prof(K_RAST_INTERP, stream);
    hipLaunchKernelGGL(kd_rast_interp<T>, dim3((unsigned)((P + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, P, (int64_t)H * W, F, D, rast, feat, interp,
                       face_idx, weights);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "rast interpolate: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

extern "C" {

int kd_rast_interpolate_f32(int B, int H, int W, int64_t F, int D, const float *rast,
                            const float *feat, float *interp, int64_t *face_idx, float *weights,
                            void *stream) {
  return rast_interp<float>(B, H, W, F, D, rast, feat, interp, face_idx, weights,
                            (hipStream_t)stream);
}
int kd_rast_interpolate_f64(int B, int H, int W, int64_t F, int D, const double *rast,
                            const double *feat, double *interp, int64_t *face_idx,
                            double *weights, void *stream) {
  return rast_interp<double>(B, H, W, F, D, rast, feat, interp, face_idx, weights,
                             (hipStream_t)stream);
}

}  // extern "C"
