// kd_texture.hip -- texture_mapping (kaolin/render/mesh/utils.py:23-76): the uv -> texture lookup
// that consumes dibr_rasterization's interpolated uvs in the DIB-R training step
// (examples/tutorial/ian_dibr.py:248-252), forward and backward.
//
// Reference: uv clamped to [0, 1] (:66), mapped to [-1, 1] with y flipped (:67-68), then
// torch.nn.functional.grid_sample(align_corners=False, padding_mode='border', mode) (:71-75).
// Restated per sample (the grid_sampler_2d arithmetic, in T, no contraction):
//   gx = u * 2 - 1;  gy = -(v * 2 - 1)
//   ix = ((gx + 1) * Wt - 1) / 2  clipped to [0, Wt - 1];  iy likewise with Ht   (border)
//   nearest:  texel (rint(ix), rint(iy))  (round half to even, like nearbyint)
//   bilinear: the four taps around (ix, iy) with weights (x_se - ix)(y_se - iy) ..., out of range
//             taps contribute nothing.
// Layout: coords (B, N, 2) (N = h * w for a dense image), texture (Bt, C, Ht, Wt) with Bt == B
// or a batch stride of 0 (one texture shared by all views: `expand` instead of the reference's
// `repeat`), output (B, N, C) -- the reference's permuted result written directly.
// One thread per sample, all C channels; each tap is C loads a plane apart.  Backward: the
// texture gradient by float atomics (texels of neighbouring samples coincide) into a buffer zeroed
// here, and for bilinear the coordinate gradient through border clipping, the y flip, the affine
// map and the clamp (0 outside [0, 1], like torch.clamp's backward).
#include "kd_capi.hpp"
#include "kd_common.hpp"

namespace kd {

enum { KD_TEX_NEAREST = 0, KD_TEX_BILINEAR = 1 };

template <typename T>
struct TexArgs {
  int64_t N;
  int C, Ht, Wt;
  const T *coords;    // (B, N, 2)
  const T *tex;       // (Bt, C, Ht, Wt)
  int64_t tex_bstride;
  T *out;             // (B, N, C)
  const T *grad_out;  // (B, N, C)
  T *grad_tex;        // same layout as tex (batch stride tex_bstride)
  T *grad_coords;     // (B, N, 2)
};

// source index along one axis (grid_sampler_compute_source_index, align_corners=False, border)
template <typename T>
__device__ __forceinline__ T tex_source(T g, int size, T &dmult) {
  T x = ((g + (T)1) * (T)size - (T)1) / (T)2;
  dmult = (T)size / (T)2;
  // clip_coordinates_set_grad: the gradient is cut where the coordinate is clipped
  if (x <= (T)0) {
    dmult = (T)0;
    return (T)0;
  }
  if (x >= (T)(size - 1)) {
    dmult = (T)0;
    return (T)(size - 1);
  }
  return x;
}

template <typename T>
__device__ __forceinline__ void tex_coord(const T *c, T &ix, T &iy, T &mx, T &my, T &cu, T &cv,
                                          int Wt, int Ht) {
  const T u = c[0], v = c[1];
  // utils.py:66; fmax / fmin map NaN to 0, which keeps every index in range
  const T uc = fmin(fmax(u, (T)0), (T)1);
  const T vc = fmin(fmax(v, (T)0), (T)1);
  cu = (u >= (T)0 && u <= (T)1) ? (T)1 : (T)0;  // clamp backward mask
  cv = (v >= (T)0 && v <= (T)1) ? (T)1 : (T)0;
  const T gx = uc * (T)2 - (T)1;     // :67
  const T gy = -(vc * (T)2 - (T)1);  // :68
  ix = tex_source<T>(gx, Wt, mx);
  iy = tex_source<T>(gy, Ht, my);
}

template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_fwd(TexArgs<T> a) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (n >= a.N) return;
  const int64_t s = (int64_t)b * a.N + n;
  T ix, iy, mx, my, cu, cv;
  tex_coord<T>(a.coords + 2 * s, ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
  const int64_t plane = (int64_t)a.Ht * a.Wt;
  const T *tex = a.tex + (int64_t)b * a.tex_bstride;
  T *out = a.out + s * a.C;
  if (MODE == KD_TEX_NEAREST) {
    const int x = (int)rint(ix), y = (int)rint(iy);
    const bool in = x >= 0 && x < a.Wt && y >= 0 && y < a.Ht;
    const T *t = tex + (int64_t)y * a.Wt + x;
    for (int c = 0; c < a.C; ++c) out[c] = in ? t[c * plane] : (T)0;
  } else {
    const T fx = floor(ix), fy = floor(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const T wnw = ((T)x1 - ix) * ((T)y1 - iy), wne = (ix - (T)x0) * ((T)y1 - iy);
    const T wsw = ((T)x1 - ix) * (iy - (T)y0), wse = (ix - (T)x0) * (iy - (T)y0);
    const bool vx0 = x0 >= 0 && x0 < a.Wt, vx1 = x1 >= 0 && x1 < a.Wt;
    const bool vy0 = y0 >= 0 && y0 < a.Ht, vy1 = y1 >= 0 && y1 < a.Ht;
    const T *t = tex + (int64_t)y0 * a.Wt + x0;
    for (int c = 0; c < a.C; ++c) {
      const T *tc = t + c * plane;
      T acc = (T)0;
      if (vy0 && vx0) acc = acc + tc[0] * wnw;
      if (vy0 && vx1) acc = acc + tc[1] * wne;
      if (vy1 && vx0) acc = acc + tc[a.Wt] * wsw;
      if (vy1 && vx1) acc = acc + tc[a.Wt + 1] * wse;
      out[c] = acc;
    }
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_bwd(TexArgs<T> a) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (n >= a.N) return;
  const int64_t s = (int64_t)b * a.N + n;
  T ix, iy, mx, my, cu, cv;
  tex_coord<T>(a.coords + 2 * s, ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
  const int64_t plane = (int64_t)a.Ht * a.Wt;
  const T *go = a.grad_out + s * a.C;
  T *gt = a.grad_tex ? a.grad_tex + (int64_t)b * a.tex_bstride : nullptr;
  if (MODE == KD_TEX_NEAREST) {
    if (gt) {
      const int x = (int)rint(ix), y = (int)rint(iy);
      if (x >= 0 && x < a.Wt && y >= 0 && y < a.Ht)
        for (int c = 0; c < a.C; ++c) atomicAdd(gt + c * plane + (int64_t)y * a.Wt + x, go[c]);
    }
    if (a.grad_coords) {  // nearest sampling has no coordinate gradient
      a.grad_coords[2 * s] = (T)0;
      a.grad_coords[2 * s + 1] = (T)0;
    }
    return;
  }
  const T fx = floor(ix), fy = floor(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  const T ex = (T)x1 - ix, wx = ix - (T)x0, ey = (T)y1 - iy, wy = iy - (T)y0;
  const bool vx0 = x0 >= 0 && x0 < a.Wt, vx1 = x1 >= 0 && x1 < a.Wt;
  const bool vy0 = y0 >= 0 && y0 < a.Ht, vy1 = y1 >= 0 && y1 < a.Ht;
  const int64_t o = (int64_t)y0 * a.Wt + x0;
  const T *tex = a.tex + (int64_t)b * a.tex_bstride + o;
  T gix = (T)0, giy = (T)0;
  for (int c = 0; c < a.C; ++c) {
    const T g = go[c];
    const T *tc = tex + c * plane;
    if (gt) {
      T *gc = gt + c * plane + o;
      if (vy0 && vx0) atomicAdd(gc, ex * ey * g);
      if (vy0 && vx1) atomicAdd(gc + 1, wx * ey * g);
      if (vy1 && vx0) atomicAdd(gc + a.Wt, ex * wy * g);
      if (vy1 && vx1) atomicAdd(gc + a.Wt + 1, wx * wy * g);
    }
    if (a.grad_coords) {
      if (vy0 && vx0) {
        const T v = tc[0];
        gix -= v * ey * g;
        giy -= v * ex * g;
      }
      if (vy0 && vx1) {
        const T v = tc[1];
        gix += v * ey * g;
        giy -= v * wx * g;
      }
      if (vy1 && vx0) {
        const T v = tc[a.Wt];
        gix -= v * wy * g;
        giy += v * ex * g;
      }
      if (vy1 && vx1) {
        const T v = tc[a.Wt + 1];
        gix += v * wy * g;
        giy += v * wx * g;
      }
    }
  }
  if (a.grad_coords) {
    // grid gradient -> [-1, 1] coords (x mx, y my) -> y flip and *2 -> clamp mask
    a.grad_coords[2 * s] = cu != (T)0 ? (mx * gix) * (T)2 : (T)0;
    a.grad_coords[2 * s + 1] = cv != (T)0 ? -(my * giy) * (T)2 : (T)0;
  }
}

template <typename T>
__global__ void kd_tex_zero(T *p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    p[i] = (T)0;
}

template <typename T>
static int tex_check(int B, int64_t N, int C, int Ht, int Wt, int mode, int64_t tex_bstride) {
  KD_CHECK_ARG(B >= 0 && B <= 65535 && N >= 0 && C >= 0, "texture_mapping: bad sizes");
  KD_CHECK_ARG(Ht >= 1 && Wt >= 1, "texture_mapping: empty texture");
  KD_CHECK_ARG(mode == KD_TEX_NEAREST || mode == KD_TEX_BILINEAR,
               "texture_mapping: mode must be 0 (nearest) or 1 (bilinear)");
  KD_CHECK_ARG(tex_bstride == 0 || tex_bstride == (int64_t)C * Ht * Wt,
               "texture_mapping: texture batch stride must be 0 or C * Ht * Wt");
  return KD_OK;
}

template <typename T>
static int tex_forward(int B, int64_t N, int C, int Ht, int Wt, const T *coords, const T *tex,
                       int64_t tex_bstride, int mode, T *out, hipStream_t stream) {
  int rc = tex_check<T>(B, N, C, Ht, Wt, mode, tex_bstride);
  if (rc != KD_OK) return rc;
  if (B == 0 || N == 0 || C == 0) return KD_OK;
  TexArgs<T> a{N, C, Ht, Wt, coords, tex, tex_bstride, out, nullptr, nullptr, nullptr};
  const dim3 grid((unsigned)((N + kBlock - 1) / kBlock), (unsigned)B);
  KD_CHECK_ARG(grid.x <= 0x7fffffffu, "texture_mapping: too many samples");
  {
    ProfScope prof(K_TEX_FWD, stream);
    if (mode == KD_TEX_NEAREST)
      hipLaunchKernelGGL((kd_tex_fwd<T, KD_TEX_NEAREST>), grid, dim3(kBlock), 0, stream, a);
    else
      hipLaunchKernelGGL((kd_tex_fwd<T, KD_TEX_BILINEAR>), grid, dim3(kBlock), 0, stream, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "texture_mapping: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
static int tex_backward(int B, int64_t N, int C, int Ht, int Wt, const T *coords, const T *tex,
                        int64_t tex_bstride, int mode, const T *grad_out, T *grad_tex,
                        T *grad_coords, hipStream_t stream) {
  int rc = tex_check<T>(B, N, C, Ht, Wt, mode, tex_bstride);
  if (rc != KD_OK) return rc;
  KD_CHECK_ARG(grad_out || (!grad_tex && !grad_coords), "texture_mapping: grad_out is NULL");
  if (grad_tex) {  // zero the texture gradient (all Bt textures)
    const int64_t nt = (tex_bstride ? (int64_t)B : 1) * C * Ht * Wt;
    const unsigned g = (unsigned)std::min<int64_t>((nt + kBlock - 1) / kBlock, 4096);
    if (nt > 0) {
      ProfScope prof(K_ZERO, stream);
      hipLaunchKernelGGL(kd_tex_zero<T>, dim3(g), dim3(kBlock), 0, stream, grad_tex, nt);
    }
  }
  if (B == 0 || N == 0 || (!grad_tex && !grad_coords)) return KD_OK;
  TexArgs<T> a{N, C, Ht, Wt, coords, tex, tex_bstride, nullptr, grad_out, grad_tex, grad_coords};
  const dim3 grid((unsigned)((N + kBlock - 1) / kBlock), (unsigned)B);
  {
    ProfScope prof(K_TEX_BWD, stream);
    if (mode == KD_TEX_NEAREST)
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_NEAREST>), grid, dim3(kBlock), 0, stream, a);
    else
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_BILINEAR>), grid, dim3(kBlock), 0, stream, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(KD_ERR_LAUNCH, "texture_mapping bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

extern "C" {

int kd_texture_mapping_forward_f32(int B, int64_t N, int C, int Ht, int Wt, const float *coords,
                                   const float *tex, int64_t tex_batch_stride, int mode,
                                   float *out, void *stream) {
  return tex_forward<float>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, out,
                            (hipStream_t)stream);
}
int kd_texture_mapping_forward_f64(int B, int64_t N, int C, int Ht, int Wt, const double *coords,
                                   const double *tex, int64_t tex_batch_stride, int mode,
                                   double *out, void *stream) {
  return tex_forward<double>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, out,
                             (hipStream_t)stream);
}
int kd_texture_mapping_backward_f32(int B, int64_t N, int C, int Ht, int Wt, const float *coords,
                                    const float *tex, int64_t tex_batch_stride, int mode,
                                    const float *grad_out, float *grad_tex, float *grad_coords,
                                    void *stream) {
  return tex_backward<float>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, grad_out,
                             grad_tex, grad_coords, (hipStream_t)stream);
}
int kd_texture_mapping_backward_f64(int B, int64_t N, int C, int Ht, int Wt,
                                    const double *coords, const double *tex,
                                    int64_t tex_batch_stride, int mode, const double *grad_out,
                                    double *grad_tex, double *grad_coords, void *stream) {
  return tex_backward<double>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, grad_out,
                              grad_tex, grad_coords, (hipStream_t)stream);
}

}  // extern "C"
