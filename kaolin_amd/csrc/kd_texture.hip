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
// texture gradient summed per 16 x 16 sample block in LDS and flushed with one float atomic per
// touched texel (kd_tex_bwd) into a buffer zeroed here, and for bilinear the coordinate gradient
// through border clipping, the y flip, the affine map and the clamp (0 outside [0, 1], like
// torch.clamp's backward).
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

// Workgroup sample block: 16 x 16 samples of a dense image (row > 0: row length), otherwise 256
// consecutive samples.
__device__ __forceinline__ int64_t tex_sample(int64_t N, int64_t row, bool &ok) {
  const int tid = threadIdx.x;
  if (row > 0) {
    const int64_t ntx = (row + 15) / 16, nrows = N / row;
    const int64_t ty = blockIdx.x / ntx, tx = blockIdx.x - ty * ntx;
    const int64_t x = tx * 16 + (tid & 15), y = ty * 16 + (tid >> 4);
    ok = x < row && y < nrows;
    return y * row + x;
  }
  const int64_t n = (int64_t)blockIdx.x * kBlock + tid;
  ok = n < N;
  return n;
}

__device__ __forceinline__ int wg_min_max(int lo, int hi, int *s, int &hi_out) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    lo = min(lo, __shfl_xor(lo, d));
    hi = max(hi, __shfl_xor(hi, d));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s[w] = lo;
    s[4 + w] = hi;
  }
  __syncthreads();
  lo = min(min(s[0], s[1]), min(s[2], s[3]));
  hi_out = max(max(s[4], s[5]), max(s[6], s[7]));
  __syncthreads();
  return lo;
}

// Backward.  The texture gradient of a sample block is summed in LDS over the block's texel
// footprint (neighbouring samples hit the same texels; same-address global atomics serialise in
// L2) and flushed with one global atomic per touched texel and channel.  A footprint too large for
// the LDS buffer falls back to per-sample global atomics.  Zero incoming gradients (the masked
// background of an image loss) add nothing and are skipped.  The uv gradient is per sample.
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_bwd(TexArgs<T> a, int64_t row) {
  constexpr int kLds = 32768 / sizeof(T);
  __shared__ T s_acc[kLds];
  __shared__ int s_red[8];
  const int b = blockIdx.y;
  bool ok;
  const int64_t n = tex_sample(a.N, row, ok);
  const int64_t s = (int64_t)b * a.N + n;
  const int64_t plane = (int64_t)a.Ht * a.Wt;
  T ix = 0, iy = 0, mx = 0, my = 0, cu = 0, cv = 0;
  if (ok) tex_coord<T>(a.coords + 2 * s, ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
  const T *go = a.grad_out + s * a.C;
  T *gt = a.grad_tex ? a.grad_tex + (int64_t)b * a.tex_bstride : nullptr;
  // taps: nearest (x0, y0) only; bilinear the 2 x 2 block at (x0, y0)
  int x0, y0;
  T ex = 0, wx = 0, ey = 0, wy = 0;
  if (MODE == KD_TEX_NEAREST) {
    x0 = (int)rint(ix);
    y0 = (int)rint(iy);
  } else {
    x0 = (int)floor(ix);
    y0 = (int)floor(iy);
    ex = (T)(x0 + 1) - ix;
    wx = ix - (T)x0;
    ey = (T)(y0 + 1) - iy;
    wy = iy - (T)y0;
  }
  constexpr int kExt = MODE == KD_TEX_NEAREST ? 0 : 1;
  bool act = false;
  if (ok && gt)
    for (int c = 0; c < a.C; ++c) act |= go[c] != (T)0;
  // texel footprint of the block's contributing samples
  int hx, hy;
  const int lx = wg_min_max(act ? x0 : INT_MAX, act ? x0 + kExt : INT_MIN, s_red, hx);
  const int ly = wg_min_max(act ? y0 : INT_MAX, act ? y0 + kExt : INT_MIN, s_red, hy);
  const int64_t bw = (int64_t)hx - lx + 1, bh = (int64_t)hy - ly + 1;
  const bool any = hx >= lx;
  const bool lds = any && bw * bh * a.C <= kLds;
  const int64_t nl = lds ? bw * bh * a.C : 0;
  for (int64_t i = threadIdx.x; i < nl; i += kBlock) s_acc[i] = (T)0;
  if (lds) __syncthreads();
  auto add = [&](int c, int x, int y, T v) {
    if (x < 0 || x >= a.Wt || y < 0 || y >= a.Ht) return;
    if (lds)
      atomicAdd(&s_acc[((int64_t)c * bh + (y - ly)) * bw + (x - lx)], v);
    else
      atomicAdd(gt + c * plane + (int64_t)y * a.Wt + x, v);
  };
  T gix = (T)0, giy = (T)0;
  if (ok) {
    const T *tex = a.tex + (int64_t)b * a.tex_bstride;
    const bool vx0 = x0 >= 0 && x0 < a.Wt, vx1 = x0 + 1 >= 0 && x0 + 1 < a.Wt;
    const bool vy0 = y0 >= 0 && y0 < a.Ht, vy1 = y0 + 1 >= 0 && y0 + 1 < a.Ht;
    const T *t0 = tex + (int64_t)y0 * a.Wt + x0;
    for (int c = 0; c < a.C; ++c) {
      const T g = go[c];
      if (act && g != (T)0) {
        if (MODE == KD_TEX_NEAREST) {
          add(c, x0, y0, g);
        } else {
          add(c, x0, y0, ex * ey * g);
          add(c, x0 + 1, y0, wx * ey * g);
          add(c, x0, y0 + 1, ex * wy * g);
          add(c, x0 + 1, y0 + 1, wx * wy * g);
        }
      }
      if (MODE == KD_TEX_BILINEAR && a.grad_coords) {
        const T *tc = t0 + c * plane;
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
      // nearest sampling has no coordinate gradient; bilinear: grid gradient -> [-1, 1] coords
      // (x mx, y my) -> y flip and * 2 -> clamp mask
      a.grad_coords[2 * s] = MODE == KD_TEX_BILINEAR && cu != (T)0 ? (mx * gix) * (T)2 : (T)0;
      a.grad_coords[2 * s + 1] =
          MODE == KD_TEX_BILINEAR && cv != (T)0 ? -(my * giy) * (T)2 : (T)0;
    }
  }
  if (!lds) return;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < nl; i += kBlock) {  // one atomic per touched texel
    const T v = s_acc[i];
    if (v == (T)0) continue;
    const int64_t c = i / (bw * bh), r = i - c * bw * bh;
    const int64_t y = ly + r / bw, x = lx + r % bw;
    atomicAdd(gt + c * plane + y * a.Wt + x, v);
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
                        int64_t tex_bstride, int mode, int64_t row, const T *grad_out,
                        T *grad_tex, T *grad_coords, hipStream_t stream) {
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
  KD_CHECK_ARG(row >= 0 && (row == 0 || N % row == 0),
               "texture_mapping: sample_row must be 0 or divide the sample count");
  TexArgs<T> a{N, C, Ht, Wt, coords, tex, tex_bstride, nullptr, grad_out, grad_tex, grad_coords};
  const int64_t blocks =
      row > 0 ? ((row + 15) / 16) * ((N / row + 15) / 16) : (N + kBlock - 1) / kBlock;
  KD_CHECK_ARG(blocks < (1ll << 31), "texture_mapping: too many samples");
  const dim3 grid((unsigned)blocks, (unsigned)B);
  {
    ProfScope prof(K_TEX_BWD, stream);
    if (mode == KD_TEX_NEAREST)
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_NEAREST>), grid, dim3(kBlock), 0, stream, a, row);
    else
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_BILINEAR>), grid, dim3(kBlock), 0, stream, a,
                         row);
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
                                    int64_t sample_row, const float *grad_out, float *grad_tex,
                                    float *grad_coords, void *stream) {
  return tex_backward<float>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, sample_row,
                             grad_out, grad_tex, grad_coords, (hipStream_t)stream);
}
int kd_texture_mapping_backward_f64(int B, int64_t N, int C, int Ht, int Wt,
                                    const double *coords, const double *tex,
                                    int64_t tex_batch_stride, int mode, int64_t sample_row,
                                    const double *grad_out, double *grad_tex,
                                    double *grad_coords, void *stream) {
  return tex_backward<double>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, sample_row,
                              grad_out, grad_tex, grad_coords, (hipStream_t)stream);
}

}  // extern "C"
