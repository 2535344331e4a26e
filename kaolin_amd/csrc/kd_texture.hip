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
#include "kd_tile.hpp"

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

// The two horizontal taps (x, x + 1) of one texture row: one 2-element load (element-aligned:
// the hardware needs dword alignment only) when x + 1 is in the row, else the first alone.
typedef float kd_f2u __attribute__((ext_vector_type(2), aligned(4)));
typedef double kd_d2u __attribute__((ext_vector_type(2), aligned(8)));
__device__ __forceinline__ void tex_pair(const float *p, bool both, float &v0, float &v1) {
  if (both) {
    const kd_f2u v = *reinterpret_cast<const kd_f2u *>(p);
    v0 = v.x;
    v1 = v.y;
  } else {
    v0 = p[0];
    v1 = 0.f;
  }
}
__device__ __forceinline__ void tex_pair(const double *p, bool both, double &v0, double &v1) {
  if (both) {
    const kd_d2u v = *reinterpret_cast<const kd_d2u *>(p);
    v0 = v.x;
    v1 = v.y;
  } else {
    v0 = p[0];
    v1 = 0.0;
  }
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
    // ix, iy are clipped to the texture: x0, y0 are in range, x1 / y1 at most one past it
    auto channel = [&](int c) {
      const T *tc = t + c * plane;
      T nw, ne, sw = (T)0, se = (T)0;
      tex_pair(tc, vx1, nw, ne);
      if (vy1) tex_pair(tc + a.Wt, vx1, sw, se);
      T acc = (T)0;
      if (vy0 && vx0) acc = acc + nw * wnw;
      if (vy0 && vx1) acc = acc + ne * wne;
      if (vy1 && vx0) acc = acc + sw * wsw;
      if (vy1 && vx1) acc = acc + se * wse;
      return acc;
    };
    if (a.C == 3) {  // (RGB: the three channels' loads together, one row store)
      const T c0 = channel(0), c1 = channel(1), c2 = channel(2);
      store3(out, c0, c1, c2);
    } else {
      for (int c = 0; c < a.C; ++c) out[c] = channel(c);
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

// DPP within 16-lane rows (row_shr:n = 0x110 + n, row_shl:1 = 0x101); lanes whose source is
// outside their row read `old`.
template <int CTRL>
__device__ __forceinline__ int tex_dpp(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ float tex_dpp_v(float x) {
  return __int_as_float(tex_dpp<CTRL>(0, __float_as_int(x)));
}
template <int CTRL>
__device__ __forceinline__ double tex_dpp_v(double x) {
  const long long u = __double_as_longlong(x);
  const int lo = tex_dpp<CTRL>(0, (int)u), hi = tex_dpp<CTRL>(0, (int)(u >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Runs of equal keys along each 16-lane row: take[k] says whether step k (distance 2^k) of the
// segmented scan adds its source (the flag recurrence of a segmented Hillis-Steele scan, so
// keys that recur after another key never merge); tail marks each run's last lane.
__device__ __forceinline__ void tex_runs16(int key, bool take[4], bool &tail) {
  int prev = tex_dpp<0x111>(INT_MIN, key), next = tex_dpp<0x101>(INT_MIN, key);
  asm volatile("" : "+v"(prev), "+v"(next));
  int flag = prev != key;  // run head (a row start reads INT_MIN)
  take[0] = !flag;
  int f1 = tex_dpp<0x111>(1, flag);
  asm volatile("" : "+v"(f1));
  flag |= f1;
  take[1] = !flag;
  int f2 = tex_dpp<0x112>(1, flag);
  asm volatile("" : "+v"(f2));
  flag |= f2;
  take[2] = !flag;
  int f4 = tex_dpp<0x114>(1, flag);
  asm volatile("" : "+v"(f4));
  flag |= f4;
  take[3] = !flag;
  tail = next != key;
}

// One step of the segmented sum.  The DPP read must run on every lane: left as
// `take ? dpp(x) : 0` the compiler may issue it under the `take` lanes only, and a source lane
// outside EXEC reads `old` (0) -- partial sums silently dropped.  The empty asm pins the read
// at this point, where the whole wave is active.
template <int CTRL, typename T>
__device__ __forceinline__ T tex_seg_step(bool take, T x) {
  T o = tex_dpp_v<CTRL>(x);
  asm volatile("" : "+v"(o));
  return x + (take ? o : (T)0);
}

// inclusive segmented sums of v over the runs of tex_runs16 (every lane of the wave active)
template <typename T, int N>
__device__ __forceinline__ void tex_seg_sum16(const bool take[4], T v[N]) {
#pragma unroll
  for (int t = 0; t < N; ++t) {
    T x = v[t];
    x = tex_seg_step<0x111>(take[0], x);
    x = tex_seg_step<0x112>(take[1], x);
    x = tex_seg_step<0x114>(take[2], x);
    x = tex_seg_step<0x118>(take[3], x);
    v[t] = x;
  }
}

// Backward.  The texture gradient of a sample block is summed in LDS over the block's texel
// footprint (neighbouring samples hit the same texels; same-address global atomics serialise in
// L2) and flushed with one global atomic per touched texel and channel.  A footprint too large for
// the LDS buffer falls back to per-sample global atomics.  Zero incoming gradients (the masked
// background of an image loss) add nothing and are skipped.  The uv gradient is per sample.
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_bwd(TexArgs<T> a, int64_t row, int dbg) {
  // 20 KB of texel sums: eight workgroups per CU (with s_red, under 160 KB / 8), and C3's block
  // footprints still fit (32 KB: five per CU, 121.7 -> 113.4 us; 8 KB sends blocks to the
  // global-atomic fallback, 148 us)
  constexpr int kLds = 20416 / sizeof(T);
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
  constexpr int kTaps = MODE == KD_TEX_NEAREST ? 1 : 4;
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
    if (!lds && ablate(dbg, 1 << 28)) return;  // (diagnostics 1 << 28: no global atomics)
    if (lds)
      atomicAdd(&s_acc[((int64_t)c * bh + (y - ly)) * bw + (x - lx)], v);
    else
      atomicAdd(gt + c * plane + (int64_t)y * a.Wt + x, v);
  };
  // Adjacent samples of a row (the 16 lanes of a DPP row: one row of the 16 x 16 block) often
  // share their texel cell when the texture is magnified: their tap values are summed over each
  // run of equal cells by a segmented scan and only the run's last lane adds them (the LDS float
  // atomics are priced per active lane).
  bool take[4], tail;
  tex_runs16(act ? y0 * a.Wt + x0 : -1, take, tail);
  T gix = (T)0, giy = (T)0;
  const T *tex = a.tex + (int64_t)b * a.tex_bstride;
  const bool vx0 = x0 >= 0 && x0 < a.Wt, vx1 = x0 + 1 >= 0 && x0 + 1 < a.Wt;
  const bool vy0 = y0 >= 0 && y0 < a.Ht, vy1 = y0 + 1 >= 0 && y0 + 1 < a.Ht;
  const T *t0 = tex + (int64_t)y0 * a.Wt + x0;
  for (int c = 0; c < a.C; ++c) {
    const T g = ok ? go[c] : (T)0;
    if (gt) {  // uniform
      T v[kTaps];
      if (MODE == KD_TEX_NEAREST) {
        v[0] = act ? g : (T)0;
      } else {
        v[0] = act ? ex * ey * g : (T)0;
        v[kTaps > 1 ? 1 : 0] = act ? wx * ey * g : (T)0;
        v[kTaps > 2 ? 2 : 0] = act ? ex * wy * g : (T)0;
        v[kTaps > 3 ? 3 : 0] = act ? wx * wy * g : (T)0;
      }
      tex_seg_sum16<T, kTaps>(take, v);
      if (tail && act) {
#pragma unroll
        for (int t = 0; t < kTaps; ++t)
          if (v[t] != (T)0) add(c, x0 + (t & 1), y0 + (t >> 1), v[t]);
      }
    }
    if (ok && MODE == KD_TEX_BILINEAR && a.grad_coords) {
      // x0, y0 are in range (ix, iy clipped); x0 + 1 / y0 + 1 at most one past it
      const T *tc = t0 + c * plane;
      T nw, ne, sw = (T)0, se = (T)0;
      tex_pair(tc, vx1, nw, ne);
      if (vy1) tex_pair(tc + a.Wt, vx1, sw, se);
      if (vy0 && vx0) {
        gix -= nw * ey * g;
        giy -= nw * ex * g;
      }
      if (vy0 && vx1) {
        gix += ne * ey * g;
        giy -= ne * wx * g;
      }
      if (vy1 && vx0) {
        gix -= sw * wy * g;
        giy += sw * ex * g;
      }
      if (vy1 && vx1) {
        gix += se * wy * g;
        giy += se * wx * g;
      }
    }
  }
  if (ok && a.grad_coords) {
    // nearest sampling has no coordinate gradient; bilinear: grid gradient -> [-1, 1] coords
    // (x mx, y my) -> y flip and * 2 -> clamp mask
    a.grad_coords[2 * s] = MODE == KD_TEX_BILINEAR && cu != (T)0 ? (mx * gix) * (T)2 : (T)0;
    a.grad_coords[2 * s + 1] = MODE == KD_TEX_BILINEAR && cv != (T)0 ? -(my * giy) * (T)2 : (T)0;
  }
  if (!lds) return;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < nl; i += kBlock) {  // one atomic per touched texel
    const T v = s_acc[i];
    if (v == (T)0) continue;
    const int64_t c = i / (bw * bh), r = i - c * bw * bh;
    const int64_t y = ly + r / bw, x = lx + r % bw;
    if (!ablate(dbg, 1 << 28)) atomicAdd(gt + c * plane + y * a.Wt + x, v);
  }
}

// ------------------------------------------------------------------------------------------
// Texel-tile backward (kd_texture_mapping_backward_tiled): the samples are listed per 32 x 32
// texel tile, so the texture gradient is summed per tile in LDS and leaves as row-contiguous
// atomics (the shape the memory-side atomic units take at full rate), whatever the uv layout:
// the per-sample-block window of kd_tex_bwd grows without bound at uv seams and poles.
//   kd_tex_tcount  kTexSpan samples per workgroup: the tiles each sample's taps touch (1 to 4)
//                  counted in LDS, one global atomic per (workgroup, tile) -- counters hit by
//                  every wave serialise at the memory side; the coordinate gradient.
//   kd_tex_tscan   one workgroup: exclusive scans of the tile counts and of their kTexChunk
//                  chunk counts; the chunk table (tile, first entry).
//   kd_tex_tfill   the same samples again: ranks from the LDS counters, one cursor atomic per
//                  (workgroup, tile), the sample appended to each touched tile's list.
//   kd_tex_tacc    persistent: one chunk (<= kTexChunk entries of one tile) at a time, its taps
//                  summed in LDS, the nonzero sums added to the zeroed gradient.  Chunks of equal
//                  size keep the magnified tiles (thousands of samples) from serialising; runs
//                  of adjacent samples in one texel cell are merged in registers first.
// ------------------------------------------------------------------------------------------
constexpr int kTexTile = 32;         // texels per tile side
constexpr int kTexAccC = 4;          // channels per LDS pass of kd_tex_tacc (32 x 33 x 4 x 4 B)
constexpr int kTexRow = kTexTile + 1;  // LDS row stride of kd_tex_tacc: a column is not one bank
constexpr int kTexPer = 2;           // samples per thread in kd_tex_tcount / kd_tex_tfill
constexpr int kTexSpan = kTexPer * kBlock;
constexpr int kTexChunk = 1024;      // list entries per kd_tex_tacc chunk (4 per thread)
constexpr int kTexMaxTiles = 4096;   // tiles per texture held in LDS (textures up to 2048 x 2048)
constexpr int kTexAccGrid = 4096;    // kd_tex_tacc workgroups (persistent over the chunks)

struct TexTiles {
  int ntx, nty, ntex;  // tiles per row / column, textures (1 when shared)
  int *count;          // [ntiles + 1]; kd_tex_tscan turns it into entry offsets
  int *cursor;         // [ntiles]
  int *nchunk;         // [1]
  int *chunk_tile;     // [max chunks]
  int *chunk_e;        // [max chunks] first list entry of the chunk
  int *list;           // [4 B N] sample indices b * N + n
};

// tiles (index within the texture) touched by the taps of sample s: 1 to 4
template <typename T, int MODE>
__device__ __forceinline__ int tex_sample_tiles(const TexArgs<T> &a, const TexTiles &tt, int64_t s,
                                                int tiles[4]) {
  T ix, iy, mx, my, cu, cv;
  tex_coord<T>(a.coords + 2 * s, ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
  int x0, y0, x1, y1;
  if (MODE == KD_TEX_NEAREST) {
    x0 = x1 = (int)rint(ix);
    y0 = y1 = (int)rint(iy);
  } else {
    x0 = (int)floor(ix);
    y0 = (int)floor(iy);
    x1 = min(x0 + 1, a.Wt - 1);
    y1 = min(y0 + 1, a.Ht - 1);
  }
  const int tx0 = x0 / kTexTile, tx1 = x1 / kTexTile, ty0 = y0 / kTexTile, ty1 = y1 / kTexTile;
  int n = 0;
  tiles[n++] = ty0 * tt.ntx + tx0;
  if (tx1 != tx0) tiles[n++] = ty0 * tt.ntx + tx1;
  if (ty1 != ty0) {
    tiles[n++] = ty1 * tt.ntx + tx0;
    if (tx1 != tx0) tiles[n++] = ty1 * tt.ntx + tx1;
  }
  return n;
}

// Adds 1 to ctr[key] (an LDS counter) for every active lane, one atomic per distinct key of the
// wave; returns the lane's rank among the adders of its key (the counter's old value + its
// position among the wave's lanes with that key).  Wave-uniform call.
__device__ __forceinline__ int wave_key_add(bool active, int key, int *ctr) {
  int pos = 0;
  uint64_t left = __ballot(active);
  while (left) {
    const int leader = __builtin_ctzll(left);
    const int k = __shfl(key, leader);
    const uint64_t m = __ballot(active && key == k);
    int base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(ctr + k, __popcll(m));
    base = __shfl(base, leader);
    if (active && key == k) pos = base + mbcnt(m);
    left &= ~m;
  }
  return pos;
}

template <typename T>
__device__ __forceinline__ bool tex_active(const TexArgs<T> &a, int64_t s) {
  const T *go = a.grad_out + s * a.C;
  bool act = false;
  for (int c = 0; c < a.C; ++c) act |= go[c] != (T)0;
  return act;
}

template <typename T, int MODE>
__device__ __forceinline__ void tex_coord_grad(const TexArgs<T> &a, int b, int64_t s) {
  T ix, iy, mx, my, cu, cv;
  tex_coord<T>(a.coords + 2 * s, ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
  T gix = (T)0, giy = (T)0;
  if (MODE == KD_TEX_BILINEAR) {
    const int x0 = (int)floor(ix), y0 = (int)floor(iy);
    const T ex = (T)(x0 + 1) - ix, wx = ix - (T)x0, ey = (T)(y0 + 1) - iy, wy = iy - (T)y0;
    const bool vx0 = x0 >= 0 && x0 < a.Wt, vx1 = x0 + 1 >= 0 && x0 + 1 < a.Wt;
    const bool vy0 = y0 >= 0 && y0 < a.Ht, vy1 = y0 + 1 >= 0 && y0 + 1 < a.Ht;
    const int64_t plane = (int64_t)a.Ht * a.Wt;
    const T *t0 = a.tex + (int64_t)b * a.tex_bstride + (int64_t)y0 * a.Wt + x0;
    const T *go = a.grad_out + s * a.C;
    for (int c = 0; c < a.C; ++c) {
      const T g = go[c];
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
  a.grad_coords[2 * s] = MODE == KD_TEX_BILINEAR && cu != (T)0 ? (mx * gix) * (T)2 : (T)0;
  a.grad_coords[2 * s + 1] = MODE == KD_TEX_BILINEAR && cv != (T)0 ? -(my * giy) * (T)2 : (T)0;
}

template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_tcount(TexArgs<T> a, TexTiles tt) {
  __shared__ int s_h[kTexMaxTiles];
  const int b = blockIdx.y;
  const int per = tt.nty * tt.ntx;
  const bool cnt = a.grad_tex != nullptr;
  if (cnt) {
    for (int i = threadIdx.x; i < per; i += kBlock) s_h[i] = 0;
    __syncthreads();
  }
  for (int k = 0; k < kTexPer; ++k) {
    const int64_t n = (int64_t)blockIdx.x * kTexSpan + k * kBlock + threadIdx.x;
    const bool ok = n < a.N;
    const int64_t s = (int64_t)b * a.N + (ok ? n : 0);
    if (cnt) {
      int tiles[4] = {0, 0, 0, 0};
      const int nt = ok && tex_active(a, s) ? tex_sample_tiles<T, MODE>(a, tt, s, tiles) : 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) wave_key_add(j < nt, tiles[j], s_h);
    }
    if (ok && a.grad_coords) tex_coord_grad<T, MODE>(a, b, s);
  }
  if (!cnt) return;
  __syncthreads();
  int *gc = tt.count + (int64_t)(a.tex_bstride ? b : 0) * per;
  for (int i = threadIdx.x; i < per; i += kBlock)
    if (s_h[i]) atomicAdd(gc + i, s_h[i]);
}

// one workgroup of 1024 threads: count[0..n) -> exclusive entry offsets (count[n] = total),
// cursors, and the chunk table
__global__ __launch_bounds__(1024) void kd_tex_tscan(TexTiles tt, int n) {
  __shared__ int s_w[2][16];
  __shared__ int s_carry[2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 2) s_carry[tid] = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n; i0 += 1024) {
    const int i = i0 + tid;
    const int v = i < n ? tt.count[i] : 0;
    const int nc = (v + kTexChunk - 1) / kTexChunk;
    const int incl = wave_incl_scan(v), incl_c = wave_incl_scan(nc);
    if (lane == 63) {
      s_w[0][w] = incl;
      s_w[1][w] = incl_c;
    }
    __syncthreads();
    int off = s_carry[0], off_c = s_carry[1];
    for (int k = 0; k < w; ++k) {
      off += s_w[0][k];
      off_c += s_w[1][k];
    }
    const int ex = off + incl - v, ex_c = off_c + incl_c - nc;
    if (i < n) {
      tt.count[i] = ex;
      tt.cursor[i] = ex;
      for (int j = 0; j < nc; ++j) {
        tt.chunk_tile[ex_c + j] = i;
        tt.chunk_e[ex_c + j] = ex + j * kTexChunk;
      }
    }
    __syncthreads();
    if (tid == 1023) {
      s_carry[0] = ex + v;
      s_carry[1] = ex_c + nc;
    }
    __syncthreads();
  }
  if (tid == 0) {
    tt.count[n] = s_carry[0];
    tt.nchunk[0] = s_carry[1];
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_tfill(TexArgs<T> a, TexTiles tt) {
  __shared__ int s_h[kTexMaxTiles];
  __shared__ int s_base[kTexMaxTiles];
  const int b = blockIdx.y;
  const int per = tt.nty * tt.ntx;
  for (int i = threadIdx.x; i < per; i += kBlock) s_h[i] = 0;
  __syncthreads();
  int slot[kTexPer][4];  // rank << 12 | tile, or -1
#pragma unroll
  for (int k = 0; k < kTexPer; ++k) {
    const int64_t n = (int64_t)blockIdx.x * kTexSpan + k * kBlock + threadIdx.x;
    const bool ok = n < a.N;
    const int64_t s = (int64_t)b * a.N + (ok ? n : 0);
    int tiles[4] = {0, 0, 0, 0};
    const int nt = ok && tex_active(a, s) ? tex_sample_tiles<T, MODE>(a, tt, s, tiles) : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wave_key_add(j < nt, tiles[j], s_h);
      slot[k][j] = j < nt ? (r << 12) | tiles[j] : -1;
    }
  }
  __syncthreads();
  int *gc = tt.cursor + (int64_t)(a.tex_bstride ? b : 0) * per;
  for (int i = threadIdx.x; i < per; i += kBlock)
    if (s_h[i]) s_base[i] = atomicAdd(gc + i, s_h[i]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kTexPer; ++k) {
    const int s = (int)((int64_t)b * a.N + (int64_t)blockIdx.x * kTexSpan + k * kBlock +
                        threadIdx.x);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (slot[k][j] >= 0) tt.list[s_base[slot[k][j] & 4095] + (slot[k][j] >> 12)] = s;
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void kd_tex_tacc(TexArgs<T> a, TexTiles tt) {
  __shared__ T s_acc[kTexAccC * kTexTile * kTexRow];
  const int per = tt.nty * tt.ntx;
  const int64_t plane = (int64_t)a.Ht * a.Wt;
  const int nchunk = tt.nchunk[0];
  constexpr int kE = kTexChunk / kBlock;
  constexpr int kTaps = MODE == KD_TEX_NEAREST ? 1 : 4;
  for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int tile = tt.chunk_tile[ch];
    const int e0 = tt.chunk_e[ch], e1 = min(e0 + kTexChunk, tt.count[tile + 1]);
    const int tb = tile / per, r = tile - tb * per;
    const int ty = r / tt.ntx, tx = r - ty * tt.ntx;
    const int X0 = tx * kTexTile, Y0 = ty * kTexTile;
    T *gt = a.grad_tex + (int64_t)tb * a.tex_bstride;
    // kE consecutive entries per thread (adjacent samples), all loads issued before any use
    int64_t s[kE];
#pragma unroll
    for (int q = 0; q < kE; ++q) {
      const int e = e0 + threadIdx.x * kE + q;
      s[q] = e < e1 ? tt.list[e] : -1;
    }
    for (int c0 = 0; c0 < a.C; c0 += kTexAccC) {
      const int nc = min(kTexAccC, a.C - c0);
      for (int i = threadIdx.x; i < nc * kTexTile * kTexRow; i += kBlock) s_acc[i] = (T)0;
      __syncthreads();
      // A magnified texture gives runs of adjacent samples in one texel cell: their tap sums
      // are merged in registers and each run costs kTaps x C LDS atomics (the LDS float atomics
      // are priced per active lane).
      int cx = INT_MIN, cy = 0;
      T acc[kTaps][kTexAccC];
      auto flush = [&]() {
        if (cx == INT_MIN) return;
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
          const int x = cx + (t & 1), y = cy + (t >> 1);
          const int lx = x - X0, ly = y - Y0;
          if (x < 0 || x >= a.Wt || y < 0 || y >= a.Ht || lx < 0 || lx >= kTexTile || ly < 0 ||
              ly >= kTexTile)
            continue;
#pragma unroll
          for (int c = 0; c < kTexAccC; ++c)
            if (c < nc && acc[t][c] != (T)0)
              atomicAdd(&s_acc[(c * kTexTile + ly) * kTexRow + lx], acc[t][c]);
        }
      };
#pragma unroll
      for (int q = 0; q < kE; ++q) {
        if (s[q] < 0) continue;
        T ix, iy, mx, my, cu, cv;
        tex_coord<T>(a.coords + 2 * s[q], ix, iy, mx, my, cu, cv, a.Wt, a.Ht);
        const T *go = a.grad_out + s[q] * a.C + c0;
        int x0, y0;
        T w[kTaps];
        if (MODE == KD_TEX_NEAREST) {
          x0 = (int)rint(ix);
          y0 = (int)rint(iy);
          w[0] = (T)1;
        } else {
          x0 = (int)floor(ix);
          y0 = (int)floor(iy);
          const T ex = (T)(x0 + 1) - ix, wx = ix - (T)x0, ey = (T)(y0 + 1) - iy,
                  wy = iy - (T)y0;
          w[0] = ex * ey;
          w[kTaps > 1 ? 1 : 0] = wx * ey;
          w[kTaps > 2 ? 2 : 0] = ex * wy;
          w[kTaps > 3 ? 3 : 0] = wx * wy;
        }
        if (x0 != cx || y0 != cy) {
          flush();
          cx = x0;
          cy = y0;
#pragma unroll
          for (int t = 0; t < kTaps; ++t)
#pragma unroll
            for (int c = 0; c < kTexAccC; ++c) acc[t][c] = (T)0;
        }
#pragma unroll
        for (int c = 0; c < kTexAccC; ++c) {
          if (c >= nc) break;
          const T g = go[c];
#pragma unroll
          for (int t = 0; t < kTaps; ++t) acc[t][c] += w[t] * g;
        }
      }
      flush();
      __syncthreads();
      // nonzero sums of the tile (rows of 32 texels: two 128-B segments per wave instruction)
      for (int i = threadIdx.x; i < nc * kTexTile * kTexTile; i += kBlock) {
        const int c = i / (kTexTile * kTexTile), q = i - c * kTexTile * kTexTile;
        const T v = s_acc[(c * kTexTile + q / kTexTile) * kTexRow + q % kTexTile];
        const int y = Y0 + q / kTexTile, x = X0 + q % kTexTile;
        if (v != (T)0 && x < a.Wt && y < a.Ht)
          atomicAdd(gt + (int64_t)(c0 + c) * plane + (int64_t)y * a.Wt + x, v);
      }
      __syncthreads();
    }
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
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_NEAREST>), grid, dim3(kBlock), 0, stream, a, row,
                         debug_flags());
    else
      hipLaunchKernelGGL((kd_tex_bwd<T, KD_TEX_BILINEAR>), grid, dim3(kBlock), 0, stream, a,
                         row, debug_flags());
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(KD_ERR_LAUNCH, "texture_mapping bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

static int64_t tex_tiles(int B, int Ht, int Wt, int shared) {
  return (int64_t)(shared ? 1 : B) * ((Ht + kTexTile - 1) / kTexTile) *
         ((Wt + kTexTile - 1) / kTexTile);
}
static int64_t tex_max_chunks(int B, int64_t N, int Ht, int Wt, int shared) {
  return tex_tiles(B, Ht, Wt, shared) + (4 * (int64_t)B * N + kTexChunk - 1) / kTexChunk;
}

size_t tex_tiled_workspace_bytes(int B, int64_t N, int Ht, int Wt, int shared) {
  return sizeof(int) * (size_t)(2 * tex_tiles(B, Ht, Wt, shared) + 2 +
                                2 * tex_max_chunks(B, N, Ht, Wt, shared) + 4 * (int64_t)B * N);
}

template <typename T>
static int tex_backward_tiled(int B, int64_t N, int C, int Ht, int Wt, const T *coords,
                              const T *tex, int64_t tex_bstride, int mode, const T *grad_out,
                              T *grad_tex, T *grad_coords, void *ws, size_t wsb,
                              hipStream_t stream) {
  int rc = tex_check<T>(B, N, C, Ht, Wt, mode, tex_bstride);
  if (rc != KD_OK) return rc;
  KD_CHECK_ARG(grad_out || (!grad_tex && !grad_coords), "texture_mapping: grad_out is NULL");
  KD_CHECK_ARG((int64_t)B * N < (1ll << 31) / 4, "texture_mapping: too many samples");
  TexTiles tt;
  tt.ntx = (Wt + kTexTile - 1) / kTexTile;
  tt.nty = (Ht + kTexTile - 1) / kTexTile;
  tt.ntex = tex_bstride ? B : 1;
  // textures past kTexMaxTiles tiles: the per-sample-block kernel
  if ((int64_t)tt.ntx * tt.nty > kTexMaxTiles)
    return tex_backward<T>(B, N, C, Ht, Wt, coords, tex, tex_bstride, mode, 0, grad_out,
                           grad_tex, grad_coords, stream);
  const size_t need = tex_tiled_workspace_bytes(B, N, Ht, Wt, tex_bstride == 0);
  if (grad_tex && (wsb < need || !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  const int ntiles = tt.ntex * tt.nty * tt.ntx;
  const int64_t mc = tex_max_chunks(B, N, Ht, Wt, tex_bstride == 0);
  tt.count = (int *)ws;
  tt.cursor = tt.count + ntiles + 1;
  tt.nchunk = tt.cursor + ntiles;
  tt.chunk_tile = tt.nchunk + 1;
  tt.chunk_e = tt.chunk_tile + mc;
  tt.list = tt.chunk_e + mc;
  if (grad_tex) {  // the gradient is added into zeros (all Bt textures)
    const int64_t nt = (int64_t)tt.ntex * C * Ht * Wt;
    if (nt > 0 && zero_words(grad_tex, sizeof(T) * (size_t)nt, stream) != hipSuccess)
      return set_error(KD_ERR_LAUNCH, "texture_mapping: memset");
  }
  if (B == 0 || N == 0 || C == 0 || (!grad_tex && !grad_coords)) return KD_OK;
  TexArgs<T> a{N, C, Ht, Wt, coords, tex, tex_bstride, nullptr, grad_out, grad_tex, grad_coords};
  const dim3 grid((unsigned)((N + kTexSpan - 1) / kTexSpan), (unsigned)B);
  const unsigned gacc = (unsigned)std::min<int64_t>(mc, kTexAccGrid);
  ProfScope prof(K_TEX_BWD, stream);
  if (grad_tex && zero_words(tt.count, sizeof(int) * (size_t)(ntiles + 1), stream) !=
                      hipSuccess)
    return set_error(KD_ERR_LAUNCH, "texture_mapping: memset");
#define KD_TEX_LAUNCH(M)                                                                   \
  do {                                                                                     \
    hipLaunchKernelGGL((kd_tex_tcount<T, M>), grid, dim3(kBlock), 0, stream, a, tt);       \
    if (grad_tex) {                                                                        \
      hipLaunchKernelGGL(kd_tex_tscan, dim3(1), dim3(1024), 0, stream, tt, ntiles);        \
      hipLaunchKernelGGL((kd_tex_tfill<T, M>), grid, dim3(kBlock), 0, stream, a, tt);      \
      hipLaunchKernelGGL((kd_tex_tacc<T, M>), dim3(gacc), dim3(kBlock), 0, stream, a, tt); \
    }                                                                                      \
  } while (0)
  if (mode == KD_TEX_NEAREST)
    KD_TEX_LAUNCH(KD_TEX_NEAREST);
  else
    KD_TEX_LAUNCH(KD_TEX_BILINEAR);
#undef KD_TEX_LAUNCH
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

size_t kd_texture_mapping_backward_workspace_size(int B, int64_t N, int Ht, int Wt,
                                                  int shared_texture) {
  if (B < 0 || N < 0 || Ht < 1 || Wt < 1) return 0;
  return tex_tiled_workspace_bytes(B, N, Ht, Wt, shared_texture);
}
int kd_texture_mapping_backward_tiled_f32(int B, int64_t N, int C, int Ht, int Wt,
                                          const float *coords, const float *tex,
                                          int64_t tex_batch_stride, int mode,
                                          const float *grad_out, float *grad_tex,
                                          float *grad_coords, void *ws, size_t wsb,
                                          void *stream) {
  return tex_backward_tiled<float>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode, grad_out,
                                   grad_tex, grad_coords, ws, wsb, (hipStream_t)stream);
}
int kd_texture_mapping_backward_tiled_f64(int B, int64_t N, int C, int Ht, int Wt,
                                          const double *coords, const double *tex,
                                          int64_t tex_batch_stride, int mode,
                                          const double *grad_out, double *grad_tex,
                                          double *grad_coords, void *ws, size_t wsb,
                                          void *stream) {
  return tex_backward_tiled<double>(B, N, C, Ht, Wt, coords, tex, tex_batch_stride, mode,
                                    grad_out, grad_tex, grad_coords, ws, wsb,
                                    (hipStream_t)stream);
}

}  // extern "C"
