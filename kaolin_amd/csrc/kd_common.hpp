// kd_common.hpp -- shared device/host helpers for the gfx950 DIB-R kernels.
//
// Numerics contract: every kernel is compiled with -ffp-contract=off and
// without fast-math, so `a*b - c*d` is two rounded products and a rounded difference, exactly as
// the reference expressions are written (and as the C oracle evaluates them); fp32 division is
// IEEE correctly rounded (hipcc default); pixel centres are computed in fp32 even for fp64 data
// (rasterization_cuda.cu:85-86, dibr_soft_mask_cuda.cu:75-76).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

namespace kd {

// Diagnostic build (kaolin_amd/_build.py build(diag=True) -> lib/libkaolin_dibr_diag.so, loaded
// with KAOLIN_AMD_DIAG=1 by the tools under tools/): the device-side ablation switches and the
// per-tile clocks exist only there.  In the production library ablate() is constant false and
// TileClock records nothing, so none of it is in the kernels.
#ifndef KD_DIAG
#define KD_DIAG 0
#endif
__host__ __device__ constexpr bool ablate(int flags, int bit) { return KD_DIAG && (flags & bit); }

// Diagnostic ablation switches (kd_debug_set, copied into FaceSet::dbg; diagnostic build only:
// the production library's debug_flags() is the constant 0, so no host path there selects a kernel
// from them).
// Bits: 1 skip the per-pixel face tests of the forward kernels, 2 skip staging face data,
//       4 skip the per-batch work entirely (bin walk only), 8 fp32 raster: lane-per-pixel
//       kernel instead of the pair pipeline, 16 / 32 skip the per-pair pass of the fp32
//       raster / soft mask, 64 record per-tile durations into the kd_debug_buffer array,
//       8192 skip the fp32 raster's per-pixel epilogue (winner reload, output writes),
//       32 also skips the fused soft mask's pair math (kd_softpair.hip soft_pairs_tile),
//       1 << 18 / 1 << 19 skip kd_bin_count's cull coefficients / its LDS tile counts,
//       1 << 16 / 1 << 23 kd_soft_lists: skip every list store / the index and type stores (the
//       host presets the indices to -1 so that the backward reads no garbage),
//       1 << 20 256-face binning chunks, 1 << 21 one count workgroup for both face sets,
//       1 << 29 the lane-per-pixel K-list backward,
//       16384 return at the start of the raster / soft pass-A tile kernels (dispatch cost),
//       1 << 24 the fused forward without its soft phase (the raster phase's instruction counts),
//       1 << 25 the DefTet backward as the raster tile kernel over the P x knum samples,
//       1 << 27 kd_dt_bwd: the sample compaction only (no per-face sums),
//       1 << 26 kd_dt_fwd: the LDS rank form for every pixel (not only past the wave form),
//       128 / 4096 the raster backward's / the soft backward items' gradient atomics skipped,
//       1 << 28 kd_tex_bwd without its global atomics.
#if KD_DIAG
int debug_flags();
#else
constexpr int debug_flags() { return 0; }
#endif
// kd_set_test_forms (KD_FORM_* of kaolin_dibr.h): run dibr_rasterization through the separate
// launches its one-launch kernels fuse (a test hook of both builds)
int test_forms();
// kd_set_tile_split: workgroups per tile of the fused fp32 forward (0: chosen by the batch size)
int tile_split();
// kd_set_coarse_tile: dibr_rasterization's coarse bin edge (0: chosen by the batch size)
int coarse_tile_hook();
// the device `stream` belongs to (null stream: the current device)
int stream_device(hipStream_t stream);
// compute units of the stream's device (cached per device on first use; 256 when unknown)
int device_cus(hipStream_t stream);
// Tile cost history of the fused fp32 DIB-R forward (kd_set_tile_history): a caller-owned
// device buffer of kTileHistCap ushort entries per device (kd_tile_history_attach; the caller
// keeps it alive while captured graphs use it), zeroed on the stream when `tag` (the call's
// shape) changes outside a capture.  nullptr: history off, no buffer attached for the stream's
// device, too many entries, or a new shape inside a stream capture.
constexpr int64_t kTileHistCap = 1 << 20;
unsigned short *tile_history(int64_t n, long long tag, hipStream_t stream);
int tile_history_attach(hipStream_t stream, void *buf, size_t bytes);
long long *debug_tile_buffer();  // kd_debug_buffer (flag 64), else nullptr

// Per-workgroup duration (wall clock, 100 MHz ticks) for diagnostics: written by thread 0 when
// the workgroup's kernel body returns.
struct TileClock {
  long long *buf;
  long long t0;
  int64_t idx;
  __device__ __forceinline__ TileClock(long long *b, int slot)
      : buf(KD_DIAG ? b : nullptr), t0(KD_DIAG && b ? wall_clock64() : 0),
        idx((int64_t)slot * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x +
            blockIdx.x) {}
  __device__ __forceinline__ ~TileClock() {
    if (KD_DIAG && buf && threadIdx.x == 0) buf[idx] = wall_clock64() - t0;
  }
  // diagnostics: also the start time, in `slot` (dispatch slot order)
  __device__ __forceinline__ void start_to(int slot) const {
    if (KD_DIAG && buf && threadIdx.x == 0)
      buf[(int64_t)slot * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] =
          t0;
  }
};

constexpr int kWave = 64;
constexpr int kBlock = 256;      // 4 waves
constexpr int kTile = 16;        // fine tile: 16x16 pixels per workgroup, 8x8 per wave
constexpr int kChunk = 512;      // faces per binning workgroup (two per thread) ...
// ... or one per thread when the batch is small, so the binning grids still fill the chip
inline int bin_chunk(int B, int64_t max_per_view) {  // (debug flag 1 << 20: always 256)
  return (int64_t)B * ((max_per_view + kChunk - 1) / kChunk) < 256 || (debug_flags() & (1 << 20))
             ? kChunk / 2
             : kChunk;
}
constexpr int kMaxCtiles = 1024; // coarse tiles per view (LDS bound of the binning kernels)

// ------------------------------------------------------------------------------------------
// pixel centres, identical to the reference expression `multiplier / width * (2*w + 1 - width)`
// ------------------------------------------------------------------------------------------
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global stores (__syncthreads' workgroup fence drains vmcnt to 0, which serialises a
// loop of store-heavy tiles on the store latency).  Global memory written before it is NOT
// visible to the other waves after it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float px_cx(float M, int W, int w) {
  return M / (float)W * (float)(2 * w + 1 - W);
}
__device__ __forceinline__ float px_cy(float M, int H, int h) {
  return M / (float)H * (float)(H - 2 * h - 1);
}

// NaN-propagating min / max of three (torch.min / torch.max over a dim propagate NaN).
template <typename T>
__device__ __forceinline__ T nmin3(T a, T b, T c) {
  T m = (b < a || isnan(b)) ? b : a;
  if (isnan(m)) return m;
  return (c < m || isnan(c)) ? c : m;
}
template <typename T>
__device__ __forceinline__ T nmax3(T a, T b, T c) {
  T m = (b > a || isnan(b)) ? b : a;
  if (isnan(m)) return m;
  return (c > m || isnan(c)) ? c : m;
}

// ------------------------------------------------------------------------------------------
// Exact pixel span of a half-open box test.  The reference rejects a pixel when
//   x0 < xmin || x0 >= xmax || y0 < ymin || y0 >= ymax
// with x0 / y0 the fp32 centres widened to T.  Centres are monotone in the pixel index (for any
// finite multiplier; a zero multiplier makes them all 0), so the accepted pixels form
// [a, b] x [c, d]; a NaN bound rejects nothing on its side (every comparison with NaN is false),
// exactly like the reference.  Positive multiplier: estimate in double, then settle the boundary
// with the exact centre formula; otherwise binary search on the exact test.
// ------------------------------------------------------------------------------------------
struct Span {
  short x0, x1, y0, y1;  // inclusive; empty when x0 > x1 or y0 > y1
};

// First index in [0, n) where a monotone predicate (false...false true...true) holds, n if none.
template <typename Pred>
__device__ inline int first_true(int n, Pred p) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p(mid))
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

// General span of `!(c(i) < lo) && !(c(i) >= hi)` for centres c(i) monotone in i (either
// direction, ties allowed: a negative or zero multiplier), by binary search on the exact test.
template <typename T, typename Centre>
__device__ inline void span_monotone(T lo, T hi, int n, bool increasing, Centre c, int &a,
                                     int &b) {
  auto ge_lo = [&](int i) { return !((T)c(i) < lo); };
  auto lt_hi = [&](int i) { return !((T)c(i) >= hi); };
  if (increasing) {  // ge_lo: F..T, lt_hi: T..F
    a = first_true(n, ge_lo);
    b = first_true(n, [&](int i) { return !lt_hi(i); }) - 1;
  } else {           // ge_lo: T..F, lt_hi: F..T
    a = first_true(n, lt_hi);
    b = first_true(n, [&](int i) { return !ge_lo(i); }) - 1;
  }
}

template <typename T>
__device__ inline void span_x(T lo, T hi, float M, int W, int &a, int &b) {
  const float s = M / (float)W;
  if (!(s > 0.f)) {  // negative or zero multiplier (finite: checked by the C ABI)
    span_monotone<T>(lo, hi, W, false, [&](int i) { return px_cx(M, W, i); }, a, b);
    return;
  }
  const double rs = 1.0 / (double)s;  // estimate only: the loops below settle it exactly
  if (isnan(lo)) {
    a = 0;
  } else {
    double t = ((double)lo * rs + (double)(W - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)W);
    a = (int)ceil(t);
    a = a < 0 ? 0 : (a > W ? W : a);
    while (a > 0 && (T)px_cx(M, W, a - 1) >= lo) --a;
    while (a < W && (T)px_cx(M, W, a) < lo) ++a;
  }
  if (isnan(hi)) {
    b = W - 1;
  } else {
    double t = ((double)hi * rs + (double)(W - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)W + 1.0);
    b = (int)ceil(t) - 1;
    b = b < -1 ? -1 : (b > W - 1 ? W - 1 : b);
    while (b < W - 1 && (T)px_cx(M, W, b + 1) < hi) ++b;
    while (b >= 0 && (T)px_cx(M, W, b) >= hi) --b;
  }
}

template <typename T>
__device__ inline void span_y(T lo, T hi, float M, int H, int &c, int &d) {
  const float s = M / (float)H;
  if (!(s > 0.f)) {  // centres increase with h for a negative multiplier
    span_monotone<T>(lo, hi, H, true, [&](int i) { return px_cy(M, H, i); }, c, d);
    return;
  }
  // rows accepted: !(cy < lo) && !(cy >= hi); cy decreases with h.
  const double rs = 1.0 / (double)s;  // estimate only: the loops below settle it exactly
  if (isnan(hi)) {
    c = 0;
  } else {  // first h with cy(h) < hi
    double t = ((double)(H - 1) - (double)hi * rs) * 0.5;
    t = fmin(fmax(t, -2.0), (double)H);
    c = (int)floor(t) + 1;
    c = c < 0 ? 0 : (c > H ? H : c);
    while (c > 0 && (T)px_cy(M, H, c - 1) < hi) --c;
    while (c < H && (T)px_cy(M, H, c) >= hi) ++c;
  }
  if (isnan(lo)) {
    d = H - 1;
  } else {  // last h with cy(h) >= lo
    double t = ((double)(H - 1) - (double)lo * rs) * 0.5;
    t = fmin(fmax(t, -2.0), (double)H);
    d = (int)floor(t);
    d = d < -1 ? -1 : (d > H - 1 ? H - 1 : d);
    while (d < H - 1 && (T)px_cy(M, H, d + 1) >= lo) ++d;
    while (d >= 0 && (T)px_cy(M, H, d) < lo) --d;
  }
}

template <typename T>
__device__ inline Span make_span(T xmin, T ymin, T xmax, T ymax, float M, int H, int W) {
  int a, b, c, d;
  span_x<T>(xmin, xmax, M, W, a, b);
  span_y<T>(ymin, ymax, M, H, c, d);
  Span s;
  if (a > b || c > d) {
    s.x0 = 1;
    s.x1 = 0;
    s.y0 = 1;
    s.y1 = 0;
  } else {
    s.x0 = (short)a;
    s.x1 = (short)b;
    s.y0 = (short)c;
    s.y1 = (short)d;
  }
  return s;
}

// The per-call constants of make_span, computed once on the host (IEEE fp32 M / W there is the
// device's quotient too): the binning kernels compute a span per face.
struct SpanConsts {
  float M, sx, sy;  // sx = M / W, sy = M / H (the first factor of px_cx / px_cy)
  double rsx, rsy;  // 1 / sx, 1 / sy (estimates only)
  int H, W;
  int fast;         // sx > 0 and sy > 0: estimate + settle; else binary search (make_span)
};

inline SpanConsts span_consts(float M, int H, int W) {
  SpanConsts k;
  k.M = M;
  k.H = H;
  k.W = W;
  k.sx = W > 0 ? M / (float)W : 0.f;
  k.sy = H > 0 ? M / (float)H : 0.f;
  k.fast = k.sx > 0.f && k.sy > 0.f;
  k.rsx = k.fast ? 1.0 / (double)k.sx : 0.0;
  k.rsy = k.fast ? 1.0 / (double)k.sy : 0.0;
  return k;
}

// First index a in [0, n] with c(a) >= lo for centres c increasing in the index (n if none), from
// the estimate e (within one index of the answer for finite inputs): one settling step each way,
// verified; the linear walk runs only if the verification fails (never for finite inputs).
template <typename T, typename Centre>
__device__ __forceinline__ int settle_first_ge(T lo, int n, int e, Centre c) {
  if (e > 0 && (T)c(e - 1) >= lo)
    --e;
  else if (e < n && (T)c(e) < lo)
    ++e;
  const bool ok = (e == 0 || (T)c(e - 1) < lo) && (e == n || (T)c(e) >= lo);
  if (__builtin_expect(!ok, 0)) {
    while (e > 0 && (T)c(e - 1) >= lo) --e;
    while (e < n && (T)c(e) < lo) ++e;
  }
  return e;
}

// make_span for a positive multiplier with host constants: the same integer span (the double
// estimates are settled against the exact fp32 centre formula, like span_x / span_y).
template <typename T>
__device__ __forceinline__ Span make_span_k(T xmin, T ymin, T xmax, T ymax, const SpanConsts &k) {
  if (!k.fast) return make_span<T>(xmin, ymin, xmax, ymax, k.M, k.H, k.W);
  const int W = k.W, H = k.H;
  const float sx = k.sx, sy = k.sy;
  auto cx = [&](int i) { return sx * (float)(2 * i + 1 - W); };  // px_cx, increasing in i
  // rows: cy(h) decreases with h; with g = H - 1 - h, cy = sy * (2 g + 1 - H) increases in g
  auto cyg = [&](int g) { return sy * (float)(2 * g + 1 - H); };
  int a = 0, b = W - 1, c = 0, d = H - 1;
  if (!isnan(xmin)) {  // a = first column with cx >= xmin
    double t = ((double)xmin * k.rsx + (double)(W - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)W);
    a = settle_first_ge<T>(xmin, W, min(max((int)ceil(t), 0), W), cx);
  }
  if (!isnan(xmax)) {  // b = last column with cx < xmax = (first with cx >= xmax) - 1
    double t = ((double)xmax * k.rsx + (double)(W - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)W);
    b = settle_first_ge<T>(xmax, W, min(max((int)ceil(t), 0), W), cx) - 1;
  }
  if (!isnan(ymax)) {  // c = first row with cy < ymax = H - (first g with cyg >= ymax)
    double t = ((double)ymax * k.rsy + (double)(H - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)H);
    c = H - settle_first_ge<T>(ymax, H, min(max((int)ceil(t), 0), H), cyg);
  }
  if (!isnan(ymin)) {  // d = last row with cy >= ymin = H - 1 - (first g with cyg >= ymin)
    double t = ((double)ymin * k.rsy + (double)(H - 1)) * 0.5;
    t = fmin(fmax(t, -1.0), (double)H);
    d = H - 1 - settle_first_ge<T>(ymin, H, min(max((int)ceil(t), 0), H), cyg);
  }
  Span s;
  if (a > b || c > d) {
    s.x0 = 1;
    s.x1 = 0;
    s.y0 = 1;
    s.y1 = 0;
  } else {
    s.x0 = (short)a;
    s.x1 = (short)b;
    s.y0 = (short)c;
    s.y1 = (short)d;
  }
  return s;
}

__device__ __forceinline__ bool span_empty(Span s) { return s.x0 > s.x1 || s.y0 > s.y1; }
__device__ __forceinline__ bool span_overlaps(Span s, int x0, int x1, int y0, int y1) {
  return !(s.x1 < x0 || s.x0 > x1 || s.y1 < y0 || s.y0 > y1 || span_empty(s));
}

// ------------------------------------------------------------------------------------------
// Face sets: where the faces of view b are, how to get a face's (scaled) corners and box.
// ------------------------------------------------------------------------------------------
template <typename T>
struct FaceSet {
  int B, H, W;
  int64_t N;                 // rows of the face arrays
  int64_t F;                 // faces per view when first_idx == nullptr
  const int64_t *first_idx;  // packed layout (device), or nullptr
  const T *fvi;              // (N, 3, 2)
  T scale;                   // corners are fvi * scale (1 for already-scaled input)
  const T *bbox;             // (N, 4) explicit box in scaled space, or nullptr
  T margin;                  // computed box enlarged by +-margin when has_margin
  int has_margin;
  const uint8_t *valid;      // (N) uint8 or nullptr
  const T *nz;               // or: face i valid iff nz[i * nz_stride] >= 0 (normals z), nullable
  int64_t nz_stride;
  float M;                   // float multiplier of the pixel centres
  int dbg;                   // diagnostic ablation flags (0 in production)
  long long *tbuf;           // diagnostic per-tile clock buffer (nullptr in production)
};

// Three / two consecutive values of a row as one store (rows of 12 / 8 bytes at their element
// alignment: a dwordx3-or-x2+x1 / dwordx2 store instead of three / two dword stores)
template <typename T>
struct alignas(sizeof(T)) Vec3 {
  T x, y, z;
};
template <typename T>
struct alignas(sizeof(T)) Vec2 {
  T x, y;
};
template <typename T>
__device__ __forceinline__ void store3(T *p, T x, T y, T z) {
  *reinterpret_cast<Vec3<T> *>(p) = Vec3<T>{x, y, z};
}
template <typename T>
__device__ __forceinline__ void store2(T *p, T x, T y) {
  *reinterpret_cast<Vec2<T> *>(p) = Vec2<T>{x, y};
}

template <typename T>
__device__ __forceinline__ void view_range(const FaceSet<T> &fs, int b, int64_t &lo,
                                           int64_t &hi) {
  if (fs.first_idx) {
    lo = fs.first_idx[b];
    hi = fs.first_idx[b + 1];
  } else {
    lo = (int64_t)b * fs.F;
    hi = lo + fs.F;
  }
}

template <typename T>
__device__ __forceinline__ void load_corners(const FaceSet<T> &fs, int64_t i, T v[6]) {
  const T *p = fs.fvi + i * 6;
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] = p[k] * fs.scale;
}

// Box exactly as the reference host code builds it: min / max over the three scaled corners
// (rasterization.py:342-344), optionally -+ boxlen*multiplier (dibr.py:34-39).
template <typename T>
__device__ __forceinline__ void face_box(const FaceSet<T> &fs, int64_t i, const T v[6], T box[4]) {
  if (fs.bbox) {
    const T *p = fs.bbox + i * 4;
    box[0] = p[0];
    box[1] = p[1];
    box[2] = p[2];
    box[3] = p[3];
    return;
  }
  box[0] = nmin3(v[0], v[2], v[4]);
  box[1] = nmin3(v[1], v[3], v[5]);
  box[2] = nmax3(v[0], v[2], v[4]);
  box[3] = nmax3(v[1], v[3], v[5]);
  if (fs.has_margin) {
    box[0] = box[0] - fs.margin;
    box[1] = box[1] - fs.margin;
    box[2] = box[2] + fs.margin;
    box[3] = box[3] + fs.margin;
  }
}

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
__device__ __forceinline__ int rdlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double rdlane(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)(unsigned)lo) | ((long long)hi << 32));
}

// Workgroup-wide ordered compaction (256 threads): position of this thread's item among the
// items of lower threads, and the total.  s_cnt: 4 ints of LDS.
__device__ __forceinline__ int wg_compact(bool pred, int *s_cnt, int &total) {
  const uint64_t m = __ballot(pred);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) s_cnt[w] = __popcll(m);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / kWave; ++k) {
    const int c = s_cnt[k];
    off += (k < w) ? c : 0;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return pred ? off + mbcnt(m) : -1;
}

// ------------------------------------------------------------------------------------------
// coarse-bin geometry shared by host and device
// ------------------------------------------------------------------------------------------
#ifndef KD_COARSE_TILE0
#define KD_COARSE_TILE0 32
#endif
constexpr int kCoarseTile0 = KD_COARSE_TILE0;  // smallest coarse tile (px); grows to <= 32 per side

struct BinGeom {
  int ct;        // coarse tile edge in pixels (a power of two, multiple of kTile)
  int sh;        // log2(ct): coarse tile of pixel coordinate x >= 0 is x >> sh
  int nctx, ncty;
  __host__ __device__ int nct() const { return nctx * ncty; }
};

// ct0: the smallest coarse tile (kCoarseTile0, or kTile for the small-batch forward of
// kd_dibr.hip, whose workgroups cover 8x8 pixels and walk 16-pixel coarse bins)
__host__ __device__ inline BinGeom bin_geom(int H, int W, int ct0 = kCoarseTile0) {
  int m = H > W ? H : W;
  int ct = ct0;
  while (((m + ct - 1) / ct) > 32) ct *= 2;
  BinGeom g;
  g.ct = ct;
  g.sh = 0;
  while ((1 << g.sh) < ct) ++g.sh;
  g.nctx = (W + ct - 1) / ct;
  g.ncty = (H + ct - 1) / ct;
  return g;
}

}  // namespace kd
