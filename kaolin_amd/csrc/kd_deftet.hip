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
//   kd_dt_bin     conservative per-cell face lists on a uniform grid over [-1, 1]^2 (dt_grid),
//                 counted per workgroup in LDS and reserved with one global atomic per touched
//                 cell; the lists are unordered.
//   kd_dt_fwd     one wave per pixel walks its cell's list (lane = face, the reference test),
//                 hits go to an LDS list.  The reference keeps the first knum hits by face
//                 index: with more hits than knum the list is cut by face rank, with more than
//                 the LDS capacity a bisection on the face index (re-walks) finds the knum-th.
//                 The kept hits are ranked by depth, descending, ties by face index (a stable
//                 order; the reference's torch.argsort is not stable, so tied depths are the one
//                 place it is unpinned), and each slot writes its face index, weights
//                 (w0, w1, 1 - (w0 + w1)) and interpolated features; empty slots get -1 / 0.
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

// Uniform grid of G x G cells over [-1, 1]^2 per view (G = 64, or 32 when the worst-case list
// reservation of G^2 * B * F entries would pass 2^29); coordinates outside are clamped to the
// border cells.  dt_cell is monotone in x, so a pixel inside a face's box (xmin <= x0 <= xmax)
// lies in a cell of the face's cell range: the binning is conservative for any coordinates (NaN
// pixels and NaN boxes never pass the box test and are skipped).
constexpr int kDtGridMax = 64;

__host__ __device__ inline int dt_grid(int64_t N) {
  return (int64_t)64 * 64 * N <= (1ll << 29) ? 64 : 32;
}

template <typename T>
__device__ __forceinline__ int dt_cell(T x, int G) {
  T t = (x + (T)1) * (T)(G / 2);
  t = fmin(fmax(t, (T)0), (T)(G - 1));  // NaN -> 0
  return (int)t;                        // floor for t >= 0
}

template <typename T>
__device__ __forceinline__ bool dt_box(const T *v, T &xmin, T &ymin, T &xmax, T &ymax) {
  xmin = nmin3(v[0], v[2], v[4]);
  xmax = nmax3(v[0], v[2], v[4]);
  ymin = nmin3(v[1], v[3], v[5]);
  ymax = nmax3(v[1], v[3], v[5]);
  return !(isnan(xmin) || isnan(xmax) || isnan(ymin) || isnan(ymax));
}

// (view, face) -> every cell its box touches: unordered lists, cell c of view b at
// lists[c * N + b * F] with room for all F faces of the view; cursor[b][c] = list length.
// Neighbouring faces share cells, so a workgroup counts its 256 faces per cell in LDS, reserves
// one range per touched cell with a single global atomic, and places its faces in it.
// Box of face row i: the caller's (xmin, ymin, xmax, ymax) when given (the op form takes the
// reference's face_bboxes argument, deftet.cpp:48-55), else the corners' min / max (deftet.py:287-289).
template <typename T>
__device__ __forceinline__ bool dt_face_box(const T *fvi, const T *bbox, int64_t i, T &xmin,
                                            T &ymin, T &xmax, T &ymax) {
  if (bbox) {
    const T *q = bbox + i * 4;
    xmin = q[0];
    ymin = q[1];
    xmax = q[2];
    ymax = q[3];
    return !(isnan(xmin) || isnan(xmax) || isnan(ymin) || isnan(ymax));
  }
  return dt_box<T>(fvi + i * 6, xmin, ymin, xmax, ymax);
}

// One atomic add per distinct key of a wave (lanes with the same key share it: a pixel grid
// puts a wave's 64 pixels into ~8 cells); RET: this lane's slot, the counter's old value plus
// the lane's rank among the lanes of its key (every atomic is issued before the first wait).
template <bool RET>
__device__ __forceinline__ int wave_key_add(int *ctr, int key, bool active) {
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t rem = __ballot(active);
  int leader = 0, rank = 0, mine = 0;
  while (rem) {
    const int l = __builtin_ctzll(rem);
    const int k = __builtin_amdgcn_readlane(key, l);
    const bool in = active && key == k;
    const uint64_t m = __ballot(in);
    if (in) {
      leader = l;
      rank = mbcnt(m);
    }
    if (lane == l) {
      if constexpr (RET)
        mine = atomicAdd(&ctr[k], __popcll(m));
      else
        atomicAdd(&ctr[k], __popcll(m));
    }
    rem &= ~m;
  }
  if constexpr (!RET) return 0;
  return __shfl(mine, leader) + rank;
}

// The cell-major walk's pixel sort, first step (workgroups past the face workgroups of the same
// launch): pixels per cell (wave-aggregated atomics), and the per-pixel hit counts zeroed.
template <typename T>
__device__ void dt_count_pixels(int64_t P, int G, const T *px, int *pcnt, int *hcnt, int64_t p) {
  const int b = blockIdx.y;
  int c = 0;
  if (p < P) {
    const int64_t pp = (int64_t)b * P + p;
    c = dt_cell(px[2 * pp + 1], G) * G + dt_cell(px[2 * pp], G);
    hcnt[pp] = 0;
  }
  wave_key_add<false>(pcnt + (int64_t)b * G * G, c, p < P);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_dt_bin(int64_t F, int64_t N, int G, const T *fvi,
                                                    const T *bbox, int *cursor, int *lists,
                                                    T *boxes, int nfb, int64_t P, const T *px,
                                                    int *pcnt, int *hcnt) {
  __shared__ int s_cnt[kDtGridMax * kDtGridMax];
  const int b = blockIdx.y, cells = G * G;
  if ((int)blockIdx.x >= nfb) {  // (uniform per workgroup)
    dt_count_pixels<T>(P, G, px, pcnt, hcnt, (int64_t)(blockIdx.x - nfb) * kBlock + threadIdx.x);
    return;
  }
  for (int i = threadIdx.x; i < cells; i += kBlock) s_cnt[i] = 0;
  __syncthreads();
  const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  T xmin = 0, ymin = 0, xmax = 0, ymax = 0;
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (f < F && dt_face_box<T>(fvi, bbox, (int64_t)b * F + f, xmin, ymin, xmax, ymax)) {
    cx0 = dt_cell(xmin, G);
    cx1 = dt_cell(xmax, G);
    cy0 = dt_cell(ymin, G);
    cy1 = dt_cell(ymax, G);
  }
  if (boxes && f < F) {  // the walk's box table (a NaN box is in no list: its value is unused)
    T *q = boxes + ((int64_t)b * F + f) * 4;
    q[0] = xmin;
    q[1] = ymin;
    q[2] = xmax;
    q[3] = ymax;
  }
  for (int cy = cy0; cy <= cy1; ++cy)
    for (int cx = cx0; cx <= cx1; ++cx) atomicAdd(&s_cnt[cy * G + cx], 1);
  __syncthreads();
  int *cur = cursor + (int64_t)b * cells;
  for (int i = threadIdx.x; i < cells; i += kBlock) {
    const int n = s_cnt[i];
    s_cnt[i] = n ? atomicAdd(&cur[i], n) : 0;  // this workgroup's range start in cell i
  }
  __syncthreads();
  for (int cy = cy0; cy <= cy1; ++cy)
    for (int cx = cx0; cx <= cx1; ++cx) {
      const int c = cy * G + cx;
      const int pos = atomicAdd(&s_cnt[c], 1);
      lists[(int64_t)c * N + (int64_t)b * F + pos] = (int)f;
    }
}

template <typename T>
__device__ __forceinline__ bool dt_face_weights(T ax, T ay, T bx, T by, T cx, T cy, T z0, T z1,
                                                T z2, T x0, T y0, T dmin, T dmax, T eps, T &w0,
                                                T &w1, T &depth);

// The reference's per-face test (deftet_cuda.cu:114-160): half-open box of the corner min / max,
// eps-normalised barycentrics (copysignf of the float eps, also for fp64 data), all >= 0, depth
// in [min, max).
template <typename T>
__device__ __forceinline__ bool dt_face_test(const T *v, const T *z, const T *bbox, T x0, T y0,
                                             T dmin, T dmax, T eps, T &w0, T &w1, T &depth) {
  const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
  T xmin, xmax, ymin, ymax;
  if (bbox) {
    xmin = bbox[0];
    ymin = bbox[1];
    xmax = bbox[2];
    ymax = bbox[3];
  } else {
    xmin = nmin3(ax, bx, cx);
    xmax = nmax3(ax, bx, cx);
    ymin = nmin3(ay, by, cy);
    ymax = nmax3(ay, by, cy);
  }
  if (!(x0 >= xmin && x0 < xmax && y0 >= ymin && y0 < ymax)) return false;
  return dt_face_weights<T>(ax, ay, bx, by, cx, cy, z[0], z[1], z[2], x0, y0, dmin, dmax, eps, w0,
                            w1, depth);
}

// The test past the box (deftet_cuda.cu:128-160), on corner values.
template <typename T>
__device__ __forceinline__ bool dt_face_weights(T ax, T ay, T bx, T by, T cx, T cy, T z0, T z1,
                                                T z2, T x0, T y0, T dmin, T dmax, T eps, T &w0,
                                                T &w1, T &depth) {
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
  if (!(w0 >= (T)0 && w1 >= (T)0 && w2 >= (T)0)) return false;
  depth = w0 * z0 + w1 * z1 + w2 * z2;   // :156
  return depth < dmax && depth >= dmin;  // :158
}

// The cell-major walk's hit records: per pixel up to kDtHitCap hits in the order found (a pixel
// with more re-walks its cell list in kd_dt_fwd).
template <typename T>
struct alignas(16) DtHit {
  int f;
  T depth, w0, w1;
};
constexpr int kDtHitCap = 64;
constexpr int kDtWalkDMax = 4;  // the cell-major path carries features up to this D
constexpr int kDtFaceChunk = 128;  // faces of a cell list per walk item

template <typename T>
struct DtArgs {
  int B;
  int64_t P, F, N;
  int K, D, C;  // C: LDS hit-list capacity per pixel (>= K)
  int G;        // grid cells per side
  float eps;
  const T *px;      // (B, P, 2)
  const T *range;   // (B, P, 2): min, max depth
  const T *fvz;     // (B, F, 3)
  const T *fvi;     // (B, F, 3, 2)
  const T *feat;    // (B, F, 3, D)
  const int *cursor, *lists;
  const T *boxes;     // (B, F, 4): xmin, ymin, xmax, ymax of every face (bbox or kd_dt_bin's)
  T *interp;          // (B, P, K, D)
  int64_t *face_idx;  // (B, P, K)
  T *weights;         // (B, P, K, 3)
  // op form (deftet_sparse_render_forward_cuda, deftet_cuda.cu:31-192): the caller's boxes, and
  // per slot in face-index order (unsorted) face, depth, w0, w1 instead of interp / weights
  const T *bbox;      // (B, F, 4) or nullptr
  T *depth, *w0, *w1; // (B, P, K) each, or nullptr (sorted mode)
  int dbg;            // diagnostic ablation flags (kd_common.hpp)
  long long *tbuf;    // diagnostics (flag 64): candidate / hit / fallback / flush counters
  // the cell-major path: kd_dt_walk's hits for kd_dt_out; the pixels it defers (more hits than
  // its records hold) for kd_dt_fwd's own walk, or nullptr: kd_dt_fwd takes every pixel
  const int *hcnt;       // (B, P) hits found
  const DtHit<T> *hits;  // (B, P, kDtHitCap)
  const T *hint;         // (B, P, kDtHitCap, D): the records' interpolated features (D <= 4)
  int *ovf, *novf;       // deferred pixels (b * P + p) and their count
};

constexpr int kDtWaves = 4;  // pixels per workgroup

// A cell's walk items: its pixels in groups of 64 against its face list cut into at most
// kDtSplitMax near-equal chunks of ~kWave faces (the long pole-cell lists spread over many waves).
constexpr int kDtSplitMax = 16;
__host__ __device__ inline int dt_splits(int nl) {
  return min((nl + kWave - 1) / kWave, kDtSplitMax);
}
__host__ __device__ inline int dt_items(int np, int nl) {
  return np > 0 && nl > 0 ? ((np + kWave - 1) / kWave) * dt_splits(nl) : 0;
}

// The pixel sort, second step (one workgroup): each cell's first slot in the sorted pixel order
// (the exclusive prefix of the pixel counts over every view's cells), and the walk's item table
// (cell, pixel group * kDtSplitMax + face chunk) and its length (nitems).
__global__ __launch_bounds__(1024) void kd_dt_pscan(int n, const int *pcnt, const int *cursor,
                                                    int *poff, int2 *items, int *nitems) {
  __shared__ int s_p[1024], s_i[1024];
  const int t = threadIdx.x, m = (n + 1023) / 1024;
  const int i0 = min(n, t * m), i1 = min(n, i0 + m);
  int sp = 0, si = 0;
  for (int i = i0; i < i1; ++i) {
    sp += pcnt[i];
    si += dt_items(pcnt[i], cursor[i]);
  }
  s_p[t] = sp;
  s_i[t] = si;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int vp = t >= d ? s_p[t - d] : 0, vi = t >= d ? s_i[t - d] : 0;
    __syncthreads();
    s_p[t] += vp;
    s_i[t] += vi;
    __syncthreads();
  }
  if (t == 1023) *nitems = s_i[t];
  int rp = s_p[t] - sp, ri = s_i[t] - si;
  for (int i = i0; i < i1; ++i) {
    poff[i] = rp;
    rp += pcnt[i];
    const int np = pcnt[i], nl = cursor[i];
    if (np == 0 || nl == 0) continue;
    const int ns = dt_splits(nl), ng = (np + kWave - 1) / kWave;
    for (int g = 0; g < ng; ++g)
      for (int fc = 0; fc < ns; ++fc) items[ri++] = make_int2(i, g * kDtSplitMax + fc);
  }
}

// Third step: every pixel into its cell's range (the order inside a cell is free: a pixel's
// result depends only on the set of its hits).
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_dt_pscatter(int64_t P, int G, const T *px,
                                                         const int *poff, int *pfill, int *spix) {
  const int b = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t pp = (int64_t)b * P + p;
  const int c = p < P ? dt_cell(px[2 * pp + 1], G) * G + dt_cell(px[2 * pp], G) : 0;
  const int64_t cb = (int64_t)b * G * G;
  const int slot = wave_key_add<true>(pfill + cb, c, p < P);
  if (p < P) spix[poff[cb + c] + slot] = (int)p;
}

template <typename T>
__device__ __forceinline__ T dt_bcast(T v, int j) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), j);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

// The cell-major walk: a wave per item (64 of a cell's sorted pixels, lane = pixel, against one
// chunk of its face list; grid-stride over the item table).  A step loads 64 faces' boxes, corners
// and depths (lane = face, one gather per step) and broadcasts them face by face: the box test is
// one compare group per face for all 64 pixels, and the exact test (dt_face_weights, the
// reference's arithmetic) runs only for faces whose box holds some lane's pixel.  A cell with one
// chunk writes its pixels' hit records directly.  With several, the wave's hits are appended to a
// wave pool in LDS (kDtPool records, each tagged with its lane and the lane's hit number) and
// flushed when it could overflow and at the end: one atomic per pixel reserves its records, then
// the wave writes the pool out.
constexpr int kDtPool = 256;
constexpr int kDtWalkWaves = 4;

// DI > 0: the hit's interpolated features (D = DI <= 4) go with its record (hint), from the face's
// features gathered with its corners -- kd_dt_out then needs no gather of its own.
template <typename T, int DI>
__global__ __launch_bounds__(kWave *kDtWalkWaves) void kd_dt_walk(DtArgs<T> a, const int *pcnt,
                                                                  const int *poff, const int *spix,
                                                                  const int2 *items,
                                                                  const int *nitems, int *hcnt,
                                                                  DtHit<T> *hits, T *hint) {
  constexpr int DP = DI > 0 ? DI : 1;
  __shared__ DtHit<T> s_pool[kDtWalkWaves][kDtPool];
  __shared__ T s_pint[kDtWalkWaves][kDtPool][DP];
  __shared__ int s_tag[kDtWalkWaves][kDtPool];  // lane | hit number << 6
  __shared__ int s_base[kDtWalkWaves][kWave];   // the lane's first record of this flush
  __shared__ int s_pp[kDtWalkWaves][kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int G = a.G, cells = G * G;
  const int n_items = *nitems;
  const T eps = (T)a.eps;
  for (int it = blockIdx.x * kDtWalkWaves + wave; it < n_items; it += gridDim.x * kDtWalkWaves) {
    const int2 item = items[it];
    const int gc = item.x, b = gc / cells, c = gc - b * cells;
    const int g = item.y / kDtSplitMax, fc = item.y - g * kDtSplitMax;
    const int np = pcnt[gc], nl = a.cursor[gc], ns = dt_splits(nl);
    const int k = g * kWave + lane;
    const bool valid = k < np;
    int64_t pp = 0;
    T x0 = 0, y0 = 0, dmin = 0, dmax = 0;
    if (valid) {
      pp = (int64_t)b * a.P + spix[poff[gc] + k];
      x0 = a.px[2 * pp];
      y0 = a.px[2 * pp + 1];
      dmin = a.range[2 * pp];
      dmax = a.range[2 * pp + 1];
    }
    const int *list = a.lists + (int64_t)c * a.N + (int64_t)b * a.F;
    const T *fvi = a.fvi + (int64_t)b * a.F * 6;
    const T *fvz = a.fvz + (int64_t)b * a.F * 3;
    const T *boxes = a.boxes + (int64_t)b * a.F * 4;
    const T *feat = DI > 0 ? a.feat + (int64_t)b * a.F * 3 * DI : nullptr;
    const int f0 = (int)((int64_t)fc * nl / ns), f1 = (int)((int64_t)(fc + 1) * nl / ns);
    const bool direct = ns == 1;
    int num = 0, pend = 0, pooled = 0;
    s_pp[wave][lane] = (int)pp;
    auto put = [&](int64_t r, const DtHit<T> &h, const T *iv) {
      hits[r] = h;
#pragma unroll
      for (int d = 0; d < DI; ++d) hint[r * DI + d] = iv[d];
    };
    auto flush = [&]() {  // (wave-uniform)
      s_base[wave][lane] = valid && pend > 0 ? atomicAdd(&hcnt[pp], pend) : 0;
      wave_lds_sync();
      for (int e = lane; e < pooled; e += kWave) {
        const int tag = s_tag[wave][e], l = tag & (kWave - 1);
        const int slot = s_base[wave][l] + (tag >> 6);
        if (slot < kDtHitCap)
          put((int64_t)s_pp[wave][l] * kDtHitCap + slot, s_pool[wave][e], s_pint[wave][e]);
      }
      wave_lds_sync();
      pend = 0;
      pooled = 0;
    };
    for (int j0 = f0; j0 < f1; j0 += kWave) {
      const int m = min(kWave, f1 - j0);
      int f = 0;
      T q[4] = {}, v[6] = {}, z[3] = {}, cf[3 * DP] = {};
      if (lane < m) {
        f = list[j0 + lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = boxes[(int64_t)f * 4 + i];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = fvi[(int64_t)f * 6 + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) z[i] = fvz[(int64_t)f * 3 + i];
#pragma unroll
        for (int i = 0; i < 3 * DI; ++i) cf[i] = feat[(int64_t)f * 3 * DI + i];
      }
      for (int jj = 0; jj < m; ++jj) {
        const T xmin = dt_bcast(q[0], jj), ymin = dt_bcast(q[1], jj);
        const T xmax = dt_bcast(q[2], jj), ymax = dt_bcast(q[3], jj);
        const bool inb = valid && x0 >= xmin && x0 < xmax && y0 >= ymin && y0 < ymax;
        if (__ballot(inb) == 0) continue;
        T w0 = 0, w1 = 0, depth = 0;
        const bool hit =
            inb && dt_face_weights<T>(dt_bcast(v[0], jj), dt_bcast(v[1], jj), dt_bcast(v[2], jj),
                                      dt_bcast(v[3], jj), dt_bcast(v[4], jj), dt_bcast(v[5], jj),
                                      dt_bcast(z[0], jj), dt_bcast(z[1], jj), dt_bcast(z[2], jj),
                                      x0, y0, dmin, dmax, eps, w0, w1, depth);
        const uint64_t hm = __ballot(hit);
        if (hm == 0) continue;
        const DtHit<T> h{dt_bcast(f, jj), depth, w0, w1};
        T iv[DP] = {};
        const T w2 = (T)1 - (w0 + w1);  // deftet.py:304
#pragma unroll
        for (int d = 0; d < DI; ++d)  // :312-313, the sum over the 3 corners in order
          iv[d] = w0 * dt_bcast(cf[d], jj) + w1 * dt_bcast(cf[DI + d], jj) +
                  w2 * dt_bcast(cf[2 * DI + d], jj);
        if (direct) {
          if (hit && num < kDtHitCap) put(pp * kDtHitCap + num, h, iv);
          num += hit ? 1 : 0;
          continue;
        }
        if (hit) {
          const int at = pooled + mbcnt(hm);
          s_pool[wave][at] = h;
#pragma unroll
          for (int d = 0; d < DI; ++d) s_pint[wave][at][d] = iv[d];
          s_tag[wave][at] = lane | (pend << 6);
          ++pend;
        }
        pooled += __popcll(hm);
        if (pooled > kDtPool - kWave) flush();
      }
    }
    if (direct) {
      if (valid) hcnt[pp] = num;
    } else if (pooled > 0) {
      flush();
    }
  }
}

template <typename T>
__host__ __device__ constexpr size_t dt_wave_lds(int C) {  // depth, w0, w1, face, face rank
  return (size_t)C * (3 * sizeof(T) + 2 * sizeof(int));
}

// One wave per pixel.  The pixel's cell list is walked 64 faces at a time (lane = face, the
// reference test), hits go to the wave's LDS list.  The reference keeps the first knum hits by
// face index: with more hits than knum the list is cut by face rank; with more than the LDS
// capacity a binary search on the face index (re-walks counting hits below a threshold) finds
// the knum-th smallest and only hits below it are collected.  The kept hits are then ranked by
// depth, descending, ties by face index, and each slot writes face index, weights
// (w0, w1, 1 - (w0 + w1)) and interpolated features; empty slots get -1 / 0.
template <typename T>
__device__ void dt_pixel_wave(const DtArgs<T> &a, int b, int64_t p, char *wave_lds) {
  const int lane = threadIdx.x & 63;
  const int K = a.K, C = a.C;
  T *dep = (T *)wave_lds;
  T *lw0 = dep + C, *lw1 = lw0 + C;
  int *fid = (int *)(lw1 + C);
  const int64_t pp = (int64_t)b * a.P + p;
  const T x0 = a.px[2 * pp], y0 = a.px[2 * pp + 1];
  const T dmin = a.range[2 * pp], dmax = a.range[2 * pp + 1];
  const T *fvi = a.fvi + (int64_t)b * a.F * 6;
  const T *fvz = a.fvz + (int64_t)b * a.F * 3;
  const T *bbox = a.bbox ? a.bbox + (int64_t)b * a.F * 4 : nullptr;
  const T eps = (T)a.eps;
  int nl;
  const int *list;
  // walk: hits with face < limit are appended (limit = F: all)
  auto walk = [&](int limit, bool store) {
    int num = 0;
    for (int j0 = 0; j0 < nl; j0 += kWave) {
      const int j = j0 + lane;
      bool hit = false;
      T w0 = 0, w1 = 0, depth = 0;
      int f = 0;
      if (j < nl) {
        f = list[j];
        if (f < limit)
          hit = dt_face_test<T>(fvi + (int64_t)f * 6, fvz + (int64_t)f * 3,
                                bbox ? bbox + (int64_t)f * 4 : nullptr, x0, y0, dmin, dmax, eps,
                                w0, w1, depth);
      }
      const uint64_t hm = __ballot(hit);
      if (store && hit) {
        const int at = num + (int)__builtin_amdgcn_mbcnt_hi(
                                 (uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
        if (at < C) {
          dep[at] = depth;
          lw0[at] = w0;
          lw1[at] = w1;
          fid[at] = f;
        }
      }
      num += __popcll(hm);
    }
    return num;
  };
  const int G = a.G;
  const int c = dt_cell(y0, G) * G + dt_cell(x0, G);
  nl = a.cursor[(int64_t)b * G * G + c];
  list = a.lists + (int64_t)c * a.N + (int64_t)b * a.F;
  int nh = walk(INT_MAX, true);
  if (nh > C) {  // more hits than the list holds: the knum smallest face indices, by bisection
    int lo = 0, hi = (int)a.F;  // count(face < hi) >= K
    while (lo < hi) {
      const int mid = lo + (hi - lo) / 2;
      if (walk(mid + 1, false) >= K)
        hi = mid;
      else
        lo = mid + 1;
    }
    wave_lds_sync();
    nh = walk(lo + 1, true);  // exactly K hits: faces <= the K-th smallest
  }
  wave_lds_sync();
  // the reference keeps the first K hits by face index: mark the others (face rank >= K)
  int *frank = fid + C;
  const int64_t row = pp * K;
  if (a.depth) {
    // op form: slot = face rank among the hits (the reference kernel's insertion order,
    // deftet_cuda.cu:166-180), unsorted; the empty slots keep -1 / -inf / 0 / 0
    // (deftet.cpp:88-94)
    for (int i = lane; i < nh; i += kWave) {
      const int fi = fid[i];
      int r = 0;
      for (int j = 0; j < nh; ++j) r += fid[j] < fi ? 1 : 0;
      if (r < K) {
        a.face_idx[row + r] = fi;
        a.depth[row + r] = dep[i];
        a.w0[row + r] = lw0[i];
        a.w1[row + r] = lw1[i];
      }
    }
    for (int s = min(nh, K) + lane; s < K; s += kWave) {
      a.face_idx[row + s] = -1;
      a.depth[row + s] = (T)-INFINITY;
      a.w0[row + s] = (T)0;
      a.w1[row + s] = (T)0;
    }
    return;
  }
  const bool cut = nh > K;
  for (int i = lane; i < nh; i += kWave) {
    int r = 0;
    if (cut) {
      const int fi = fid[i];
      for (int j = 0; j < nh; ++j) r += fid[j] < fi ? 1 : 0;
    }
    frank[i] = r;
  }
  wave_lds_sync();
  // rank the kept hits: depth descending, then face index (deftet.py:300-303, stable order)
  const int n = cut ? K : nh;
  const int D = a.D;
  const T *feat = a.feat + (int64_t)b * a.F * 3 * D;
  for (int i = lane; i < nh; i += kWave) {
    if (frank[i] >= K) continue;
    const T di = dep[i];
    const int fi = fid[i];
    int r = 0;
    for (int j = 0; j < nh; ++j) {
      const T dj = dep[j];
      r += (frank[j] < K && (dj > di || (dj == di && fid[j] < fi))) ? 1 : 0;
    }
    const T w0 = lw0[i], w1 = lw1[i];
    const T w2 = (T)1 - (w0 + w1);  // deftet.py:304
    const int64_t o = row + r;
    a.face_idx[o] = fi;
    a.weights[3 * o] = w0;
    a.weights[3 * o + 1] = w1;
    a.weights[3 * o + 2] = w2;
    const T *cf = feat + (int64_t)fi * 3 * D;
    T *out = a.interp + o * D;
    for (int d = 0; d < D; ++d)  // :312-313, the sum over the 3 corners in order
      out[d] = w0 * cf[d] + w1 * cf[D + d] + w2 * cf[2 * D + d];
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
__global__ __launch_bounds__(kWave *kDtWaves) void kd_dt_fwd(DtArgs<T> a) {
  extern __shared__ __align__(16) char dt_lds[];
  const int w = threadIdx.x >> 6;
  char *lds = dt_lds + (size_t)w * dt_wave_lds<T>(a.C);
  // a pixel per wave, or (ovf without hits) the pixels kd_dt_out deferred, grid-stride
  const bool deferred = a.ovf && !a.hits;
  const int n = deferred ? *a.novf : 0;
  for (int i = blockIdx.x * kDtWaves + w;; i += gridDim.x * kDtWaves) {
    int b = blockIdx.y;
    int64_t p = i;
    if (deferred) {
      if (i >= n) return;
      const int pp = a.ovf[i];
      b = (int)(pp / a.P);
      p = pp - (int64_t)b * a.P;
    } else if (i >= a.P || i >= (int)(blockIdx.x + 1) * kDtWaves) {
      return;  // whole wave (one pixel per wave)
    }
    dt_pixel_wave<T>(a, b, p, lds);
    wave_lds_sync();
  }
}

// x / m and x % m for 0 <= x < 2^22 (a float reciprocal and one correction step)
__device__ __forceinline__ int dt_divmod(int x, int m, float inv, int &r) {
  int q = (int)((float)x * inv);
  r = x - q * m;
  if (r < 0) {
    --q;
    r += m;
  } else if (r >= m) {
    ++q;
    r -= m;
  }
  return q;
}

// The cell-major path's outputs: a workgroup per kDtOutPix consecutive pixels.  Their hit records
// (and interpolated features, DI = D) go to LDS packed one after another, a thread per record
// (~6 per pixel on the bench mesh, so every phase is one or two rounds of the workgroup); each
// record's thread finds its face rank (the reference keeps the first knum hits by face index) and
// its slot -- depth descending, ties by face index (deftet.py:300-303), or, in the op form, the
// face rank itself; then the block's contiguous outputs are written in memory order from LDS, a
// thread per (pixel, slot).  A pixel with more hits than its records hold, or past the block's
// kDtOutPool records, is deferred to kd_dt_fwd's walk (its list).
constexpr int kDtOutPix = 32;
constexpr int kDtOutThreads = 128;
constexpr int kDtOutPool = 1024;

template <typename T, int DI>
__global__ __launch_bounds__(kDtOutThreads) void kd_dt_out(DtArgs<T> a) {
  constexpr int DP = DI > 0 ? DI : 1;
  __shared__ int s_n[kDtOutPix], s_off[kDtOutPix], s_total;
  __shared__ DtHit<T> s_h[kDtOutPool];                     // the block's records
  __shared__ T s_hi[kDtOutPool][DP];                       // their features
  __shared__ unsigned char s_own[kDtOutPool], s_fr[kDtOutPool];  // record -> pixel, face rank
  __shared__ short s_slot[kDtOutPix][kDtHitCap];           // (pixel, slot) -> record
  const int t = threadIdx.x, b = blockIdx.y;
  const int K = a.K;
  const bool raw = a.depth != nullptr;
  const int64_t p0 = (int64_t)blockIdx.x * kDtOutPix;
  const int npx = (int)min<int64_t>(kDtOutPix, a.P - p0);
  const int64_t pp0 = (int64_t)b * a.P + p0;
  if (t < kWave) {
    const int n = t < npx ? a.hcnt[pp0 + t] : 0;
    const int incl = wave_incl_scan(n <= kDtHitCap ? n : 0);
    const bool defer = t < npx && (n > kDtHitCap || incl > kDtOutPool);
    const int slot = wave_key_add<true>(a.novf, 0, defer);
    if (defer) a.ovf[slot] = (int)(pp0 + t);
    const int nk = defer ? 0 : n;
    if (t < kDtOutPix) {
      s_n[t] = defer ? -1 : n;
      s_off[t] = incl - nk;
      for (int i = 0; i < nk; ++i) s_own[incl - nk + i] = (unsigned char)t;
    }
    const int last = wave_incl_scan(nk);
    if (t == kWave - 1) s_total = last;
  }
  __syncthreads();
  const int H = s_total;
  for (int e = t; e < H; e += kDtOutThreads) {
    const int px = s_own[e];
    const int64_t r = (pp0 + px) * kDtHitCap + (e - s_off[px]);
    s_h[e] = a.hits[r];
#pragma unroll
    for (int d = 0; d < DI; ++d) s_hi[e][d] = a.hint[r * DI + d];
  }
  __syncthreads();
  for (int e = t; e < H; e += kDtOutThreads) {
    const int px = s_own[e], n = s_n[px], o = s_off[px];
    int fr = 0;
    if (raw || n > K) {
      const int fj = s_h[e].f;
      for (int i = 0; i < n; ++i) fr += s_h[o + i].f < fj ? 1 : 0;
    }
    s_fr[e] = (unsigned char)fr;
  }
  __syncthreads();
  for (int e = t; e < H; e += kDtOutThreads) {
    if (s_fr[e] >= K) continue;
    const int px = s_own[e];
    if (raw) {
      s_slot[px][s_fr[e]] = (short)e;
      continue;
    }
    const int n = s_n[px], o = s_off[px];
    const T de = s_h[e].depth;
    const int fe = s_h[e].f;
    int r = 0;
    for (int i = o; i < o + n; ++i) {
      const T di = s_h[i].depth;
      r += (s_fr[i] < K && (di > de || (di == de && s_h[i].f < fe))) ? 1 : 0;
    }
    s_slot[px][r] = (short)e;
  }
  __syncthreads();
  // the block's outputs, a thread per (pixel, slot) in memory order (a deferred pixel's rows are
  // kd_dt_fwd's)
  const int64_t o0 = pp0 * K;
  const float invK = 1.0f / (float)K;
  for (int e = t; e < npx * K; e += kDtOutThreads) {
    int s;
    const int px = dt_divmod(e, K, invK, s), n = s_n[px];
    if (n < 0) continue;
    const bool on = s < min(n, K);
    const int rec = on ? s_slot[px][s] : 0;
    const DtHit<T> h = s_h[rec];
    const int64_t o = o0 + e;
    a.face_idx[o] = on ? (int64_t)h.f : -1;
    if (raw) {  // deftet.cpp:88-94's padding
      a.depth[o] = on ? h.depth : (T)-INFINITY;
      a.w0[o] = on ? h.w0 : (T)0;
      a.w1[o] = on ? h.w1 : (T)0;
      continue;
    }
    a.weights[3 * o] = on ? h.w0 : (T)0;
    a.weights[3 * o + 1] = on ? h.w1 : (T)0;
    a.weights[3 * o + 2] = on ? (T)1 - (h.w0 + h.w1) : (T)0;
#pragma unroll
    for (int d = 0; d < DI; ++d) a.interp[o * DI + d] = on ? s_hi[rec][d] : (T)0;
  }
}

// Workspace: [cursor | pixel counts | pixel fill] (one memset), the cell lists, the face boxes,
// and the cell-major walk's pixel offsets, sorted pixels, hit counts and hit records.
struct DtLayout {
  size_t cursor, lists, boxes, poff, spix, hcnt, hits, hint, items, ovf, total;
};
static DtLayout dt_layout(int B, int64_t P, int64_t F, int D, size_t esize) {
  const int64_t N = (int64_t)B * F;
  const size_t cells = (size_t)dt_grid(N) * dt_grid(N);
  DtLayout l;
  size_t o = 0;
  l.cursor = o;  // cursor, pixel counts, pixel fill, the item count, the deferred pixel count
  o += align_up(3 * sizeof(int) * (size_t)B * cells + 2 * sizeof(int));
  l.lists = o;
  o += align_up(sizeof(int) * cells * (size_t)(N > 0 ? N : 1));
  l.boxes = o;
  o += align_up(4 * esize * (size_t)N);
  l.poff = o;
  o += align_up(sizeof(int) * (size_t)B * cells);
  l.spix = o;
  o += align_up(sizeof(int) * (size_t)B * (size_t)P);
  l.hcnt = o;
  o += align_up(sizeof(int) * (size_t)B * (size_t)P);
  l.hits = o;
  o += align_up((esize == 8 ? 32 : 16) * (size_t)kDtHitCap * (size_t)B * (size_t)P);
  l.hint = o;
  o += align_up(esize * (size_t)(D <= kDtWalkDMax ? D : 0) * kDtHitCap * (size_t)B * (size_t)P);
  l.items = o;  // at most (pixel groups + cells) * kDtSplitMax per view
  o += align_up(sizeof(int2) * (size_t)kDtSplitMax * (size_t)B *
                ((size_t)(P + kWave - 1) / kWave + cells));
  l.ovf = o;
  o += align_up(sizeof(int) * (size_t)B * (size_t)P);
  l.total = o;
  return l;
}
static size_t dt_workspace(int B, int64_t P, int64_t F, int D, size_t esize) {
  return dt_layout(B, P, F, D, esize).total;
}

static int dt_capacity(int K) { return K < 256 ? 256 : K; }

// The cell-major walk and its outputs (DI: the features the records carry).
template <typename T, int DI>
static void dt_cell_launch(const DtArgs<T> &a, const int *pcnt, const int *poff, const int *spix,
                           const int2 *items, const int *nitems, hipStream_t stream) {
  {
    ProfScope prof(K_DT_WALK, stream);
    // as many workgroups as fit at once (the items are dealt statically, grid-stride)
    constexpr size_t lds = (sizeof(DtHit<T>) + sizeof(T) * (DI > 0 ? DI : 1) + sizeof(int)) *
                               kDtPool * kDtWalkWaves +
                           2 * sizeof(int) * kWave * kDtWalkWaves;
    const int per_cu = (int)std::min<size_t>(8, (160 * 1024) / lds);
    hipLaunchKernelGGL((kd_dt_walk<T, DI>), dim3((unsigned)(device_cus(stream) * per_cu)),
                       dim3(kWave * kDtWalkWaves), 0, stream, a, pcnt, poff, spix, items, nitems,
                       (int *)a.hcnt, (DtHit<T> *)a.hits, (T *)a.hint);
  }
  ProfScope prof(K_DT_OUT, stream);
  hipLaunchKernelGGL((kd_dt_out<T, DI>), dim3((unsigned)((a.P + kDtOutPix - 1) / kDtOutPix), a.B),
                     dim3(kDtOutThreads), 0, stream, a);
}

template <typename T>
static int dt_forward(int B, int64_t P, int64_t F, int K, int D, const T *px, const T *range,
                      const T *fvz, const T *fvi, const T *feat, float eps, T *interp,
                      int64_t *face_idx, T *weights, void *ws, size_t wsb, hipStream_t stream,
                      const T *bbox = nullptr, T *depth = nullptr, T *w0 = nullptr,
                      T *w1 = nullptr) {
  KD_CHECK_ARG(B >= 0 && B <= 65535 && P >= 0 && F >= 0 && D >= 0, "deftet: bad sizes");
  KD_CHECK_ARG(K >= 1, "deftet: knum must be >= 1");
  KD_CHECK_ARG(F < (1ll << 31) && (int64_t)B * F < (1ll << 40), "deftet: too many faces");
  const int C = dt_capacity(K);
  const size_t lds = dt_wave_lds<T>(C) * kDtWaves;
  KD_CHECK_ARG(lds <= 160 * 1024, "deftet: knum too large for the LDS list (fp32 <= 2048, "
                                  "fp64 <= 1280)");
  static_assert(sizeof(DtHit<T>) == (sizeof(T) == 8 ? 32 : 16), "hit record size");
  const DtLayout lay = dt_layout(B, P, F, depth ? 0 : D, sizeof(T));
  const size_t need = lay.total;
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  if (B == 0 || P == 0) return KD_OK;
  KD_CHECK_ARG((int64_t)B * P < (1ll << 31), "deftet: more than 2^31 pixels");
  const int64_t N = (int64_t)B * F;
  const int G = dt_grid(N);
  const size_t cells = (size_t)G * G;
  char *w = (char *)ws;
  int *cursor = (int *)(w + lay.cursor);
  int *pcnt = cursor + (size_t)B * cells, *pfill = pcnt + (size_t)B * cells;
  int *lists = (int *)(w + lay.lists);
  T *boxes = (T *)(w + lay.boxes);
  int *poff = (int *)(w + lay.poff), *spix = (int *)(w + lay.spix), *hcnt = (int *)(w + lay.hcnt);
  DtHit<T> *hits = (DtHit<T> *)(w + lay.hits);
  T *hint = (T *)(w + lay.hint);
  int2 *items = (int2 *)(w + lay.items);
  int *nitems = pfill + (size_t)B * cells, *novf = nitems + 1;
  int *ovf = (int *)(w + lay.ovf);
  // the cell-major path (the default; KD_FORM_DT_PIXEL: every pixel walks its list in kd_dt_fwd),
  // with the features carried by the records for D <= kDtWalkDMax (the op form has none)
  const int DI = depth ? 0 : D;
  const bool cellwalk = F > 0 && !(test_forms() & KD_FORM_DT_PIXEL) && DI <= kDtWalkDMax;
  hipError_t e = zero_words(cursor, 3 * sizeof(int) * (size_t)B * cells + 2 * sizeof(int), stream);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "deftet: %s", hipGetErrorString(e));
  const int nfb = (int)((F + kBlock - 1) / kBlock);
  const int64_t npb = cellwalk ? (P + kBlock - 1) / kBlock : 0;
  KD_CHECK_ARG(nfb + npb < (1ll << 31), "deftet: too many faces / pixels");
  if (nfb + npb > 0) {
    ProfScope prof(K_DT_BIN, stream);
    hipLaunchKernelGGL(kd_dt_bin<T>, dim3((unsigned)(nfb + npb), B), dim3(kBlock), 0, stream, F,
                       N, G, fvi, bbox, cursor, lists, bbox ? nullptr : boxes, nfb, P, px, pcnt,
                       hcnt);
  }
  DtArgs<T> a{B,   P,      F,     N,      K,       D,        C,       G,
              eps, px,     range, fvz,    fvi,     feat,     cursor,  lists,
              bbox ? bbox : boxes, interp, face_idx, weights, bbox, depth, w0, w1,
              debug_flags(), debug_tile_buffer(), hcnt, hits, hint, ovf, novf};
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void *)kd_dt_fwd<T>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (cellwalk) {
    {
      ProfScope prof(K_DT_SORT, stream);
      hipLaunchKernelGGL(kd_dt_pscan, dim3(1), dim3(1024), 0, stream, (int)(B * cells), pcnt,
                         cursor, poff, items, nitems);
      hipLaunchKernelGGL(kd_dt_pscatter<T>, dim3((unsigned)npb, B), dim3(kBlock), 0, stream, P,
                         G, px, poff, pfill, spix);
    }
    switch (DI) {
      case 0: dt_cell_launch<T, 0>(a, pcnt, poff, spix, items, nitems, stream); break;
      case 1: dt_cell_launch<T, 1>(a, pcnt, poff, spix, items, nitems, stream); break;
      case 2: dt_cell_launch<T, 2>(a, pcnt, poff, spix, items, nitems, stream); break;
      case 3: dt_cell_launch<T, 3>(a, pcnt, poff, spix, items, nitems, stream); break;
      default: dt_cell_launch<T, 4>(a, pcnt, poff, spix, items, nitems, stream); break;
    }
    // the deferred pixels (grid-stride over the list kd_dt_out left: ovf without hits)
    DtArgs<T> af = a;
    af.hcnt = nullptr;
    af.hits = nullptr;
    ProfScope prof(K_DT_FWD, stream);
    hipLaunchKernelGGL(kd_dt_fwd<T>, dim3((unsigned)(device_cus(stream) * 4)),
                       dim3(kWave * kDtWaves), lds, stream, af);
  } else {
    const int64_t gx = (P + kDtWaves - 1) / kDtWaves;
    KD_CHECK_ARG(gx < (1ll << 31), "deftet: too many pixels");
    DtArgs<T> ap = a;  // every pixel walks its list
    ap.ovf = nullptr;
    ProfScope prof(K_DT_FWD, stream);
    hipLaunchKernelGGL(kd_dt_fwd<T>, dim3((unsigned)gx, B), dim3(kWave * kDtWaves), lds, stream,
                       ap);
  }
  e = hipGetLastError();
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

size_t kd_deftet_workspace_size(int B, int64_t P, int64_t F, int D, int double_precision) {
  if (B < 0 || P < 0 || F < 0 || D < 0) return 0;
  return dt_workspace(B, P, F, D, double_precision ? sizeof(double) : sizeof(float));
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
int kd_deftet_sparse_render_forward_raw_f32(int B, int64_t P, int64_t F, int knum,
                                            const float *fvz, const float *fvi,
                                            const float *face_bboxes, const float *pixel_coords,
                                            const float *render_ranges, float eps,
                                            int64_t *face_idx, float *pixel_depths, float *w0,
                                            float *w1, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(face_idx && pixel_depths && w0 && w1, "deftet: NULL output");
  return dt_forward<float>(B, P, F, knum, 0, pixel_coords, render_ranges, fvz, fvi, nullptr, eps,
                           nullptr, face_idx, nullptr, ws, wsb, (hipStream_t)stream, face_bboxes,
                           pixel_depths, w0, w1);
}
int kd_deftet_sparse_render_forward_raw_f64(int B, int64_t P, int64_t F, int knum,
                                            const double *fvz, const double *fvi,
                                            const double *face_bboxes,
                                            const double *pixel_coords,
                                            const double *render_ranges, float eps,
                                            int64_t *face_idx, double *pixel_depths, double *w0,
                                            double *w1, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(face_idx && pixel_depths && w0 && w1, "deftet: NULL output");
  return dt_forward<double>(B, P, F, knum, 0, pixel_coords, render_ranges, fvz, fvi, nullptr,
                            eps, nullptr, face_idx, nullptr, ws, wsb, (hipStream_t)stream,
                            face_bboxes, pixel_depths, w0, w1);
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
