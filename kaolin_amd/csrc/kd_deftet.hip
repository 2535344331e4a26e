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

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_dt_bin(int64_t F, int64_t N, int G, const T *fvi,
                                                    const T *bbox, int *cursor, int *lists,
                                                    T *boxes) {
  __shared__ int s_cnt[kDtGridMax * kDtGridMax];
  const int b = blockIdx.y, cells = G * G;
  const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (int i = threadIdx.x; i < cells; i += kBlock) s_cnt[i] = 0;
  __syncthreads();
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
};

constexpr int kDtWaves = 4;  // pixels per workgroup

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
  const int G = a.G;
  const int c = dt_cell(y0, G) * G + dt_cell(x0, G);
  const int nl = a.cursor[(int64_t)b * G * G + c];
  const int *list = a.lists + (int64_t)c * a.N + (int64_t)b * a.F;
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
  const int64_t p = (int64_t)blockIdx.x * kDtWaves + w;
  if (p >= a.P) return;  // whole wave
  dt_pixel_wave<T>(a, blockIdx.y, p, dt_lds + (size_t)w * dt_wave_lds<T>(a.C));
}

// Pooled forward (knum <= kDtMaxK): one wave (its own workgroup) takes 16 consecutive pixels.
//   walk      the pixels' cell lists, four pixels at a time (four independent list -> box load
//             chains in flight), with the box test only (one 16-byte box per lane); the faces
//             whose half-open box holds the pixel go to the wave's LDS candidate ring, tagged with
//             the pixel (~25 per pixel on the bench's sphere: the boxes of its thin triangles are
//             large next to the ~2 hits)
//   test      whenever the ring holds 64 candidates, the reference's exact test (eps-normalised
//             divisions, depth range) runs on them with every lane busy -- the per-pixel walk ran
//             its divisions for every 64-face step with ~3% of the lanes inside a box; hits go to
//             the wave's hit pool
//   rank      face rank within the pixel (the reference keeps the first knum hits by face index),
//             then depth rank (descending, ties by face index) -> slot table
//   store     the group's outputs are one contiguous run per array: written in memory order
// Walk, test, rank and store run per group of four pixels, so the hit pool holds four pixels'
// hits (~5.5 per pixel at the bench row, more at poles) and the ranking loops stay short.
// A pixel with a hit beyond the pool is redone by the per-pixel wave path (dt_pixel_wave, with its
// bisection for any number of hits), in LDS the pool no longer uses.  Candidate order is
// irrelevant: selection and output order depend on face index and depth only.
constexpr int kDtPx = 4;       // pixels per wave (= workgroup)
constexpr int kDtRing = 512;   // candidate ring (< 64 + 4 x 64 entries live)
constexpr int kDtHits = 256;   // hit pool per wave
constexpr int kDtMaxK = 32;    // knum bound of the pooled path (slot table)
constexpr int kDtMaxD = 4;     // feature bound of the pooled path (interpolated-feature table)

template <typename T>
struct DtPoolLDS {
  struct Work {
    int cface[kDtRing];      // candidates: face, pixel
    uint8_t cpix[kDtRing];
    int hface[kDtHits];      // hits: face, depth, w0, w1, pixel, face rank within the pixel
    T hdep[kDtHits], hw0[kDtHits], hw1[kDtHits];
    uint8_t hpix[kDtHits];
    short hrank[kDtHits];
  };
  union {
    Work w;
    char fb[dt_wave_lds<T>(256)];  // the per-pixel fallback's lists (C = 256)
  } u;
  T x[kDtPx], y[kDtPx], dmin[kDtPx], dmax[kDtPx];
  int64_t lofs[kDtPx];
  int nl[kDtPx], nh[kDtPx];
  short slot[4][kDtMaxK];  // the current group of four pixels
  T ival[4][kDtMaxK][kDtMaxD];  // its interpolated features
  unsigned ovf;  // pixels whose hits did not all fit the pool
};

template <typename T>
__device__ __forceinline__ void dt_load_box(const T *boxes, int64_t i, T bx[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 q = *(const float4 *)(boxes + i * 4);
    bx[0] = q.x;
    bx[1] = q.y;
    bx[2] = q.z;
    bx[3] = q.w;
  } else {
    const double2 q0 = *(const double2 *)(boxes + i * 4);
    const double2 q1 = *(const double2 *)(boxes + i * 4 + 2);
    bx[0] = q0.x;
    bx[1] = q0.y;
    bx[2] = q1.x;
    bx[3] = q1.y;
  }
}

// e / d for the store loops' small operands (e < 2^12, d < 2^10): (e + 0.5) / d is at least
// 0.5 / d from an integer, far beyond the float product's error
__device__ __forceinline__ int small_div(int e, float inv_d) {
  return (int)(((float)e + 0.5f) * inv_d);
}

// lane j's value to every lane (j wave-uniform)
__device__ __forceinline__ float lane_bcast(float x, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
}
__device__ __forceinline__ double lane_bcast(double x, int j) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), j),
                          __builtin_amdgcn_readlane(__double2loint(x), j));
}

__device__ __forceinline__ int lane_rank(uint64_t m) {  // set lanes of m below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <typename T>
__global__ __launch_bounds__(kWave) void kd_dt_fwd_pool(DtArgs<T> a) {
  __shared__ DtPoolLDS<T> s;
  typename DtPoolLDS<T>::Work &wk = s.u.w;
  const int lane = threadIdx.x;
  // diagnostics (flag 64): duration, start, and the ends of the walk / rank / store phases
  TileClock clk(a.tbuf, 0);
  clk.start_to(1);
  auto stamp = [&](int slot) {
    if (KD_DIAG && a.tbuf && lane == 0)
      a.tbuf[(int64_t)slot * gridDim.x * gridDim.y + (int64_t)blockIdx.y * gridDim.x +
             blockIdx.x] = wall_clock64();
  };
  const int b = blockIdx.y, K = a.K, G = a.G;
  const int64_t p0 = (int64_t)blockIdx.x * kDtPx;
  const int npx = (int)min((int64_t)kDtPx, a.P - p0);
  if (lane < kDtPx) {
    int n = 0;
    int64_t lofs = 0;
    if (lane < npx) {
      const int64_t pp = (int64_t)b * a.P + p0 + lane;
      const T x0 = a.px[2 * pp], y0 = a.px[2 * pp + 1];
      s.x[lane] = x0;
      s.y[lane] = y0;
      s.dmin[lane] = a.range[2 * pp];
      s.dmax[lane] = a.range[2 * pp + 1];
      const int c = dt_cell(y0, G) * G + dt_cell(x0, G);
      n = a.cursor[(int64_t)b * G * G + c];
      lofs = (int64_t)c * a.N + (int64_t)b * a.F;
    }
    s.nl[lane] = n;
    s.lofs[lane] = lofs;
    s.nh[lane] = 0;
  }
  if (lane == 0) s.ovf = 0;
  wave_lds_sync();
  const T *boxes = a.boxes + (int64_t)b * a.F * 4;
  const T *fvi = a.fvi + (int64_t)b * a.F * 6;
  const T *fvz = a.fvz + (int64_t)b * a.F * 3;
  const T *bbox = a.bbox ? a.bbox + (int64_t)b * a.F * 4 : nullptr;
  const T eps = (T)a.eps;
  int head = 0, tail = 0, nhit = 0;  // wave-uniform
  // the exact test on ring entries [head, head + m)
  auto flush = [&](int m) {
    const int idx = (head + lane) & (kDtRing - 1);
    bool hit = false;
    int q = 0, f = 0;
    T w0 = 0, w1 = 0, depth = 0;
    if (lane < m && !ablate(a.dbg, 1)) {  // (diagnostics: 1 = no exact tests)
      q = wk.cpix[idx];
      f = wk.cface[idx];
      hit = dt_face_test<T>(fvi + (int64_t)f * 6, fvz + (int64_t)f * 3,
                            bbox ? bbox + (int64_t)f * 4 : nullptr, s.x[q], s.y[q], s.dmin[q],
                            s.dmax[q], eps, w0, w1, depth);
      if (ablate(a.dbg, 4) && hit) hit = depth == (T)12345;  // diagnostics: tests, no hits
    }
    const uint64_t hm = __ballot(hit);
    if (hit) {
      const int at = nhit + lane_rank(hm);
      if (at < kDtHits) {
        wk.hface[at] = f;
        wk.hdep[at] = depth;
        wk.hw0[at] = w0;
        wk.hw1[at] = w1;
        wk.hpix[at] = (uint8_t)q;
      }
    }
    // per-pixel hit counts and pool overflow by ballots (LDS atomics are priced per lane)
    const uint64_t hov = __ballot(hit && nhit + lane_rank(hm) >= kDtHits);
#pragma unroll
    for (int u = 0; u < kDtPx; ++u) {
      const uint64_t mu = __ballot(hit && q == u);
      if (lane == 0 && mu) {
        s.nh[u] += __popcll(mu & ~hov);
        if (mu & hov) s.ovf |= 1u << u;
      }
    }
    nhit += __popcll(hm);
    head += m;
    wave_lds_sync();
  };
  constexpr int U = 4;
  const int D = a.D;
  const T *feat = a.feat ? a.feat + (int64_t)b * a.F * 3 * D : nullptr;
  for (int g = 0; g < kDtPx / U; ++g) {
    const int qg = g * U;
    if (qg >= npx) break;  // wave-uniform
    int n[U], steps = 0;
    int64_t lofs[U];
    T x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = qg + u;
      n[u] = s.nl[q];
      lofs[u] = s.lofs[q];
      x[u] = s.x[q];
      y[u] = s.y[q];
      steps = max(steps, (n[u] + kWave - 1) / kWave);
    }
    for (int t = 0; t < steps; ++t) {
      const int j = t * kWave + lane;
      int f[U];
#pragma unroll
      for (int u = 0; u < U; ++u) f[u] = j < n[u] ? a.lists[lofs[u] + j] : -1;
      if (ablate(a.dbg, 2)) continue;  // diagnostics: list loads only
      T bx[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (f[u] >= 0) dt_load_box<T>(boxes, f[u], bx[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // the reference's half-open box test (deftet_cuda.cu:124-127)
        const bool in = f[u] >= 0 && x[u] >= bx[u][0] && x[u] < bx[u][2] && y[u] >= bx[u][1] &&
                        y[u] < bx[u][3];
        const uint64_t m = __ballot(in);
        if (in) {
          const int at = (tail + lane_rank(m)) & (kDtRing - 1);
          wk.cface[at] = f[u];
          wk.cpix[at] = (uint8_t)(qg + u);
        }
        tail += __popcll(m);
      }
      wave_lds_sync();
      while (tail - head >= kWave) flush(kWave);
    }
    if (tail > head) flush(tail - head);
    stamp(2);
    // ranks within each pixel of the group: lane = hit i, the other hits j broadcast from
    // registers a block of 64 at a time (readlane, no LDS round trip per j)
    const int nk = min(nhit, kDtHits);
    const unsigned ovf = s.ovf;
    bool need_frank = a.depth != nullptr;  // the face rank: for a cut and the op form's slots
    for (int u = 0; u < U; ++u) need_frank |= s.nh[qg + u] > K;
    for (int i0 = 0; i0 < nk; i0 += kWave) {
      const int i = i0 + lane;
      const int qi = i < nk ? wk.hpix[i] : 255, fi = i < nk ? wk.hface[i] : 0;
      int r = 0;
      if (need_frank)
        for (int j0 = 0; j0 < nk; j0 += kWave) {
          const int jl = j0 + lane;
          const int qj = jl < nk ? wk.hpix[jl] : 254, fj = jl < nk ? wk.hface[jl] : 0;
          const int m = min(kWave, nk - j0);
          for (int jj = 0; jj < m; ++jj)
            r += (__builtin_amdgcn_readlane(qj, jj) == qi &&
                  __builtin_amdgcn_readlane(fj, jj) < fi)
                     ? 1
                     : 0;
        }
      if (i < nk) wk.hrank[i] = (short)r;
    }
    wave_lds_sync();
    for (int i0 = 0; i0 < nk; i0 += kWave) {
      const int i = i0 + lane;
      const bool vi = i < nk;
      const int qi = vi ? wk.hpix[i] : 255, fi = vi ? wk.hface[i] : 0;
      const int ri = vi ? wk.hrank[i] : K;
      const T di = vi ? wk.hdep[i] : (T)0;
      int r = ri;  // op form: slot = face rank (deftet_cuda.cu:166-180), unsorted
      if (!a.depth) {  // depth descending, then face index (deftet.py:300-303, stable order)
        r = 0;
        for (int j0 = 0; j0 < nk; j0 += kWave) {
          const int jl = j0 + lane;
          const bool vj = jl < nk;
          // pixel, or 254 when not kept (face rank >= K)
          const int qj = vj && wk.hrank[jl] < K ? wk.hpix[jl] : 254;
          const int fj = vj ? wk.hface[jl] : 0;
          const T dj = vj ? wk.hdep[jl] : (T)0;
          const int m = min(kWave, nk - j0);
          for (int jj = 0; jj < m; ++jj) {
            const T db = lane_bcast(dj, jj);
            r += (__builtin_amdgcn_readlane(qj, jj) == qi &&
                  (db > di || (db == di && __builtin_amdgcn_readlane(fj, jj) < fi)))
                     ? 1
                     : 0;
          }
        }
      }
      if (vi && ri < K && !((ovf >> qi) & 1) && !ablate(a.dbg, 512))
        s.slot[qi - qg][r] = (short)i;
    }
    wave_lds_sync();
    stamp(3);
    // stores: the group's rows are one contiguous run per array.  First the interpolated
    // features into LDS (their gathers are the only global loads; a load issued after a store
    // would wait for that store too: vmcnt counts both), then every output in memory order,
    // consecutive lanes on consecutive elements.
    const int ng = min(U, npx - qg);
    const int64_t row0 = ((int64_t)b * a.P + p0 + qg) * K;
    auto slot_hit = [&](int qq, int sl) {  // -2: redone by the fallback, -1: empty slot
      const int q = qg + qq;
      if (((ovf >> q) & 1) && !ablate(a.dbg, 1 << 15)) return -2;
      const int kept = ablate(a.dbg, 512) || ((ovf >> q) & 1) ? 0 : min(s.nh[q], K);
      return sl < kept ? (int)s.slot[qq][sl] : -1;
    };
    const float invK = 1.f / (float)K;
    if (a.depth) {  // op form: empty slots -1 / -inf / 0 / 0 (deftet.cpp:88-94)
      for (int e = lane; e < ng * K; e += kWave) {
        const int qq = small_div(e, invK), h = slot_hit(qq, e - qq * K);
        if (h == -2) continue;
        const int64_t o = row0 + e;
        a.face_idx[o] = h >= 0 ? (int64_t)wk.hface[h] : -1;
        a.depth[o] = h >= 0 ? wk.hdep[h] : (T)-INFINITY;
        a.w0[o] = h >= 0 ? wk.hw0[h] : (T)0;
        a.w1[o] = h >= 0 ? wk.hw1[h] : (T)0;
      }
    } else {
      const int KD = K * D;
      const float invKD = 1.f / (float)KD, invD = 1.f / (float)max(D, 1), invK3 = 1.f / (3.f * K);
      for (int e = lane; e < ng * KD; e += kWave) {
        const int qq = small_div(e, invKD), rem = e - qq * KD, sl = small_div(rem, invD),
                  d = rem - sl * D;
        const int h = slot_hit(qq, sl);
        if (h < 0) continue;
        const T w0 = wk.hw0[h], w1 = wk.hw1[h];
        const T w2 = (T)1 - (w0 + w1);  // deftet.py:304
        const T *cf = feat + (int64_t)wk.hface[h] * 3 * D;
        // :312-313, the sum over the 3 corners in order
        s.ival[qq][sl][d] = w0 * cf[d] + w1 * cf[D + d] + w2 * cf[2 * D + d];
      }
      wave_lds_sync();
      for (int e = lane; e < ng * K; e += kWave) {
        const int qq = small_div(e, invK), h = slot_hit(qq, e - qq * K);
        if (h != -2) a.face_idx[row0 + e] = h >= 0 ? (int64_t)wk.hface[h] : -1;
      }
      for (int e = lane; e < ng * K * 3; e += kWave) {
        const int qq = small_div(e, invK3), rem = e - qq * 3 * K, sl = small_div(rem, 1.f / 3.f),
                  c = rem - sl * 3;
        const int h = slot_hit(qq, sl);
        if (h == -2) continue;
        T v = (T)0;
        if (h >= 0) {
          const T w0 = wk.hw0[h], w1 = wk.hw1[h];
          v = c == 0 ? w0 : c == 1 ? w1 : (T)1 - (w0 + w1);
        }
        a.weights[3 * row0 + e] = v;
      }
      for (int e = lane; e < ng * KD; e += kWave) {
        const int qq = small_div(e, invKD), rem = e - qq * KD, sl = small_div(rem, invD),
                  d = rem - sl * D;
        const int h = slot_hit(qq, sl);
        if (h != -2) a.interp[row0 * D + e] = h >= 0 ? s.ival[qq][sl][d] : (T)0;
      }
    }
    stamp(4);
    if (ovf && !ablate(a.dbg, 1 << 15)) {  // wave-uniform (diagnostics: no fallback)
      wave_lds_sync();  // the pool's LDS becomes the fallback's
      for (int u = 0; u < ng; ++u)
        if ((ovf >> (qg + u)) & 1) dt_pixel_wave<T>(a, b, p0 + qg + u, s.u.fb);
      if (lane == 0) s.ovf = 0;
    }
    head = tail = nhit = 0;
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// Cell-major forward (knum <= kDtCellK, debug flag 1024, a workspace with room for the pixel
// sort: kd_deftet_workspace_size_p).  Every pixel of one grid cell walks the same face list, so:
//   kd_dt_pix_count    cell of every pixel, counted per (view, cell) with one atomic per distinct
//                      cell of a wave (ballot groups: neighbouring pixels share cells); the
//                      pixel's position in its cell
//   kd_dt_pix_scan     per view: exclusive scans of the cell counts (pixel offsets) and of their
//                      64-pixel chunks (work items)
//   kd_dt_pix_scatter  pixels in cell order
//   kd_dt_fwd_cell     one wave per work item: lane = pixel (up to 64 of one cell).  The cell's
//                      list is read 64 faces at a time -- lane j loads face j's box, corners and
//                      depths -- and broadcast face by face (readlane): every pixel lane runs the
//                      reference's box test, and the exact test where it is inside.  A round trip
//                      serves 64 pixels instead of one.  Each lane keeps the knum hits with the
//                      smallest face indices in LDS (the reference keeps the first knum by index:
//                      a further hit replaces the largest kept index when it is smaller), ranks
//                      them (depth descending, ties by face index; op form: by face index) and the
//                      wave writes each pixel's rows in turn, lanes across the row.
//   kd_dt_interp       the interpolated features from face_idx / weights (flat, one thread per
//                      (pixel, slot); the gathers would otherwise sit between the stores)
constexpr int kDtCellK = 32;

__host__ __device__ inline int64_t dt_max_items(int64_t P, int G) {
  return (P + kWave - 1) / kWave + (int64_t)G * G;
}

struct DtCellBuf {
  int *cell_cnt;   // [B][G*G]
  int *cell_off;   // [B][G*G]
  int *n_items;    // [B]
  int2 *items;     // [B][max_items] (cell, chunk)
  int2 *pix_cell;  // [B][P] (cell, position in the cell)
  int *sorted;     // [B][P] pixel indices in cell order
  int64_t max_items;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_dt_pix_count(int64_t P, int G, const T *px,
                                                          DtCellBuf cb) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int c = -1;
  if (p < P) {
    const int64_t pp = (int64_t)b * P + p;
    c = dt_cell(px[2 * pp + 1], G) * G + dt_cell(px[2 * pp], G);
  }
  int *cnt = cb.cell_cnt + (int64_t)b * G * G;
  uint64_t todo = __ballot(c >= 0);
  int pos = 0;
  while (todo) {  // wave-uniform: one group of lanes in one cell per pass
    const int leader = __builtin_ctzll(todo);
    const int c0 = __builtin_amdgcn_readlane(c, leader);
    const uint64_t m = __ballot(c == c0);
    int base = 0;
    if (lane == leader) base = atomicAdd(&cnt[c0], __popcll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    if (c == c0) pos = base + lane_rank(m);
    todo &= ~m;
  }
  if (p < P) cb.pix_cell[(int64_t)b * P + p] = make_int2(c, pos);
}

__global__ __launch_bounds__(kBlock) void kd_dt_pix_scan(int G, DtCellBuf cb) {
  __shared__ int s_scan[kBlock / kWave];
  const int b = blockIdx.x, tid = threadIdx.x, cells = G * G;
  const int per = (cells + kBlock - 1) / kBlock;  // 16 (G = 64) or 4 (G = 32)
  const int *cnt = cb.cell_cnt + (int64_t)b * cells;
  int np = 0, nc = 0;
  for (int k = 0; k < per; ++k) {
    const int c = tid * per + k;
    const int n = c < cells ? cnt[c] : 0;
    np += n;
    nc += (n + kWave - 1) / kWave;
  }
  int tot_p, tot_c;
  int op = wg_exclusive_scan(np, s_scan, tot_p);
  int oc = wg_exclusive_scan(nc, s_scan, tot_c);
  int *off = cb.cell_off + (int64_t)b * cells;
  int2 *items = cb.items + (int64_t)b * cb.max_items;
  for (int k = 0; k < per; ++k) {
    const int c = tid * per + k;
    if (c >= cells) break;
    const int n = cnt[c];
    off[c] = op;
    op += n;
    for (int j = 0; j < (n + kWave - 1) / kWave; ++j) items[oc + j] = make_int2(c, j);
    oc += (n + kWave - 1) / kWave;
  }
  if (tid == 0) cb.n_items[b] = tot_c;
}

__global__ __launch_bounds__(kBlock) void kd_dt_pix_scatter(int64_t P, int G, DtCellBuf cb) {
  const int b = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= P) return;
  const int2 cp = cb.pix_cell[(int64_t)b * P + p];
  cb.sorted[(int64_t)b * P + cb.cell_off[(int64_t)b * G * G + cp.x] + cp.y] = (int)p;
}

// LDS of kd_dt_fwd_cell per wave: kept hits [64 pixels][KP] (KP odd: lane = pixel walks a row
// with an odd word stride, conflict-free), face / depth / w0 / w1 and the rank (bytes).
__host__ __device__ inline int dt_cell_kp(int K) { return K | 1; }
template <typename T>
__host__ __device__ inline size_t dt_cell_lds(int K) {
  const int kp = dt_cell_kp(K);
  return (size_t)kWave * kp * (sizeof(int) + 3 * sizeof(T)) + (size_t)kWave * (kp + 3) / 4 * 4 + 16;
}

template <typename T>
__device__ __forceinline__ T bcast(T x, int j) {
  return lane_bcast(x, j);
}

template <typename T>
__global__ __launch_bounds__(kWave) void kd_dt_fwd_cell(DtArgs<T> a, DtCellBuf cb) {
  extern __shared__ __align__(16) char dc_lds[];
  const int lane = threadIdx.x, b = blockIdx.y, K = a.K, KP = dt_cell_kp(K), G = a.G;
  TileClock clk(a.tbuf, 0);  // diagnostics (flag 64): duration, start, list length
  clk.start_to(1);
  if ((int)blockIdx.x >= cb.n_items[b]) return;  // wave-uniform
  T *hd = (T *)dc_lds;  // [64][KP] each
  T *h0 = hd + kWave * KP, *h1 = h0 + kWave * KP;
  int *hf = (int *)(h1 + kWave * KP);
  uint8_t *rk = (uint8_t *)(hf + kWave * KP);
  const int RB = (KP + 3) / 4 * 4;  // rank row bytes
  const int2 item = cb.items[(int64_t)b * cb.max_items + blockIdx.x];
  const int c = item.x;
  const int ncell = cb.cell_cnt[(int64_t)b * G * G + c];
  const int k = item.y * kWave + lane;
  const bool live = k < ncell;
  int p = 0;
  T x0 = 0, y0 = 0, dmin = 0, dmax = 0;
  if (live) {
    p = cb.sorted[(int64_t)b * a.P + cb.cell_off[(int64_t)b * G * G + c] + k];
    const int64_t pp = (int64_t)b * a.P + p;
    x0 = a.px[2 * pp];
    y0 = a.px[2 * pp + 1];
    dmin = a.range[2 * pp];
    dmax = a.range[2 * pp + 1];
  }
  const int nl = a.cursor[(int64_t)b * G * G + c];
  if (KD_DIAG && a.tbuf && lane == 0) a.tbuf[2 * (int64_t)gridDim.x * gridDim.y + blockIdx.x] = nl;
  const int *list = a.lists + (int64_t)c * a.N + (int64_t)b * a.F;
  const T *boxes = a.boxes + (int64_t)b * a.F * 4;
  const T *fvi = a.fvi + (int64_t)b * a.F * 6;
  const T *fvz = a.fvz + (int64_t)b * a.F * 3;
  const T eps = (T)a.eps;
  int nh = 0, maxf = -1, maxs = 0;  // per lane: kept hits, the largest kept face index and its slot
  T *myd = hd + lane * KP, *my0 = h0 + lane * KP, *my1 = h1 + lane * KP;
  int *myf = hf + lane * KP;
  for (int j0 = 0; j0 < nl; j0 += kWave) {
    const int j = j0 + lane;
    int f = -1;
    T bx[4] = {0, 0, 0, 0}, v[6] = {0, 0, 0, 0, 0, 0}, z[3] = {0, 0, 0};
    if (j < nl) {
      f = list[j];
      dt_load_box<T>(boxes, f, bx);
#pragma unroll
      for (int q = 0; q < 6; ++q) v[q] = fvi[(int64_t)f * 6 + q];
#pragma unroll
      for (int q = 0; q < 3; ++q) z[q] = fvz[(int64_t)f * 3 + q];
    }
    const int m = ablate(a.dbg, 2) ? 0 : min(kWave, nl - j0);  // (diagnostics: no face loop)
    for (int jj = 0; jj < m; ++jj) {
      // the reference's half-open box test (deftet_cuda.cu:124-127)
      const T bx0 = bcast(bx[0], jj), by0 = bcast(bx[1], jj);
      const T bx1 = bcast(bx[2], jj), by1 = bcast(bx[3], jj);
      const bool in = live && x0 >= bx0 && x0 < bx1 && y0 >= by0 && y0 < by1;
      if (!__ballot(in) || ablate(a.dbg, 1)) continue;  // wave-uniform (diag: box tests only)
      const T ax = bcast(v[0], jj), ay = bcast(v[1], jj), bxx = bcast(v[2], jj);
      const T byy = bcast(v[3], jj), cx = bcast(v[4], jj), cy = bcast(v[5], jj);
      const T z0 = bcast(z[0], jj), z1 = bcast(z[1], jj), z2 = bcast(z[2], jj);
      const int fj = __builtin_amdgcn_readlane(f, jj);
      T w0, w1, depth;
      if (in && dt_face_weights<T>(ax, ay, bxx, byy, cx, cy, z0, z1, z2, x0, y0, dmin, dmax, eps,
                                   w0, w1, depth)) {
        int slot = -1;
        if (nh < K) {
          slot = nh++;
          if (fj > maxf) {
            maxf = fj;
            maxs = slot;
          }
        } else if (fj < maxf) {  // keep the K smallest face indices
          slot = maxs;
        }
        if (slot >= 0) {
          myf[slot] = fj;
          myd[slot] = depth;
          my0[slot] = w0;
          my1[slot] = w1;
          if (nh == K && slot == maxs) {  // a replacement: find the new largest index
            maxf = -1;
            for (int e = 0; e < K; ++e)
              if (myf[e] > maxf) {
                maxf = myf[e];
                maxs = e;
              }
          }
        }
      }
    }
  }
  // ranks: sorted form -- depth descending, then face index (deftet.py:300-303, stable order);
  // op form -- face index (the reference kernel's insertion order, deftet_cuda.cu:166-180)
  for (int e = 0; e < nh; ++e) {
    const int fe = myf[e];
    const T de = myd[e];
    int r = 0;
    for (int q = 0; q < nh; ++q) {
      const int fq = myf[q];
      r += (a.depth ? fq < fe : (myd[q] > de || (myd[q] == de && fq < fe))) ? 1 : 0;
    }
    rk[lane * RB + e] = (uint8_t)r;
  }
  wave_lds_sync();
  // rows, pixel by pixel: lanes across the row; entry e goes to slot rank[e], slots >= n are empty
  const uint64_t lv = __ballot(live);
  for (int i = 0; i < kWave; ++i) {
    if (!((lv >> i) & 1)) continue;  // wave-uniform
    const int pi = __builtin_amdgcn_readlane(p, i), ni = __builtin_amdgcn_readlane(nh, i);
    const int64_t row0 = ((int64_t)b * a.P + pi) * K;
    const uint8_t *ri = rk + i * RB;
    if (lane < K) {
      const bool h = lane < ni;
      const int slot = h ? ri[lane] : lane;
      const int64_t o = row0 + slot;
      if (a.depth) {  // op form: empty slots -1 / -inf / 0 / 0 (deftet.cpp:88-94)
        a.face_idx[o] = h ? (int64_t)hf[i * KP + lane] : -1;
        a.depth[o] = h ? hd[i * KP + lane] : (T)-INFINITY;
        a.w0[o] = h ? h0[i * KP + lane] : (T)0;
        a.w1[o] = h ? h1[i * KP + lane] : (T)0;
      } else {
        a.face_idx[o] = h ? (int64_t)hf[i * KP + lane] : -1;
      }
    }
    if (!a.depth)
      for (int t = lane; t < 3 * K; t += kWave) {
        const int e = small_div(t, 1.f / 3.f), cc = t - 3 * e;
        const bool h = e < ni;
        T val = (T)0;
        if (h) {
          const T w0 = h0[i * KP + e], w1 = h1[i * KP + e];
          val = cc == 0 ? w0 : cc == 1 ? w1 : (T)1 - (w0 + w1);  // deftet.py:304
        }
        a.weights[3 * (row0 + (h ? ri[e] : e)) + cc] = val;
      }
  }
}

// interp (B, P, K, D) from face_idx and weights: deftet.py:312-313, the sum over the 3 corners
template <typename T>
__global__ __launch_bounds__(kBlock) void kd_dt_interp(int64_t PK, int64_t F, int D,
                                                       const int64_t *face_idx, const T *weights,
                                                       const T *feat, T *interp, int64_t n) {
  for (int64_t o = (int64_t)blockIdx.x * kBlock + threadIdx.x; o < n;
       o += (int64_t)gridDim.x * kBlock) {
    const int64_t f = face_idx[o];
    T *out = interp + o * D;
    if (f < 0) {
      for (int d = 0; d < D; ++d) out[d] = (T)0;
      continue;
    }
    const T w0 = weights[3 * o], w1 = weights[3 * o + 1], w2 = weights[3 * o + 2];
    const T *cf = feat + ((o / PK) * F + f) * 3 * D;
    for (int d = 0; d < D; ++d) out[d] = w0 * cf[d] + w1 * cf[D + d] + w2 * cf[2 * D + d];
  }
}

// Workspace: [cursor | cell_cnt] (one memset), the cell lists, the face boxes; with P >= 0 also
// the cell-major forward's pixel sort (kd_deftet_workspace_size_p).
static size_t dt_workspace(int B, int64_t F, size_t esize, int64_t P = -1) {
  const int64_t N = (int64_t)B * F;
  const int G = dt_grid(N);
  const int64_t cells = (int64_t)G * G;
  size_t n = align_up(2 * sizeof(int) * (size_t)B * cells) +
             align_up(sizeof(int) * (size_t)cells * (size_t)(N > 0 ? N : 1)) +
             align_up(4 * esize * (size_t)N);  // the face boxes
  if (P >= 0)
    n += align_up(sizeof(int) * (size_t)B * cells) + align_up(sizeof(int) * (size_t)B) +
         align_up(sizeof(int2) * (size_t)B * dt_max_items(P, G)) +
         align_up(sizeof(int2) * (size_t)B * P) + align_up(sizeof(int) * (size_t)B * P);
  return n;
}

static int dt_capacity(int K) { return K < 256 ? 256 : K; }

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
  const size_t need = dt_workspace(B, F, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  if (B == 0 || P == 0) return KD_OK;
  const int64_t N = (int64_t)B * F;
  const int G = dt_grid(N);
  const size_t cells = (size_t)G * G;
  char *w = (char *)ws;
  int *cursor = (int *)w;
  int *cell_cnt = cursor + (size_t)B * cells;
  w += align_up(2 * sizeof(int) * (size_t)B * cells);
  int *lists = (int *)w;
  w += align_up(sizeof(int) * cells * (size_t)(N > 0 ? N : 1));
  T *boxes = (T *)w;
  w += align_up(4 * sizeof(T) * (size_t)N);
  hipError_t e = hipMemsetAsync(cursor, 0, 2 * sizeof(int) * (size_t)B * cells, stream);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "deftet: %s", hipGetErrorString(e));
  if (F > 0) {
    ProfScope prof(K_DT_BIN, stream);
    hipLaunchKernelGGL(kd_dt_bin<T>, dim3((unsigned)((F + kBlock - 1) / kBlock), B),
                       dim3(kBlock), 0, stream, F, N, G, fvi, bbox, cursor, lists,
                       bbox ? nullptr : boxes);
  }
  DtArgs<T> a{B,   P,      F,     N,      K,       D,        C,       G,
              eps, px,     range, fvz,    fvi,     feat,     cursor,  lists,
              bbox ? bbox : boxes, interp, face_idx, weights, bbox, depth, w0, w1,
              debug_flags(), debug_tile_buffer()};
  // kernel choice: the per-pixel waves, unless debug flag 1024 selects the cell-major forward
  // (knum <= 32, a workspace that holds the pixel sort: kd_deftet_workspace_size_p) or 2048 the
  // pooled one -- both bit-identical and measured slower
  const bool cellmajor = K <= kDtCellK && wsb >= dt_workspace(B, F, sizeof(T), P) &&
                         (debug_flags() & 1024) && !(debug_flags() & 2048);
  const bool pooled = K <= kDtMaxK && D <= kDtMaxD && (debug_flags() & 2048);
  if (cellmajor) {
    KD_CHECK_ARG(P < (1ll << 31), "deftet: too many pixels");
    DtCellBuf cb;
    cb.cell_cnt = cell_cnt;
    cb.cell_off = (int *)w;
    w += align_up(sizeof(int) * (size_t)B * cells);
    cb.n_items = (int *)w;
    w += align_up(sizeof(int) * (size_t)B);
    cb.max_items = dt_max_items(P, G);
    cb.items = (int2 *)w;
    w += align_up(sizeof(int2) * (size_t)B * cb.max_items);
    cb.pix_cell = (int2 *)w;
    w += align_up(sizeof(int2) * (size_t)B * P);
    cb.sorted = (int *)w;
    const unsigned pb = (unsigned)((P + kBlock - 1) / kBlock);
    {
      ProfScope prof(K_DT_BIN, stream);
      hipLaunchKernelGGL(kd_dt_pix_count<T>, dim3(pb, B), dim3(kBlock), 0, stream, P, G, px, cb);
      hipLaunchKernelGGL(kd_dt_pix_scan, dim3(B), dim3(kBlock), 0, stream, G, cb);
      hipLaunchKernelGGL(kd_dt_pix_scatter, dim3(pb, B), dim3(kBlock), 0, stream, P, G, cb);
    }
    {
      ProfScope prof(K_DT_FWD, stream);
      const size_t lds = dt_cell_lds<T>(K);
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void *)kd_dt_fwd_cell<T>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kd_dt_fwd_cell<T>, dim3((unsigned)cb.max_items, B), dim3(kWave), lds,
                         stream, a, cb);
      const int64_t n = (int64_t)B * P * K;
      if (!depth && D > 0)
        hipLaunchKernelGGL(kd_dt_interp<T>,
                           dim3((unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 1 << 20)),
                           dim3(kBlock), 0, stream, P * K, F, D, face_idx, weights, feat, interp,
                           n);
    }
  } else {
    const int64_t gx = pooled ? (P + kDtPx - 1) / kDtPx : (P + kDtWaves - 1) / kDtWaves;
    KD_CHECK_ARG(gx < (1ll << 31), "deftet: too many pixels");
    ProfScope prof(K_DT_FWD, stream);
    if (pooled) {
      hipLaunchKernelGGL(kd_dt_fwd_pool<T>, dim3((unsigned)gx, B), dim3(kWave), 0, stream, a);
    } else {
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void *)kd_dt_fwd<T>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kd_dt_fwd<T>, dim3((unsigned)gx, B), dim3(kWave * kDtWaves), lds, stream,
                         a);
    }
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

size_t kd_deftet_workspace_size(int B, int64_t F, int double_precision) {
  if (B < 0 || F < 0) return 0;
  return dt_workspace(B, F, double_precision ? sizeof(double) : sizeof(float));
}
size_t kd_deftet_workspace_size_p(int B, int64_t P, int64_t F, int double_precision) {
  if (B < 0 || F < 0 || P < 0) return 0;
  return dt_workspace(B, F, double_precision ? sizeof(double) : sizeof(float), P);
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
