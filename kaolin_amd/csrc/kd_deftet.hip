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
//   kd_dt_bwd     the rasterize backward's per-sample math (deftet_cuda.cu:238-402 ==
//                 rasterization_cuda.cu:238-402, kd_raster_bwd.hpp) over the (pixel, slot)
//                 samples that hold a face: a workgroup takes kDtBwdSpan consecutive samples,
//                 compacts the occupied ones into LDS (most slots are empty) and sums their terms
//                 per face 256 at a time (raster_bwd_group), one atomic per (group, face, term).
// The eps of the box-normalisation is the reference's float parameter (copysignf of it), also for
// fp64 data.
#include "kd_capi.hpp"
#include "kd_common.hpp"
#include "kd_raster.hpp"
#include "kd_raster_bwd.hpp"
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

// The reference's per-face test (deftet_cuda.cu:114-160): half-open box of the corner min / max
// (or the caller's face_bboxes), eps-normalised barycentrics (copysignf of the float eps, also for
// fp64 data), all >= 0, depth in [min, max).  (Reading kd_dt_bin's box table and the depths for
// every candidate instead measured 192 -> 198 us: more bytes per candidate than the min / max.)
template <typename T>
__device__ __forceinline__ bool dt_face_test(const T *v, const T *z, const T *box, T x0, T y0,
                                             T dmin, T dmax, T eps, T &w0, T &w1, T &depth) {
  const T ax = v[0], ay = v[1], bx = v[2], by = v[3], cx = v[4], cy = v[5];
  T xmin, xmax, ymin, ymax;
  if (box) {
    xmin = box[0];
    ymin = box[1];
    xmax = box[2];
    ymax = box[3];
  } else {
    // listed faces have no NaN corner (kd_dt_bin drops NaN boxes), so the plain min / max equal
    // the NaN-propagating ones here (and +-0 compare equal): v_min3 / v_max3, no branches
    xmin = fmin(fmin(ax, bx), cx);
    xmax = fmax(fmax(ax, bx), cx);
    ymin = fmin(fmin(ay, by), cy);
    ymax = fmax(fmax(ay, by), cy);
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

constexpr int kDtWaves = 1;  // pixels per workgroup: one wave (finer dispatch of uneven pixels)

template <typename T>
__host__ __device__ constexpr size_t dt_wave_lds(int C) {  // depth, w0, w1, face, face rank
  return (size_t)C * (3 * sizeof(T) + 2 * sizeof(int));
}

// The pixel's outputs when its hits fit the wave without the first-K cut (nh <= 64, and nh <= K
// unless op form).  Lanes form (hit i, group g) pairs: NI >= nh lanes a group, G = 64 / NI
// groups; lane (i, g) compares hit i with hits j = g, g + G, ... and the groups' counts are summed
// by lane shuffles, so a rank costs nh / G comparisons instead of nh.  The same comparisons as the
// LDS form below (bit-identical outputs).
template <typename T>
__device__ __forceinline__ void dt_pixel_out_wave(const DtArgs<T> &a, int b, int64_t row, int nh,
                                                  const T *dep, const T *lw0, const T *lw1,
                                                  const int *fid) {
  const int lane = threadIdx.x & 63;
  const int K = a.K;
  const int lg = nh <= 1 ? 0 : 32 - __builtin_clz((unsigned)(nh - 1));  // NI = 2^lg >= nh
  const int NI = 1 << lg, G = kWave >> lg;
  const int i = lane & (NI - 1), g = lane >> lg;
  const bool has = i < nh;
  T di = (T)0;
  int fi = INT_MAX;
  if (has) {
    di = dep[i];
    fi = fid[i];
  }
  int r = 0;
  if (a.depth) {  // op form: slot = face rank among the hits (deftet_cuda.cu:166-180)
    if (has) {
#pragma unroll 4
      for (int j = g; j < nh; j += G) r += fid[j] < fi ? 1 : 0;
    }
  } else {  // depth descending, then face index (deftet.py:300-303, stable order)
    if (has) {
#pragma unroll 4
      for (int j = g; j < nh; j += G) {
        const T dj = dep[j];
        r += (dj > di || (dj == di && fid[j] < fi)) ? 1 : 0;
      }
    }
  }
  for (int s = NI; s < kWave; s <<= 1) r += __shfl_xor(r, s);
  const bool st = has && g == 0;
  const int n = min(nh, K);
  if (a.depth) {  // unsorted; the empty slots keep -1 / -inf / 0 / 0 (deftet.cpp:88-94)
    if (st && r < K) {
      a.face_idx[row + r] = fi;
      a.depth[row + r] = di;
      a.w0[row + r] = lw0[i];
      a.w1[row + r] = lw1[i];
    }
    for (int s = n + lane; s < K; s += kWave) {
      a.face_idx[row + s] = -1;
      a.depth[row + s] = (T)-INFINITY;
      a.w0[row + s] = (T)0;
      a.w1[row + s] = (T)0;
    }
    return;
  }
  const int D = a.D;
  if (st) {
    const T *feat = a.feat + (int64_t)b * a.F * 3 * D;
    const T w0 = lw0[i], w1 = lw1[i];
    const T w2 = (T)1 - (w0 + w1);  // deftet.py:304
    const int64_t o = row + r;
    a.face_idx[o] = fi;
    store3(a.weights + 3 * o, w0, w1, w2);
    const T *cf = feat + (int64_t)fi * 3 * D;
    T *out = a.interp + o * D;
    if (D == 2) {  // (uv features: one 8-byte store)
      store2(out, w0 * cf[0] + w1 * cf[2] + w2 * cf[4], w0 * cf[1] + w1 * cf[3] + w2 * cf[5]);
    } else {
      for (int d = 0; d < D; ++d)  // :312-313, the sum over the 3 corners in order
        out[d] = w0 * cf[d] + w1 * cf[D + d] + w2 * cf[2 * D + d];
    }
  }
  for (int s = n + lane; s < K; s += kWave) {
    const int64_t o = row + s;
    a.face_idx[o] = -1;
    store3(a.weights + 3 * o, (T)0, (T)0, (T)0);
    if (D == 2)
      store2(a.interp + o * 2, (T)0, (T)0);
    else
      for (int d = 0; d < D; ++d) a.interp[o * D + d] = (T)0;
  }
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
    int fn = lane < nl ? list[lane] : 0;  // the next step's list entry, loaded a step ahead
    for (int j0 = 0; j0 < nl; j0 += kWave) {
      const int j = j0 + lane;
      bool hit = false;
      T w0 = 0, w1 = 0, depth = 0;
      int f = 0;
      const int fc = fn;
      if (j + kWave < nl) fn = list[j + kWave];
      if (j < nl) {
        f = fc;
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
  const int64_t row = pp * K;
  if (nh <= kWave && (a.depth || nh <= K) && !ablate(a.dbg, 1 << 26)) {
    dt_pixel_out_wave<T>(a, b, row, nh, dep, lw0, lw1, fid);
    return;
  }
  // the reference keeps the first K hits by face index: mark the others (face rank >= K)
  int *frank = fid + C;
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
    store3(a.weights + 3 * o, w0, w1, w2);
    const T *cf = feat + (int64_t)fi * 3 * D;
    T *out = a.interp + o * D;
    if (D == 2) {  // (uv features: one 8-byte store)
      store2(out, w0 * cf[0] + w1 * cf[2] + w2 * cf[4], w0 * cf[1] + w1 * cf[3] + w2 * cf[5]);
    } else {
      for (int d = 0; d < D; ++d)  // :312-313, the sum over the 3 corners in order
        out[d] = w0 * cf[d] + w1 * cf[D + d] + w2 * cf[2 * D + d];
    }
  }
  for (int s = n + lane; s < K; s += kWave) {
    const int64_t o = row + s;
    a.face_idx[o] = -1;
    store3(a.weights + 3 * o, (T)0, (T)0, (T)0);
    if (D == 2)
      store2(a.interp + o * 2, (T)0, (T)0);
    else
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

// Workspace: [cursor | cell_cnt] (one memset), the cell lists, the face boxes.
static size_t dt_workspace(int B, int64_t F, size_t esize) {
  const int64_t N = (int64_t)B * F;
  const int G = dt_grid(N);
  const int64_t cells = (int64_t)G * G;
  size_t n = align_up(2 * sizeof(int) * (size_t)B * cells) +
             align_up(sizeof(int) * (size_t)cells * (size_t)(N > 0 ? N : 1)) +
             align_up(4 * esize * (size_t)N);  // the face boxes
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
  w += align_up(2 * sizeof(int) * (size_t)B * cells);
  int *lists = (int *)w;
  w += align_up(sizeof(int) * cells * (size_t)(N > 0 ? N : 1));
  T *boxes = (T *)w;
  w += align_up(4 * sizeof(T) * (size_t)N);
  hipError_t e = zero_words(cursor, 2 * sizeof(int) * (size_t)B * cells, stream);
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
  {
    const int64_t gx = (P + kDtWaves - 1) / kDtWaves;
    KD_CHECK_ARG(gx < (1ll << 31), "deftet: too many pixels");
    ProfScope prof(K_DT_FWD, stream);
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void *)kd_dt_fwd<T>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kd_dt_fwd<T>, dim3((unsigned)gx, B), dim3(kWave * kDtWaves), lds, stream, a);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "deftet fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

constexpr int kDtBwdSpan = 512;  // samples per workgroup: 2 per lane

template <typename T, int DMAX>
__global__ __launch_bounds__(kBlock) void kd_dt_bwd(RasterBwdArgs<T> ra) {
  constexpr int PER = kDtBwdSpan / kBlock;
  __shared__ short s_hit[kDtBwdSpan];
  __shared__ int s_scan[4];
  const int64_t PK = (int64_t)ra.H * ra.W;
  const int64_t total = ra.B * PK;
  const int tid = threadIdx.x;
  // XCD-aware as the raster tiles: XCD x gets a contiguous band of groups (neighbouring pixels
  // share faces)
  int d = blockIdx.x;
  const int n = gridDim.x;
  if ((n & 7) == 0) d = (d & 7) * (n >> 3) + (d >> 3);
  const int64_t e0 = (int64_t)d * kDtBwdSpan;
  // occupied samples of the span, in sample order
  bool hit[PER];
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int64_t e = e0 + tid * PER + i;
    const int64_t f = e < total ? ra.face_idx[e] : -1;
    hit[i] = f >= 0 && f < ra.F;
    cnt += hit[i];
  }
  int nh;
  int o = wg_exclusive_scan(cnt, s_scan, nh);
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (hit[i]) s_hit[o++] = (short)(tid * PER + i);
  __syncthreads();
  if (ablate(ra.dbg, 1 << 27)) return;
  for (int base = 0; base < nh; base += kBlock) {
    if (base) __syncthreads();  // the previous group is done with the LDS table
    int64_t p = -1;
    int b = 0;
    if (base + tid < nh) {
      p = e0 + s_hit[base + tid];
      b = ra.B == 1 ? 0 : (int)(p / PK);
    }
    raster_bwd_group<T, DMAX, false, true>(ra, p, b);
  }
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
  const int64_t total = (int64_t)B * P * K;
  if (D > 8 || nf >= (1ll << 31) || (debug_flags() & (1 << 25)))
    // (pixel, slot) samples as a P x K image (one atomic per sample and term past 8 features)
    return raster_backward_launch<T>(B, (int)P, K, F, D, grad, face_idx, weights, fvi, feat, eps,
                                     gfvi, gfeat, stream);
  const int64_t nblk = (total + kDtBwdSpan - 1) / kDtBwdSpan;
  KD_CHECK_ARG(nblk < (1ll << 31), "deftet: too many samples");
  const RasterBwdArgs<T> ra{B,       (int)P, K,   F,    D,     grad, face_idx,
                            weights, fvi,    feat, eps, gfvi, gfeat, debug_flags()};
  {
    ProfScope prof(K_DT_BWD, stream);
    if (D <= 3)
      hipLaunchKernelGGL((kd_dt_bwd<T, 3>), dim3((unsigned)nblk), dim3(kBlock), 0, stream, ra);
    else if (D <= 4)
      hipLaunchKernelGGL((kd_dt_bwd<T, 4>), dim3((unsigned)nblk), dim3(kBlock), 0, stream, ra);
    else
      hipLaunchKernelGGL((kd_dt_bwd<T, 8>), dim3((unsigned)nblk), dim3(kBlock), 0, stream, ra);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "deftet bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

extern "C" {

size_t kd_deftet_workspace_size(int B, int64_t F, int double_precision) {
  if (B < 0 || F < 0) return 0;
  return dt_workspace(B, F, double_precision ? sizeof(double) : sizeof(float));
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
