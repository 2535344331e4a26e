// kd_softmask.hip -- DIB-R soft mask forward / backward for gfx950.
//
// Forward (replaces dibr_soft_mask_forward_cuda_kernel, dibr_soft_mask_cuda.cu:27-184):
//   one 256-thread workgroup per 16x16 pixel tile (one wave per 8x8 sub-tile) walks the ordered
//   coarse bin of ENLARGED boxes (all faces, no culling: dibr.py:201-208), stages the faces
//   touching the tile in LDS, and each wave compacts those touching its sub-tile.  Uncovered
//   pixels are then processed one at a time by the whole wave, lane = candidate face: a ballot
//   of the exact box test gives the hits, their rank (mbcnt) is the slot, so "the first K faces in
//   index order" comes out of one prefix count per 64 faces and the K-list of a pixel is written
//   as contiguous, coalesced stores.  soft = 1 - prod(1 - p) is accumulated in slot order with
//   the reference's double promotion.  With `LISTS` false the close lists are not materialised
//   at all; only close_last (the K-th close face when the list is full) is kept for the backward.
// Backward:
//   kd_soft_bwd_atomic -- general form (any close lists), one thread per pixel, float atomics.
//   kd_soft_bwd_gather -- autograd form: one thread per face walks the uncovered pixels of its
//                         enlarged box, decides membership from close_last, recomputes the
//                         (bit-identical) distance type / probability and sums its own gradient.
#include "../../include/kaolin_dibr.h"
#include "kd_binning.hpp"
#include "kd_capi.hpp"

namespace kd {

#define KD_SOFT_EPS 1e-7  // dibr_soft_mask_cuda.cu:23 (a double literal)

__device__ __forceinline__ float kexp(float x) { return expf(x); }
__device__ __forceinline__ double kexp(double x) { return exp(x); }

// dibr_soft_mask_cuda.cu:100-163: squared distance type (0..5) and probability of one face.
template <typename T>
__device__ __forceinline__ void soft_face_dist(T x0, T y0, const T v[6], float M, float sigmainv,
                                               int &edgeid, T &prob) {
  T pdis[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = (i + 1) % 3;
    const T x1 = v[i * 2], y1 = v[i * 2 + 1], x2 = v[j * 2], y2 = v[j * 2 + 1];
    const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const T up = A * x0 + Bc * y0 + C;
    const T down = A * A + Bc * Bc;
    T x3 = Bc * Bc * x0 - A * Bc * y0 - A * C;
    T y3 = A * A * y0 - A * Bc * x0 - Bc * C;
    x3 = (T)((double)x3 / ((double)down + KD_SOFT_EPS));
    y3 = (T)((double)y3 / ((double)down + KD_SOFT_EPS));
    const T direct = (x3 - x1) * (x3 - x2) + (y3 - y1) * (y3 - y2);
    if (direct > (T)0)
      pdis[i] = (T)(4.0f * M * M);
    else
      pdis[i] = (T)((double)(up * up) / ((double)down + KD_SOFT_EPS));
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T x1 = v[i * 2], y1 = v[i * 2 + 1];
    pdis[i + 3] = (x0 - x1) * (x0 - x1) + (y0 - y1) * (y0 - y1);
  }
  edgeid = 0;
  T d = pdis[0];
#pragma unroll
  for (int i = 1; i < 6; ++i)
    if (d > pdis[i]) {
      d = pdis[i];
      edgeid = i;
    }
  const T z = (T)sigmainv * d / (T)M / (T)M;
  prob = kexp(-z);
}

template <typename T>
struct SoftFwdArgs {
  FaceSet<T> fs;
  BinBuffers bb;
  const int64_t *face_idx;
  int K;
  float sigmainv;
  T *soft;
  T *prob;
  int64_t *cidx;
  uint8_t *ctype;
  int32_t *last;
};

template <typename T>
struct SoftCap {
  static constexpr int value = 512;
};
template <>
struct SoftCap<double> {
  static constexpr int value = 256;
};

template <typename T, bool LISTS>
__global__ __launch_bounds__(kBlock) void kd_soft_fwd(SoftFwdArgs<T> a) {
  constexpr int CAP = SoftCap<T>::value;
  __shared__ int s_f[CAP];
  __shared__ Span s_span[CAP];
  __shared__ T s_geo[10][CAP];  // x0 y0 x1 y1 x2 y2 (scaled corners), xmin ymin xmax ymax
  __shared__ unsigned short s_sub[4][CAP];
  __shared__ int s_cnt[4];

  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const float M = fs.M;
  const int b = blockIdx.y;
  const int ntx = (W + kTile - 1) / kTile;
  const int tx = blockIdx.x % ntx, ty = blockIdx.x / ntx;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);

  const int X0 = tx * kTile, Y0 = ty * kTile;
  const int X1 = min(X0 + kTile - 1, W - 1), Y1 = min(Y0 + kTile - 1, H - 1);
  const int WX0 = X0 + (w & 1) * 8, WY0 = Y0 + (w >> 1) * 8;
  const int WX1 = min(WX0 + 7, W - 1), WY1 = min(WY0 + 7, H - 1);
  const int px = WX0 + (lane & 7), py = WY0 + (lane >> 3);
  const bool inimg = px < W && py < H;
  const bool wave_live = WX0 < W && WY0 < H;
  const T x0 = (T)px_cx(M, W, px);
  const T y0 = (T)px_cy(M, H, py);
  const int64_t p = ((int64_t)b * H + py) * W + px;
  const bool covered = inimg && a.face_idx[p] >= 0;
  const uint64_t umask = __ballot(inimg && !covered);

  int my_kid = 0, my_last = -1;
  T my_prod = (T)1.0;
  bool any_sub = false;

  const BinGeom &g = a.bb.g;
  const int ct = (Y0 / g.ct) * g.nctx + (X0 / g.ct);
  const int n = a.bb.totals[(int64_t)b * g.nct() + ct];
  const int *bin = a.bb.bins + (int64_t)ct * fs.N + lo;

  int cnt = 0;
  for (int base = 0; base < n; base += kBlock) {
    const int e = base + tid;
    int f = 0;
    bool ov = false;
    Span sp;
    if (e < n) {
      f = bin[e];
      sp = a.bb.spans[lo + f];
      ov = span_overlaps(sp, X0, X1, Y0, Y1);
    }
    int tot;
    const int pos = wg_compact(ov, s_cnt, tot);
    if (ov) {
      s_f[cnt + pos] = f;
      s_span[cnt + pos] = sp;
    }
    cnt += tot;
    if (cnt > CAP - kBlock || base + kBlock >= n) {
      __syncthreads();
      for (int k = tid; k < cnt; k += kBlock) {
        const int64_t fi = lo + s_f[k];
        T v[6], box[4];
        load_corners(fs, fi, v);
        face_box(fs, fi, v, box);
#pragma unroll
        for (int q = 0; q < 6; ++q) s_geo[q][k] = v[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) s_geo[6 + q][k] = box[q];
      }
      int nsub = 0;
      for (int k0 = 0; k0 < cnt; k0 += kWave) {
        const int k = k0 + lane;
        const bool ok = wave_live && k < cnt && span_overlaps(s_span[k], WX0, WX1, WY0, WY1);
        const uint64_t m = __ballot(ok);
        if (ok) s_sub[w][nsub + mbcnt(m)] = (unsigned short)k;
        nsub += __popcll(m);
      }
      __syncthreads();
      if (umask && nsub > 0) {
        any_sub = true;
        for (uint64_t mm = umask; mm; mm &= mm - 1) {
          const int q = __builtin_ctzll(mm);
          int kid = rdlane_i(my_kid, q);
          if (kid >= K) continue;
          T prod = rdlane(my_prod, q);
          int last = rdlane_i(my_last, q);
          const T qx = rdlane(x0, q), qy = rdlane(y0, q);
          const int64_t qp = ((int64_t)b * H + WY0 + (q >> 3)) * W + WX0 + (q & 7);
          for (int j0 = 0; j0 < nsub && kid < K; j0 += kWave) {
            const int j = j0 + lane;
            bool hit = false;
            int k = 0;
            if (j < nsub) {
              k = s_sub[w][j];
              hit = !(qx < s_geo[6][k] || qx >= s_geo[8][k] || qy < s_geo[7][k] ||
                      qy >= s_geo[9][k]);  // :95
            }
            const uint64_t hm = __ballot(hit);
            if (!hm) continue;
            const int rank = mbcnt(hm);
            const bool take = hit && rank < K - kid;
            T pr = (T)0;
            int fl = 0;
            if (take) {
              T v[6];
#pragma unroll
              for (int c = 0; c < 6; ++c) v[c] = s_geo[c][k];
              int et;
              soft_face_dist<T>(qx, qy, v, M, a.sigmainv, et, pr);
              fl = s_f[k];
              if (LISTS) {
                const int64_t o = qp * K + kid + rank;
                a.prob[o] = pr;
                a.cidx[o] = fl;
                a.ctype[o] = (uint8_t)(et + 1);
              }
            }
            uint64_t tm = __ballot(take);
            const int ntake = __popcll(tm);
            if (kid + ntake == K) last = rdlane_i(fl, 63 - __builtin_clzll(tm));
            while (tm) {  // :174-178, in slot order
              const int l = __builtin_ctzll(tm);
              prod = (T)((double)prod * (1.0 - (double)rdlane(pr, l)));
              tm &= tm - 1;
            }
            kid += ntake;
          }
          if (lane == q) {
            my_kid = kid;
            my_prod = prod;
            my_last = last;
          }
        }
      }
      __syncthreads();
      cnt = 0;
    }
  }

  if (!wave_live) return;
  if (inimg) {
    a.soft[p] = covered ? (T)1.0 : (T)(1.0 - (double)my_prod);  // :69, :181
    if (a.last) a.last[p] = (my_kid >= K) ? my_last : -1;
  }
  if (!LISTS) return;
  // -1 / 0 / 0 padding of every slot not written above (dibr_soft_mask.cpp:86-97 pre-fill).
  const int nx = WX1 - WX0 + 1;
  if (!any_sub) {
    const int per_row = nx * K;
    for (int r = 0; r <= WY1 - WY0; ++r) {
      const int64_t e0 = (((int64_t)b * H + WY0 + r) * W + WX0) * K;
      for (int e = lane; e < per_row; e += kWave) {
        a.prob[e0 + e] = (T)0;
        a.cidx[e0 + e] = -1;
        a.ctype[e0 + e] = 0;
      }
    }
  } else {
    const uint64_t imask = __ballot(inimg);
    for (uint64_t mm = imask; mm; mm &= mm - 1) {
      const int q = __builtin_ctzll(mm);
      const int kid = rdlane_i(my_kid, q);
      const int64_t e0 = (((int64_t)b * H + WY0 + (q >> 3)) * W + WX0 + (q & 7)) * K;
      for (int s = kid + lane; s < K; s += kWave) {
        a.prob[e0 + s] = (T)0;
        a.cidx[e0 + s] = -1;
        a.ctype[e0 + s] = 0;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward terms of one (pixel, close face) pair, dibr_soft_mask_cuda.cu:281-348; adds to the
// face's 6 corner gradients (already divided by M per term, like the reference).
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void soft_bwd_terms(T x0, T y0, const T v[6], int edgeid, T prob,
                                               T dLdp, T allprob, float sigmainv, float M,
                                               T g[6]) {
  const T dLdz = (T)(-1.0 * (double)sigmainv * (double)dLdp * (1.0 - (double)allprob) /
                     (1.0 - (double)prob + KD_SOFT_EPS) * (double)prob);
  if (edgeid >= 3) {
    const int ps = (edgeid - 3) * 2;
    const T x1 = v[ps], y1 = v[ps + 1];
    const T dLdx1 = dLdz * (T)2 * (x1 - x0);
    const T dLdy1 = dLdz * (T)2 * (y1 - y0);
    g[ps] += dLdx1 / (T)M;
    g[ps + 1] += dLdy1 / (T)M;
  } else {
    const int ps = edgeid * 2, ps2 = ((edgeid + 1) % 3) * 2;
    const T x1 = v[ps], y1 = v[ps + 1], x2 = v[ps2], y2 = v[ps2 + 1];
    const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const T up = A * x0 + Bc * y0 + C;
    const T down = A * A + Bc * Bc;
    const T dissquare = (T)((double)(up * up) / ((double)down + KD_SOFT_EPS));
    const T dzdA = (T)((double)((T)2 * (x0 * up - dissquare * A)) / ((double)down + KD_SOFT_EPS));
    const T dzdB = (T)((double)((T)2 * (y0 * up - dissquare * Bc)) / ((double)down + KD_SOFT_EPS));
    const T dzdC = (T)((double)((T)2 * up) / ((double)down + KD_SOFT_EPS));
    const T dLdx1 = dLdz * (dzdB - y2 * dzdC);
    const T dLdy1 = dLdz * (x2 * dzdC - dzdA);
    const T dLdx2 = dLdz * (y1 * dzdC - dzdB);
    const T dLdy2 = dLdz * (dzdA - x1 * dzdC);
    g[ps] += dLdx1 / (T)M;
    g[ps + 1] += dLdy1 / (T)M;
    g[ps2] += dLdx2 / (T)M;
    g[ps2 + 1] += dLdy2 / (T)M;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_soft_bwd_atomic(
    int B, int H, int W, int64_t F, int K, const T *__restrict__ grad_soft,
    const T *__restrict__ soft, const int64_t *__restrict__ face_idx, const T *__restrict__ prob,
    const int64_t *__restrict__ cidx, const uint8_t *__restrict__ ctype,
    const T *__restrict__ fvi, float sigmainv, float M, T *grad_fvi) {
  const int64_t P = (int64_t)H * W;
  const int64_t total = (int64_t)B * P;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * kBlock) {
    if (face_idx[p] >= 0) continue;
    const int64_t b = p / P;
    const int64_t rem = p - b * P;
    const int h = (int)(rem / W), x = (int)(rem - (int64_t)h * W);
    const T x0 = (T)px_cx(M, W, x), y0 = (T)px_cy(M, H, h);
    const T dLdp = grad_soft[p], allprob = soft[p];
    for (int kid = 0; kid < K; ++kid) {
      const int64_t f = cidx[p * K + kid];
      if (f < 0) break;
      const int64_t sf = b * F + f;
      T v[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) v[c] = fvi[sf * 6 + c];
      T g[6] = {0, 0, 0, 0, 0, 0};
      soft_bwd_terms<T>(x0, y0, v, (int)ctype[p * K + kid] - 1, prob[p * K + kid], dLdp,
                        allprob, sigmainv, M, g);
#pragma unroll
      for (int c = 0; c < 6; ++c)
        if (g[c] != (T)0) atomicAdd(grad_fvi + sf * 6 + c, g[c]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_soft_bwd_gather(
    FaceSet<T> fs, const T *__restrict__ grad_soft, const T *__restrict__ soft,
    const int64_t *__restrict__ face_idx, const int32_t *__restrict__ last, float sigmainv,
    T *grad_fvi) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= fs.N) return;
  const int b = (int)(i / fs.F);
  const int f = (int)(i - (int64_t)b * fs.F);
  const float M = fs.M;
  T g[6] = {0, 0, 0, 0, 0, 0};
  T v[6], box[4];
  load_corners(fs, i, v);
  face_box(fs, i, v, box);
  const Span s = make_span<T>(box[0], box[1], box[2], box[3], M, fs.H, fs.W);
  if (!span_empty(s)) {
    for (int y = s.y0; y <= s.y1; ++y) {
      const T y0 = (T)px_cy(M, fs.H, y);
      const int64_t row = ((int64_t)b * fs.H + y) * fs.W;
      for (int x = s.x0; x <= s.x1; ++x) {
        const int64_t p = row + x;
        if (face_idx[p] >= 0) continue;
        const int32_t l = last[p];
        if (l >= 0 && f > l) continue;  // not among the pixel's first K close faces
        const T x0 = (T)px_cx(M, fs.W, x);
        if (x0 < box[0] || x0 >= box[2] || y0 < box[1] || y0 >= box[3]) continue;
        int et;
        T pr;
        soft_face_dist<T>(x0, y0, v, M, sigmainv, et, pr);
        soft_bwd_terms<T>(x0, y0, v, et, pr, grad_soft[p], soft[p], sigmainv, M, g);
      }
    }
  }
  T *go = grad_fvi + i * 6;
#pragma unroll
  for (int c = 0; c < 6; ++c) go[c] = g[c];
}

template <typename T>
__global__ void kd_zero_s(T *p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (T)0;
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
template <typename T>
int soft_forward(const FaceSet<T> &fs, const int64_t *face_idx, int K, float sigmainv, T *soft,
                 T *prob, int64_t *cidx, uint8_t *ctype, int32_t *last, void *ws,
                 size_t ws_bytes, hipStream_t stream) {
  const size_t need = bin_workspace_bytes(fs.B, fs.H, fs.W, fs.N, fs.F);
  if (ws_bytes < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  if (fs.B == 0 || fs.H == 0 || fs.W == 0) return KD_OK;
  size_t off = 0;
  BinBuffers bb = bin_carve(ws, off, fs.B, fs.H, fs.W, fs.N, fs.F);
  hipError_t e = bin_faces<T>(fs, bb, stream);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "binning: %s", hipGetErrorString(e));
  SoftFwdArgs<T> a{fs, bb, face_idx, K, sigmainv, soft, prob, cidx, ctype, last};
  const int ntiles = ((fs.W + kTile - 1) / kTile) * ((fs.H + kTile - 1) / kTile);
  if (prob)
    hipLaunchKernelGGL((kd_soft_fwd<T, true>), dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
  else
    hipLaunchKernelGGL((kd_soft_fwd<T, false>), dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft fwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int soft_backward(int B, int H, int W, int64_t F, int K, const T *grad_soft, const T *soft,
                  const int64_t *face_idx, const T *prob, const int64_t *cidx,
                  const uint8_t *ctype, const T *fvi, float sigmainv, float M, T *grad_fvi,
                  hipStream_t stream) {
  const int64_t nf = (int64_t)B * F;
  if (nf > 0) hipLaunchKernelGGL(kd_zero_s<T>, dim3(1024), dim3(256), 0, stream, grad_fvi, nf * 6);
  const int64_t total = (int64_t)B * H * W;
  if (total > 0 && nf > 0 && K > 0) {
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(kd_soft_bwd_atomic<T>, dim3((unsigned)(blocks < 65536 ? blocks : 65536)),
                       dim3(kBlock), 0, stream, B, H, W, F, K, grad_soft, soft, face_idx, prob,
                       cidx, ctype, fvi, sigmainv, M, grad_fvi);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
FaceSet<T> fused_faceset(int B, int H, int W, int64_t F, const T *fvi, double M, double boxlen) {
  FaceSet<T> fs{};
  fs.B = B;
  fs.H = H;
  fs.W = W;
  fs.N = (int64_t)B * F;
  fs.F = F;
  fs.fvi = fvi;
  fs.scale = (T)M;
  fs.margin = (T)(boxlen * M);
  fs.has_margin = 1;
  fs.M = (float)M;
  return fs;
}

template <typename T>
int soft_backward_gather(int B, int H, int W, int64_t F, const T *grad_soft, const T *soft,
                         const int64_t *face_idx, const int32_t *last, const T *fvi, double M,
                         double boxlen, float sigmainv, T *grad_fvi, hipStream_t stream) {
  FaceSet<T> fs = fused_faceset<T>(B, H, W, F, fvi, M, boxlen);
  if (fs.N > 0)
    hipLaunchKernelGGL(kd_soft_bwd_gather<T>, dim3((unsigned)((fs.N + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, fs, grad_soft, soft, face_idx, last, sigmainv,
                       grad_fvi);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(KD_ERR_LAUNCH, "soft bwd gather: %s", hipGetErrorString(e));
  return KD_OK;
}

}  // namespace kd

using namespace kd;

template <typename T>
static int soft_fwd_raw(int B, int H, int W, int64_t F, int K, const T *fvi, const T *bbox,
                        const int64_t *fidx, float sigmainv, float M, T *soft, T *prob,
                        int64_t *cidx, uint8_t *ctype, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(K >= 1, "knum must be >= 1");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  KD_CHECK_ARG(prob && cidx && ctype, "close lists are required");
  FaceSet<T> fs{};
  fs.B = B;
  fs.H = H;
  fs.W = W;
  fs.N = (int64_t)B * F;
  fs.F = F;
  fs.fvi = fvi;
  fs.scale = (T)1;
  fs.bbox = bbox;
  fs.M = M;
  return soft_forward<T>(fs, fidx, K, sigmainv, soft, prob, cidx, ctype, nullptr, ws, wsb,
                         (hipStream_t)stream);
}

template <typename T>
static int soft_fwd_fused(int B, int H, int W, int64_t F, int K, const T *fvi, double M,
                          double boxlen, const int64_t *fidx, float sigmainv, T *soft, T *prob,
                          int64_t *cidx, uint8_t *ctype, int32_t *last, void *ws, size_t wsb,
                          void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(K >= 1, "knum must be >= 1");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  KD_CHECK_ARG((prob && cidx && ctype) || (!prob && !cidx && !ctype),
               "close lists must be all set or all NULL");
  FaceSet<T> fs = fused_faceset<T>(B, H, W, F, fvi, M, boxlen);
  return soft_forward<T>(fs, fidx, K, sigmainv, soft, prob, cidx, ctype, last, ws, wsb,
                         (hipStream_t)stream);
}

extern "C" {

int kd_dibr_soft_mask_forward_f32(int B, int H, int W, int64_t F, int K, const float *fvi,
                                  const float *bbox, const int64_t *fidx, float sigmainv, float M,
                                  float *soft, float *prob, int64_t *cidx, uint8_t *ctype,
                                  void *ws, size_t wsb, void *stream) {
  return soft_fwd_raw<float>(B, H, W, F, K, fvi, bbox, fidx, sigmainv, M, soft, prob, cidx, ctype,
                             ws, wsb, stream);
}
int kd_dibr_soft_mask_forward_f64(int B, int H, int W, int64_t F, int K, const double *fvi,
                                  const double *bbox, const int64_t *fidx, float sigmainv,
                                  float M, double *soft, double *prob, int64_t *cidx,
                                  uint8_t *ctype, void *ws, size_t wsb, void *stream) {
  return soft_fwd_raw<double>(B, H, W, F, K, fvi, bbox, fidx, sigmainv, M, soft, prob, cidx,
                              ctype, ws, wsb, stream);
}

int kd_dibr_soft_mask_forward_fused_f32(int B, int H, int W, int64_t F, int K, const float *fvi,
                                        double M, double boxlen, const int64_t *fidx,
                                        float sigmainv, float *soft, float *prob, int64_t *cidx,
                                        uint8_t *ctype, int32_t *last, void *ws, size_t wsb,
                                        void *stream) {
  return soft_fwd_fused<float>(B, H, W, F, K, fvi, M, boxlen, fidx, sigmainv, soft, prob, cidx,
                               ctype, last, ws, wsb, stream);
}
int kd_dibr_soft_mask_forward_fused_f64(int B, int H, int W, int64_t F, int K, const double *fvi,
                                        double M, double boxlen, const int64_t *fidx,
                                        float sigmainv, double *soft, double *prob,
                                        int64_t *cidx, uint8_t *ctype, int32_t *last, void *ws,
                                        size_t wsb, void *stream) {
  return soft_fwd_fused<double>(B, H, W, F, K, fvi, M, boxlen, fidx, sigmainv, soft, prob, cidx,
                                ctype, last, ws, wsb, stream);
}

int kd_dibr_soft_mask_backward_f32(int B, int H, int W, int64_t F, int K, const float *gs,
                                   const float *soft, const int64_t *fidx, const float *prob,
                                   const int64_t *cidx, const uint8_t *ctype, const float *fvi,
                                   float sigmainv, float M, float *gfvi, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && K >= 0, "negative size");
  return soft_backward<float>(B, H, W, F, K, gs, soft, fidx, prob, cidx, ctype, fvi, sigmainv, M,
                              gfvi, (hipStream_t)stream);
}
int kd_dibr_soft_mask_backward_f64(int B, int H, int W, int64_t F, int K, const double *gs,
                                   const double *soft, const int64_t *fidx, const double *prob,
                                   const int64_t *cidx, const uint8_t *ctype, const double *fvi,
                                   float sigmainv, float M, double *gfvi, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && K >= 0, "negative size");
  return soft_backward<double>(B, H, W, F, K, gs, soft, fidx, prob, cidx, ctype, fvi, sigmainv,
                               M, gfvi, (hipStream_t)stream);
}

int kd_dibr_soft_mask_backward_gather_f32(int B, int H, int W, int64_t F, const float *gs,
                                          const float *soft, const int64_t *fidx,
                                          const int32_t *last, const float *fvi, double M,
                                          double boxlen, float sigmainv, float *gfvi, void *ws,
                                          size_t wsb, void *stream) {
  (void)ws;
  (void)wsb;
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  return soft_backward_gather<float>(B, H, W, F, gs, soft, fidx, last, fvi, M, boxlen, sigmainv,
                                     gfvi, (hipStream_t)stream);
}
int kd_dibr_soft_mask_backward_gather_f64(int B, int H, int W, int64_t F, const double *gs,
                                          const double *soft, const int64_t *fidx,
                                          const int32_t *last, const double *fvi, double M,
                                          double boxlen, float sigmainv, double *gfvi, void *ws,
                                          size_t wsb, void *stream) {
  (void)ws;
  (void)wsb;
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  return soft_backward_gather<double>(B, H, W, F, gs, soft, fidx, last, fvi, M, boxlen, sigmainv,
                                      gfvi, (hipStream_t)stream);
}

}  // extern "C"
