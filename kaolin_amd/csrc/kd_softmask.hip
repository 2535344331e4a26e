// kd_softmask.hip -- DIB-R soft mask forward / backward for gfx950.
//
// Forward (replaces dibr_soft_mask_forward_cuda_kernel, dibr_soft_mask_cuda.cu:27-184).
//   Per 16x16 tile (kd_tile.hpp): the ordered list of faces whose ENLARGED box touches the tile
//   (all faces, no culling: dibr.py:201-208) is staged in LDS.  Each wave then works on the
//   uncovered pixels of its 8x8 sub-tile in three passes over a per-wave (pixel, face) pair list:
//     A  per pixel, lane = candidate face: ballot of the exact box test; the first K hits by face
//        index are the lowest ballot ranks (mbcnt), appended to the pair list in slot order;
//     B  lane = pair: distance type and probability (the reference arithmetic), stored in LDS and,
//        when the close lists are requested, written out (consecutive lanes = consecutive slots,
//        coalesced);
//     C  lane = pixel: soft = 1 - prod(1 - p) over the pixel's pairs in slot order with the
//        reference's double promotion per step.
//   The expensive distance math (9 double divisions) thus runs with every lane busy, once per
//   (pixel, close face) pair.  With the close lists not requested nothing but soft (and
//   optionally close_last) is written.
// This file serves the reference's op forms (_C.render.mesh.dibr_soft_mask_forward_cuda /
// _backward_cuda: explicit boxes, close lists in and out); the autograd path is the pair
// pipeline of kd_softpair.hip.
// Backward.
//   kd_soft_bwd_atomic -- general form of the reference op (any given close lists), one thread
//                         per pixel, float atomics (dibr_soft_mask_cuda.cu:230-353).
#include "../../include/kaolin_dibr.h"
#include "kd_soft.hpp"

namespace kd {

template <typename T, bool LISTS>
__global__ __launch_bounds__(kBlock) void kd_soft_fwd(SoftArgs<T> a) {
  TileClock clk(a.fs.tbuf, 1);
  __shared__ TileLists L;
  __shared__ T s_geo[6][kCap];  // scaled corners
  __shared__ PairBook P;
  __shared__ T s_val[4][kPairCap];  // probability of each pair

  const FaceSet<T> &fs = a.fs;
  const int H = fs.H, W = fs.W, K = a.K;
  const float M = fs.M;
  const int b = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int64_t lo, hi;
  view_range(fs, b, lo, hi);
  const TileGeom t = tile_geom(H, W);
  const int64_t p = ((int64_t)b * H + t.py) * W + t.px;
  const bool covered = t.inimg && a.face_idx[p] >= 0;
  const bool unc = t.inimg && !covered;
  const uint64_t umask = __ballot(unc);
  int my_kid = 0;
  T my_prod = (T)1.0;
  bool any_sub = false;

  if (__syncthreads_or(unc)) {
    auto stage = [&](int k, int64_t fi) { soft_stage(fs, s_geo, k, fi); };
    auto flush = [&](int npairs) {  // passes B and C
      if (ablate(fs.dbg, 32)) npairs = 0;
      wave_lds_sync();
      for (int e = lane; e < npairs; e += kWave) {
        const int pr = P.pair[w][e];
        const int q = pr >> 8, k = pr & 255;
        const int qx = t.WX0 + (q & 7), qy = t.WY0 + (q >> 3);
        T v[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) v[c] = s_geo[c][k];
        int et;
        T pb;
        soft_face_dist<T>((T)px_cx(M, W, qx), (T)px_cy(M, H, qy), v, M, a.sigmainv, et, pb);
        s_val[w][e] = pb;
        const int slot = P.base[w][q] + (e - P.start[w][q]);
        const int64_t qp = ((int64_t)b * H + qy) * W + qx;
        if (LISTS) {
          const int64_t o = qp * K + slot;
          a.prob[o] = pb;
          a.cidx[o] = L.f[k];
          a.ctype[o] = (uint8_t)(et + 1);
        }
        if (a.last && slot == K - 1) a.last[qp] = L.f[k];
      }
      wave_lds_sync();
      const int nq = P.n[w][lane];
      const int sq = P.start[w][lane];
      for (int i = 0; i < nq; ++i)  // dibr_soft_mask_cuda.cu:174-178, slot order
        my_prod = (T)((double)my_prod * (1.0 - (double)s_val[w][sq + i]));
      wave_lds_sync();
      P.n[w][lane] = 0;
      wave_lds_sync();
    };
    auto round = [&](int nsub, int) {
      if (!umask || nsub == 0 || ablate(fs.dbg, 1)) return;
      any_sub = true;
      const SubSpans ss = load_subspans(L, nsub);
      soft_pass_a(ss, nsub, P, umask, K, t, my_kid, flush);
    };
    // once every uncovered pixel of the tile holds K close faces, later faces cannot enter
    auto done = [&]() { return __syncthreads_and(!unc || my_kid >= K) != 0; };
    tile_rounds(L, a.bb, (int)(hi - lo), b, lo, t, stage, round, fs.dbg, done);
  }

  if (!t.wave_live) return;
  if (t.inimg) {
    a.soft[p] = covered ? (T)1.0 : (T)(1.0 - (double)my_prod);  // :69, :181
    if (a.last && my_kid < K) a.last[p] = -1;
  }
  if (!LISTS) return;
  // -1 / 0 / 0 padding of every slot not written above (dibr_soft_mask.cpp:86-97 pre-fill).
  const int nx = t.WX1 - t.WX0 + 1;
  if (!any_sub) {
    const int per_row = nx * K;
    for (int r = 0; r <= t.WY1 - t.WY0; ++r) {
      const int64_t e0 = (((int64_t)b * H + t.WY0 + r) * W + t.WX0) * K;
      for (int e = lane; e < per_row; e += kWave) {
        a.prob[e0 + e] = (T)0;
        a.cidx[e0 + e] = -1;
        a.ctype[e0 + e] = 0;
      }
    }
  } else {
    const uint64_t imask = __ballot(t.inimg);
    for (uint64_t mm = imask; mm; mm &= mm - 1) {
      const int q = __builtin_ctzll(mm);
      const int kid = rdlane_i(my_kid, q);
      const int64_t e0 = (((int64_t)b * H + t.WY0 + (q >> 3)) * W + t.WX0 + (q & 7)) * K;
      for (int s = kid + lane; s < K; s += kWave) {
        a.prob[e0 + s] = (T)0;
        a.cidx[e0 + s] = -1;
        a.ctype[e0 + s] = 0;
      }
    }
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

// The same backward over given close lists, per 16x16 tile of pixels (grid-stride): the tile's
// uncovered pixels whose terms can be nonzero are compacted in LDS with their factor
// s_p = -sigmainv * dL/dsoft * (1 - soft); each half-wave (K <= 32) or wave (K > 32, 64 slots at
// a time) takes one listed pixel's row of K slots -- consecutive lanes, consecutive elements,
// the slot's face, probability and type loaded together -- and its lanes up to the row's first
// -1 (a ballot: the reference's loop stops there, dibr_soft_mask_cuda.cu:273-276) add their
// pair's terms s_p * h_j (kd_soft.hpp soft_pair_coef: the coefficients of the fused path, the
// reference's factors, dibr_soft_mask_cuda.cu:281-348, up to rounding).  The terms are summed per
// face in an LDS hash table (a face is close to many pixels of a tile) and each (tile, face,
// coordinate) sum goes out with one float atomic; a pair whose face finds no slot (a full table)
// adds its terms directly.  Load chain per tile: face_idx / grad / soft -> the rows -> the
// faces' corners.  Small LDS (11 KB fp32), so several tiles per CU hide it.
constexpr int kListHash = 256;  // LDS face slots per tile

template <typename T>
__global__ __launch_bounds__(kBlock) void kd_soft_bwd_lists(
    int B, int H, int W, int64_t F, int K, const T *__restrict__ grad_soft,
    const T *__restrict__ soft, const int64_t *__restrict__ face_idx, const T *__restrict__ prob,
    const int64_t *__restrict__ cidx, const uint8_t *__restrict__ ctype,
    const T *__restrict__ fvi, float sigmainv, float M, T *grad_fvi, int dbg,
    const int32_t *__restrict__ row_n) {
  __shared__ int64_t s_pix[kBlock];  // listed pixel: image index | tile pixel << 48
  __shared__ double s_sp[kBlock];    // its s_p
  __shared__ int s_cnt[kBlock / kWave];
  __shared__ int s_key[kListHash];
  __shared__ T s_acc[kListHash][6];
  const int ntx = (W + kTile - 1) / kTile, nty = (H + kTile - 1) / kTile;
  const int64_t ntiles = (int64_t)B * ntx * nty;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int i = tid; i < kListHash; i += kBlock) {
    s_key[i] = -1;
#pragma unroll
    for (int c = 0; c < 6; ++c) s_acc[i][c] = (T)0;
  }
  // one (pixel, slot) pair with a face (c >= 0): its terms into the tile's face sums
  auto pair = [&](int b, int x, int h, int64_t c, T pr, int et, double sp) {
    const int64_t sf = (int64_t)b * F + c;
    T v[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) v[q] = fvi[sf * 6 + q];
    SoftCoef<T> cf;
    soft_pair_coef<T>((T)px_cx(M, W, x), (T)px_cy(M, H, h), v, et, pr, M, cf.h);
    T g[6] = {0, 0, 0, 0, 0, 0};
    soft_add_pair<T>(g, et, sp, cf);
    if (ablate(dbg, 1 << 22)) {  // diagnostics: no accumulation (one plain store keeps the math)
      if (g[0] + g[1] + g[2] + g[3] + g[4] + g[5] == (T)12345) grad_fvi[0] = (T)1;
      return;
    }
    unsigned u = ((unsigned)sf * 2654435761u) >> 24;  // 8 bits
    int slot = -1;
    for (int probe = 0; probe < 32; ++probe) {
      const int old = atomicCAS(&s_key[u], -1, (int)sf);
      if (old == -1 || old == (int)sf) {
        slot = (int)u;
        break;
      }
      u = (u + 1) & (kListHash - 1);
    }
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (g[q] != (T)0) {
        if (slot >= 0)
          atomicAdd(&s_acc[slot][q], g[q]);
        else
          atomicAdd(grad_fvi + sf * 6 + q, g[q]);
      }
  };
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = (int)(tile / ((int64_t)ntx * nty));
    const int tl = (int)(tile - (int64_t)b * ntx * nty);
    const int X0 = (tl % ntx) * kTile, Y0 = (tl / ntx) * kTile;
    const int px = X0 + (tid & 15), py = Y0 + (tid >> 4);
    const bool in = px < W && py < H;
    const int64_t p = ((int64_t)b * H + py) * W + px;
    int64_t fi = 0;
    T gsv = (T)0, sov = (T)0;
    if (in) {  // (independent loads, issued together)
      fi = face_idx[p];
      gsv = grad_soft[p];
      sov = soft[p];
    }
    // a listed pixel needs its rows read unless every term of its row is exactly zero: soft 1
    // (the factor 1 - soft) or a zero incoming gradient -- with both finite (a NaN or inf must
    // reach the gradients as in the reference).  soft 0 is NOT such a case: it only says that
    // every 1 - prob rounded to 1 (dibr_soft_mask_cuda.cu:174-181), and a probability of ~2^-25
    // still gives the nonzero terms dLdz * geometry of dibr_soft_mask_cuda.cu:283-348.
    // row_n (nullable; the fused lists forward's row lengths, kd_dibr_rasterization_forward_lists):
    // a row without listed faces has no terms at all -- known without reading it
    const bool zero_terms = ((sov == (T)1 || gsv == (T)0) && isfinite(sov) && isfinite(gsv)) ||
                            (row_n && in && row_n[p] == 0);
    const bool live = in && fi < 0 && !zero_terms;
    int n;
    const int pos = wg_compact(live, s_cnt, n);  // (its barriers also order the table reset)
    if (live) {
      s_pix[pos] = ((int64_t)tid << 48) | p;  // tile pixel + image pixel
      s_sp[pos] = -(double)sigmainv * (double)gsv * (1.0 - (double)sov);
    }
    __syncthreads();
    if (K <= 32) {  // two rows per wave step (half-waves), rows dealt to the waves in turn
      const int half = lane >> 5, s = lane & 31;
      for (int i0 = 2 * w; i0 < n; i0 += 2 * (kBlock / kWave)) {
        const int i = i0 + half;
        const bool in2 = i < n && s < K;
        const int64_t ent = i < n ? s_pix[i] : 0;
        const int64_t e = (ent & 0xffffffffffffll) * K + s;
        int64_t c = -1;
        T pr = (T)0;
        int ty = 0;
        if (in2) {  // the slot's face, probability and type together
          c = cidx[e];
          pr = prob[e];
          ty = ctype[e];
        }
        const uint64_t sm = __ballot(!in2 || c < 0);
        const uint32_t hm = (uint32_t)(sm >> (32 * half));  // this half's stops
        const int first = hm ? __builtin_ctz(hm) : 32;
        if (in2 && s < first) {
          const int q = (int)(ent >> 48);
          pair(b, X0 + (q & 15), Y0 + (q >> 4), c, pr, ty - 1, s_sp[i]);
        }
      }
    } else {  // one row per wave, 64 slots at a time until its first -1
      for (int i = w; i < n; i += kBlock / kWave) {
        const int64_t ent = s_pix[i];
        const int64_t pp = ent & 0xffffffffffffll;
        const int q = (int)(ent >> 48);
        const double sp = s_sp[i];
        for (int s0 = 0; s0 < K; s0 += kWave) {
          const int s = s0 + lane;
          int64_t c = -1;
          T pr = (T)0;
          int ty = 0;
          if (s < K) {
            c = cidx[pp * K + s];
            pr = prob[pp * K + s];
            ty = ctype[pp * K + s];
          }
          const uint64_t sm = __ballot(c < 0);
          const int first = sm ? __builtin_ctzll(sm) : kWave;
          if (lane < first) pair(b, X0 + (q & 15), Y0 + (q >> 4), c, pr, ty - 1, sp);
          if (sm) break;
        }
      }
    }
    __syncthreads();
    // flush the tile's face sums (one atomic per nonzero (face, coordinate)) and reset the table
    for (int i = tid; i < kListHash; i += kBlock) {
      const int key = s_key[i];
      if (key < 0) continue;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const T v = s_acc[i][c];
        if (v != (T)0) atomicAdd(grad_fvi + (int64_t)key * 6 + c, v);
        s_acc[i][c] = (T)0;
      }
      s_key[i] = -1;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
template <typename T>
int soft_forward(SoftArgs<T> &a, void *ws, size_t ws_bytes, bool build_bins,
                 hipStream_t stream) {
  const FaceSet<T> &fs = a.fs;
  const size_t need = bin_workspace_bytes(fs.B, fs.H, fs.W, fs.N, fs.F);
  if (ws_bytes < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  if (fs.B == 0 || fs.H == 0 || fs.W == 0) return KD_OK;
  size_t off = 0;
  a.bb = bin_carve(ws, off, fs.B, fs.H, fs.W, fs.N, fs.F);
  a.bb.cull = nullptr;
  a.fs.dbg = debug_flags();
  a.fs.tbuf = debug_tile_buffer();
  if (build_bins) {
    hipError_t e = bin_faces<T>(fs, a.bb, stream);
    if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "binning: %s", hipGetErrorString(e));
  }
  const int ntiles = ((fs.W + kTile - 1) / kTile) * ((fs.H + kTile - 1) / kTile);
  {
    ProfScope prof(K_SOFT_FWD, stream);
    if (a.prob)
      hipLaunchKernelGGL((kd_soft_fwd<T, true>), dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
    else
      hipLaunchKernelGGL((kd_soft_fwd<T, false>), dim3(ntiles, fs.B), dim3(kBlock), 0, stream, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft mask: %s", hipGetErrorString(e));
  return KD_OK;
}

template <typename T>
int soft_backward(int B, int H, int W, int64_t F, int K, const T *grad_soft, const T *soft,
                  const int64_t *face_idx, const T *prob, const int64_t *cidx,
                  const uint8_t *ctype, const T *fvi, float sigmainv, float M, T *grad_fvi,
                  hipStream_t stream, const int32_t *row_n = nullptr) {
  const int64_t nf = (int64_t)B * F;
  if (nf > 0) {  // (a kernel, not a memset node: see zero_buffers)
    const int rc = zero_buffers<T>(grad_fvi, nf * 6, (T *)nullptr, 0, stream);
    if (rc != KD_OK) return rc;
  }
  const int64_t total = (int64_t)B * H * W;
  if (total > 0 && nf > 0 && K > 0) {
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    ProfScope prof(K_SOFT_BWD_ATOMIC, stream);
    const int64_t tiles = (int64_t)B * ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    const unsigned grid = (unsigned)(blocks < 8192 ? blocks : 8192);
    const unsigned tgrid = (unsigned)(tiles < 8192 ? tiles : 8192);
    bool atomic_form = false;  // diagnostics: the lane-per-pixel form (flag 1 << 29)
    if constexpr (KD_DIAG) {
      atomic_form = (debug_flags() & (1 << 29)) != 0;
      if (atomic_form)
        hipLaunchKernelGGL(kd_soft_bwd_atomic<T>, dim3(grid), dim3(kBlock), 0, stream, B, H, W,
                           F, K, grad_soft, soft, face_idx, prob, cidx, ctype, fvi, sigmainv, M,
                           grad_fvi);
    }
    if (!atomic_form)
      hipLaunchKernelGGL(kd_soft_bwd_lists<T>, dim3(tgrid), dim3(kBlock), 0, stream, B, H, W, F,
                         K, grad_soft, soft, face_idx, prob, cidx, ctype, fvi, sigmainv, M,
                         grad_fvi, debug_flags(), row_n);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "soft bwd: %s", hipGetErrorString(e));
  return KD_OK;
}

template int soft_backward<float>(int, int, int, int64_t, int, const float *, const float *,
                                  const int64_t *, const float *, const int64_t *,
                                  const uint8_t *, const float *, float, float, float *,
                                  hipStream_t, const int32_t *);
template int soft_backward<double>(int, int, int, int64_t, int, const double *, const double *,
                                   const int64_t *, const double *, const int64_t *,
                                   const uint8_t *, const double *, float, float, double *,
                                   hipStream_t, const int32_t *);

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

}  // namespace kd

using namespace kd;

template <typename T>
static int soft_fwd_raw(int B, int H, int W, int64_t F, int K, const T *fvi, const T *bbox,
                        const int64_t *fidx, float sigmainv, float M, T *soft, T *prob,
                        int64_t *cidx, uint8_t *ctype, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(K >= 1, "knum must be >= 1");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  KD_CHECK_ARG(prob && cidx && ctype, "close lists are required");
  SoftArgs<T> a{};
  a.fs.B = B;
  a.fs.H = H;
  a.fs.W = W;
  a.fs.N = (int64_t)B * F;
  a.fs.F = F;
  a.fs.fvi = fvi;
  a.fs.scale = (T)1;
  a.fs.bbox = bbox;
  a.fs.M = M;
  a.face_idx = fidx;
  a.K = K;
  a.sigmainv = sigmainv;
  a.soft = soft;
  a.prob = prob;
  a.cidx = cidx;
  a.ctype = ctype;
  return soft_forward<T>(a, ws, wsb, true, (hipStream_t)stream);
}

template <typename T>
static int soft_fwd_fused(int B, int H, int W, int64_t F, int K, const T *fvi, double M,
                          double boxlen, const int64_t *fidx, float sigmainv, T *soft, T *prob,
                          int64_t *cidx, uint8_t *ctype, int32_t *last, int want_grad, void *ws,
                          size_t wsb, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(K >= 1 && K <= 65535, "knum must be in [1, 65535]");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  KD_CHECK_ARG((prob && cidx && ctype) || (!prob && !cidx && !ctype),
               "close lists must be all set or all NULL");
  KD_CHECK_ARG(soft, "soft_mask is NULL");
  SoftArgs<T> a{};
  a.fs = fused_faceset<T>(B, H, W, F, fvi, M, boxlen);
  a.face_idx = fidx;
  a.K = K;
  a.sigmainv = sigmainv;
  a.soft = soft;
  a.prob = prob;
  a.cidx = cidx;
  a.ctype = ctype;
  a.last = last;
  return soft_pairs_forward<T>(a, ws, wsb, want_grad != 0, true, (hipStream_t)stream);
}

template <typename T>
static int soft_bwd_binned(int B, int H, int W, int64_t F, int K, const T *gs, const T *soft,
                           const int64_t *fidx, const T *fvi, double M, double boxlen,
                           float sigmainv, T *gfvi, void *ws, size_t wsb, int bins_ready,
                           void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0, "negative size");
  KD_CHECK_ARG(K >= 1 && K <= 65535, "knum must be in [1, 65535]");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  const int64_t nf = (int64_t)B * F;
  if (nf > 0) {  // (a kernel, not a memset node: see zero_buffers)
    const int rc = zero_buffers<T>(gfvi, nf * 6, (T *)nullptr, 0, (hipStream_t)stream);
    if (rc != KD_OK) return rc;
  }
  SoftArgs<T> a{};
  a.fs = fused_faceset<T>(B, H, W, F, fvi, M, boxlen);
  a.face_idx = fidx;
  a.K = K;
  a.sigmainv = sigmainv;
  a.grad_soft = gs;
  a.soft_in = soft;
  a.grad_fvi = gfvi;
  if (!bins_ready) {  // no forward workspace: rebuild the records and their coefficients
    const int rc = soft_pairs_forward<T>(a, ws, wsb, true, false, (hipStream_t)stream);
    if (rc != KD_OK) return rc;
  }
  return soft_pairs_backward<T>(a, ws, wsb, (hipStream_t)stream);
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

size_t kd_soft_mask_workspace_size(int B, int H, int W, int64_t F, int knum,
                                   int double_precision) {
  if (B < 0 || H < 0 || W < 0 || F < 0 || knum < 1) return 0;
  return soft_pair_workspace_bytes(B, H, W, (int64_t)B * F, F, knum, double_precision ? 8 : 4);
}

int kd_dibr_soft_mask_forward_fused_f32(int B, int H, int W, int64_t F, int K, const float *fvi,
                                        double M, double boxlen, const int64_t *fidx,
                                        float sigmainv, float *soft, float *prob, int64_t *cidx,
                                        uint8_t *ctype, int32_t *last, int want_grad, void *ws,
                                        size_t wsb, void *stream) {
  return soft_fwd_fused<float>(B, H, W, F, K, fvi, M, boxlen, fidx, sigmainv, soft, prob, cidx,
                               ctype, last, want_grad, ws, wsb, stream);
}
int kd_dibr_soft_mask_forward_fused_f64(int B, int H, int W, int64_t F, int K, const double *fvi,
                                        double M, double boxlen, const int64_t *fidx,
                                        float sigmainv, double *soft, double *prob,
                                        int64_t *cidx, uint8_t *ctype, int32_t *last,
                                        int want_grad, void *ws, size_t wsb, void *stream) {
  return soft_fwd_fused<double>(B, H, W, F, K, fvi, M, boxlen, fidx, sigmainv, soft, prob, cidx,
                                ctype, last, want_grad, ws, wsb, stream);
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

int kd_dibr_soft_mask_backward_binned_f32(int B, int H, int W, int64_t F, int K, const float *gs,
                                          const float *soft, const int64_t *fidx,
                                          const float *fvi, double M, double boxlen,
                                          float sigmainv, float *gfvi, void *ws, size_t wsb,
                                          int bins_ready, void *stream) {
  return soft_bwd_binned<float>(B, H, W, F, K, gs, soft, fidx, fvi, M, boxlen, sigmainv, gfvi, ws,
                                wsb, bins_ready, stream);
}
int kd_dibr_soft_mask_backward_binned_f64(int B, int H, int W, int64_t F, int K,
                                          const double *gs, const double *soft,
                                          const int64_t *fidx, const double *fvi, double M,
                                          double boxlen, float sigmainv, double *gfvi, void *ws,
                                          size_t wsb, int bins_ready, void *stream) {
  return soft_bwd_binned<double>(B, H, W, F, K, gs, soft, fidx, fvi, M, boxlen, sigmainv, gfvi,
                                 ws, wsb, bins_ready, stream);
}

}  // extern "C"
