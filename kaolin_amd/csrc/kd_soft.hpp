// kd_soft.hpp -- shared pieces of the DIB-R soft-mask kernels (kd_softmask.hip, kd_softpair.hip):
// the reference's per-pair arithmetic (distance type / probability, backward terms), the per-wave
// (pixel, face) pair book and pass A (first K close faces per pixel over the tile lists).
#pragma once

#include "kd_binning.hpp"
#include "kd_capi.hpp"
#include "kd_raster.hpp"
#include "kd_softdist.hpp"
#include "kd_tile.hpp"

#include <type_traits>

namespace kd {

// dibr_soft_mask_cuda.cu:100-163: squared distance type (0..5) and probability of one face,
// bit-identical to the reference (kd_softdist.hpp; fp32: one double reciprocal per edge for its
// three quotients, quo_f).
template <typename T>
__device__ __forceinline__ void soft_face_dist(T x0, T y0, const T v[6], float M, float sigmainv,
                                               int &edgeid, T &prob) {
  soft_face_dist_ref<T, std::is_same<T, float>::value>(x0, y0, v, M, sigmainv, edgeid, prob);
}

// backward terms of one (pixel, close face) pair, dibr_soft_mask_cuda.cu:281-348; adds to the
// face's 6 corner gradients (already divided by M per term, like the reference).
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

constexpr int kPairCap = 512;  // (pixel, face) pairs per wave batch

template <typename T>
struct SoftArgs {
  FaceSet<T> fs;
  BinBuffers bb;
  const int64_t *face_idx;
  int K;
  float sigmainv;
  // forward outputs
  T *soft;
  T *prob;
  int64_t *cidx;
  uint8_t *ctype;
  int32_t *last;
  // backward
  const T *grad_soft;
  const T *soft_in;
  T *grad_fvi;
  // buffers the soft reduction zeroes on the side (the fused backward's gradients), nullable
  T *zero0, *zero1;
  int64_t nzero0, nzero1;
  // mask_iou(soft_mask, iou_gt) fused in: the forward adds each view's
  // (U_b, D_b) = (sum s g, sum (s + g - s g)) into iou_acc (fp64, B x 2); the backward adds
  // d loss / d soft (kaolin/metrics/render.py:18-40 through autograd, from iou_stats (B x 2, T)
  // and the device scalar iou_grad) to grad_soft.  iou_gt nullptr: no IoU.
  const T *iou_gt;
  double *iou_acc;  // [B][kIouParts] (U, D) partials: a tile adds to partial tile % kIouParts
  const T *iou_stats;
  const T *iou_grad;
  int iou_B;
  VertexOut<T> vo;  // backward: vo.grad set -> vertex gradients instead of grad_fvi (VTX bodies)
};

// d loss / d soft of the fused backward at pixel gp of view b: the incoming grad_soft (nullable)
// plus, with iou_gt, mask_iou's gradient w.r.t. its left mask -- kd_iou_bwd's arithmetic
// (kd_metrics.hip), so the sum is that of rasterize + dibr_soft_mask + mask_iou's autograd.
template <typename T>
__device__ __forceinline__ T soft_grad_at(const SoftArgs<T> &a, int b, int64_t gp) {
  T g = a.grad_soft ? a.grad_soft[gp] : (T)0;
  if (a.iou_gt) {
    const T gi = -(*a.iou_grad / (T)a.iou_B);
    const T U = a.iou_stats[2 * b], Dp = a.iou_stats[2 * b + 1] + (T)1e-10;
    const T gu = gi / Dp;
    const T gd = -gi * U / (Dp * Dp);
    const T gm = gu - gd;
    const T gl = gm * a.iou_gt[gp] + gd;
    g = a.grad_soft ? g + gl : gl;
  }
  return g;
}

constexpr int kIouParts = 32;  // fp64 (U, D) partials per view of the fused mask_iou

// Per-wave pair list of the current batch and its per-pixel bookkeeping.
struct PairBook {
  unsigned short pair[4][kPairCap];  // (q << 8) | k, q = pixel lane, k = tile-list entry
  short start[4][64], n[4][64], base[4][64];
};

// Pass A over the uncovered pixels of this wave for one batch of tile faces: per pixel, the
// first K - kid hits (ascending face order = ascending ballot rank) are appended to the pair
// list.  flush(npairs) runs passes B / C whenever the list is full and at the end.
template <typename Flush>
__device__ __forceinline__ void soft_pass_a(const SubSpans &ss, int nsub, PairBook &P,
                                            uint64_t umask, int K, const TileGeom &t,
                                            int &my_kid, Flush flush) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int npairs = 0;
  P.n[w][lane] = 0;
  for (uint64_t mm = umask; mm; mm &= mm - 1) {
    const int q = __builtin_ctzll(mm);
    int kid = rdlane_i(my_kid, q);
    if (kid >= K) continue;
    const int qx = t.WX0 + (q & 7), qy = t.WY0 + (q >> 3);
    int start = npairs, base = kid;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c * kWave >= nsub || kid >= K) break;
      const bool hit = pspan_has(ss.s[c], qx, qy);  // dibr_soft_mask_cuda.cu:95, exact
      const uint64_t hm = __ballot(hit);
      if (!hm) continue;
      const int need = K - kid;
      const int nh = __popcll(hm);
      const int ntake = nh < need ? nh : need;
      if (npairs + ntake > kPairCap) {
        if (lane == 0) {
          P.start[w][q] = (short)start;
          P.n[w][q] = (short)(npairs - start);
          P.base[w][q] = (short)base;
        }
        flush(npairs);
        npairs = 0;
        start = 0;
        base = kid;
      }
      const int rank = mbcnt(hm);
      if (hit && rank < need) P.pair[w][npairs + rank] = (unsigned short)((q << 8) | ss.k[c]);
      npairs += ntake;
      kid += ntake;
    }
    if (lane == 0) {
      P.start[w][q] = (short)start;
      P.n[w][q] = (short)(npairs - start);
      P.base[w][q] = (short)base;
    }
    if (lane == q) my_kid = kid;
  }
  flush(npairs);
}

template <typename T>
__device__ __forceinline__ void soft_stage(const FaceSet<T> &fs, T (*geo)[kCap], int k,
                                           int64_t fi) {
  T v[6];
  load_corners(fs, fi, v);
#pragma unroll
  for (int q = 0; q < 6; ++q) geo[q][k] = v[q];
}

// ------------------------------------------------------------------------------------------
// pair pipeline of the autograd path (kd_softpair.hip)
// ------------------------------------------------------------------------------------------
struct SoftPairRec {
  int32_t row;    // face row (view offset + face index)
  uint16_t slot;  // close-face slot of the pixel, 0..K-1
  uint8_t q;      // pixel of the tile (tile_geom thread index)
  uint8_t type;   // distance type 0..5 (set by the pair math, while the line is in L2)
};
// (soft_chunk_write stores a record as one 64-bit word: row | slot << 32 | q << 48 | type << 56)
static_assert(sizeof(SoftPairRec) == 8 && offsetof(SoftPairRec, slot) == 4 &&
                  offsetof(SoftPairRec, q) == 6 && offsetof(SoftPairRec, type) == 7,
              "SoftPairRec layout");

template <typename T>
struct SoftCoef {
  T h[4];
};

// Backward coefficients h_j of one pair (kd_softpair.hip, file comment); the geometric factors are the
// reference's expressions (dibr_soft_mask_cuda.cu:288-343) in T.
template <typename T>
__device__ __forceinline__ void soft_pair_coef(T x0, T y0, const T v[6], int et, T prob, float M,
                                               T h[4]) {
  if constexpr (std::is_same<T, float>::value) {
    {
      // fp32 with hardware reciprocals (1 ulp): the gradient's accuracy is that of the
      // reference's fp32 terms, whose double divisions end in float roundings too
      const float s = prob * __builtin_amdgcn_rcpf((1.f - prob + 1e-7f) * M);
      if (et >= 3) {
        const int ps = (et - 3) * 2;
        h[0] = s * (2.f * (v[ps] - x0));
        h[1] = s * (2.f * (v[ps + 1] - y0));
        h[2] = 0.f;
        h[3] = 0.f;
      } else {
        const int ps = et * 2, ps2 = ((et + 1) % 3) * 2;
        const float x1 = v[ps], y1 = v[ps + 1], x2 = v[ps2], y2 = v[ps2 + 1];
        const float A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
        const float up = A * x0 + Bc * y0 + C;
        const float rd = __builtin_amdgcn_rcpf(A * A + Bc * Bc + 1e-7f);
        const float dissquare = up * up * rd;
        const float dzdA = 2.f * (x0 * up - dissquare * A) * rd;
        const float dzdB = 2.f * (y0 * up - dissquare * Bc) * rd;
        const float dzdC = 2.f * up * rd;
        h[0] = s * (dzdB - y2 * dzdC);
        h[1] = s * (x2 * dzdC - dzdA);
        h[2] = s * (y1 * dzdC - dzdB);
        h[3] = s * (dzdA - x1 * dzdC);
      }
      return;
    }
  }
  // the backward's coefficients need gradient accuracy, not bit-exactness: reciprocals
  const double s = (double)prob * (1.0 / ((1.0 - (double)prob + KD_SOFT_EPS) * (double)M));
  if (et >= 3) {
    const int ps = (et - 3) * 2;
    h[0] = (T)(s * (double)((T)2 * (v[ps] - x0)));
    h[1] = (T)(s * (double)((T)2 * (v[ps + 1] - y0)));
    h[2] = (T)0;
    h[3] = (T)0;
  } else {
    const int ps = et * 2, ps2 = ((et + 1) % 3) * 2;
    const T x1 = v[ps], y1 = v[ps + 1], x2 = v[ps2], y2 = v[ps2 + 1];
    const T A = y2 - y1, Bc = x1 - x2, C = x2 * y1 - x1 * y2;
    const T up = A * x0 + Bc * y0 + C;
    const T down = A * A + Bc * Bc;
    const double rd = 1.0 / ((double)down + KD_SOFT_EPS);
    const T dissquare = (T)((double)(up * up) * rd);
    const T dzdA = (T)((double)((T)2 * (x0 * up - dissquare * A)) * rd);
    const T dzdB = (T)((double)((T)2 * (y0 * up - dissquare * Bc)) * rd);
    const T dzdC = (T)((double)((T)2 * up) * rd);
    h[0] = (T)(s * (double)(dzdB - y2 * dzdC));
    h[1] = (T)(s * (double)(x2 * dzdC - dzdA));
    h[2] = (T)(s * (double)(y1 * dzdC - dzdB));
    h[3] = (T)(s * (double)(dzdA - x1 * dzdC));
  }
}

// Adds one pair's contribution s_p * h_j to the register sums g[6] of its face's corners.
template <typename T>
__device__ __forceinline__ void soft_add_pair(T g[6], int et, double sp, const SoftCoef<T> &c) {
  const int ps = et >= 3 ? (et - 3) * 2 : et * 2;
  const int ps2 = et >= 3 ? -8 : ((et + 1) % 3) * 2;  // vertex types touch one corner only
  T v0, v1, v2, v3;
  if (std::is_same<T, float>::value) {
    const T spf = (T)sp;
    v0 = spf * c.h[0];
    v1 = spf * c.h[1];
    v2 = spf * c.h[2];
    v3 = spf * c.h[3];
  } else {
    v0 = (T)(sp * (double)c.h[0]);
    v1 = (T)(sp * (double)c.h[1]);
    v2 = (T)(sp * (double)c.h[2]);
    v3 = (T)(sp * (double)c.h[3]);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
    g[i] += i == ps ? v0 : i == ps + 1 ? v1 : i == ps2 ? v2 : i == ps2 + 1 ? v3 : (T)0;
}


constexpr int kFuseSlots = 32;           // knum bound of the one-launch soft mask (LDS slot table)
constexpr int kPoolPairsPerPixel = kFuseSlots;  // record pool: min(knum, 32) records per pixel

// One backward / pair-math work item: up to 256 consecutive records of one tile.
struct PairItem {
  int64_t start;  // first record
  int32_t tile;   // view * tiles + fine tile
  int32_t n;      // records (<= 256)
};

// The record pool (12 B per pair in fp32: the record and its probability).  A tile reserves,
// with one device atomic at the start of its soft phase, room for the most records it can
// produce -- its uncovered pixels x min(knum, faces of its soft coarse bin) -- and pass A fills
// it in order (face-major runs per wave chunk, an LDS counter); reserved room that stays unused
// is never touched.  The pair math and the backward find the records through PairItems.  The
// pool holds min(knum, 32) records per pixel, so with knum <= 32 every tile fits: then each tile
// simply owns 256 knum records (no atomic; `fixed`).  Otherwise (or
// under kd_set_pool_limits) a tile whose reservation does not fit computes its soft mask without
// records (`ovf` list, kd_soft_ovf_fwd) and its backward recomputes the pairs
// (kd_soft_ovf_bwd).
template <typename T>
struct SoftPairBuf {
  SoftPairRec *rec;    // [cap]
  T *sprob;            // [cap] probability of each record
  int64_t *tbase;      // [tiles] first record of each tile
  int32_t *npix;       // [P] close faces of each uncovered pixel (split pipeline)
  int32_t *ntile;      // [tiles] records of each tile
  PairItem *items;     // [cap / 256 + tiles]
  int32_t *tiles;      // [tiles] tiles with records (split pipeline's reduce)
  int32_t *ovf;        // [tiles] tiles that computed their soft mask without records
  int32_t *counters;   // [4]: items, tiles with records, overflow tiles, (unused); then the 64-bit
                       // record cursor (all zeroed by kd_bin_count: n_clear = 6)
  unsigned long long *cursor;
  int64_t ntiles, npixels, cap, lim;  // lim: records a forward may use (kd_set_pool_limits)
  int64_t icap;                        // entries of `items` (its allocation)
  int fixed;  // knum <= 32 and the whole pool usable: tile t owns records [t * 256 K, +256 K)
  int ntx;
};

constexpr int kPairClear = 6;  // ints of SoftPairBuf::counters (with the cursor) to zero

// bins + pair buffers for B views of F faces, K close faces, element size esize
size_t soft_pair_workspace_bytes(int B, int H, int W, int64_t N, int64_t F, int K, int esize,
                                 int ct0 = kCoarseTile0);
// pair buffers carved from a workspace after the soft mask's bins
template <typename T>
SoftPairBuf<T> soft_pair_carve(void *ws, size_t &off, int B, int H, int W, int K);
// pass A + pair math + (when reduce) the soft mask, over already built bins (a.bb) whose
// kd_bin_count cleared pb.counters
template <typename T>
int soft_pairs_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, bool grad, bool reduce,
                      hipStream_t stream);
// the backward over the records of soft_pairs_launch(grad = true), adding into a.grad_fvi
template <typename T>
int soft_pairs_backward_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, hipStream_t stream);
// The raster forward (fp32 pair pipeline) and the fused soft mask in one launch, when both apply.
template <typename T>
struct RasterFwdArgs;
bool dibr_fwd_fusable(const RasterFwdArgs<double> &ra, const SoftArgs<double> &a);
int dibr_fwd_fused_launch(RasterFwdArgs<double> &ra, SoftArgs<double> &a, SoftPairBuf<double> &pb,
                          hipStream_t stream);
bool dibr_fwd_fusable(const RasterFwdArgs<float> &ra, const SoftArgs<float> &a);
// workgroups per tile (1, 2, 4) the fused fp32 forward will use for B views
int dibr_fwd_split(const SoftPairBuf<float> &pb, int K, int B, bool history, hipStream_t stream);
int dibr_fwd_fused_launch(RasterFwdArgs<float> &ra, SoftArgs<float> &a, SoftPairBuf<float> &pb,
                          hipStream_t stream);
// The soft-mask backward and the raster backward (kd_raster_bwd.hpp, D <= 3) in one launch.
template <typename T>
struct RasterBwdArgs;
template <typename T>
int dibr_backward_merged_launch(SoftArgs<T> &a, SoftPairBuf<T> &pb, const RasterBwdArgs<T> &ra,
                                hipStream_t stream);
// bins + pass A + pair math (+ backward coefficients when grad) + (when reduce) the soft mask
template <typename T>
int soft_pairs_forward(SoftArgs<T> &a, void *ws, size_t ws_bytes, bool grad, bool reduce,
                       hipStream_t stream);
template <typename T>
int soft_pairs_backward(SoftArgs<T> &a, void *ws, size_t ws_bytes, hipStream_t stream);

}  // namespace kd
