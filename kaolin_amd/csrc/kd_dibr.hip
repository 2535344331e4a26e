// kd_dibr.hip -- dibr_rasterization (kaolin/render/mesh/dibr.py:119-209) as one forward and one
// backward launch sequence.
//
// The reference composes rasterize (valid faces = face_normals_z >= 0, dibr.py:195) and
// dibr_soft_mask (all faces, dibr.py:201-208) as two autograd functions.  Fused here:
//   forward   one binning pass for both face sets (the raster's tight boxes of the valid faces
//             and the soft mask's enlarged boxes of all faces: kd_binning bin_faces2), the
//             raster kernel, then the soft-mask pair pipeline on its face_idx.  face_vertices_z
//             and face_normals_z are read through strides, so views of prepare_vertices'
//             outputs need no copies.
//   backward  one zero fill for both gradients, the raster backward and the soft-mask backward
//             accumulating into the same grad_fvi (no separate buffers and no sum kernel).
// Results are exactly those of rasterize + dibr_soft_mask.
#include "../../include/kaolin_dibr.h"
#include "kd_raster.hpp"
#include "kd_prep.hpp"
#include "kd_raster_bwd.hpp"
#include "kd_soft.hpp"

#include <type_traits>
#include <vector>

namespace kd {

// Coarse bin edge (kd_binning bin_geom ct0) of a call: the test / tuning hook's, else 32 px.
// Measured at C3 (bench.py --coarse-tile, same box; profiles/r04/ab_ct*.txt): with 16-px bins
// (each fine tile walks only its own faces) the fused forward at 1 view drops from 55.1 to
// 48.9 us, but the scatter's per-chunk membership masks grow with the bin count (10.3 -> 18.4
// us; 21.6 -> 60.5 us at 8 views) and the count's LDS atomics with the bins a face touches:
// 1 view 0.1098 -> 0.1161 ms, 2 views 0.1382 -> 0.1553, 8 views 0.3017 -> 0.3590.  A function
// of the hook only, so forward and backward agree (the pair buffers lead the workspace anyway).
static int dibr_ct0(int, int, int) {
  const int hook = coarse_tile_hook();
  return hook > 0 ? hook : kCoarseTile0;
}

size_t dibr_workspace_bytes(int B, int H, int W, int64_t F, int K, int esize) {
  // sized for the smallest coarse tile (the most bins): covers every dibr_ct0 choice
  const int64_t N = (int64_t)B * F;
  return bin_workspace_bytes(B, H, W, N, F, kTile) +
         soft_pair_workspace_bytes(B, H, W, N, F, K, esize, kTile);
}

template <typename T>
struct DibrBuffers {
  BinBuffers rbb;      // raster bins (+ cull coefficients)
  BinBuffers sbb;      // soft-mask bins
  SoftPairBuf<T> pb;   // soft-mask records
};

// The pair buffers first: their place does not depend on the coarse tile (dibr_ct0), so a
// backward finds its forward's records whatever it would choose.
template <typename T>
static DibrBuffers<T> dibr_carve(void *ws, int B, int H, int W, int64_t F, int K) {
  const int64_t N = (int64_t)B * F;
  const int ct0 = dibr_ct0(B, H, W);
  DibrBuffers<T> d;
  size_t off = 0;
  d.pb = soft_pair_carve<T>(ws, off, B, H, W, K);
  d.rbb = bin_carve(ws, off, B, H, W, N, F, ct0);
  d.sbb = bin_carve(ws, off, B, H, W, N, F, ct0);
  return d;
}

template <typename T>
static FaceSet<T> dibr_faceset(int B, int H, int W, int64_t F, const T *fvi, double M) {
  FaceSet<T> fs{};
  fs.B = B;
  fs.H = H;
  fs.W = W;
  fs.N = (int64_t)B * F;
  fs.F = F;
  fs.fvi = fvi;
  fs.scale = (T)M;
  fs.M = (float)M;
  return fs;
}

// mask_iou(soft, gt) fused into dibr_rasterization: inputs / outputs of the
// forward (gt nullptr: none) and of the backward
template <typename T>
struct IouIo {
  const T *gt;     // (B, H, W) the right-hand mask
  T *loss;         // () forward
  T *stats;        // (B, 2) (U_b, D_b) in T: forward out, backward in
  double *acc;     // (B, kIouParts, 2) fp64 partials, forward
  const T *grad;   // () device scalar d(outer)/d loss, backward
};

template <typename T>
int iou_finish_launch(int B, int nparts, const double *acc, T *stats, T *loss,
                      hipStream_t stream);

template <typename T>
static int dibr_fwd(int B, int H, int W, int64_t F, int D, const T *fvz, int64_t fvz_fs,
                    int64_t fvz_cs, const T *fvi, const T *feat, const T *nz, int64_t nz_stride,
                    double M, float eps, float sigmainv, double boxlen, int K, T *interp,
                    int64_t *face_idx, T *weights, T *soft, int want_grad, T *gz_fvi,
                    T *gz_feat, void *ws, size_t wsb, void *stream_,
                    const IouIo<T> &iou = IouIo<T>{}, const PrepOut<T> *prep = nullptr,
                    T *prob = nullptr, int64_t *cidx = nullptr, uint8_t *ctype = nullptr) {
  hipStream_t stream = (hipStream_t)stream_;
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  KD_CHECK_ARG(K >= 1 && K <= 65535, "knum must be in [1, 65535]");
  KD_CHECK_ARG(H < 32768 && W < 32768, "image side must be < 32768");
  KD_CHECK_ARG(std::isfinite((float)M), "multiplier must be finite");
  KD_CHECK_ARG((int64_t)B * F < (1ll << 31), "too many faces");
  const size_t need = dibr_workspace_bytes(B, H, W, F, K, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  KD_CHECK_ARG(!iou.gt || (iou.loss && iou.stats && iou.acc), "mask_iou: NULL output");
  KD_CHECK_ARG(!prob == !cidx && !prob == !ctype, "close lists: give all three outputs or none");
  KD_CHECK_ARG(!prob || F < (1ll << 28), "close lists: more than 2^28 faces per view");
  KD_CHECK_ARG(!iou.gt || (K <= kFuseSlots && pool_limit_pairs() >= 1.f &&
                            !(test_forms() & KD_FORM_SOFT_SPLIT)),
               "fused mask_iou needs knum <= 32 (the one-launch soft mask)");
  const int64_t nf = (int64_t)B * F;
  if (!want_grad) gz_fvi = gz_feat = nullptr;
  if (B == 0 || H == 0 || W == 0) {
    const int rc = zero_buffers<T>(gz_fvi, nf * 6, gz_feat, gz_feat ? nf * 3 * D : 0, stream);
    if (rc != KD_OK || !iou.gt || B == 0) return rc;
    if (zero_words(iou.acc, sizeof(double) * 2 * kIouParts * B, stream) != hipSuccess)
      return set_error(KD_ERR_LAUNCH, "mask_iou: memset");
    return iou_finish_launch<T>(B, kIouParts, iou.acc, iou.stats, iou.loss, stream);
  }
  DibrBuffers<T> d = dibr_carve<T>(ws, B, H, W, F, K);
  // raster: valid faces (normals z >= 0, dibr.py:195), tight boxes; soft: all faces, +-boxlen*M
  FaceSet<T> rfs = dibr_faceset<T>(B, H, W, F, fvi, M);
  rfs.nz = nz;
  rfs.nz_stride = nz_stride;
  FaceSet<T> sfs = dibr_faceset<T>(B, H, W, F, fvi, M);
  sfs.margin = (T)(boxlen * M);
  sfs.has_margin = 1;
  if (!raster_uses_cull<T>()) d.rbb.cull = nullptr;
  d.rbb.cull_eps = eps;
  d.sbb.cull = nullptr;
  d.sbb.clear = d.pb.counters;
  d.sbb.n_clear = kPairClear;  // the pair pipeline's counters and record cursor
  if (iou.gt) {  // the IoU accumulators start at zero (kd_bin_count)
    d.sbb.clear_b = (int *)iou.acc;
    d.sbb.n_clear_b = 4 * kIouParts * B;
  }
  RasterFwdArgs<T> ra{rfs, d.rbb, fvz, fvz_fs, fvz_cs, feat, D, eps, interp, face_idx, weights};
  SoftArgs<T> sa{};
  sa.fs = sfs;
  sa.bb = d.sbb;
  sa.face_idx = face_idx;
  sa.K = K;
  sa.sigmainv = sigmainv;
  sa.soft = soft;
  // the backward's gradient buffers are zeroed by the soft reduction (latency-bound, so the
  // fill is nearly free there) instead of a fill launch of the backward
  sa.zero0 = gz_fvi;
  sa.nzero0 = gz_fvi ? nf * 6 : 0;
  sa.zero1 = gz_feat;
  sa.nzero1 = gz_feat ? nf * 3 * D : 0;
  sa.iou_gt = iou.gt;
  sa.iou_acc = iou.acc;
  sa.iou_B = B;
  sa.prob = prob;  // the close-face lists (dibr_soft_mask_cuda.cu:165-171)
  sa.cidx = cidx;
  sa.ctype = ctype;
  const bool fusable = dibr_fwd_fusable(ra, sa);  // (fp32 and fp64)
  // the one-launch fp32 forward's tile history (kd_set_tile_history): the previous same-shape
  // call's tile durations order this call's tiles (tile_order) and this call records its own --
  // only on the launch that writes it (the fused forward), so no other form reads a history
  if (std::is_same<T, float>::value && fusable) {
    const int64_t nt = (int64_t)((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    uint64_t tag = 1469598103934665603ull;  // FNV-1a over the shape and the hooks
    for (const int64_t x : {(int64_t)B, (int64_t)H, (int64_t)W, F, (int64_t)K,
                            (int64_t)tile_split(), (int64_t)coarse_tile_hook(),
                            (int64_t)(prob != nullptr)})  // (the lists path runs whole tiles)
      tag = (tag ^ (uint64_t)x) * 1099511628211ull;
    d.rbb.hist = tile_history(4 * (int64_t)B * nt, (long long)(tag >> 1), stream);
    ra.bb.hist = d.rbb.hist;
  }
  hipError_t e = bin_faces2<T>(rfs, d.rbb, sfs, d.sbb, stream, prep);
  if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "binning: %s", hipGetErrorString(e));
  int rc = KD_OK;
  bool done = false;
  if (fusable) {
    rc = dibr_fwd_fused_launch(ra, sa, d.pb, stream);
    done = true;
  }
  if (!done) {
    rc = raster_launch<T>(ra, stream);
    if (rc == KD_OK) rc = soft_pairs_launch<T>(sa, d.pb, want_grad != 0, true, stream);
  }
  if (rc != KD_OK || !iou.gt) return rc;
  return iou_finish_launch<T>(B, kIouParts, iou.acc, iou.stats, iou.loss, stream);
}

// prepare_vertices (camera transform form) + dibr_rasterization's forward, the projection done
// by the binning count (kd_bin_count PREP), which also writes prepare_vertices' outputs: the
// DIB-R training step's forward without a kd_prepare_fwd launch and without reading the corners
// back.
template <typename T>
int prep_vertices_forward(int B, int Bv, int64_t V, int64_t F, const T *vert, const int64_t *faces,
                          const T *proj, const T *tf, T *fvc, T *fvi, T *nrm, void *stream);

template <typename T>
static int dibr_fwd_vertices(int B, int H, int W, int Bv, int64_t V, int64_t F, int D,
                             const T *vert, const int64_t *faces, const T *proj, const T *tf,
                             const T *feat, double M, float eps, float sigmainv, double boxlen,
                             int K, T *fvc, T *fvi, T *nrm, T *interp, int64_t *face_idx,
                             T *weights, T *soft, int want_grad, T *gz_fvi, T *gz_feat, void *ws,
                             size_t wsb, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0 && V >= 0, "negative size");
  KD_CHECK_ARG(Bv == 1 || Bv == B, "vertex batch must be 1 or the view count");
  KD_CHECK_ARG((int64_t)B * F == 0 || (vert && faces && proj && tf && fvc && fvi && nrm),
               "from vertices: NULL input or output");
  if ((int64_t)B * F == 0 || H == 0 || W == 0) {  // no binning: prepare_vertices alone
    const int rc = prep_vertices_forward<T>(B, Bv, V, F, vert, faces, proj, tf, fvc, fvi, nrm,
                                            stream);
    if (rc != KD_OK) return rc;
    return dibr_fwd<T>(B, H, W, F, D, fvc + 2, 9, 3, fvi, feat, nrm + 2, 3, M, eps, sigmainv,
                       boxlen, K, interp, face_idx, weights, soft, want_grad, gz_fvi, gz_feat,
                       ws, wsb, stream);
  }
  const PrepOut<T> prep{PrepArgs<T>{B, Bv, V, F, vert, faces, proj, tf}, fvc, fvi, nrm};
  return dibr_fwd<T>(B, H, W, F, D, fvc + 2, 9, 3, fvi, feat, nrm + 2, 3, M, eps, sigmainv,
                     boxlen, K, interp, face_idx, weights, soft, want_grad, gz_fvi, gz_feat, ws,
                     wsb, stream, IouIo<T>{}, &prep);
}

template <typename T>
static int dibr_bwd(int B, int H, int W, int64_t F, int D, const T *grad_interp,
                    const T *grad_soft, const int64_t *face_idx, const T *weights, const T *soft,
                    const T *fvi, const T *feat, float eps, double M, double boxlen,
                    float sigmainv, int K, T *gfvi, T *gfeat, int zeroed, void *ws, size_t wsb,
                    void *stream_, const IouIo<T> &iou = IouIo<T>{}) {
  hipStream_t stream = (hipStream_t)stream_;
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0, "negative size");
  KD_CHECK_ARG(K >= 1 && K <= 65535, "knum must be in [1, 65535]");
  KD_CHECK_ARG(gfvi, "grad_fvi is NULL");
  const size_t need = dibr_workspace_bytes(B, H, W, F, K, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  const int64_t nf = (int64_t)B * F;
  int rc = zeroed ? KD_OK : zero_buffers<T>(gfvi, nf * 6, gfeat, gfeat ? nf * 3 * D : 0, stream);
  if (rc != KD_OK || B == 0 || H == 0 || W == 0) return rc;
  KD_CHECK_ARG(!iou.gt || (iou.stats && iou.grad), "mask_iou: NULL stats / gradient");
  if (grad_soft || iou.gt) {
    DibrBuffers<T> d = dibr_carve<T>(ws, B, H, W, F, K);
    SoftArgs<T> sa{};
    sa.fs = dibr_faceset<T>(B, H, W, F, fvi, M);
    sa.fs.margin = (T)(boxlen * M);
    sa.fs.has_margin = 1;
    sa.bb = d.sbb;
    sa.face_idx = face_idx;
    sa.K = K;
    sa.sigmainv = sigmainv;
    sa.grad_soft = grad_soft;
    sa.soft_in = soft;
    sa.grad_fvi = gfvi;
    sa.iou_gt = iou.gt;
    sa.iou_stats = iou.stats;
    sa.iou_grad = iou.grad;
    sa.iou_B = B;
    if (grad_interp && D <= 3 && !(test_forms() & KD_FORM_SPLIT_BWD)) {
      // both backwards in one launch (kd_dibr_bwd)
      const RasterBwdArgs<T> ra{B,   H,    W,   F,    D,     grad_interp, face_idx,
                                weights, fvi, feat, eps, gfvi, gfeat, debug_flags()};
      return dibr_backward_merged_launch<T>(sa, d.pb, ra, stream);
    }
    rc = soft_pairs_backward_launch<T>(sa, d.pb, stream);
    if (rc != KD_OK) return rc;
  }
  if (grad_interp)
    rc = raster_backward_launch<T>(B, H, W, F, D, grad_interp, face_idx, weights, fvi, feat, eps,
                                   gfvi, gfeat, stream);
  return rc;
}

// The backward with the face -> vertex step fused (VertexOut): the raster and
// soft-mask corner gradients go straight to the vertex gradient (Bv, V, 3); no grad_fvi.
template <typename T>
static int dibr_bwd_vtx(int B, int H, int W, int64_t F, int D, const T *grad_interp,
                        const T *grad_soft, const int64_t *face_idx, const T *weights,
                        const T *soft, const T *fvi, const T *feat, float eps, double M,
                        double boxlen, float sigmainv, int K, int Bv, int64_t V,
                        const int64_t *faces, const T *fvc, const T *proj, const T *tf,
                        T *gvert, T *gfeat, int feat_zeroed, void *ws, size_t wsb,
                        void *stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && D >= 0 && V >= 0, "negative size");
  KD_CHECK_ARG(K >= 1 && K <= 65535, "knum must be in [1, 65535]");
  KD_CHECK_ARG(D <= 3, "vertex backward: feature dim > 3 (use the grad_fvi backward)");
  KD_CHECK_ARG(Bv == 1 || Bv == B, "vertex batch must be 1 or the view count");
  KD_CHECK_ARG(gvert && (F == 0 || (faces && fvc && proj && tf)), "vertex backward: NULL input");
  const size_t need = dibr_workspace_bytes(B, H, W, F, K, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  if ((int64_t)Bv * V > 0) {
    const hipError_t e = zero_words(gvert, sizeof(T) * 3 * (size_t)Bv * (size_t)V, stream);
    if (e != hipSuccess) return set_error(KD_ERR_LAUNCH, "memset: %s", hipGetErrorString(e));
  }
  const int64_t nf = (int64_t)B * F;
  int rc = feat_zeroed || !gfeat ? KD_OK
                                 : zero_buffers<T>(gfeat, nf * 3 * D, (T *)nullptr, 0, stream);
  if (rc != KD_OK || B == 0 || H == 0 || W == 0 || F == 0) return rc;
  DibrBuffers<T> d = dibr_carve<T>(ws, B, H, W, F, K);
  const VertexOut<T> vo{gvert, faces, fvc, proj, tf, F, V, Bv};
  SoftArgs<T> sa{};
  sa.fs = dibr_faceset<T>(B, H, W, F, fvi, M);
  sa.fs.margin = (T)(boxlen * M);
  sa.fs.has_margin = 1;
  sa.bb = d.sbb;
  sa.face_idx = face_idx;
  sa.K = K;
  sa.sigmainv = sigmainv;
  sa.grad_soft = grad_soft;
  sa.soft_in = soft;
  sa.vo = vo;
  const RasterBwdArgs<T> ra{B,   H,    W,   F,     D,     grad_interp,   face_idx, weights,
                            fvi, feat, eps, nullptr, gfeat, debug_flags(), vo};
  return dibr_backward_merged_launch<T>(sa, d.pb, ra, stream);
}

}  // namespace kd

using namespace kd;

extern "C" {

size_t kd_dibr_workspace_size(int B, int H, int W, int64_t F, int knum, int double_precision) {
  if (B < 0 || H < 0 || W < 0 || F < 0 || knum < 1) return 0;
  return dibr_workspace_bytes(B, H, W, F, knum, double_precision ? 8 : 4);
}

int64_t kd_dibr_pair_count(const void *ws, int B, int H, int W, int64_t F, int knum,
                           int double_precision, void *stream) {
  if (!ws || B <= 0 || H <= 0 || W <= 0 || knum < 1) return 0;
  void *w = const_cast<void *>(ws);
  // the records are those of the work items (every fused form writes them)
  const int32_t *counters = double_precision ? dibr_carve<double>(w, B, H, W, F, knum).pb.counters
                                             : dibr_carve<float>(w, B, H, W, F, knum).pb.counters;
  const PairItem *items = double_precision ? dibr_carve<double>(w, B, H, W, F, knum).pb.items
                                           : dibr_carve<float>(w, B, H, W, F, knum).pb.items;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return -1;
  int32_t nitems = 0;
  if (hipMemcpy(&nitems, counters, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  std::vector<PairItem> it((size_t)std::max(nitems, 0));
  if (nitems > 0 && hipMemcpy(it.data(), items, sizeof(PairItem) * it.size(),
                              hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  int64_t n = 0;
  for (const PairItem &x : it) n += x.n;
  return n;
}

int kd_dibr_rasterization_forward_f32(int B, int H, int W, int64_t F, int D, const float *fvz,
                                      int64_t fvz_face_stride, int64_t fvz_corner_stride,
                                      const float *fvi, const float *feat,
                                      const float *normals_z, int64_t normals_z_stride, double M,
                                      float eps, float sigmainv, double boxlen, int knum,
                                      float *interp, int64_t *face_idx, float *weights,
                                      float *soft, int want_grad, float *grad_fvi_zero,
                                      float *grad_feat_zero, void *ws, size_t wsb, void *stream) {
  return dibr_fwd<float>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                         normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                         face_idx, weights, soft, want_grad, grad_fvi_zero, grad_feat_zero, ws,
                         wsb, stream);
}
int kd_dibr_rasterization_forward_lists_f32(
    int B, int H, int W, int64_t F, int D, const float *fvz, int64_t fvz_face_stride,
    int64_t fvz_corner_stride, const float *fvi, const float *feat, const float *normals_z,
    int64_t normals_z_stride, double M, float eps, float sigmainv, double boxlen, int knum,
    float *interp, int64_t *face_idx, float *weights, float *soft, float *prob, int64_t *cidx,
    uint8_t *ctype, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(prob && cidx && ctype, "close lists: NULL output");
  return dibr_fwd<float>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                         normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                         face_idx, weights, soft, 0, nullptr, nullptr, ws, wsb, stream,
                         IouIo<float>{}, nullptr, prob, cidx, ctype);
}
int kd_dibr_rasterization_forward_lists_f64(
    int B, int H, int W, int64_t F, int D, const double *fvz, int64_t fvz_face_stride,
    int64_t fvz_corner_stride, const double *fvi, const double *feat, const double *normals_z,
    int64_t normals_z_stride, double M, float eps, float sigmainv, double boxlen, int knum,
    double *interp, int64_t *face_idx, double *weights, double *soft, double *prob,
    int64_t *cidx, uint8_t *ctype, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(prob && cidx && ctype, "close lists: NULL output");
  return dibr_fwd<double>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                          normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                          face_idx, weights, soft, 0, nullptr, nullptr, ws, wsb, stream,
                          IouIo<double>{}, nullptr, prob, cidx, ctype);
}
}  // extern "C"

namespace kd {
template <typename T>
int soft_backward(int B, int H, int W, int64_t F, int K, const T *grad_soft, const T *soft,
                  const int64_t *face_idx, const T *prob, const int64_t *cidx,
                  const uint8_t *ctype, const T *fvi, float sigmainv, float M, T *grad_fvi,
                  hipStream_t stream, const int32_t *row_n);

// dibr_soft_mask's backward over the close-face lists of kd_dibr_rasterization_forward_lists_*,
// with that forward's workspace: its per-pixel row lengths let the lists backward skip the rows
// without listed faces exactly (their terms are all zero), without reading them.
template <typename T>
static int soft_bwd_lists_ws(int B, int H, int W, int64_t F, int K, const T *gs, const T *soft,
                             const int64_t *fidx, const T *prob, const int64_t *cidx,
                             const uint8_t *ctype, const T *fvi_scaled, float sigmainv, float M,
                             T *gfvi, const void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(B >= 0 && H >= 0 && W >= 0 && F >= 0 && K >= 1, "negative size");
  const size_t need = dibr_workspace_bytes(B, H, W, F, K, sizeof(T));
  if (wsb < need || (need && !ws))
    return set_error(KD_ERR_WORKSPACE, "workspace too small: %zu < %zu", wsb, need);
  const int32_t *row_n =
      (B && H && W) ? dibr_carve<T>(const_cast<void *>(ws), B, H, W, F, K).pb.npix : nullptr;
  return soft_backward<T>(B, H, W, F, K, gs, soft, fidx, prob, cidx, ctype, fvi_scaled, sigmainv,
                          M, gfvi, (hipStream_t)stream, row_n);
}
}  // namespace kd

extern "C" {

int kd_dibr_rasterization_soft_backward_lists_f32(
    int B, int H, int W, int64_t F, int knum, const float *grad_soft, const float *soft,
    const int64_t *face_idx, const float *prob, const int64_t *cidx, const uint8_t *ctype,
    const float *fvi_scaled, float sigmainv, float M, float *grad_fvi, const void *ws,
    size_t wsb, void *stream) {
  return soft_bwd_lists_ws<float>(B, H, W, F, knum, grad_soft, soft, face_idx, prob, cidx, ctype,
                                  fvi_scaled, sigmainv, M, grad_fvi, ws, wsb, stream);
}
int kd_dibr_rasterization_soft_backward_lists_f64(
    int B, int H, int W, int64_t F, int knum, const double *grad_soft, const double *soft,
    const int64_t *face_idx, const double *prob, const int64_t *cidx, const uint8_t *ctype,
    const double *fvi_scaled, float sigmainv, float M, double *grad_fvi, const void *ws,
    size_t wsb, void *stream) {
  return soft_bwd_lists_ws<double>(B, H, W, F, knum, grad_soft, soft, face_idx, prob, cidx,
                                   ctype, fvi_scaled, sigmainv, M, grad_fvi, ws, wsb, stream);
}
int kd_dibr_rasterization_forward_vertices_f32(
    int B, int H, int W, int vertex_batch, int64_t V, int64_t F, int D, const float *vertices,
    const int64_t *faces, const float *camera_proj, const float *camera_transform,
    const float *feat, double M, float eps, float sigmainv, double boxlen, int knum, float *fvc,
    float *fvi, float *normals, float *interp, int64_t *face_idx, float *weights, float *soft,
    int want_grad, float *grad_fvi_zero, float *grad_feat_zero, void *ws, size_t wsb,
    void *stream) {
  return dibr_fwd_vertices<float>(B, H, W, vertex_batch, V, F, D, vertices, faces, camera_proj,
                                  camera_transform, feat, M, eps, sigmainv, boxlen, knum, fvc, fvi,
                                  normals, interp, face_idx, weights, soft, want_grad,
                                  grad_fvi_zero, grad_feat_zero, ws, wsb, stream);
}
int kd_dibr_rasterization_forward_vertices_f64(
    int B, int H, int W, int vertex_batch, int64_t V, int64_t F, int D, const double *vertices,
    const int64_t *faces, const double *camera_proj, const double *camera_transform,
    const double *feat, double M, float eps, float sigmainv, double boxlen, int knum, double *fvc,
    double *fvi, double *normals, double *interp, int64_t *face_idx, double *weights,
    double *soft, int want_grad, double *grad_fvi_zero, double *grad_feat_zero, void *ws,
    size_t wsb, void *stream) {
  return dibr_fwd_vertices<double>(B, H, W, vertex_batch, V, F, D, vertices, faces, camera_proj,
                                   camera_transform, feat, M, eps, sigmainv, boxlen, knum, fvc,
                                   fvi, normals, interp, face_idx, weights, soft, want_grad,
                                   grad_fvi_zero, grad_feat_zero, ws, wsb, stream);
}
int kd_dibr_rasterization_forward_f64(int B, int H, int W, int64_t F, int D, const double *fvz,
                                      int64_t fvz_face_stride, int64_t fvz_corner_stride,
                                      const double *fvi, const double *feat,
                                      const double *normals_z, int64_t normals_z_stride,
                                      double M, float eps, float sigmainv, double boxlen,
                                      int knum, double *interp, int64_t *face_idx,
                                      double *weights, double *soft, int want_grad,
                                      double *grad_fvi_zero, double *grad_feat_zero, void *ws,
                                      size_t wsb, void *stream) {
  return dibr_fwd<double>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                          normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                          face_idx, weights, soft, want_grad, grad_fvi_zero, grad_feat_zero, ws,
                          wsb, stream);
}
int kd_dibr_rasterization_backward_f32(int B, int H, int W, int64_t F, int D,
                                       const float *grad_interp, const float *grad_soft,
                                       const int64_t *face_idx, const float *weights,
                                       const float *soft, const float *fvi, const float *feat,
                                       float eps, double M, double boxlen, float sigmainv,
                                       int knum, float *grad_fvi, float *grad_feat,
                                       int grads_zeroed, void *ws, size_t wsb, void *stream) {
  return dibr_bwd<float>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft, fvi,
                         feat, eps, M, boxlen, sigmainv, knum, grad_fvi, grad_feat, grads_zeroed,
                         ws, wsb, stream);
}
int kd_dibr_rasterization_backward_f64(int B, int H, int W, int64_t F, int D,
                                       const double *grad_interp, const double *grad_soft,
                                       const int64_t *face_idx, const double *weights,
                                       const double *soft, const double *fvi,
                                       const double *feat, float eps, double M, double boxlen,
                                       float sigmainv, int knum, double *grad_fvi,
                                       double *grad_feat, int grads_zeroed, void *ws,
                                       size_t wsb, void *stream) {
  return dibr_bwd<double>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft, fvi,
                          feat, eps, M, boxlen, sigmainv, knum, grad_fvi, grad_feat,
                          grads_zeroed, ws, wsb, stream);
}

int kd_dibr_rasterization_iou_forward_f32(
    int B, int H, int W, int64_t F, int D, const float *fvz, int64_t fvz_face_stride,
    int64_t fvz_corner_stride, const float *fvi, const float *feat, const float *normals_z,
    int64_t normals_z_stride, double M, float eps, float sigmainv, double boxlen, int knum,
    const float *gt_mask, float *interp, int64_t *face_idx, float *weights, float *soft,
    float *iou_loss, float *iou_stats, double *iou_acc, int want_grad, float *grad_fvi_zero,
    float *grad_feat_zero, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(gt_mask, "mask_iou: gt_mask is NULL");
  return dibr_fwd<float>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                         normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                         face_idx, weights, soft, want_grad, grad_fvi_zero, grad_feat_zero, ws,
                         wsb, stream, IouIo<float>{gt_mask, iou_loss, iou_stats, iou_acc, nullptr});
}
int kd_dibr_rasterization_iou_forward_f64(
    int B, int H, int W, int64_t F, int D, const double *fvz, int64_t fvz_face_stride,
    int64_t fvz_corner_stride, const double *fvi, const double *feat, const double *normals_z,
    int64_t normals_z_stride, double M, float eps, float sigmainv, double boxlen, int knum,
    const double *gt_mask, double *interp, int64_t *face_idx, double *weights, double *soft,
    double *iou_loss, double *iou_stats, double *iou_acc, int want_grad, double *grad_fvi_zero,
    double *grad_feat_zero, void *ws, size_t wsb, void *stream) {
  KD_CHECK_ARG(gt_mask, "mask_iou: gt_mask is NULL");
  return dibr_fwd<double>(B, H, W, F, D, fvz, fvz_face_stride, fvz_corner_stride, fvi, feat,
                          normals_z, normals_z_stride, M, eps, sigmainv, boxlen, knum, interp,
                          face_idx, weights, soft, want_grad, grad_fvi_zero, grad_feat_zero, ws,
                          wsb, stream,
                          IouIo<double>{gt_mask, iou_loss, iou_stats, iou_acc, nullptr});
}
int kd_dibr_rasterization_iou_backward_f32(
    int B, int H, int W, int64_t F, int D, const float *grad_interp, const float *grad_soft,
    const float *grad_iou_loss, const float *gt_mask, const float *iou_stats,
    const int64_t *face_idx, const float *weights, const float *soft, const float *fvi,
    const float *feat, float eps, double M, double boxlen, float sigmainv, int knum,
    float *grad_fvi, float *grad_feat, int grads_zeroed, void *ws, size_t wsb, void *stream) {
  return dibr_bwd<float>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft, fvi,
                         feat, eps, M, boxlen, sigmainv, knum, grad_fvi, grad_feat, grads_zeroed,
                         ws, wsb, stream,
                         IouIo<float>{grad_iou_loss ? gt_mask : nullptr, nullptr,
                                      const_cast<float *>(iou_stats), nullptr, grad_iou_loss});
}
int kd_dibr_rasterization_iou_backward_f64(
    int B, int H, int W, int64_t F, int D, const double *grad_interp, const double *grad_soft,
    const double *grad_iou_loss, const double *gt_mask, const double *iou_stats,
    const int64_t *face_idx, const double *weights, const double *soft, const double *fvi,
    const double *feat, float eps, double M, double boxlen, float sigmainv, int knum,
    double *grad_fvi, double *grad_feat, int grads_zeroed, void *ws, size_t wsb, void *stream) {
  return dibr_bwd<double>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft, fvi,
                          feat, eps, M, boxlen, sigmainv, knum, grad_fvi, grad_feat, grads_zeroed,
                          ws, wsb, stream,
                          IouIo<double>{grad_iou_loss ? gt_mask : nullptr, nullptr,
                                        const_cast<double *>(iou_stats), nullptr,
                                        grad_iou_loss});
}

int kd_dibr_rasterization_backward_vertices_f32(
    int B, int H, int W, int64_t F, int D, const float *grad_interp, const float *grad_soft,
    const int64_t *face_idx, const float *weights, const float *soft, const float *fvi,
    const float *feat, float eps, double M, double boxlen, float sigmainv, int knum,
    int vertex_batch, int64_t num_vertices, const int64_t *faces, const float *fvc,
    const float *camera_proj, const float *camera_transform, float *grad_vertices,
    float *grad_feat, int feat_zeroed, void *ws, size_t wsb, void *stream) {
  return dibr_bwd_vtx<float>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft, fvi,
                             feat, eps, M, boxlen, sigmainv, knum, vertex_batch, num_vertices,
                             faces, fvc, camera_proj, camera_transform, grad_vertices, grad_feat,
                             feat_zeroed, ws, wsb, stream);
}
int kd_dibr_rasterization_backward_vertices_f64(
    int B, int H, int W, int64_t F, int D, const double *grad_interp, const double *grad_soft,
    const int64_t *face_idx, const double *weights, const double *soft, const double *fvi,
    const double *feat, float eps, double M, double boxlen, float sigmainv, int knum,
    int vertex_batch, int64_t num_vertices, const int64_t *faces, const double *fvc,
    const double *camera_proj, const double *camera_transform, double *grad_vertices,
    double *grad_feat, int feat_zeroed, void *ws, size_t wsb, void *stream) {
  return dibr_bwd_vtx<double>(B, H, W, F, D, grad_interp, grad_soft, face_idx, weights, soft,
                              fvi, feat, eps, M, boxlen, sigmainv, knum, vertex_batch,
                              num_vertices, faces, fvc, camera_proj, camera_transform,
                              grad_vertices, grad_feat, feat_zeroed, ws, wsb, stream);
}

}  // extern "C"
