/*
 * kaolin_dibr.h -- C ABI of the MI355X (gfx950) DIB-R rasterization hot path.
 *
 * Plain C: pointers are DEVICE pointers (hipMalloc / torch caching allocator) unless noted,
 * sizes are plain integers, `stream` is a hipStream_t passed as void*.  Every function is
 * asynchronous on `stream`, never synchronises the host, never allocates, never frees and never
 * keeps a pointer past its return.  Every output element is written (no pre-fill needed).
 * Return value: KD_OK (0) or a KD_ERR_* code; kd_last_error() gives the message (thread-local).
 *
 * Layouts are the reference's (contiguous row-major):
 *   face_vertices_z      (B, F, 3)        face_vertices_image (B, F, 3, 2)
 *   face_features        (B, F, 3, D)     face_idx            (B, H, W) int64, -1 = empty
 *   interpolated_features(B, H, W, D)     weights             (B, H, W, 3)
 *   soft_mask            (B, H, W)        close_face_{prob,idx,dist_type} (B, H, W, K)
 * "packed" inputs are the reference's packed layout: faces of view b are rows
 * [first_idx[b], first_idx[b+1]) of (Fp, ...) arrays; first_idx (B+1) int64 lives on the device.
 *
 * The `_f32` / `_f64` suffix is the scalar type (reference: AT_DISPATCH float / double).
 */
#ifndef KAOLIN_DIBR_H_
#define KAOLIN_DIBR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KD_OK 0
#define KD_ERR_INVALID_ARGUMENT 1
#define KD_ERR_LAUNCH 2
#define KD_ERR_WORKSPACE 3

/* Workspace kinds for kd_workspace_size(). */
#define KD_WS_RASTER_PACKED 1 /* kd_packed_rasterize_forward_*      */
#define KD_WS_RASTER 2        /* kd_rasterize_forward_*             */
#define KD_WS_SOFT_MASK 3     /* kd_dibr_soft_mask_forward_* (op form)                    */

/* Bytes of device workspace the call of `kind` needs.  num_faces_total = rows of the face arrays
 * (Fp for the packed layout, B*F otherwise); max_faces_per_view = the largest per-view count
 * (Fp when unknown on the host, F otherwise). */
size_t kd_workspace_size(int kind, int batch, int height, int width, int64_t num_faces_total,
                         int64_t max_faces_per_view);

const char *kd_last_error(void);
int kd_version(void);

/* In-library kernel timing (HIP events recorded around every launch on the launch stream).
 * kd_profile_enable(1) starts recording; kd_profile_collect() waits for the recorded events,
 * adds each kernel's elapsed milliseconds / launch count into total_ms[id] / launches[id]
 * (arrays of n entries), clears the records and returns min(n, number of kernel ids).
 * kd_profile_kernel_name(id) names them.  Not for use under stream capture. */
void kd_profile_enable(int on);
int kd_profile_collect(double *total_ms, int64_t *launches, int n);
const char *kd_profile_kernel_name(int id);

/* Diagnostics only: ablation switches read by the kernels of the diagnostic build
 * (libkaolin_dibr_diag.so), and (flag 64) a device int64 array of 3 * views * tiles entries
 * receiving per-tile durations (100 MHz ticks) of the raster forward / soft forward / soft
 * backward tile kernels.  The production library reads no flags: kd_debug_set returns
 * KD_ERR_INVALID_ARGUMENT there for any nonzero value. */
int kd_debug_set(int flags);
int kd_debug_buffer(void *device_ptr);

/* Launch forms (a test hook; 0 by default).  dibr_rasterization's forward and backward run as one
 * launch each; the same tile bodies also run as separate launches, which other entry points use
 * (the op forms, knum > 32, D > 3).  A test sets these bits to run dibr_rasterization through the
 * separate launches and compare.  Bits: KD_FORM_SPLIT_FWD raster then soft mask as two launches,
 * KD_FORM_SPLIT_BWD the two backwards as two launches, KD_FORM_SOFT_SPLIT the soft mask's pass A,
 * pair math and product as three launches (the K-list pipeline without the lists). */
#define KD_FORM_SPLIT_FWD 1
#define KD_FORM_SPLIT_BWD 2
#define KD_FORM_SOFT_SPLIT 4
int kd_set_test_forms(int forms);

/* Workgroups per 16x16 tile of dibr_rasterization's fp32 forward (a test and tuning hook; 0 by
 * default = chosen from the batch's tile count against the device's workgroup slots).  With 2 or
 * 4, each tile is rendered by that many workgroups (half / quarter tiles, several waves per 8x8
 * sub-tile), so that a small batch's heavy tiles spread over more CUs; results are identical.
 * Used only when the soft mask's record pool is the fixed one (knum <= 32, no pool limit). */
int kd_set_tile_split(int split);

/* Coarse bin edge of dibr_rasterization in pixels (a test and tuning hook; 0 by default = 32;
 * larger images grow it to at most 32 bins per side).  Results never depend on it.  It fixes the workspace layout of a call:
 * hold it constant between a forward and its backward (kd_dibr_workspace_size covers every
 * choice). */
int kd_set_coarse_tile(int px);

/* Tile cost history of dibr_rasterization's fp32 forward (a tuning hook; 1 by default).  The
 * one-launch forward records each 16x16 tile's duration in a CALLER-OWNED device buffer (one per
 * device, attached with kd_tile_history_attach), and the next call of the same shape dispatches
 * its tiles heaviest-first by those durations instead of by their coarse bins' face counts (a
 * silhouette tile's soft-mask work shows only after its raster phase).  Results never depend on
 * it; 0 turns it off, and so does attaching no buffer. */
int kd_set_tile_history(int on);

/* The device a stream belongs to (the null stream: the calling thread's current device) -- the
 * device whose per-device state (tile history, CU count) a call on that stream uses -- and, when
 * compute_units is not NULL, that device's CU count as the launchers see it.  Support. */
int kd_stream_device(void *stream, int *compute_units);

/* Bytes of one device's tile history buffer (2 MB). */
size_t kd_tile_history_bytes(void);

/* Attach a caller-owned device buffer of >= kd_tile_history_bytes() bytes as the tile history of
 * the device `stream` belongs to (NULL detaches).  The library never allocates or frees it and
 * keeps only its address: the caller keeps it alive while any call or captured graph on that
 * device may use it (kaolin_amd._C allocates one per device from the PyTorch caching allocator
 * and holds it for the process).  Every stream, thread and graph of the device shares it; the
 * library zeroes it on the stream when the call's shape changes outside a capture. */
int kd_tile_history_attach(void *stream, void *device_buffer, size_t bytes);

/* Pool limits (a test and tuning hook; both 1 by default).  The workspaces hold two bounded
 * pools whose layout depends only on the call's sizes: the coarse bins (16 entries per face row)
 * and the soft mask's (pixel, close face) records (min(knum, 12) per pixel plus block slack).
 * A forward uses the given fraction of each; what does not fit takes the overflow paths (a bin
 * walks all faces of its view; a tile computes its soft mask without records and its backward
 * recomputes them), which change the time, never the results.  Values in [0, 1]. */
int kd_set_pool_limits(double bin_fraction, double pair_fraction);

/* ---------------------------------------------------------------------------------------------
 * Packed rasterize forward.  Replaces _C.render.mesh.packed_rasterize_forward_cuda
 * (reference kaolin/csrc/bindings.cpp:77 -> kaolin/csrc/render/mesh/rasterization.cpp:49-104,
 * kernel rasterization_cuda.cu:43-192).  fvi and bboxes are already multiplied by `multiplier`
 * (rasterization.py:337-344).  face_idx receives the PACKED-LOCAL index (row - first_idx[b]).
 * ------------------------------------------------------------------------------------------- */
int kd_packed_rasterize_forward_f32(int batch, int height, int width, int64_t num_faces,
                                    int feat_dim, const float *fvz, const float *fvi,
                                    const float *bboxes, const float *feat,
                                    const int64_t *first_idx, float multiplier, float eps,
                                    float *interp, int64_t *face_idx, float *weights,
                                    void *workspace, size_t workspace_bytes, void *stream);
int kd_packed_rasterize_forward_f64(int batch, int height, int width, int64_t num_faces,
                                    int feat_dim, const double *fvz, const double *fvi,
                                    const double *bboxes, const double *feat,
                                    const int64_t *first_idx, float multiplier, float eps,
                                    double *interp, int64_t *face_idx, double *weights,
                                    void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Batched rasterize forward (no packing, no host sync).  Replaces RasterizeCuda.forward
 * (kaolin/render/mesh/rasterization.py:289-369: torch.where packing, x multiplier, bboxes,
 * packed->original remap) fused with the packed kernel.  fvi is NOT scaled; `valid` (B, F) uint8
 * may be NULL (all faces valid).  face_idx receives the ORIGINAL face index, exactly as
 * rasterize() returns it.  `multiplier` is the Python value (scaling is done in the scalar type
 * like torch's `tensor * multiplier`; pixel centres use (float)multiplier like the kernel).
 * ------------------------------------------------------------------------------------------- */
int kd_rasterize_forward_f32(int batch, int height, int width, int64_t num_faces, int feat_dim,
                             const float *fvz, const float *fvi, const float *feat,
                             const uint8_t *valid, double multiplier, float eps, float *interp,
                             int64_t *face_idx, float *weights, void *workspace,
                             size_t workspace_bytes, void *stream);
int kd_rasterize_forward_f64(int batch, int height, int width, int64_t num_faces, int feat_dim,
                             const double *fvz, const double *fvi, const double *feat,
                             const uint8_t *valid, double multiplier, float eps, double *interp,
                             int64_t *face_idx, double *weights, void *workspace,
                             size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Rasterize backward, general form.  Replaces _C.render.mesh.rasterize_backward_cuda
 * (bindings.cpp:78 -> rasterization.cpp:106-168, kernel rasterization_cuda.cu:238-402).  Any
 * face_idx is accepted (original index, -1 = none).  fvi is NOT scaled.  grad_feat may be NULL.
 * Pixels of one face are summed per 16x16 tile in LDS, then added with float atomics: the
 * summation order, hence the last bits, vary run to run (as in the reference).
 * ------------------------------------------------------------------------------------------- */
int kd_rasterize_backward_f32(int batch, int height, int width, int64_t num_faces, int feat_dim,
                              const float *grad_interp, const int64_t *face_idx,
                              const float *weights, const float *fvi, const float *feat,
                              float eps, float *grad_fvi, float *grad_feat, void *stream);
int kd_rasterize_backward_f64(int batch, int height, int width, int64_t num_faces, int feat_dim,
                              const double *grad_interp, const int64_t *face_idx,
                              const double *weights, const double *fvi, const double *feat,
                              float eps, double *grad_fvi, double *grad_feat, void *stream);

/* ---------------------------------------------------------------------------------------------
 * DIB-R soft mask forward.  Replaces _C.render.mesh.dibr_soft_mask_forward_cuda
 * (bindings.cpp:79 -> kaolin/csrc/render/mesh/dibr_soft_mask.cpp:48-108, kernel
 * dibr_soft_mask_cuda.cu:27-184).  fvi_scaled = fvi * multiplier, large_bboxes (B, F, 4) as
 * computed by DibrSoftMaskCuda.forward (dibr.py:31-39).  face_idx (B, H, W): >= 0 = covered.
 * close_face_idx receives the face index within the view, -1 padded.
 * ------------------------------------------------------------------------------------------- */
int kd_dibr_soft_mask_forward_f32(int batch, int height, int width, int64_t num_faces, int knum,
                                  const float *fvi_scaled, const float *large_bboxes,
                                  const int64_t *face_idx, float sigmainv, float multiplier,
                                  float *soft_mask, float *close_face_prob,
                                  int64_t *close_face_idx, uint8_t *close_face_dist_type,
                                  void *workspace, size_t workspace_bytes, void *stream);
int kd_dibr_soft_mask_forward_f64(int batch, int height, int width, int64_t num_faces, int knum,
                                  const double *fvi_scaled, const double *large_bboxes,
                                  const int64_t *face_idx, float sigmainv, float multiplier,
                                  double *soft_mask, double *close_face_prob,
                                  int64_t *close_face_idx, uint8_t *close_face_dist_type,
                                  void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * DIB-R soft mask forward from UNSCALED fvi (DibrSoftMaskCuda.forward dibr.py:29-55 fused: the
 * x multiplier and the +-boxlen*multiplier bounding boxes are computed in the kernels).
 * close_last (B, H, W) int32, if not NULL, receives per pixel the K-th close face when the list
 * is full, else -1.  The three close_face_* lists may all be NULL (then they are not
 * materialised).  Workspace: kd_soft_mask_workspace_size().  With want_grad != 0 the workspace
 * also receives every (pixel, close face) pair's backward coefficients; keep it for
 * kd_dibr_soft_mask_backward_binned_* (bins_ready = 1).
 * ------------------------------------------------------------------------------------------- */
size_t kd_soft_mask_workspace_size(int batch, int height, int width, int64_t num_faces, int knum,
                                   int double_precision);
int kd_dibr_soft_mask_forward_fused_f32(int batch, int height, int width, int64_t num_faces,
                                        int knum, const float *fvi, double multiplier,
                                        double boxlen, const int64_t *face_idx, float sigmainv,
                                        float *soft_mask, float *close_face_prob,
                                        int64_t *close_face_idx, uint8_t *close_face_dist_type,
                                        int32_t *close_last, int want_grad, void *workspace,
                                        size_t workspace_bytes, void *stream);
int kd_dibr_soft_mask_forward_fused_f64(int batch, int height, int width, int64_t num_faces,
                                        int knum, const double *fvi, double multiplier,
                                        double boxlen, const int64_t *face_idx, float sigmainv,
                                        double *soft_mask, double *close_face_prob,
                                        int64_t *close_face_idx, uint8_t *close_face_dist_type,
                                        int32_t *close_last, int want_grad, void *workspace,
                                        size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * DIB-R soft mask backward, general form.  Replaces _C.render.mesh.dibr_soft_mask_backward_cuda
 * (bindings.cpp:80 -> dibr_soft_mask.cpp:110-183, kernel dibr_soft_mask_cuda.cu:230-353).
 * Returns the gradient w.r.t. the unscaled coordinates, like the reference op.  Float atomics.
 * ------------------------------------------------------------------------------------------- */
int kd_dibr_soft_mask_backward_f32(int batch, int height, int width, int64_t num_faces, int knum,
                                   const float *grad_soft_mask, const float *soft_mask,
                                   const int64_t *face_idx, const float *close_face_prob,
                                   const int64_t *close_face_idx,
                                   const uint8_t *close_face_dist_type, const float *fvi_scaled,
                                   float sigmainv, float multiplier, float *grad_fvi,
                                   void *stream);
int kd_dibr_soft_mask_backward_f64(int batch, int height, int width, int64_t num_faces, int knum,
                                   const double *grad_soft_mask, const double *soft_mask,
                                   const int64_t *face_idx, const double *close_face_prob,
                                   const int64_t *close_face_idx,
                                   const uint8_t *close_face_dist_type, const double *fvi_scaled,
                                   float sigmainv, float multiplier, double *grad_fvi,
                                   void *stream);

/* ---------------------------------------------------------------------------------------------
 * DIB-R soft mask backward, autograd form (DibrSoftMaskCuda.backward dibr.py:57-73 without close
 * lists).  `workspace` is the fused forward's (want_grad = 1, same fvi / multiplier / boxlen /
 * knum, bins_ready != 0): every pair's stored coefficients times the pixel's
 * -sigmainv * grad * (1 - soft) are summed per face and tile in LDS and added with float atomics
 * (the reference's terms dibr_soft_mask_cuda.cu:281-348, up to rounding order).  With
 * bins_ready == 0 the pairs and coefficients are rebuilt first.  fvi is NOT scaled; grad_fvi is
 * the gradient w.r.t. fvi.
 * ------------------------------------------------------------------------------------------- */
int kd_dibr_soft_mask_backward_binned_f32(int batch, int height, int width, int64_t num_faces,
                                          int knum, const float *grad_soft_mask,
                                          const float *soft_mask, const int64_t *face_idx,
                                          const float *fvi, double multiplier, double boxlen,
                                          float sigmainv, float *grad_fvi, void *workspace,
                                          size_t workspace_bytes, int bins_ready, void *stream);
int kd_dibr_soft_mask_backward_binned_f64(int batch, int height, int width, int64_t num_faces,
                                          int knum, const double *grad_soft_mask,
                                          const double *soft_mask, const int64_t *face_idx,
                                          const double *fvi, double multiplier, double boxlen,
                                          float sigmainv, double *grad_fvi, void *workspace,
                                          size_t workspace_bytes, int bins_ready, void *stream);

/* ---------------------------------------------------------------------------------------------
 * dibr_rasterization (kaolin/render/mesh/dibr.py:119-209) fused: rasterize of the faces with
 * normals_z >= 0 (dibr.py:195) + dibr_soft_mask of all faces (dibr.py:201-208), one binning
 * pass for both.  fvi UNSCALED (B, F, 3, 2); face_vertices_z read at
 * fvz[(b * F + f) * fvz_face_stride + j * fvz_corner_stride] and normals_z at
 * normals_z[(b * F + f) * normals_z_stride] (views of prepare_vertices' outputs: 9, 3 and 3);
 * normals_z NULL = all faces valid.  Outputs interp (B, H, W, D), face_idx (B, H, W) int64,
 * weights (B, H, W, 3), soft (B, H, W).  With want_grad the workspace keeps what the backward
 * needs; pass the same workspace to the backward.  Workspace: kd_dibr_workspace_size().
 * The backward writes grad_fvi (B, F, 3, 2) = raster + soft-mask gradients (one buffer) and
 * grad_feat (nullable); grad_interp / grad_soft NULL = zero.  A forward with want_grad may zero
 * the backward's gradient buffers (grad_fvi_zero (B, F, 3, 2), grad_feat_zero (B, F, 3, D),
 * nullable) inside one of its kernels; the backward then takes them with grads_zeroed = 1 and
 * skips its own fill launch.
 * ------------------------------------------------------------------------------------------- */
size_t kd_dibr_workspace_size(int batch, int height, int width, int64_t num_faces, int knum,
                              int double_precision);
/* Diagnostics: number of (pixel, close face) pairs a forward left in `workspace` (synchronises
 * `stream`, copies the per-tile counts to the host). */
int64_t kd_dibr_pair_count(const void *workspace, int batch, int height, int width,
                           int64_t num_faces, int knum, int double_precision, void *stream);
int kd_dibr_rasterization_forward_f32(int batch, int height, int width, int64_t num_faces,
                                      int feat_dim, const float *fvz, int64_t fvz_face_stride,
                                      int64_t fvz_corner_stride, const float *fvi,
                                      const float *feat, const float *normals_z,
                                      int64_t normals_z_stride, double multiplier, float eps,
                                      float sigmainv, double boxlen, int knum, float *interp,
                                      int64_t *face_idx, float *weights, float *soft,
                                      int want_grad, float *grad_fvi_zero, float *grad_feat_zero,
                                      void *workspace, size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_forward_f64(int batch, int height, int width, int64_t num_faces,
                                      int feat_dim, const double *fvz, int64_t fvz_face_stride,
                                      int64_t fvz_corner_stride, const double *fvi,
                                      const double *feat, const double *normals_z,
                                      int64_t normals_z_stride, double multiplier, float eps,
                                      float sigmainv, double boxlen, int knum, double *interp,
                                      int64_t *face_idx, double *weights, double *soft,
                                      int want_grad, double *grad_fvi_zero, double *grad_feat_zero,
                                      void *workspace, size_t workspace_bytes, void *stream);
/* The same forward keeping the close-face lists of its soft mask (dibr.py's DibrSoftMaskCuda
 * inside the reference composition, dibr.py:193-208, dibr_soft_mask_cuda.cu:165-171): prob
 * (B, H, W, knum), cidx (B, H, W, knum) int64 (-1 = empty), ctype (B, H, W, knum) uint8, read
 * by kd_dibr_soft_mask_backward_* (with kd_rasterize_backward_* for the raster part).  No
 * workspace backward (want_grad 0). */
/* dibr_soft_mask's backward (as kd_dibr_soft_mask_backward_*) over the close-face lists that
 * kd_dibr_rasterization_forward_lists_* wrote, given that forward's workspace (ws, wsb as it was
 * called with): its per-pixel row lengths let the rows without listed faces be skipped exactly,
 * without reading them.  fvi_scaled = face_vertices_image * multiplier.  Replaces the soft half
 * of the reference composition's backward (dibr.py:57-73 -> dibr_soft_mask.cpp:110-183). */
int kd_dibr_rasterization_soft_backward_lists_f32(
    int batch, int height, int width, int64_t num_faces, int knum, const float *grad_soft,
    const float *soft_mask, const int64_t *face_idx, const float *close_prob,
    const int64_t *close_idx, const uint8_t *close_type, const float *fvi_scaled,
    float sigmainv, float multiplier, float *grad_fvi, const void *workspace,
    size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_soft_backward_lists_f64(
    int batch, int height, int width, int64_t num_faces, int knum, const double *grad_soft,
    const double *soft_mask, const int64_t *face_idx, const double *close_prob,
    const int64_t *close_idx, const uint8_t *close_type, const double *fvi_scaled,
    float sigmainv, float multiplier, double *grad_fvi, const void *workspace,
    size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_forward_lists_f32(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const float *fvz,
    int64_t fvz_face_stride, int64_t fvz_corner_stride, const float *fvi, const float *feat,
    const float *normals_z, int64_t normals_z_stride, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, float *interp, int64_t *face_idx, float *weights,
    float *soft, float *prob, int64_t *cidx, uint8_t *ctype, void *workspace,
    size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_forward_lists_f64(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const double *fvz,
    int64_t fvz_face_stride, int64_t fvz_corner_stride, const double *fvi, const double *feat,
    const double *normals_z, int64_t normals_z_stride, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, double *interp, int64_t *face_idx, double *weights,
    double *soft, double *prob, int64_t *cidx, uint8_t *ctype, void *workspace,
    size_t workspace_bytes, void *stream);
/* The same forward from the vertices (prepare_vertices, camera transform form,
 * kaolin/render/mesh/utils.py:128-175, followed by dibr_rasterization of its outputs, the DIB-R
 * training step of examples/tutorial/ian_dibr.py): vertices (vertex_batch, V, 3) with
 * vertex_batch 1 or batch, faces (F, 3) int64, camera_proj (3), camera_transform (batch, 4, 3).
 * Writes prepare_vertices' outputs fvc (batch, F, 3, 3), fvi (batch, F, 3, 2) and normals
 * (batch, F, 3) -- the projection runs inside the binning launch, which writes them -- and
 * renders with face_vertices_z = fvc[..., 2], face_vertices_image = fvi, face_normals_z =
 * normals[..., 2]; every output equals kd_prepare_vertices_forward followed by
 * kd_dibr_rasterization_forward.  Its backward: kd_dibr_rasterization_backward_* for grad_fvi,
 * then kd_prepare_vertices_backward_*; or kd_dibr_rasterization_backward_vertices_*. */
int kd_dibr_rasterization_forward_vertices_f32(
    int batch, int height, int width, int vertex_batch, int64_t num_vertices, int64_t num_faces,
    int feat_dim, const float *vertices, const int64_t *faces, const float *camera_proj,
    const float *camera_transform, const float *feat, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, float *fvc, float *fvi, float *normals,
    float *interp, int64_t *face_idx, float *weights, float *soft, int want_grad,
    float *grad_fvi_zero, float *grad_feat_zero, void *workspace, size_t workspace_bytes,
    void *stream);
int kd_dibr_rasterization_forward_vertices_f64(
    int batch, int height, int width, int vertex_batch, int64_t num_vertices, int64_t num_faces,
    int feat_dim, const double *vertices, const int64_t *faces, const double *camera_proj,
    const double *camera_transform, const double *feat, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, double *fvc, double *fvi, double *normals,
    double *interp, int64_t *face_idx, double *weights, double *soft, int want_grad,
    double *grad_fvi_zero, double *grad_feat_zero, void *workspace, size_t workspace_bytes,
    void *stream);
int kd_dibr_rasterization_backward_f32(int batch, int height, int width, int64_t num_faces,
                                       int feat_dim, const float *grad_interp,
                                       const float *grad_soft, const int64_t *face_idx,
                                       const float *weights, const float *soft, const float *fvi,
                                       const float *feat, float eps, double multiplier,
                                       double boxlen, float sigmainv, int knum, float *grad_fvi,
                                       float *grad_feat, int grads_zeroed, void *workspace,
                                       size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_backward_f64(int batch, int height, int width, int64_t num_faces,
                                       int feat_dim, const double *grad_interp,
                                       const double *grad_soft, const int64_t *face_idx,
                                       const double *weights, const double *soft,
                                       const double *fvi, const double *feat, float eps,
                                       double multiplier, double boxlen, float sigmainv,
                                       int knum, double *grad_fvi, double *grad_feat,
                                       int grads_zeroed, void *workspace, size_t workspace_bytes,
                                       void *stream);
/* dibr_rasterization with the silhouette loss fused in (mask_iou of
 * kaolin/metrics/render.py:18-40 applied to the soft mask, as in the DIB-R training loop
 * examples/tutorial/ian_dibr.py:264-265): the forward above, plus
 *   iou_loss (scalar) = 1 - mean_b(U_b / (D_b + 1e-10)),  U_b = sum(s g), D_b = sum(s + g - s g)
 * over soft_mask s and gt_mask g (B, H, W), with the per-pixel terms in T, accumulated in fp64
 * inside the soft mask's tile launch (iou_acc, B x 32 x 2 doubles of partials, scratch) and
 * finished like
 * kd_mask_iou_forward_* does; iou_stats = (U_b, D_b) in T, B x 2.  knum <= 32.
 * The backward adds d iou_loss / d soft_mask -- the arithmetic of kd_mask_iou_backward_*, its
 * incoming gradient the DEVICE scalar grad_iou_loss (nullable) -- to grad_soft (nullable) per pixel
 * inside the soft mask's backward: no (B, H, W) gradient of the mask is materialised. */
int kd_dibr_rasterization_iou_forward_f32(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const float *fvz,
    int64_t fvz_face_stride, int64_t fvz_corner_stride, const float *fvi, const float *feat,
    const float *normals_z, int64_t normals_z_stride, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, const float *gt_mask, float *interp,
    int64_t *face_idx, float *weights, float *soft, float *iou_loss, float *iou_stats,
    double *iou_acc, int want_grad, float *grad_fvi_zero, float *grad_feat_zero,
    void *workspace, size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_iou_forward_f64(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const double *fvz,
    int64_t fvz_face_stride, int64_t fvz_corner_stride, const double *fvi, const double *feat,
    const double *normals_z, int64_t normals_z_stride, double multiplier, float eps,
    float sigmainv, double boxlen, int knum, const double *gt_mask, double *interp,
    int64_t *face_idx, double *weights, double *soft, double *iou_loss, double *iou_stats,
    double *iou_acc, int want_grad, double *grad_fvi_zero, double *grad_feat_zero,
    void *workspace, size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_iou_backward_f32(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const float *grad_interp,
    const float *grad_soft, const float *grad_iou_loss, const float *gt_mask,
    const float *iou_stats, const int64_t *face_idx, const float *weights, const float *soft,
    const float *fvi, const float *feat, float eps, double multiplier, double boxlen,
    float sigmainv, int knum, float *grad_fvi, float *grad_feat, int grads_zeroed,
    void *workspace, size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_iou_backward_f64(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const double *grad_interp,
    const double *grad_soft, const double *grad_iou_loss, const double *gt_mask,
    const double *iou_stats, const int64_t *face_idx, const double *weights, const double *soft,
    const double *fvi, const double *feat, float eps, double multiplier, double boxlen,
    float sigmainv, int knum, double *grad_fvi, double *grad_feat, int grads_zeroed,
    void *workspace, size_t workspace_bytes, void *stream);
/* The same backward with the face -> vertex step of prepare_vertices fused in (SURVEY.md §8 f1;
 * reference: the gather backward of kaolin/ops/mesh/mesh.py:24-45 with the projection and camera
 * transform of kaolin/render/mesh/utils.py:164-167 and render/camera/legacy.py:120-139): the raster
 * and soft-mask corner gradients go straight to grad_vertices (vertex_batch, num_vertices, 3) --
 * summed over the views when vertex_batch == 1 -- with no (B, F, 3, 2) gradient in between.
 * fvi / fvc are prepare_vertices' outputs for faces (F, 3) int64, camera_proj (3),
 * camera_transform (B, 4, 3); feat_dim <= 3.  grad_vertices is zeroed here; grad_feat (nullable)
 * is zeroed here unless feat_zeroed (the forward's grad_feat_zero). */
int kd_dibr_rasterization_backward_vertices_f32(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const float *grad_interp,
    const float *grad_soft, const int64_t *face_idx, const float *weights, const float *soft,
    const float *fvi, const float *feat, float eps, double multiplier, double boxlen,
    float sigmainv, int knum, int vertex_batch, int64_t num_vertices, const int64_t *faces,
    const float *fvc, const float *camera_proj, const float *camera_transform,
    float *grad_vertices, float *grad_feat, int feat_zeroed, void *workspace,
    size_t workspace_bytes, void *stream);
int kd_dibr_rasterization_backward_vertices_f64(
    int batch, int height, int width, int64_t num_faces, int feat_dim, const double *grad_interp,
    const double *grad_soft, const int64_t *face_idx, const double *weights, const double *soft,
    const double *fvi, const double *feat, float eps, double multiplier, double boxlen,
    float sigmainv, int knum, int vertex_batch, int64_t num_vertices, const int64_t *faces,
    const double *fvc, const double *camera_proj, const double *camera_transform,
    double *grad_vertices, double *grad_feat, int feat_zeroed, void *workspace,
    size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * prepare_vertices (kaolin/render/mesh/utils.py:128-175 with camera_transform): camera
 * transform (pad(v, 1) @ T), perspective projection (legacy.py:120-139), per-face gather
 * (ops/mesh/mesh.py:24-45) and unit face normals (ops/mesh/trianglemesh.py:313-336), fused.
 * vertices (Bv, V, 3) with Bv == 1 (shared by all views) or Bv == B; faces (F, 3) int64;
 * camera_proj (3); camera_transform (B, 4, 3).  Outputs fvc (B, F, 3, 3), fvi (B, F, 3, 2),
 * normals (B, F, 3).
 * The backward walks each vertex's incident (face, corner) list -- CSR adjacency: adj_offsets
 * (V + 1) int64, adj (3F) int32 entries f * 3 + corner, grouped by vertex -- and writes
 * grad_vertices (Bv, V, 3) (summed over the views when Bv == 1).  adj_ranges (num_ranges + 1)
 * int32 are the workgroups' entry ranges from kd_prepare_vertices_ranges (once per topology):
 * each vertex is summed in LDS and stored once -- no pre-fill, no global atomics.  Any of the three incoming gradients may be NULL
 * (zero).  fvc is the forward's output.
 * ------------------------------------------------------------------------------------------- */
int kd_prepare_vertices_forward_f32(int batch, int vertex_batch, int64_t num_vertices,
                                    int64_t num_faces, const float *vertices,
                                    const int64_t *faces, const float *camera_proj,
                                    const float *camera_transform, float *fvc, float *fvi,
                                    float *normals, void *stream);
int kd_prepare_vertices_forward_f64(int batch, int vertex_batch, int64_t num_vertices,
                                    int64_t num_faces, const double *vertices,
                                    const int64_t *faces, const double *camera_proj,
                                    const double *camera_transform, double *fvc, double *fvi,
                                    double *normals, void *stream);
int kd_prepare_vertices_backward_f32(int batch, int vertex_batch, int64_t num_vertices,
                                     int64_t num_faces, const int64_t *faces,
                                     const float *camera_proj, const float *camera_transform,
                                     const float *fvc, const float *grad_fvc,
                                     const float *grad_fvi, const float *grad_normals,
                                     const int64_t *adj_offsets, const int32_t *adj,
                                     const int32_t *adj_ranges, int64_t num_ranges,
                                     float *grad_vertices, void *stream);
int kd_prepare_vertices_backward_f64(int batch, int vertex_batch, int64_t num_vertices,
                                     int64_t num_faces, const int64_t *faces,
                                     const double *camera_proj, const double *camera_transform,
                                     const double *fvc, const double *grad_fvc,
                                     const double *grad_fvi, const double *grad_normals,
                                     const int64_t *adj_offsets, const int32_t *adj,
                                     const int32_t *adj_ranges, int64_t num_ranges,
                                     double *grad_vertices, void *stream);
/* The same backward for grad_fvi alone (grad_fvc and grad_normals zero: the DIB-R training
 * step, where face_vertices_z and the normals only select faces), from the vertices instead of
 * fvc: each corner's camera-space point is recomputed per view with the forward's arithmetic (the
 * bits of fvc), so only the corner's grad_fvi is gathered per (entry, view).  Same result, bit
 * for bit, as kd_prepare_vertices_backward_* with the forward's fvc (up to the order of the
 * LDS sums of a vertex's entries).  adj_vertex (3F) int32: the vertex of each CSR entry (the
 * chain entry -> face row -> vertex becomes one load). */
int kd_prepare_vertices_backward_vertices_f32(int batch, int vertex_batch, int64_t num_vertices,
                                              int64_t num_faces, const float *vertices,
                                              const int64_t *faces, const float *camera_proj,
                                              const float *camera_transform,
                                              const float *grad_fvi, const int64_t *adj_offsets,
                                              const int32_t *adj, const int32_t *adj_vertex,
                                              const int32_t *adj_ranges,
                                              int64_t num_ranges, float *grad_vertices,
                                              void *stream);
int kd_prepare_vertices_backward_vertices_f64(int batch, int vertex_batch, int64_t num_vertices,
                                              int64_t num_faces, const double *vertices,
                                              const int64_t *faces, const double *camera_proj,
                                              const double *camera_transform,
                                              const double *grad_fvi, const int64_t *adj_offsets,
                                              const int32_t *adj, const int32_t *adj_vertex,
                                              const int32_t *adj_ranges,
                                              int64_t num_ranges, double *grad_vertices,
                                              void *stream);
/* Host function (host memory): workgroup entry ranges of the prepare_vertices backward from the
 * CSR offsets (V + 1): greedy, whole vertices, at most `cap` (<= 256) entries per range unless one
 * vertex alone has more.  ranges_out holds at least V + 2 values; returns the range count. */
int64_t kd_prepare_vertices_ranges(const int64_t *adj_offsets, int64_t num_vertices, int32_t cap,
                                   int32_t *ranges_out);

/* ---------------------------------------------------------------------------------------------
 * mask_iou (kaolin/metrics/render.py:18-40): loss = 1 - mean_b(U_b / (D_b + 1e-10)) with
 * U_b = sum(l * r), D_b = sum(l + r - l * r) over the `pixels` elements of view b.  lhs / rhs
 * (B, pixels) contiguous.  The forward writes the scalar loss, stats (B, 2) = (U_b, D_b) for the
 * backward and, when `iou` is not NULL, the per-view IoU (B).  Workspace:
 * kd_mask_iou_workspace_size.  The backward reads the incoming gradient from the DEVICE scalar
 * grad_loss and writes grad_lhs / grad_rhs (either may be NULL).
 * ------------------------------------------------------------------------------------------- */
size_t kd_mask_iou_workspace_size(int batch, int64_t pixels, int double_precision);
int kd_mask_iou_forward_f32(int batch, int64_t pixels, const float *lhs, const float *rhs,
                            float *loss, float *stats, float *iou, void *workspace,
                            size_t workspace_bytes, void *stream);
int kd_mask_iou_forward_f64(int batch, int64_t pixels, const double *lhs, const double *rhs,
                            double *loss, double *stats, double *iou, void *workspace,
                            size_t workspace_bytes, void *stream);
int kd_mask_iou_backward_f32(int batch, int64_t pixels, const float *lhs, const float *rhs,
                             const float *stats, const float *grad_loss, float *grad_lhs,
                             float *grad_rhs, void *stream);
int kd_mask_iou_backward_f64(int batch, int64_t pixels, const double *lhs, const double *rhs,
                             const double *stats, const double *grad_loss, double *grad_lhs,
                             double *grad_rhs, void *stream);

/* ---------------------------------------------------------------------------------------------
 * texture_mapping (kaolin/render/mesh/utils.py:23-76): clamp uv to [0, 1], flip v, then
 * grid_sample(align_corners=False, padding_mode='border').  coords (B, N, 2) with N = h * w for a
 * dense image or the number of points; texture (Bt, C, Ht, Wt) contiguous per view with
 * tex_batch_stride C * Ht * Wt (Bt == B) or 0 (one texture shared by every view); out (B, N, C).
 * mode 0 = nearest, 1 = bilinear.  The backward zeroes and fills grad_tex (the texture's layout
 * and batch stride; shared texture: summed over views) and grad_coords (B, N, 2); either may be
 * NULL.  sample_row = w for a dense (h, w) image (samples are grouped in 16 x 16 blocks whose
 * texture gradient is summed in LDS), 0 for sparse points.
 * ------------------------------------------------------------------------------------------- */
int kd_texture_mapping_forward_f32(int batch, int64_t num_samples, int channels, int tex_height,
                                   int tex_width, const float *coords, const float *tex,
                                   int64_t tex_batch_stride, int mode, float *out, void *stream);
int kd_texture_mapping_forward_f64(int batch, int64_t num_samples, int channels, int tex_height,
                                   int tex_width, const double *coords, const double *tex,
                                   int64_t tex_batch_stride, int mode, double *out, void *stream);
int kd_texture_mapping_backward_f32(int batch, int64_t num_samples, int channels, int tex_height,
                                    int tex_width, const float *coords, const float *tex,
                                    int64_t tex_batch_stride, int mode, int64_t sample_row,
                                    const float *grad_out, float *grad_tex, float *grad_coords,
                                    void *stream);
int kd_texture_mapping_backward_f64(int batch, int64_t num_samples, int channels,
                                    int tex_height, int tex_width, const double *coords,
                                    const double *tex, int64_t tex_batch_stride, int mode,
                                    int64_t sample_row, const double *grad_out,
                                    double *grad_tex, double *grad_coords, void *stream);
/* The same backward with the samples listed per 32 x 32 texel tile: the samples with a nonzero
 * incoming gradient are listed per tile their taps touch (LDS-aggregated counting pass, scan,
 * fill), each tile's list is cut into chunks of 1024 entries, and each chunk's taps are summed in
 * LDS and added to the zeroed texture gradient as row-contiguous atomics.  Independent of the uv
 * layout (the per-block kernel above has an unbounded texel window at uv seams and poles, but is
 * faster on rendered uvs and is the one texture_mapping runs);
 * textures of more than 4096 tiles (2048 x 2048) run the per-block kernel.  Same results up to
 * float summation order.  Workspace: kd_texture_mapping_backward_workspace_size
 * (shared_texture = tex_batch_stride == 0). */
size_t kd_texture_mapping_backward_workspace_size(int batch, int64_t num_samples, int tex_height,
                                                  int tex_width, int shared_texture);
int kd_texture_mapping_backward_tiled_f32(int batch, int64_t num_samples, int channels,
                                          int tex_height, int tex_width, const float *coords,
                                          const float *tex, int64_t tex_batch_stride, int mode,
                                          const float *grad_out, float *grad_tex,
                                          float *grad_coords, void *workspace,
                                          size_t workspace_bytes, void *stream);
int kd_texture_mapping_backward_tiled_f64(int batch, int64_t num_samples, int channels,
                                          int tex_height, int tex_width, const double *coords,
                                          const double *tex, int64_t tex_batch_stride, int mode,
                                          const double *grad_out, double *grad_tex,
                                          double *grad_coords, void *workspace,
                                          size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * nvdiffrast_fwd compatibility (kaolin/render/mesh/rasterization.py:145-241): from an external
 * forward's rast buffer (B, H, W, 4) = (u, v, z/w, triangle_id + 1) and the per-face features
 * (B, F, 3, D), writes interp (B, H, W, D) (u * a0 + v * a1 + (1 - (u + v)) * a2, 0 where empty),
 * face_idx (B, H, W) = id - 1 and weights (B, H, W, 3) = (u, v, 1 - (u + v)) -- the inputs of
 * kd_rasterize_backward_*.
 * ------------------------------------------------------------------------------------------- */
int kd_rast_interpolate_f32(int batch, int height, int width, int64_t num_faces, int feat_dim,
                            const float *rast, const float *feat, float *interp,
                            int64_t *face_idx, float *weights, void *stream);
int kd_rast_interpolate_f64(int batch, int height, int width, int64_t num_faces, int feat_dim,
                            const double *rast, const double *feat, double *interp,
                            int64_t *face_idx, double *weights, void *stream);

/* ---------------------------------------------------------------------------------------------
 * deftet_sparse_render (kaolin/render/mesh/deftet.py:269-417 -> deftet.cpp / deftet_cuda.cu):
 * per pixel (pixel_coords (B, P, 2), any image coordinates; render_ranges (B, P, 2) = [min, max)
 * depth) the first knum faces by index whose box holds the pixel, whose eps-normalised
 * barycentric weights are >= 0 and whose interpolated depth is in range, sorted by depth
 * descending (ties: face order).  Outputs: interp (B, P, knum, D), face_idx (B, P, knum) (-1 =
 * empty), weights (B, P, knum, 3) = (w0, w1, 1 - (w0 + w1)) for the backward.  Workspace:
 * kd_deftet_workspace_size.  The backward writes grad_fvi (B, F, 3, 2) and grad_feat
 * (B, F, 3, D) (NULL: skipped).
 * ------------------------------------------------------------------------------------------- */
size_t kd_deftet_workspace_size(int batch, int64_t num_faces, int double_precision);
int kd_deftet_sparse_render_forward_f32(int batch, int64_t num_pixels, int64_t num_faces,
                                        int knum, int feat_dim, const float *pixel_coords,
                                        const float *render_ranges, const float *fvz,
                                        const float *fvi, const float *feat, float eps,
                                        float *interp, int64_t *face_idx, float *weights,
                                        void *workspace, size_t workspace_bytes, void *stream);
int kd_deftet_sparse_render_forward_f64(int batch, int64_t num_pixels, int64_t num_faces,
                                        int knum, int feat_dim, const double *pixel_coords,
                                        const double *render_ranges, const double *fvz,
                                        const double *fvi, const double *feat, float eps,
                                        double *interp, int64_t *face_idx, double *weights,
                                        void *workspace, size_t workspace_bytes, void *stream);
/* The reference's op form, _C.render.mesh.deftet_sparse_render_forward_cuda (bindings.cpp:81,
 * deftet.cpp:48-106, called at deftet.py:292-299): the caller's face_bboxes (B, F, 4) =
 * (xmin, ymin, xmax, ymax) for the half-open box test, and per pixel the first knum hits in
 * face-index order, unsorted: face_idx (B, P, knum) int64, pixel_depths, w0, w1 (B, P, knum);
 * empty slots -1 / -inf / 0 / 0 (deftet.cpp:88-94).  Same workspace as above. */
int kd_deftet_sparse_render_forward_raw_f32(int batch, int64_t num_pixels, int64_t num_faces,
                                            int knum, const float *fvz, const float *fvi,
                                            const float *face_bboxes, const float *pixel_coords,
                                            const float *render_ranges, float eps,
                                            int64_t *face_idx, float *pixel_depths, float *w0,
                                            float *w1, void *workspace, size_t workspace_bytes,
                                            void *stream);
int kd_deftet_sparse_render_forward_raw_f64(int batch, int64_t num_pixels, int64_t num_faces,
                                            int knum, const double *fvz, const double *fvi,
                                            const double *face_bboxes,
                                            const double *pixel_coords,
                                            const double *render_ranges, float eps,
                                            int64_t *face_idx, double *pixel_depths, double *w0,
                                            double *w1, void *workspace, size_t workspace_bytes,
                                            void *stream);
int kd_deftet_sparse_render_backward_f32(int batch, int64_t num_pixels, int64_t num_faces,
                                         int knum, int feat_dim, const float *grad_interp,
                                         const int64_t *face_idx, const float *weights,
                                         const float *fvi, const float *feat, float eps,
                                         float *grad_fvi, float *grad_feat, void *stream);
int kd_deftet_sparse_render_backward_f64(int batch, int64_t num_pixels, int64_t num_faces,
                                         int knum, int feat_dim, const double *grad_interp,
                                         const int64_t *face_idx, const double *weights,
                                         const double *fvi, const double *feat, float eps,
                                         double *grad_fvi, double *grad_feat, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KAOLIN_DIBR_H_ */
