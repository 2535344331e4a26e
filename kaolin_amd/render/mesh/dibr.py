"""``dibr_soft_mask`` / ``dibr_rasterization`` -- drop-in for kaolin/render/mesh/dibr.py:75-209.

The reference's ``DibrSoftMaskCuda`` (dibr.py:27-73) scales the coordinates, builds enlarged
boxes, runs the per-pixel all-faces scan and saves the (B, H, W, K) close-face lists
(prob / int64 idx / uint8 type, 13*K bytes per pixel) for its backward.  Here the scaling and
boxes are computed in the kernel, the scan runs over ordered tile bins, and by default the lists
are NOT materialised: the forward keeps, per (pixel, close face) pair, the face and the pair's
backward coefficients in its workspace (kd_softpair.hip), and the backward multiplies them by the
incoming gradient and sums them per face and tile.  Inside ``with close_lists():`` the lists are
materialised and the reference-structured atomic backward is used instead (same results up to
float-sum order); the switch is per thread, so it never changes another thread's graphs.
"""
import contextlib
import threading

import torch
from torch.autograd import Function

from ... import _C, _lib
from .rasterization import rasterize

__all__ = ['dibr_soft_mask', 'dibr_rasterization', 'dibr_rasterization_from_vertices',
           'close_lists']

_tls = threading.local()


def _lists_enabled():
    return getattr(_tls, 'lists', False)


@contextlib.contextmanager
def close_lists(enabled=True):
    """Within the block (this thread only), the autograd path materialises the (B, H, W, K)
    close-face lists and uses the reference-structured backward (dibr.py:27-73)."""
    old = _lists_enabled()
    _tls.lists = bool(enabled)
    try:
        yield
    finally:
        _tls.lists = old


class DibrSoftMaskCuda(Function):
    """torch.autograd.Function for ``dibr_soft_mask`` (dibr.py:27-73)."""

    @staticmethod
    def forward(ctx, face_vertices_image, selected_face_idx, sigmainv, boxlen, knum,
                multiplier):
        face_vertices_image = face_vertices_image.contiguous()
        selected_face_idx = selected_face_idx.contiguous()
        lists = _lists_enabled()
        want_grad = face_vertices_image.requires_grad and not lists
        soft_mask, workspace, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_fused(
            face_vertices_image, selected_face_idx, sigmainv, boxlen, knum, multiplier,
            with_lists=lists, want_grad=want_grad)
        ctx.multiplier = multiplier
        ctx.sigmainv = sigmainv
        ctx.boxlen = boxlen
        ctx.knum = knum
        ctx.lists = lists
        if lists:
            ctx.save_for_backward(soft_mask, face_vertices_image, selected_face_idx, prob, cidx,
                                  ctype)
        else:
            # the workspace (records + probabilities) is a saved tensor like the reference's
            # K-lists (dibr.py:51-54): it lives until autograd frees the graph, so a second
            # backward over a retained graph reads the same records
            ctx.save_for_backward(soft_mask, face_vertices_image, selected_face_idx, workspace)
        return soft_mask

    @staticmethod
    def backward(ctx, grad_soft_mask):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        grad_soft_mask = grad_soft_mask.contiguous()
        if ctx.lists:
            soft_mask, fvi, face_idx, prob, cidx, ctype = ctx.saved_tensors
            grad = _C.render.mesh.dibr_soft_mask_backward_cuda(
                grad_soft_mask, soft_mask, face_idx, prob, cidx, ctype,
                (fvi * ctx.multiplier).contiguous(), ctx.sigmainv, ctx.multiplier)
        else:
            soft_mask, fvi, face_idx, workspace = ctx.saved_tensors
            grad = _C.render.mesh.dibr_soft_mask_backward_binned(
                grad_soft_mask, soft_mask, face_idx, fvi, ctx.multiplier, ctx.boxlen,
                ctx.sigmainv, ctx.knum, workspace)
        return grad, None, None, None, None, None


def dibr_soft_mask(face_vertices_image, selected_face_idx, sigmainv=7000, boxlen=0.02, knum=30,
                   multiplier=1000.):
    r"""Soft silhouette mask of DIB-R (dibr.py:75-117): ``1 - prod(1 - exp(-sigmainv d^2))`` over
    the first ``knum`` faces (by index) whose box enlarged by ``boxlen`` holds the pixel; 1 on
    covered pixels.  Returns (B, H, W)."""
    return DibrSoftMaskCuda.apply(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum,
                                  multiplier)


class DibrRasterizationHip(Function):
    """Fused dibr_rasterization (kd_dibr.hip): one binning pass for the raster and the soft
    mask, one backward writing both gradients into one buffer.  Same results as
    rasterize + dibr_soft_mask."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features,
                face_normals_z, sigmainv, boxlen, knum, multiplier, eps):
        want_grad = face_vertices_image.requires_grad or face_features.requires_grad
        # the kernels read dense rows; the backward must read the same copies the forward did
        # (an expanded or permuted input would otherwise be read through the wrong strides)
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        # the backward's gradient buffers, zeroed inside the forward's soft reduction
        bufs = None
        if want_grad:
            bufs = (torch.empty(face_vertices_image.shape, device=face_vertices_image.device,
                                dtype=face_vertices_image.dtype),
                    torch.empty(face_features.shape, device=face_features.device,
                                dtype=face_features.dtype) if face_features.requires_grad
                    else None)
        interp, face_idx, weights, soft, ws = _C.render.mesh.dibr_rasterization_forward_fused(
            height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z,
            sigmainv, boxlen, knum, multiplier, eps, want_grad=want_grad, grad_buffers=bufs)
        # the workspace is saved like the reference's K-lists (dibr.py:51-54): freed with the
        # graph, kept for a second backward over a retained graph
        ctx.save_for_backward(face_idx, weights, soft, face_vertices_image, face_features,
                              ws if want_grad else None)
        ctx.grad_buffers = bufs
        ctx.params = (eps, multiplier, boxlen, sigmainv, knum)
        ctx.mark_non_differentiable(face_idx)
        ctx.set_materialize_grads(False)
        return interp, soft, face_idx

    @staticmethod
    def backward(ctx, grad_interp, grad_soft, grad_face_idx):
        need_fvi, need_feat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        if not (need_fvi or need_feat) or (grad_interp is None and grad_soft is None):
            return (None,) * 11
        face_idx, weights, soft, fvi, feat, workspace = ctx.saved_tensors
        eps, multiplier, boxlen, sigmainv, knum = ctx.params
        # the forward zeroed one set of gradient buffers: the first backward fills them; a
        # second backward (retained graph) gets fresh ones, zeroed by the backward itself
        bufs, ctx.grad_buffers = ctx.grad_buffers, None
        gfvi, gfeat = _C.render.mesh.dibr_rasterization_backward_fused(
            grad_interp, grad_soft, face_idx, weights, soft, fvi, feat, eps, multiplier, boxlen,
            sigmainv, knum, workspace, need_feat=need_feat, grad_buffers=bufs)
        return (None, None, None, gfvi if need_fvi else None, gfeat, None, None, None, None,
                None, None)


class DibrRasterizationListsHip(Function):
    """dibr_rasterization inside ``close_lists()``: the fused forward also writes the soft
    mask's close-face lists (kd_dibr_rasterization_forward_lists: one binning pass, one launch for
    the raster and the soft mask, then the lists writer), and the backward is the reference
    composition's (dibr.py:193-208): rasterize's (rasterization_cuda.cu) plus dibr_soft_mask's over
    the lists (dibr_soft_mask_cuda.cu), summed into grad_fvi as autograd sums the two uses."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features,
                face_normals_z, sigmainv, boxlen, knum, multiplier, eps):
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        interp, face_idx, weights, soft, ws, prob, cidx, ctype = \
            _C.render.mesh.dibr_rasterization_forward_fused(
                height, width, face_vertices_z, face_vertices_image, face_features,
                face_normals_z, sigmainv, boxlen, knum, multiplier, eps, want_grad=False,
                with_lists=True)
        # (the workspace's per-pixel row lengths let the lists backward skip empty rows)
        ctx.save_for_backward(face_idx, weights, soft, face_vertices_image, face_features, prob,
                              cidx, ctype, ws)
        ctx.params = (eps, multiplier, sigmainv)
        ctx.mark_non_differentiable(face_idx)
        ctx.set_materialize_grads(False)
        return interp, soft, face_idx

    @staticmethod
    def backward(ctx, grad_interp, grad_soft, grad_face_idx):
        need_fvi, need_feat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        if not (need_fvi or need_feat) or (grad_interp is None and grad_soft is None):
            return (None,) * 11
        face_idx, weights, soft, fvi, feat, prob, cidx, ctype, ws = ctx.saved_tensors
        eps, multiplier, sigmainv = ctx.params
        gfvi = gfeat = None
        if grad_interp is not None:
            gfvi, gfeat = _C.render.mesh.rasterize_backward_autograd(
                grad_interp.contiguous(), face_idx, weights, fvi, feat, eps, need_feat=need_feat)
        if grad_soft is not None and need_fvi:
            gs = _C.render.mesh.dibr_soft_mask_backward_lists_ws(
                grad_soft.contiguous(), soft, face_idx, prob, cidx, ctype,
                (fvi * multiplier).contiguous(), sigmainv, multiplier, ws)
            gfvi = gs if gfvi is None else gfvi + gs
        return (None, None, None, gfvi if need_fvi else None, gfeat if need_feat else None, None,
                None, None, None, None, None)


# Inside close_lists(): the fused forward with lists (True) or the two ops of the reference
# composition (False; the tests compare both)
LISTS_FUSED = True


def dibr_rasterization(height, width, face_vertices_z, face_vertices_image, face_features,
                       face_normals_z, sigmainv=7000, boxlen=0.02, knum=30, multiplier=None,
                       eps=None, rast_backend='cuda'):
    r"""DIB-R renderer (dibr.py:119-209): rasterize the front faces (normal z >= 0), then the
    soft mask over all faces.  Returns (interpolated_features, soft_mask, face_idx).

    Runs as one fused forward / backward (DibrRasterizationHip); inside ``close_lists()`` the
    fused forward keeps the close-face lists and the backward is the reference composition's
    (DibrRasterizationListsHip)."""
    _multiplier = 1000. if multiplier is None else multiplier
    if (_lists_enabled() and not LISTS_FUSED) or rast_backend != 'cuda':
        # the reference composition (dibr.py:193-208); other backends go through rasterize
        interpolated_features, face_idx = rasterize(
            height, width, face_vertices_z, face_vertices_image, face_features,
            face_normals_z >= 0., multiplier, eps, rast_backend)
        soft_mask = dibr_soft_mask(face_vertices_image, face_idx, sigmainv, boxlen, knum,
                                   _multiplier)
        return interpolated_features, soft_mask, face_idx
    _eps = 1e-8 if eps is None else eps
    _rmult = 1000 if multiplier is None else multiplier  # rasterize's default (an int)
    if float(_rmult) != float(_multiplier):
        raise RuntimeError('internal: multiplier defaults disagree')
    feats = torch.cat(face_features, dim=-1) \
        if isinstance(face_features, (list, tuple)) else face_features
    fn = DibrRasterizationListsHip if _lists_enabled() else DibrRasterizationHip
    interp, soft, face_idx = fn.apply(
        height, width, face_vertices_z, face_vertices_image, feats, face_normals_z, sigmainv,
        boxlen, knum, _multiplier, _eps)
    if isinstance(face_features, (list, tuple)):
        out, cur = [], 0
        for f in face_features:
            out.append(interp[..., cur:cur + f.shape[-1]])
            cur += f.shape[-1]
        interp = tuple(out)
    return interp, soft, face_idx


# The from-vertices node's backward: False = the DIB-R backward's grad_fvi then prepare_vertices'
# gather kernel (the faster form, measured below); True = the face -> vertex step inside the
# DIB-R backward kernel (kd_dibr_rasterization_backward_vertices).
FUSED_VERTEX_BACKWARD = False
# The gather kernel from the vertices (kd_prepare_vertices_backward_vertices: each corner's
# camera-space point recomputed per view, only grad_fvi gathered) rather than from the forward's
# fvc (kd_prepare_vertices_backward): the same bits.
PREPARE_BWD_FROM_VERTICES = True


class DibrRenderHip(Function):
    """prepare_vertices + dibr_rasterization as one autograd node.

    Forward: kd_dibr_rasterization_forward_vertices -- the projection runs inside the binning
    launch, which also writes prepare_vertices' outputs, so no kd_prepare_fwd launch runs and the
    corners are not read back.  Backward: the DIB-R backward's grad_fvi, then prepare_vertices'
    gather kernel over the vertex -> corner CSR (kd_prepare_bwd); or, with
    FUSED_VERTEX_BACKWARD, the face -> vertex step inside the DIB-R backward kernel
    (kd_dibr_rasterization_backward_vertices), which measured slower at C3 (same box, bench.py
    --vertex-bwd fused, profiles/r04/ab_vtx*.txt): 156 us against 68.6 + 18.5 us for the two
    kernels at 8 views, 31 against 18.7 + 10.7 at 1 view -- the vertex atomics (3 per corner,
    every vertex shared by ~6 faces and every view) serialise where the per-face grad_fvi
    atomics did not (per-(tile, vertex) LDS sums before the projection did not change that)."""

    @staticmethod
    def forward(ctx, vertices, faces, camera_proj, camera_transform, face_features, height,
                width, sigmainv, boxlen, knum, multiplier, eps):
        need_v = vertices.requires_grad
        need_feat = face_features.requires_grad
        want_grad = need_v or need_feat
        fused_vtx = FUSED_VERTEX_BACKWARD
        B, F = camera_transform.shape[0], faces.shape[0]
        opts = dict(device=vertices.device, dtype=vertices.dtype)
        gfvi_buf = torch.empty((B, F, 3, 2), **opts) if want_grad and not fused_vtx else None
        gfeat_buf = torch.empty(face_features.shape, **opts) if want_grad and need_feat else None
        fvc, fvi, nrm, interp, face_idx, weights, soft, ws = \
            _C.render.mesh.dibr_rasterization_forward_vertices(
                height, width, vertices, faces, camera_proj, camera_transform, face_features,
                sigmainv, boxlen, knum, multiplier, eps, want_grad=want_grad,
                grad_buffers=(gfvi_buf, gfeat_buf) if want_grad else None)
        ctx.save_for_backward(face_idx, weights, soft, fvi, fvc, face_features, faces,
                              camera_proj.contiguous(), camera_transform.contiguous(),
                              ws if want_grad else None, vertices)
        ctx.bufs = (gfvi_buf, gfeat_buf)
        ctx.fused_vtx = fused_vtx
        from .utils import _adjacency
        ctx.adj = _adjacency(faces, vertices.shape[1]) if need_v and not fused_vtx else None
        ctx.params = (eps, multiplier, boxlen, sigmainv, knum)
        ctx.vshape = (vertices.shape[0], vertices.shape[1])
        ctx.mark_non_differentiable(face_idx)
        ctx.set_materialize_grads(False)
        return interp, soft, face_idx

    @staticmethod
    def backward(ctx, grad_interp, grad_soft, grad_face_idx):
        need_v, need_feat = ctx.needs_input_grad[0], ctx.needs_input_grad[4]
        if not (need_v or need_feat) or (grad_interp is None and grad_soft is None):
            return (None,) * 12
        (face_idx, weights, soft, fvi, fvc, feat, faces, proj, tf,
         workspace, vertices) = ctx.saved_tensors
        eps, multiplier, boxlen, sigmainv, knum = ctx.params
        # the forward zeroed one set of gradient buffers: the first backward fills them, a second
        # one (retained graph) gets fresh buffers zeroed by the backward itself
        bufs, ctx.bufs = ctx.bufs, (None, None)
        if ctx.fused_vtx:
            gvert, gfeat = _C.render.mesh.dibr_rasterization_backward_vertices(
                grad_interp, grad_soft, face_idx, weights, soft, fvi, feat, eps, multiplier,
                boxlen, sigmainv, knum, workspace, faces, fvc, proj, tf, ctx.vshape[0],
                ctx.vshape[1], need_feat=need_feat, grad_feat_buffer=bufs[1])
        else:
            gfvi, gfeat = _C.render.mesh.dibr_rasterization_backward_fused(
                grad_interp, grad_soft, face_idx, weights, soft, fvi, feat, eps, multiplier,
                boxlen, sigmainv, knum, workspace, need_feat=need_feat,
                grad_buffers=bufs if bufs[0] is not None else None)
            gvert = None
            if need_v:
                from .utils import _adjacency
                adj = ctx.adj if ctx.adj is not None else _adjacency(faces, ctx.vshape[1])
                if PREPARE_BWD_FROM_VERTICES:
                    gvert = _C.prepare_vertices_backward_from_vertices(vertices, faces, proj, tf,
                                                                       gfvi, adj)
                else:
                    gvert = _C.prepare_vertices_backward(faces, proj, tf, fvc, None, gfvi, None,
                                                         adj, ctx.vshape[0], ctx.vshape[1])
        return (gvert if need_v else None, None, None, None, gfeat if need_feat else None, None,
                None, None, None, None, None, None)


def dibr_rasterization_from_vertices(height, width, vertices, faces, camera_proj,
                                     camera_transform, face_features, sigmainv=7000,
                                     boxlen=0.02, knum=30, multiplier=None, eps=None):
    r"""``prepare_vertices`` (utils.py:128-175, camera_transform form) followed by
    ``dibr_rasterization`` of its outputs (the DIB-R training step, examples/tutorial/
    ian_dibr.py), as one autograd node (DibrRenderHip: the projection inside the binning launch;
    SURVEY.md §8 f1).  vertices (1 or B, V, 3), faces (F, 3) int64, camera_proj (3, 1),
    camera_transform (B, 4, 3), face_features (B, F, 3, D) (or a list, concatenated).  Returns
    (interpolated_features, soft_mask, face_idx), the same values as
    ``dibr_rasterization(h, w, fvc[..., 2], fvi, face_features, normals[..., 2], ...)``; the
    gradients flow to vertices and face_features.  Falls back to that composition when it
    cannot fuse (camera tensors requiring grad, close_lists mode, feature dim > 3 with
    FUSED_VERTEX_BACKWARD)."""
    feats = torch.cat(face_features, dim=-1) \
        if isinstance(face_features, (list, tuple)) else face_features
    _multiplier = 1000. if multiplier is None else multiplier
    _eps = 1e-8 if eps is None else eps
    if ((FUSED_VERTEX_BACKWARD and feats.shape[-1] > 3) or camera_proj.requires_grad or
            camera_transform.requires_grad or _lists_enabled()):
        from .utils import prepare_vertices
        fvc, fvi, nrm = prepare_vertices(vertices, faces, camera_proj,
                                         camera_transform=camera_transform)
        return dibr_rasterization(height, width, fvc[..., 2], fvi, face_features, nrm[..., 2],
                                  sigmainv, boxlen, knum, multiplier, eps)
    interp, soft, face_idx = DibrRenderHip.apply(vertices, faces, camera_proj, camera_transform,
                                                 feats, height, width, sigmainv, boxlen, knum,
                                                 _multiplier, _eps)
    if isinstance(face_features, (list, tuple)):
        out, cur = [], 0
        for f in face_features:
            out.append(interp[..., cur:cur + f.shape[-1]])
            cur += f.shape[-1]
        interp = tuple(out)
    return interp, soft, face_idx


class DibrRasterizationIouHip(Function):
    """dibr_rasterization + mask_iou(soft_mask, gt_mask) fused (kd_dibr_rasterization_iou_*,
    SURVEY.md §8 f2): the IoU sums are accumulated inside the soft mask's tile launch and the
    IoU's gradient is formed per pixel inside the soft mask's backward, so neither the standalone
    IoU kernels nor a (B, H, W) gradient of the mask run."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features,
                face_normals_z, gt_mask, sigmainv, boxlen, knum, multiplier, eps):
        want_grad = face_vertices_image.requires_grad or face_features.requires_grad
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        gt_mask = gt_mask.contiguous()
        bufs = None
        if want_grad:
            bufs = (torch.empty(face_vertices_image.shape, device=face_vertices_image.device,
                                dtype=face_vertices_image.dtype),
                    torch.empty(face_features.shape, device=face_features.device,
                                dtype=face_features.dtype) if face_features.requires_grad
                    else None)
        interp, face_idx, weights, soft, ws, loss, stats = \
            _C.render.mesh.dibr_rasterization_forward_fused(
                height, width, face_vertices_z, face_vertices_image, face_features,
                face_normals_z, sigmainv, boxlen, knum, multiplier, eps, want_grad=want_grad,
                grad_buffers=bufs, iou_gt=gt_mask)
        ctx.save_for_backward(face_idx, weights, soft, face_vertices_image, face_features,
                              ws if want_grad else None, gt_mask, stats)
        ctx.grad_buffers = bufs
        ctx.params = (eps, multiplier, boxlen, sigmainv, knum)
        ctx.mark_non_differentiable(face_idx)
        ctx.set_materialize_grads(False)
        return interp, soft, face_idx, loss

    @staticmethod
    def backward(ctx, grad_interp, grad_soft, grad_face_idx, grad_loss):
        need_fvi, need_feat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        none = (None,) * 12
        if not (need_fvi or need_feat) or (grad_interp is None and grad_soft is None and
                                           grad_loss is None):
            return none
        face_idx, weights, soft, fvi, feat, workspace, gt, stats = ctx.saved_tensors
        eps, multiplier, boxlen, sigmainv, knum = ctx.params
        bufs, ctx.grad_buffers = ctx.grad_buffers, None
        iou = None if grad_loss is None else (gt, stats, grad_loss.reshape(()))
        gfvi, gfeat = _C.render.mesh.dibr_rasterization_backward_fused(
            grad_interp, grad_soft, face_idx, weights, soft, fvi, feat, eps, multiplier, boxlen,
            sigmainv, knum, workspace, need_feat=need_feat, grad_buffers=bufs, iou=iou)
        return (None, None, None, gfvi if need_fvi else None, gfeat, None, None, None, None,
                None, None, None)


def dibr_rasterization_with_mask_iou(height, width, face_vertices_z, face_vertices_image,
                                     face_features, face_normals_z, gt_mask, sigmainv=7000,
                                     boxlen=0.02, knum=30, multiplier=None, eps=None):
    r"""``dibr_rasterization`` (dibr.py:119-209) followed by the DIB-R silhouette loss
    ``kaolin.metrics.render.mask_iou(soft_mask, gt_mask)`` (metrics/render.py:18-40; the training
    loop of examples/tutorial/ian_dibr.py:264-265), fused.  gt_mask (B, H, W)
    of the features' dtype.  Returns (interpolated_features, soft_mask, face_idx, iou_loss), the
    values of the composition; gradients of any of the outputs flow to face_vertices_image and
    face_features.  Falls back to the composition where it cannot fuse (knum > 32, close_lists
    mode, a pool-limit test hook)."""
    from ...metrics.render import mask_iou
    _multiplier = 1000. if multiplier is None else multiplier
    _eps = 1e-8 if eps is None else eps
    feats = torch.cat(face_features, dim=-1) \
        if isinstance(face_features, (list, tuple)) else face_features
    if (int(knum) > 32 or _lists_enabled() or _lib.pool_limits_active() or
            gt_mask.requires_grad or _lib.split_soft_mask_forced()):
        interp, soft, face_idx = dibr_rasterization(
            height, width, face_vertices_z, face_vertices_image, face_features, face_normals_z,
            sigmainv, boxlen, knum, multiplier, eps)
        return interp, soft, face_idx, mask_iou(soft, gt_mask)
    interp, soft, face_idx, loss = DibrRasterizationIouHip.apply(
        height, width, face_vertices_z, face_vertices_image, feats, face_normals_z, gt_mask,
        sigmainv, boxlen, knum, _multiplier, _eps)
    if isinstance(face_features, (list, tuple)):
        out, cur = [], 0
        for f in face_features:
            out.append(interp[..., cur:cur + f.shape[-1]])
            cur += f.shape[-1]
        interp = tuple(out)
    return interp, soft, face_idx, loss
