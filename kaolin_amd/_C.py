"""Drop-in for the reference's native module ``kaolin._C.render.mesh`` (hot path only).

Reference binding: kaolin/csrc/bindings.cpp:75-80.  Same four function names, positional
signatures, return tuples, output allocation and error class (RuntimeError) as the reference
wrappers kaolin/csrc/render/mesh/rasterization.cpp:49-168 and dibr_soft_mask.cpp:48-183.
Each call validates its arguments like ``at::checkAllSameGPU`` / ``checkAllContiguous`` /
``checkSize``, allocates the outputs with ``torch.empty`` (the kernels write every element, so the
reference's ``at::full(-1)`` / ``at::zeros`` pre-fills are not needed) and launches on the
current HIP stream of the inputs' device.

Also the reference's two DefTet operators (bindings.cpp:81-82, deftet.cpp:48-160) with their
positional signatures: ``deftet_sparse_render_forward_cuda`` / ``_backward_cuda``.

Extra entry points (used by kaolin_amd.render.mesh's autograd functions, not in the reference):
``rasterize_forward_fused``, ``rasterize_backward_autograd``, ``dibr_soft_mask_forward_fused``,
``dibr_soft_mask_backward_binned``.
"""
import types

import torch

from . import _lib

_SFX = {torch.float32: 'f32', torch.float64: 'f64'}


def _sfx(t, fname):
    try:
        return _SFX[t.dtype]
    except KeyError:
        raise RuntimeError(f'"{fname}" not implemented for \'{t.dtype}\'') from None


def _check_same_gpu(fname, **tensors):
    dev = None
    for name, t in tensors.items():
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f'{fname}: expected tensor for argument "{name}" to be on a GPU '
                               f'(got {t.device})')
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f'{fname}: expected all tensors to be on the same GPU, but found '
                               f'{dev} and {t.device} (argument "{name}")')
    return dev


def _check_contiguous(fname, **tensors):
    for name, t in tensors.items():
        if t is not None and not t.is_contiguous():
            raise RuntimeError(f'{fname}: expected contiguous tensor for argument "{name}"')


def _check_size(fname, name, t, size):
    if tuple(t.shape) != tuple(size):
        raise RuntimeError(f'{fname}: expected tensor for argument "{name}" to have size '
                           f'{list(size)}, but got {list(t.shape)}')


def _check_dtype(fname, ref, **tensors):
    for name, t in tensors.items():
        if t is not None and t.dtype != ref.dtype:
            raise RuntimeError(f'{fname}: expected {name} to have dtype {ref.dtype}, '
                               f'got {t.dtype}')


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _workspace(kind, dev, B, H, W, n_total, max_per_view):
    nb = _lib.workspace_size(kind, B, H, W, n_total, max_per_view)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    return ws, nb


# -------------------------------------------------------------------------------------------
# the reference's four operators
# -------------------------------------------------------------------------------------------
def packed_rasterize_forward_cuda(height, width, face_vertices_z, face_vertices_image,
                                  face_bboxes, face_features, first_idx_face_per_mesh,
                                  multiplier, eps):
    """rasterization.cpp:49-104 -> [interpolated_features, selected_face_idx, output_weights]"""
    fn = 'packed_rasterize_forward_cuda'
    dev = _check_same_gpu(fn, face_vertices_z=face_vertices_z,
                          face_vertices_image=face_vertices_image, face_bboxes=face_bboxes,
                          face_features=face_features,
                          first_idx_face_per_mesh=first_idx_face_per_mesh)
    _check_contiguous(fn, face_vertices_z=face_vertices_z,
                      face_vertices_image=face_vertices_image, face_bboxes=face_bboxes,
                      face_features=face_features,
                      first_idx_face_per_mesh=first_idx_face_per_mesh)
    num_faces = face_vertices_z.shape[0]
    batch_size = first_idx_face_per_mesh.shape[0] - 1
    feat_dim = face_features.shape[2]
    _check_size(fn, 'face_vertices_z', face_vertices_z, (num_faces, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (num_faces, 3, 2))
    _check_size(fn, 'face_bboxes', face_bboxes, (num_faces, 4))
    _check_size(fn, 'face_features', face_features, (num_faces, 3, feat_dim))
    _check_size(fn, 'first_idx_face_per_mesh', first_idx_face_per_mesh, (batch_size + 1,))
    sfx = _sfx(face_vertices_z, fn)
    _check_dtype(fn, face_vertices_z, face_vertices_image=face_vertices_image,
                 face_bboxes=face_bboxes, face_features=face_features)
    if first_idx_face_per_mesh.dtype != torch.int64:
        raise RuntimeError(f'{fn}: first_idx_face_per_mesh must be int64')
    opts = dict(device=dev, dtype=face_vertices_z.dtype)
    interp = torch.empty((batch_size, height, width, feat_dim), **opts)
    face_idx = torch.empty((batch_size, height, width), device=dev, dtype=torch.long)
    weights = torch.empty((batch_size, height, width, 3), **opts)
    ws, nb = _workspace(_lib.KD_WS_RASTER_PACKED, dev, batch_size, height, width, num_faces,
                        num_faces)
    _lib.call(f'kd_packed_rasterize_forward_{sfx}', batch_size, height, width, num_faces,
              feat_dim, _ptr(face_vertices_z), _ptr(face_vertices_image), _ptr(face_bboxes),
              _ptr(face_features), _ptr(first_idx_face_per_mesh), float(multiplier), float(eps),
              _ptr(interp), _ptr(face_idx), _ptr(weights), _ptr(ws), nb, _stream(dev))
    return [interp, face_idx, weights]


def rasterize_backward_cuda(grad_interpolated_features, interpolated_features,
                            selected_face_idx, output_weights, face_vertices_image,
                            face_features, eps):
    """rasterization.cpp:106-168 -> [grad_face_vertices_image, grad_face_features]"""
    fn = 'rasterize_backward_cuda'
    dev = _check_same_gpu(fn, grad_interpolated_features=grad_interpolated_features,
                          interpolated_features=interpolated_features,
                          selected_face_idx=selected_face_idx, output_weights=output_weights,
                          face_vertices_image=face_vertices_image, face_features=face_features)
    _check_contiguous(fn, grad_interpolated_features=grad_interpolated_features,
                      interpolated_features=interpolated_features,
                      selected_face_idx=selected_face_idx, output_weights=output_weights,
                      face_vertices_image=face_vertices_image, face_features=face_features)
    B, H, W, D = grad_interpolated_features.shape
    F = face_vertices_image.shape[1]
    _check_size(fn, 'interpolated_features', interpolated_features, (B, H, W, D))
    _check_size(fn, 'selected_face_idx', selected_face_idx, (B, H, W))
    _check_size(fn, 'output_weights', output_weights, (B, H, W, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    sfx = _sfx(grad_interpolated_features, fn)
    _check_dtype(fn, grad_interpolated_features, output_weights=output_weights,
                 face_vertices_image=face_vertices_image, face_features=face_features)
    gfvi = torch.empty_like(face_vertices_image)
    gfeat = torch.empty_like(face_features)
    _lib.call(f'kd_rasterize_backward_{sfx}', B, H, W, F, D, _ptr(grad_interpolated_features),
              _ptr(selected_face_idx), _ptr(output_weights), _ptr(face_vertices_image),
              _ptr(face_features), float(eps), _ptr(gfvi), _ptr(gfeat), _stream(dev))
    return [gfvi, gfeat]


def dibr_soft_mask_forward_cuda(face_vertices_image, face_large_bboxes, selected_face_idx,
                                sigmainv, knum, multiplier):
    """dibr_soft_mask.cpp:48-108 ->
    [soft_mask, close_face_prob, close_face_idx, close_face_dist_type]"""
    fn = 'dibr_soft_mask_forward_cuda'
    dev = _check_same_gpu(fn, face_vertices_image=face_vertices_image,
                          face_large_bboxes=face_large_bboxes,
                          selected_face_idx=selected_face_idx)
    _check_contiguous(fn, face_vertices_image=face_vertices_image,
                      face_large_bboxes=face_large_bboxes, selected_face_idx=selected_face_idx)
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:3]
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_bboxes', face_large_bboxes, (B, F, 4))
    _check_size(fn, 'selected_face_idx', selected_face_idx, (B, H, W))
    sfx = _sfx(face_vertices_image, fn)
    _check_dtype(fn, face_vertices_image, face_large_bboxes=face_large_bboxes)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    opts = dict(device=dev, dtype=face_vertices_image.dtype)
    soft = torch.empty((B, H, W), **opts)
    prob = torch.empty((B, H, W, knum), **opts)
    cidx = torch.empty((B, H, W, knum), device=dev, dtype=torch.long)
    ctype = torch.empty((B, H, W, knum), device=dev, dtype=torch.uint8)
    ws, nb = _workspace(_lib.KD_WS_SOFT_MASK, dev, B, H, W, B * F, F)
    _lib.call(f'kd_dibr_soft_mask_forward_{sfx}', B, H, W, F, knum, _ptr(face_vertices_image),
              _ptr(face_large_bboxes), _ptr(selected_face_idx), float(sigmainv),
              float(multiplier), _ptr(soft), _ptr(prob), _ptr(cidx), _ptr(ctype), _ptr(ws), nb,
              _stream(dev))
    return [soft, prob, cidx, ctype]


def dibr_soft_mask_backward_cuda(grad_soft_mask, soft_mask, selected_face_idx, close_face_prob,
                                 close_face_idx, close_face_dist_type, face_vertices_image,
                                 sigmainv, multiplier):
    """dibr_soft_mask.cpp:110-183 -> grad_face_vertices_image"""
    fn = 'dibr_soft_mask_backward_cuda'
    dev = _check_same_gpu(fn, grad_soft_mask=grad_soft_mask, soft_mask=soft_mask,
                          close_face_idx=close_face_idx,
                          close_face_dist_type=close_face_dist_type,
                          close_face_prob=close_face_prob,
                          face_vertices_image=face_vertices_image)
    _check_contiguous(fn, grad_soft_mask=grad_soft_mask, soft_mask=soft_mask,
                      close_face_prob=close_face_prob, close_face_idx=close_face_idx,
                      close_face_dist_type=close_face_dist_type,
                      face_vertices_image=face_vertices_image)
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:3]
    K = close_face_idx.shape[-1]
    _check_size(fn, 'grad_soft_mask', grad_soft_mask, (B, H, W))
    _check_size(fn, 'soft_mask', soft_mask, (B, H, W))
    _check_size(fn, 'selected_face_idx', selected_face_idx, (B, H, W))
    _check_size(fn, 'close_face_prob', close_face_prob, (B, H, W, K))
    _check_size(fn, 'close_face_idx', close_face_idx, (B, H, W, K))
    _check_size(fn, 'close_face_dist_type', close_face_dist_type, (B, H, W, K))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    sfx = _sfx(face_vertices_image, fn)
    _check_dtype(fn, face_vertices_image, grad_soft_mask=grad_soft_mask, soft_mask=soft_mask,
                 close_face_prob=close_face_prob)
    selected_face_idx = selected_face_idx.contiguous()
    g = torch.empty_like(face_vertices_image)
    _lib.call(f'kd_dibr_soft_mask_backward_{sfx}', B, H, W, F, K, _ptr(grad_soft_mask),
              _ptr(soft_mask), _ptr(selected_face_idx), _ptr(close_face_prob),
              _ptr(close_face_idx), _ptr(close_face_dist_type), _ptr(face_vertices_image),
              float(sigmainv), float(multiplier), _ptr(g), _stream(dev))
    return g


# -------------------------------------------------------------------------------------------
# fused entry points used by the autograd functions of kaolin_amd.render.mesh
# -------------------------------------------------------------------------------------------
def rasterize_forward_fused(height, width, face_vertices_z, face_vertices_image, face_features,
                            valid_faces, multiplier, eps):
    """RasterizeCuda.forward (rasterization.py:289-369) with packing / scaling / bbox / remap in
    the kernel.  Inputs contiguous (B,F,3), (B,F,3,2), (B,F,3,D); valid_faces (B,F) bool/uint8 or
    None.  Returns (interp, face_idx [original index], weights)."""
    fn = 'rasterize'
    dev = _check_same_gpu(fn, face_vertices_z=face_vertices_z,
                          face_vertices_image=face_vertices_image, face_features=face_features,
                          valid_faces=valid_faces)
    B, F = face_vertices_z.shape[:2]
    D = face_features.shape[-1]
    _check_size(fn, 'face_vertices_z', face_vertices_z, (B, F, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    sfx = _sfx(face_vertices_z, fn)
    _check_dtype(fn, face_vertices_z, face_vertices_image=face_vertices_image,
                 face_features=face_features)
    if valid_faces is not None:
        _check_size(fn, 'valid_faces', valid_faces, (B, F))
        valid_faces = valid_faces.contiguous()
        if valid_faces.dtype != torch.uint8:
            valid_faces = valid_faces.to(torch.uint8) if valid_faces.dtype != torch.bool \
                else valid_faces.view(torch.uint8)
    opts = dict(device=dev, dtype=face_vertices_z.dtype)
    interp = torch.empty((B, height, width, D), **opts)
    face_idx = torch.empty((B, height, width), device=dev, dtype=torch.long)
    weights = torch.empty((B, height, width, 3), **opts)
    ws, nb = _workspace(_lib.KD_WS_RASTER, dev, B, height, width, B * F, F)
    _lib.call(f'kd_rasterize_forward_{sfx}', B, height, width, F, D, _ptr(face_vertices_z),
              _ptr(face_vertices_image), _ptr(face_features), _ptr(valid_faces),
              float(multiplier), float(eps), _ptr(interp), _ptr(face_idx), _ptr(weights),
              _ptr(ws), nb, _stream(dev))
    return interp, face_idx, weights, valid_faces


def rasterize_backward_autograd(grad_interp, face_idx, weights, face_vertices_image,
                                face_features, eps, need_feat=True):
    """RasterizeCuda.backward: the tile kernel, grad of the features only when needed."""
    dev = grad_interp.device
    B, H, W, D = grad_interp.shape
    F = face_vertices_image.shape[1]
    sfx = _sfx(face_vertices_image, 'rasterize_backward')
    gfvi = torch.empty_like(face_vertices_image)
    gfeat = torch.empty_like(face_features) if need_feat else None
    _lib.call(f'kd_rasterize_backward_{sfx}', B, H, W, F, D, _ptr(grad_interp), _ptr(face_idx),
              _ptr(weights), _ptr(face_vertices_image), _ptr(face_features), float(eps),
              _ptr(gfvi), _ptr(gfeat), _stream(dev))
    return gfvi, gfeat


def dibr_soft_mask_forward_fused(face_vertices_image, selected_face_idx, sigmainv, boxlen, knum,
                                 multiplier, with_lists=False, want_grad=True):
    """DibrSoftMaskCuda.forward (dibr.py:29-55) with the x multiplier and the enlarged boxes in
    the kernel.  Returns (soft, workspace, prob, cidx, ctype) (lists None unless with_lists); with
    want_grad the workspace holds the (pixel, face) records and backward coefficients that
    dibr_soft_mask_backward_binned consumes."""
    fn = 'dibr_soft_mask'
    dev = _check_same_gpu(fn, face_vertices_image=face_vertices_image,
                          selected_face_idx=selected_face_idx)
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:3]
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'selected_face_idx', selected_face_idx, (B, H, W))
    sfx = _sfx(face_vertices_image, fn)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    opts = dict(device=dev, dtype=face_vertices_image.dtype)
    soft = torch.empty((B, H, W), **opts)
    prob = cidx = ctype = None
    if with_lists:
        prob = torch.empty((B, H, W, knum), **opts)
        cidx = torch.empty((B, H, W, knum), device=dev, dtype=torch.long)
        ctype = torch.empty((B, H, W, knum), device=dev, dtype=torch.uint8)
    nb = _lib.soft_mask_workspace_size(B, H, W, F, knum, face_vertices_image.dtype == torch.float64)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    _lib.call(f'kd_dibr_soft_mask_forward_fused_{sfx}', B, H, W, F, knum,
              _ptr(face_vertices_image), float(multiplier), float(boxlen),
              _ptr(selected_face_idx), float(sigmainv), _ptr(soft), _ptr(prob), _ptr(cidx),
              _ptr(ctype), None, 1 if want_grad else 0, _ptr(ws), nb, _stream(dev))
    return soft, ws, prob, cidx, ctype


def dibr_soft_mask_backward_binned(grad_soft, soft, selected_face_idx, face_vertices_image,
                                   multiplier, boxlen, sigmainv, knum, workspace):
    """DibrSoftMaskCuda.backward without close lists, from the forward's workspace (records and
    backward coefficients, kd_softpair.hip)."""
    dev = grad_soft.device
    B, F = face_vertices_image.shape[:2]
    H, W = selected_face_idx.shape[1:3]
    sfx = _sfx(face_vertices_image, 'dibr_soft_mask_backward')
    g = torch.empty_like(face_vertices_image)
    _lib.call(f'kd_dibr_soft_mask_backward_binned_{sfx}', B, H, W, F, int(knum), _ptr(grad_soft),
              _ptr(soft), _ptr(selected_face_idx), _ptr(face_vertices_image), float(multiplier),
              float(boxlen), float(sigmainv), _ptr(g), _ptr(workspace), workspace.numel(), 1,
              _stream(dev))
    return g


# -------------------------------------------------------------------------------------------
# prepare_vertices (kaolin/render/mesh/utils.py:128-175), SURVEY §8 f1
# -------------------------------------------------------------------------------------------
def vertex_face_adjacency(faces, num_vertices):
    """CSR of each vertex's incident (face, corner) entries f * 3 + corner, grouped by vertex
    (stable order), and the backward's workgroup entry ranges (whole vertices, <= 256 entries;
    kd_prepare_vertices_ranges).  Returns (offsets (V+1) int64, adj (3F) int32, ranges (R+1)
    int32, vertex of each entry (3F) int32) on the faces' device.  Built once per topology (one
    device->host copy of offsets)."""
    import numpy as np
    flat = faces.reshape(-1)
    order = torch.argsort(flat, stable=True)
    counts = torch.bincount(flat, minlength=num_vertices)
    offsets = torch.zeros(num_vertices + 1, dtype=torch.long, device=faces.device)
    torch.cumsum(counts, 0, out=offsets[1:])
    off_h = np.ascontiguousarray(offsets.cpu().numpy())
    rng = np.empty(num_vertices + 2, np.int32)
    n = int(_lib.load().kd_prepare_vertices_ranges(off_h.ctypes.data, num_vertices, 256,
                                                   rng.ctypes.data))
    if n < 0:
        raise RuntimeError('vertex_face_adjacency: kd_prepare_vertices_ranges failed')
    ranges = torch.from_numpy(rng[:n + 1].copy()).to(faces.device)
    return offsets, order.to(torch.int32), ranges, flat[order].to(torch.int32)


def prepare_vertices_forward(vertices, faces, camera_proj, camera_transform):
    """vertices (Bv, V, 3) with Bv in {1, B}, faces (F, 3) int64, camera_proj (3, 1),
    camera_transform (B, 4, 3) -> (fvc (B, F, 3, 3), fvi (B, F, 3, 2), normals (B, F, 3))."""
    fn = 'prepare_vertices'
    dev = _check_same_gpu(fn, vertices=vertices, faces=faces, camera_proj=camera_proj,
                          camera_transform=camera_transform)
    Bv, V = vertices.shape[:2]
    B, F = camera_transform.shape[0], faces.shape[0]
    _check_size(fn, 'vertices', vertices, (Bv, V, 3))
    _check_size(fn, 'faces', faces, (F, 3))
    _check_size(fn, 'camera_transform', camera_transform, (B, 4, 3))
    if Bv not in (1, B):
        raise RuntimeError(f'{fn}: vertices batch {Bv} must be 1 or the camera batch {B}')
    if faces.dtype != torch.int64:
        raise RuntimeError(f'{fn}: faces must be int64')
    sfx = _sfx(vertices, fn)
    _check_dtype(fn, vertices, camera_proj=camera_proj, camera_transform=camera_transform)
    opts = dict(device=dev, dtype=vertices.dtype)
    fvc = torch.empty((B, F, 3, 3), **opts)
    fvi = torch.empty((B, F, 3, 2), **opts)
    nrm = torch.empty((B, F, 3), **opts)
    _lib.call(f'kd_prepare_vertices_forward_{sfx}', B, Bv, V, F, _ptr(vertices), _ptr(faces),
              _ptr(camera_proj), _ptr(camera_transform), _ptr(fvc), _ptr(fvi), _ptr(nrm),
              _stream(dev))
    return fvc, fvi, nrm


def prepare_vertices_backward(faces, camera_proj, camera_transform, fvc, grad_fvc, grad_fvi,
                              grad_nrm, adjacency, vertex_batch, num_vertices):
    """Gradient w.r.t. the vertices (vertex_batch, V, 3); None gradients count as zero."""
    dev = fvc.device
    B, F = fvc.shape[:2]
    sfx = _sfx(fvc, 'prepare_vertices_backward')
    offsets, adj, ranges = adjacency[:3]
    g = torch.empty((vertex_batch, num_vertices, 3), device=dev, dtype=fvc.dtype)
    _lib.call(f'kd_prepare_vertices_backward_{sfx}', B, vertex_batch, num_vertices, F,
              _ptr(faces), _ptr(camera_proj), _ptr(camera_transform), _ptr(fvc),
              _ptr(grad_fvc), _ptr(grad_fvi), _ptr(grad_nrm), _ptr(offsets), _ptr(adj),
              _ptr(ranges), ranges.numel() - 1, _ptr(g), _stream(dev))
    return g


def prepare_vertices_backward_from_vertices(vertices, faces, camera_proj, camera_transform,
                                            grad_fvi, adjacency):
    """The vertex gradient (Bv, V, 3) from grad_fvi alone, each corner's camera-space point
    recomputed from the vertices (kd_prepare_vertices_backward_vertices): the same bits as
    prepare_vertices_backward(..., fvc, None, grad_fvi, None, ...)."""
    dev = vertices.device
    Bv, V = vertices.shape[:2]
    B, F = grad_fvi.shape[:2]
    sfx = _sfx(vertices, 'prepare_vertices_backward')
    offsets, adj, ranges, vid = adjacency
    g = torch.empty((Bv, V, 3), device=dev, dtype=vertices.dtype)
    _lib.call(f'kd_prepare_vertices_backward_vertices_{sfx}', B, Bv, V, F,
              _ptr(vertices.contiguous()), _ptr(faces), _ptr(camera_proj),
              _ptr(camera_transform), _ptr(grad_fvi.contiguous()), _ptr(offsets), _ptr(adj),
              _ptr(vid), _ptr(ranges), ranges.numel() - 1, _ptr(g), _stream(dev))
    return g


# -------------------------------------------------------------------------------------------
# dibr_rasterization fused (kd_dibr.hip)
# -------------------------------------------------------------------------------------------
def _rows_view(t, F, inner):
    """(pointer tensor, face stride, inner stride) of a (B, F[, inner]) view whose faces are
    evenly strided across the batch; a contiguous copy otherwise."""
    if t.dim() == 2:
        s0, s1 = t.stride()
        if s0 == F * s1 or t.shape[0] == 1:
            return t, s1, 1
    else:
        s0, s1, s2 = t.stride()
        if s0 == F * s1 or t.shape[0] == 1:
            return t, s1, s2
    t = t.contiguous()
    return t, (inner if t.dim() == 3 else 1), 1


def dibr_rasterization_forward_fused(height, width, face_vertices_z, face_vertices_image,
                                     face_features, face_normals_z, sigmainv, boxlen, knum,
                                     multiplier, eps, want_grad=True, grad_buffers=None,
                                     iou_gt=None, with_lists=False):
    """rasterize(valid = normals_z >= 0) + dibr_soft_mask in one launch sequence.  Returns
    (interp, face_idx, weights, soft, workspace), and with iou_gt (B, H, W) also (iou_loss,
    iou_stats): mask_iou(soft, iou_gt) fused in (kd_dibr_rasterization_iou_forward).
    grad_buffers = (grad_fvi, grad_feat or None): buffers of the backward that this forward
    zeroes (see kd_dibr_rasterization_forward).  with_lists: also the soft mask's close-face
    lists (prob, cidx, ctype) (B, H, W, knum), appended to the returns (no workspace backward;
    kd_dibr_rasterization_forward_lists)."""
    fn = 'dibr_rasterization'
    dev = _check_same_gpu(fn, face_vertices_z=face_vertices_z,
                          face_vertices_image=face_vertices_image, face_features=face_features,
                          face_normals_z=face_normals_z)
    B, F = face_vertices_image.shape[:2]
    D = face_features.shape[-1]
    _check_size(fn, 'face_vertices_z', face_vertices_z, (B, F, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    _check_size(fn, 'face_normals_z', face_normals_z, (B, F))
    sfx = _sfx(face_vertices_image, fn)
    _check_dtype(fn, face_vertices_image, face_vertices_z=face_vertices_z,
                 face_features=face_features, face_normals_z=face_normals_z)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    fvz, fvz_fs, fvz_cs = _rows_view(face_vertices_z, F, 3)
    nz, nz_s, _ = _rows_view(face_normals_z, F, 1)
    fvi = face_vertices_image.contiguous()
    feat = face_features.contiguous()
    opts = dict(device=dev, dtype=fvi.dtype)
    interp = torch.empty((B, height, width, D), **opts)
    face_idx = torch.empty((B, height, width), device=dev, dtype=torch.long)
    weights = torch.empty((B, height, width, 3), **opts)
    soft = torch.empty((B, height, width), **opts)
    if with_lists and iou_gt is not None:
        raise ValueError(f'{fn}: the close-face lists (with_lists) and the fused mask_iou '
                         f'(iou_gt) cannot be combined')
    nb = int(_lib.load().kd_dibr_workspace_size(B, height, width, F, knum,
                                                1 if fvi.dtype == torch.float64 else 0))
    if fvi.dtype == torch.float32:
        _lib.tile_history_buffer(dev)  # the caller-owned tile history (kd_tile_history_attach)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    if iou_gt is not None:
        _check_size(fn, 'gt_mask', iou_gt, (B, height, width))
        _check_dtype(fn, face_vertices_image, gt_mask=iou_gt)
        if iou_gt.device != dev:
            raise RuntimeError(f'{fn}: gt_mask must be on {dev}')
        gt = iou_gt.contiguous()
        loss = torch.empty((), **opts)
        stats = torch.empty((B, 2), **opts)
        acc = torch.empty((B, 32, 2), device=dev, dtype=torch.float64)  # kIouParts partials
        _lib.call(f'kd_dibr_rasterization_iou_forward_{sfx}', B, height, width, F, D, _ptr(fvz),
                  fvz_fs, fvz_cs, _ptr(fvi), _ptr(feat), _ptr(nz), nz_s, float(multiplier),
                  float(eps), float(sigmainv), float(boxlen), knum, _ptr(gt), _ptr(interp),
                  _ptr(face_idx), _ptr(weights), _ptr(soft), _ptr(loss), _ptr(stats), _ptr(acc),
                  1 if want_grad else 0, _ptr(grad_buffers[0]) if grad_buffers else None,
                  _ptr(grad_buffers[1]) if grad_buffers else None, _ptr(ws), nb, _stream(dev))
        return interp, face_idx, weights, soft, ws, loss, stats
    if with_lists:
        prob = torch.empty((B, height, width, knum), **opts)
        cidx = torch.empty((B, height, width, knum), device=dev, dtype=torch.long)
        ctype = torch.empty((B, height, width, knum), device=dev, dtype=torch.uint8)
        _lib.call(f'kd_dibr_rasterization_forward_lists_{sfx}', B, height, width, F, D, _ptr(fvz),
                  fvz_fs, fvz_cs, _ptr(fvi), _ptr(feat), _ptr(nz), nz_s, float(multiplier),
                  float(eps), float(sigmainv), float(boxlen), knum, _ptr(interp), _ptr(face_idx),
                  _ptr(weights), _ptr(soft), _ptr(prob), _ptr(cidx), _ptr(ctype), _ptr(ws), nb,
                  _stream(dev))
        return interp, face_idx, weights, soft, ws, prob, cidx, ctype
    _lib.call(f'kd_dibr_rasterization_forward_{sfx}', B, height, width, F, D, _ptr(fvz), fvz_fs,
              fvz_cs, _ptr(fvi), _ptr(feat), _ptr(nz), nz_s, float(multiplier), float(eps),
              float(sigmainv), float(boxlen), knum, _ptr(interp), _ptr(face_idx), _ptr(weights),
              _ptr(soft), 1 if want_grad else 0,
              _ptr(grad_buffers[0]) if grad_buffers else None,
              _ptr(grad_buffers[1]) if grad_buffers else None, _ptr(ws), nb, _stream(dev))
    return interp, face_idx, weights, soft, ws


def dibr_rasterization_forward_vertices(height, width, vertices, faces, camera_proj,
                                        camera_transform, face_features, sigmainv, boxlen, knum,
                                        multiplier, eps, want_grad=True, grad_buffers=None):
    """prepare_vertices (camera transform form) + the fused DIB-R forward with the projection
    inside the binning launch (kd_dibr_rasterization_forward_vertices).  Returns (fvc, fvi,
    normals, interp, face_idx, weights, soft, workspace); grad_buffers as in
    dibr_rasterization_forward_fused."""
    fn = 'dibr_rasterization_from_vertices'
    dev = _check_same_gpu(fn, vertices=vertices, faces=faces, camera_proj=camera_proj,
                          camera_transform=camera_transform, face_features=face_features)
    Bv, V = vertices.shape[:2]
    B, F = camera_transform.shape[0], faces.shape[0]
    D = face_features.shape[-1]
    _check_size(fn, 'vertices', vertices, (Bv, V, 3))
    _check_size(fn, 'faces', faces, (F, 3))
    _check_size(fn, 'camera_transform', camera_transform, (B, 4, 3))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    if Bv not in (1, B):
        raise RuntimeError(f'{fn}: vertices batch {Bv} must be 1 or the camera batch {B}')
    if faces.dtype != torch.int64:
        raise RuntimeError(f'{fn}: faces must be int64')
    sfx = _sfx(vertices, fn)
    _check_dtype(fn, vertices, camera_proj=camera_proj, camera_transform=camera_transform,
                 face_features=face_features)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    vertices, faces = vertices.contiguous(), faces.contiguous()
    camera_proj, camera_transform = camera_proj.contiguous(), camera_transform.contiguous()
    feat = face_features.contiguous()
    opts = dict(device=dev, dtype=vertices.dtype)
    fvc = torch.empty((B, F, 3, 3), **opts)
    fvi = torch.empty((B, F, 3, 2), **opts)
    nrm = torch.empty((B, F, 3), **opts)
    interp = torch.empty((B, height, width, D), **opts)
    face_idx = torch.empty((B, height, width), device=dev, dtype=torch.long)
    weights = torch.empty((B, height, width, 3), **opts)
    soft = torch.empty((B, height, width), **opts)
    nb = int(_lib.load().kd_dibr_workspace_size(B, height, width, F, knum,
                                                1 if vertices.dtype == torch.float64 else 0))
    if vertices.dtype == torch.float32:
        _lib.tile_history_buffer(dev)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    _lib.call(f'kd_dibr_rasterization_forward_vertices_{sfx}', B, height, width, Bv, V, F, D,
              _ptr(vertices), _ptr(faces), _ptr(camera_proj), _ptr(camera_transform), _ptr(feat),
              float(multiplier), float(eps), float(sigmainv), float(boxlen), knum, _ptr(fvc),
              _ptr(fvi), _ptr(nrm), _ptr(interp), _ptr(face_idx), _ptr(weights), _ptr(soft),
              1 if want_grad else 0, _ptr(grad_buffers[0]) if grad_buffers else None,
              _ptr(grad_buffers[1]) if grad_buffers else None, _ptr(ws), nb, _stream(dev))
    return fvc, fvi, nrm, interp, face_idx, weights, soft, ws


def dibr_soft_mask_backward_lists_ws(grad_soft, soft, face_idx, close_prob, close_idx,
                                     close_type, fvi_scaled, sigmainv, multiplier, workspace):
    """dibr_soft_mask_backward_cuda over the lists of dibr_rasterization_forward_fused(...,
    with_lists=True), given that call's workspace: the rows without listed faces are skipped
    exactly (kd_dibr_rasterization_soft_backward_lists)."""
    fn = 'dibr_soft_mask_backward'
    dev = _check_same_gpu(fn, grad_soft=grad_soft, soft=soft, close_prob=close_prob)
    B, H, W, K = close_prob.shape
    F = fvi_scaled.shape[1]
    sfx = _sfx(fvi_scaled, fn)
    g = torch.empty_like(fvi_scaled)
    _lib.call(f'kd_dibr_rasterization_soft_backward_lists_{sfx}', B, H, W, F, K,
              _ptr(grad_soft.contiguous()), _ptr(soft), _ptr(face_idx), _ptr(close_prob),
              _ptr(close_idx), _ptr(close_type), _ptr(fvi_scaled), float(sigmainv),
              float(multiplier), _ptr(g), _ptr(workspace), workspace.numel(), _stream(dev))
    return g


def dibr_rasterization_backward_fused(grad_interp, grad_soft, face_idx, weights, soft,
                                      face_vertices_image, face_features, eps, multiplier,
                                      boxlen, sigmainv, knum, workspace, need_feat=True,
                                      grad_buffers=None, iou=None):
    """Gradients (grad_fvi, grad_feat or None) of the fused forward, from its workspace;
    grad_buffers: the (grad_fvi, grad_feat) the forward zeroed, filled in place.  iou =
    (gt_mask, iou_stats, grad_iou_loss (device scalar)): the fused mask_iou's gradient is added
    to grad_soft inside the kernel (kd_dibr_rasterization_iou_backward)."""
    dev = face_idx.device
    B, F = face_vertices_image.shape[:2]
    H, W = face_idx.shape[1:3]
    D = face_features.shape[-1]
    sfx = _sfx(face_vertices_image, 'dibr_rasterization_backward')
    zeroed = grad_buffers is not None and (grad_buffers[1] is not None or not need_feat)
    if zeroed:
        gfvi, gfeat = grad_buffers[0], grad_buffers[1] if need_feat else None
    else:
        gfvi = torch.empty_like(face_vertices_image)
        gfeat = torch.empty_like(face_features) if need_feat else None
    c = (lambda t: None if t is None else t.contiguous())  # noqa: E731
    if iou is not None:
        gt, stats, g_loss = iou
        _lib.call(f'kd_dibr_rasterization_iou_backward_{sfx}', B, H, W, F, D,
                  _ptr(c(grad_interp)), _ptr(c(grad_soft)), _ptr(c(g_loss)), _ptr(c(gt)),
                  _ptr(stats), _ptr(face_idx), _ptr(weights), _ptr(soft),
                  _ptr(face_vertices_image), _ptr(face_features), float(eps), float(multiplier),
                  float(boxlen), float(sigmainv), int(knum), _ptr(gfvi), _ptr(gfeat),
                  1 if zeroed else 0, _ptr(workspace), workspace.numel(), _stream(dev))
        return gfvi, gfeat
    _lib.call(f'kd_dibr_rasterization_backward_{sfx}', B, H, W, F, D, _ptr(c(grad_interp)),
              _ptr(c(grad_soft)), _ptr(face_idx), _ptr(weights), _ptr(soft),
              _ptr(face_vertices_image), _ptr(face_features), float(eps), float(multiplier),
              float(boxlen), float(sigmainv), int(knum), _ptr(gfvi), _ptr(gfeat),
              1 if zeroed else 0, _ptr(workspace), workspace.numel(), _stream(dev))
    return gfvi, gfeat


def dibr_rasterization_backward_vertices(grad_interp, grad_soft, face_idx, weights, soft,
                                         face_vertices_image, face_features, eps, multiplier,
                                         boxlen, sigmainv, knum, workspace, faces, fvc,
                                         camera_proj, camera_transform, vertex_batch,
                                         num_vertices, need_feat=True, grad_feat_buffer=None):
    """Gradients (grad_vertices (vertex_batch, V, 3), grad_feat or None) of prepare_vertices +
    the fused DIB-R forward, with the face -> vertex step inside the backward kernel
    (kd_dibr_rasterization_backward_vertices).  grad_feat_buffer: the grad_feat the forward
    zeroed (filled in place)."""
    dev = face_idx.device
    B, F = face_vertices_image.shape[:2]
    H, W = face_idx.shape[1:3]
    D = face_features.shape[-1]
    sfx = _sfx(face_vertices_image, 'dibr_rasterization_backward')
    gvert = torch.empty((vertex_batch, num_vertices, 3), device=dev,
                        dtype=face_vertices_image.dtype)
    zeroed = need_feat and grad_feat_buffer is not None
    gfeat = (grad_feat_buffer if zeroed else torch.empty_like(face_features)) if need_feat \
        else None
    c = (lambda t: None if t is None else t.contiguous())  # noqa: E731
    _lib.call(f'kd_dibr_rasterization_backward_vertices_{sfx}', B, H, W, F, D,
              _ptr(c(grad_interp)), _ptr(c(grad_soft)), _ptr(face_idx), _ptr(weights),
              _ptr(soft), _ptr(face_vertices_image), _ptr(face_features), float(eps),
              float(multiplier), float(boxlen), float(sigmainv), int(knum), int(vertex_batch),
              int(num_vertices), _ptr(faces), _ptr(fvc), _ptr(camera_proj),
              _ptr(camera_transform), _ptr(gvert), _ptr(gfeat), 1 if zeroed else 0,
              _ptr(workspace), workspace.numel(), _stream(dev))
    return gvert, gfeat


# -------------------------------------------------------------------------------------------
# mask_iou (kaolin/metrics/render.py:18-40) and texture_mapping (render/mesh/utils.py:23-76),
# SURVEY §8 f2
# -------------------------------------------------------------------------------------------
def mask_iou_forward(lhs, rhs):
    """lhs, rhs (B, H, W) -> (loss (), stats (B, 2) = (U_b, D_b), iou (B,))."""
    fn = 'mask_iou'
    dev = _check_same_gpu(fn, lhs_mask=lhs, rhs_mask=rhs)
    if lhs.dim() != 3:
        raise RuntimeError(f'{fn}: expected (batch, height, width) masks, got {list(lhs.shape)}')
    _check_size(fn, 'rhs_mask', rhs, lhs.shape)
    sfx = _sfx(lhs, fn)
    _check_dtype(fn, lhs, rhs_mask=rhs)
    B = lhs.shape[0]
    P = lhs.shape[1] * lhs.shape[2]
    lhs, rhs = lhs.contiguous(), rhs.contiguous()
    opts = dict(device=dev, dtype=lhs.dtype)
    loss = torch.empty((), **opts)
    stats = torch.empty((B, 2), **opts)
    iou = torch.empty((B,), **opts)
    nb = int(_lib.load().kd_mask_iou_workspace_size(B, P, 1 if lhs.dtype == torch.float64 else 0))
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    _lib.call(f'kd_mask_iou_forward_{sfx}', B, P, _ptr(lhs), _ptr(rhs), _ptr(loss), _ptr(stats),
              _ptr(iou), _ptr(ws), nb, _stream(dev))
    return loss, stats, iou


def mask_iou_backward(grad_loss, lhs, rhs, stats, need_lhs=True, need_rhs=True):
    """Gradients (grad_lhs or None, grad_rhs or None); grad_loss is a device scalar."""
    dev = lhs.device
    B = lhs.shape[0]
    P = lhs.shape[1] * lhs.shape[2]
    sfx = _sfx(lhs, 'mask_iou_backward')
    lhs, rhs = lhs.contiguous(), rhs.contiguous()
    g = grad_loss.reshape(()).to(lhs.dtype).contiguous()
    gl = torch.empty_like(lhs) if need_lhs else None
    gr = torch.empty_like(rhs) if need_rhs else None
    _lib.call(f'kd_mask_iou_backward_{sfx}', B, P, _ptr(lhs), _ptr(rhs), _ptr(stats), _ptr(g),
              _ptr(gl), _ptr(gr), _stream(dev))
    return gl, gr


_TEX_MODES = {'nearest': 0, 'bilinear': 1}


def _texture_args(fn, coords, tex, mode):
    dev = _check_same_gpu(fn, texture_coordinates=coords, texture_maps=tex)
    if mode not in _TEX_MODES:
        raise RuntimeError(f'{fn}: mode must be "nearest" or "bilinear", got {mode!r}')
    if coords.shape[-1] != 2 or coords.dim() < 3:
        raise RuntimeError(f'{fn}: texture_coordinates must be (batch, ..., 2), got '
                           f'{list(coords.shape)}')
    if tex.dim() != 4:
        raise RuntimeError(f'{fn}: texture_maps must be (batch, channels, h, w), got '
                           f'{list(tex.shape)}')
    B = coords.shape[0]
    if tex.shape[0] not in (1, B):
        raise RuntimeError(f'{fn}: texture batch {tex.shape[0]} must be 1 or the coordinate '
                           f'batch {B}')
    sfx = _sfx(tex, fn)
    _check_dtype(fn, tex, texture_coordinates=coords)
    C, Ht, Wt = tex.shape[1:]
    tex_c = tex.contiguous()
    # a batch-1 texture is shared by every view (read in place, batch stride 0)
    bstride = C * Ht * Wt if tex.shape[0] == B else 0
    N = coords[0, ..., 0].numel() if B > 0 else 0
    return dev, sfx, B, N, C, Ht, Wt, tex_c, bstride


def texture_mapping_forward(coords, tex, mode):
    """coords (B, ..., 2), texture (B, C, Ht, Wt) -> (B, ..., C)."""
    fn = 'texture_mapping'
    dev, sfx, B, N, C, Ht, Wt, tex_c, bs = _texture_args(fn, coords, tex, mode)
    coords = coords.contiguous()
    out = torch.empty((*coords.shape[:-1], C), device=dev, dtype=tex.dtype)
    _lib.call(f'kd_texture_mapping_forward_{sfx}', B, N, C, Ht, Wt, _ptr(coords), _ptr(tex_c), bs,
              _TEX_MODES[mode], _ptr(out), _stream(dev))
    return out


def texture_mapping_backward(grad_out, coords, tex, mode, need_coords=True, need_tex=True):
    """(grad_coords or None, grad_tex or None); a shared (batch-1) texture gets the gradient
    summed over the views."""
    fn = 'texture_mapping_backward'
    dev, sfx, B, N, C, Ht, Wt, tex_c, bs = _texture_args(fn, coords, tex, mode)
    coords = coords.contiguous()
    go = grad_out.contiguous()
    gc = torch.empty_like(coords) if need_coords else None
    gt = None
    if need_tex:
        gt = torch.empty(tex.shape, device=dev, dtype=tex.dtype)
    # per-block backward: dense (B, h, w, 2) coordinates as 16 x 16 sample blocks, runs of
    # same-cell samples summed across the lanes of a row (DPP), LDS texel sums (kd_tex_bwd);
    # faster than the texel-tile lists (kd_texture_mapping_backward_tiled) on the C3 render
    row = coords.shape[2] if coords.dim() == 4 else 0  # dense (B, h, w, 2): 16 x 16 blocks
    _lib.call(f'kd_texture_mapping_backward_{sfx}', B, N, C, Ht, Wt, _ptr(coords), _ptr(tex_c),
              bs, _TEX_MODES[mode], row, _ptr(go), _ptr(gt), _ptr(gc), _stream(dev))
    return gc, gt


# -------------------------------------------------------------------------------------------
# nvdiffrast_fwd compatibility (rasterization.py:145-241), SURVEY §8 f4
# -------------------------------------------------------------------------------------------
def rast_interpolate(rast, face_features):
    """rast (B, H, W, 4) from an external forward, features (B, F, 3, D) ->
    (interp (B, H, W, D), face_idx (B, H, W) int64, weights (B, H, W, 3))."""
    fn = 'rast_interpolate'
    dev = _check_same_gpu(fn, rast=rast, face_features=face_features)
    if rast.dim() != 4 or rast.shape[-1] != 4:
        raise RuntimeError(f'{fn}: rast must be (batch, height, width, 4), got {list(rast.shape)}')
    B, H, W = rast.shape[:3]
    if face_features.dim() != 4 or face_features.shape[0] != B or face_features.shape[2] != 3:
        raise RuntimeError(f'{fn}: face_features must be (batch, num_faces, 3, D), got '
                           f'{list(face_features.shape)}')
    F, D = face_features.shape[1], face_features.shape[3]
    sfx = _sfx(face_features, fn)
    rast = rast.to(face_features.dtype).contiguous()
    feat = face_features.contiguous()
    opts = dict(device=dev, dtype=feat.dtype)
    interp = torch.empty((B, H, W, D), **opts)
    face_idx = torch.empty((B, H, W), device=dev, dtype=torch.long)
    weights = torch.empty((B, H, W, 3), **opts)
    _lib.call(f'kd_rast_interpolate_{sfx}', B, H, W, F, D, _ptr(rast), _ptr(feat), _ptr(interp),
              _ptr(face_idx), _ptr(weights), _stream(dev))
    return interp, face_idx, weights


# -------------------------------------------------------------------------------------------
# deftet_sparse_render (deftet.py:269-417 -> deftet.cpp), SURVEY §8 f3
# -------------------------------------------------------------------------------------------
def deftet_sparse_render_forward(pixel_coords, render_ranges, face_vertices_z,
                                 face_vertices_image, face_features, knum, eps):
    """-> (interp (B, P, knum, D), face_idx (B, P, knum), weights (B, P, knum, 3))."""
    fn = 'deftet_sparse_render'
    dev = _check_same_gpu(fn, pixel_coords=pixel_coords, render_ranges=render_ranges,
                          face_vertices_z=face_vertices_z,
                          face_vertices_image=face_vertices_image, face_features=face_features)
    B, F = face_vertices_z.shape[:2]
    P = pixel_coords.shape[1]
    D = face_features.shape[-1]
    _check_size(fn, 'pixel_coords', pixel_coords, (B, P, 2))
    _check_size(fn, 'render_ranges', render_ranges, (B, P, 2))
    _check_size(fn, 'face_vertices_z', face_vertices_z, (B, F, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    sfx = _sfx(face_vertices_image, fn)
    _check_dtype(fn, face_vertices_image, pixel_coords=pixel_coords, render_ranges=render_ranges,
                 face_vertices_z=face_vertices_z, face_features=face_features)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    c = [t.contiguous() for t in (pixel_coords, render_ranges, face_vertices_z,
                                  face_vertices_image, face_features)]
    opts = dict(device=dev, dtype=face_vertices_image.dtype)
    interp = torch.empty((B, P, knum, D), **opts)
    face_idx = torch.empty((B, P, knum), device=dev, dtype=torch.long)
    weights = torch.empty((B, P, knum, 3), **opts)
    nb = int(_lib.load().kd_deftet_workspace_size(B, F, 1 if sfx == 'f64' else 0))
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    _lib.call(f'kd_deftet_sparse_render_forward_{sfx}', B, P, F, knum, D, *(_ptr(t) for t in c),
              float(eps), _ptr(interp), _ptr(face_idx), _ptr(weights), _ptr(ws), nb,
              _stream(dev))
    return interp, face_idx, weights


def deftet_sparse_render_backward(grad_interp, face_idx, weights, face_vertices_image,
                                  face_features, eps, need_feat=True):
    """-> (grad_face_vertices_image, grad_face_features or None)."""
    dev = face_idx.device
    B, P, K = face_idx.shape
    F, D = face_vertices_image.shape[1], face_features.shape[-1]
    sfx = _sfx(face_vertices_image, 'deftet_sparse_render_backward')
    gfvi = torch.empty_like(face_vertices_image)
    gfeat = torch.empty_like(face_features) if need_feat else None
    _lib.call(f'kd_deftet_sparse_render_backward_{sfx}', B, P, F, K, D,
              _ptr(grad_interp.contiguous()), _ptr(face_idx), _ptr(weights),
              _ptr(face_vertices_image), _ptr(face_features), float(eps), _ptr(gfvi),
              _ptr(gfeat), _stream(dev))
    return gfvi, gfeat


def deftet_sparse_render_forward_cuda(face_vertices_z, face_vertices_image, face_bboxes,
                                      pixel_coords, pixel_depth_ranges, knum, eps):
    """deftet.cpp:48-106 (bindings.cpp:81) -> [selected_face_idx, pixel_depths, w0, w1]: per
    pixel the first knum hits in face-index order, unsorted; empty slots -1 / -inf / 0 / 0."""
    fn = 'deftet_sparse_render_forward_cuda'
    dev = _check_same_gpu(fn, face_vertices_z=face_vertices_z,
                          face_vertices_image=face_vertices_image, face_bboxes=face_bboxes,
                          pixel_coords=pixel_coords, pixel_depth_ranges=pixel_depth_ranges)
    _check_contiguous(fn, face_vertices_z=face_vertices_z,
                      face_vertices_image=face_vertices_image, face_bboxes=face_bboxes,
                      pixel_coords=pixel_coords, pixel_depth_ranges=pixel_depth_ranges)
    B, F = face_vertices_z.shape[:2]
    P = pixel_coords.shape[1]
    _check_size(fn, 'face_vertices_z', face_vertices_z, (B, F, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_bboxes', face_bboxes, (B, F, 4))
    _check_size(fn, 'pixel_coords', pixel_coords, (B, P, 2))
    _check_size(fn, 'pixel_depth_ranges', pixel_depth_ranges, (B, P, 2))
    sfx = _sfx(face_vertices_z, fn)
    _check_dtype(fn, face_vertices_z, face_vertices_image=face_vertices_image,
                 face_bboxes=face_bboxes, pixel_coords=pixel_coords,
                 pixel_depth_ranges=pixel_depth_ranges)
    knum = int(knum)
    if knum < 1:
        raise RuntimeError(f'{fn}: knum must be >= 1, got {knum}')
    opts = dict(device=dev, dtype=face_vertices_z.dtype)
    face_idx = torch.empty((B, P, knum), device=dev, dtype=torch.long)
    depths = torch.empty((B, P, knum), **opts)
    w0 = torch.empty((B, P, knum), **opts)
    w1 = torch.empty((B, P, knum), **opts)
    nb = int(_lib.load().kd_deftet_workspace_size(B, F, 1 if sfx == 'f64' else 0))
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    _lib.call(f'kd_deftet_sparse_render_forward_raw_{sfx}', B, P, F, knum, _ptr(face_vertices_z),
              _ptr(face_vertices_image), _ptr(face_bboxes), _ptr(pixel_coords),
              _ptr(pixel_depth_ranges), float(eps), _ptr(face_idx), _ptr(depths), _ptr(w0),
              _ptr(w1), _ptr(ws), nb, _stream(dev))
    return [face_idx, depths, w0, w1]


def deftet_sparse_render_backward_cuda(grad_interpolated_features, face_idx, weights,
                                       face_vertices_image, face_features, eps):
    """deftet.cpp:108-160 (bindings.cpp:82) -> [grad_face_vertices_image, grad_face_features]"""
    fn = 'deftet_sparse_render_backward_cuda'
    _check_same_gpu(fn, grad_interpolated_features=grad_interpolated_features,
                    face_idx=face_idx, weights=weights, face_vertices_image=face_vertices_image,
                    face_features=face_features)
    _check_contiguous(fn, grad_interpolated_features=grad_interpolated_features,
                      face_idx=face_idx, weights=weights,
                      face_vertices_image=face_vertices_image, face_features=face_features)
    B, P, K, D = grad_interpolated_features.shape
    F = face_vertices_image.shape[1]
    _check_size(fn, 'face_idx', face_idx, (B, P, K))
    _check_size(fn, 'weights', weights, (B, P, K, 3))
    _check_size(fn, 'face_vertices_image', face_vertices_image, (B, F, 3, 2))
    _check_size(fn, 'face_features', face_features, (B, F, 3, D))
    _sfx(face_vertices_image, fn)
    _check_dtype(fn, face_vertices_image, grad_interpolated_features=grad_interpolated_features,
                 weights=weights, face_features=face_features)
    gfvi, gfeat = deftet_sparse_render_backward(grad_interpolated_features, face_idx, weights,
                                                face_vertices_image, face_features, eps)
    return [gfvi, gfeat]


render = types.SimpleNamespace(mesh=types.SimpleNamespace(
    packed_rasterize_forward_cuda=packed_rasterize_forward_cuda,
    rasterize_backward_cuda=rasterize_backward_cuda,
    dibr_soft_mask_forward_cuda=dibr_soft_mask_forward_cuda,
    dibr_soft_mask_backward_cuda=dibr_soft_mask_backward_cuda,
    rasterize_forward_fused=rasterize_forward_fused,
    rasterize_backward_autograd=rasterize_backward_autograd,
    dibr_soft_mask_forward_fused=dibr_soft_mask_forward_fused,
    dibr_soft_mask_backward_binned=dibr_soft_mask_backward_binned,
    dibr_rasterization_forward_fused=dibr_rasterization_forward_fused,
    dibr_rasterization_forward_vertices=dibr_rasterization_forward_vertices,
    dibr_rasterization_backward_fused=dibr_rasterization_backward_fused,
    dibr_soft_mask_backward_lists_ws=dibr_soft_mask_backward_lists_ws,
    dibr_rasterization_backward_vertices=dibr_rasterization_backward_vertices,
    prepare_vertices_forward=prepare_vertices_forward,
    prepare_vertices_backward=prepare_vertices_backward,
    prepare_vertices_backward_from_vertices=prepare_vertices_backward_from_vertices,
    texture_mapping_forward=texture_mapping_forward,
    texture_mapping_backward=texture_mapping_backward,
    rast_interpolate=rast_interpolate,
    deftet_sparse_render_forward=deftet_sparse_render_forward,
    deftet_sparse_render_backward=deftet_sparse_render_backward,
    deftet_sparse_render_forward_cuda=deftet_sparse_render_forward_cuda,
    deftet_sparse_render_backward_cuda=deftet_sparse_render_backward_cuda,
))
metrics = types.SimpleNamespace(mask_iou_forward=mask_iou_forward,
                                mask_iou_backward=mask_iou_backward)
