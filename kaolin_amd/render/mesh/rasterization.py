"""``rasterize`` -- drop-in for kaolin/render/mesh/rasterization.py:390-506 (backend 'cuda').

The reference's ``RasterizeCuda`` (rasterization.py:243-388) packs the valid faces with
``torch.where`` (a device->host sync), scales, builds boxes, calls the packed kernel and remaps
the packed index.  Here all of that happens inside one HIP launch sequence (binning + tile
raster, kaolin_amd/csrc/kd_raster.hip) with no host sync; the outputs are bit-identical.
The backward is the tile kernel (per-tile LDS sums, one atomic per tile and face), same math
as rasterization_cuda.cu:238-402.
"""
import torch
from torch.autograd import Function

from ... import _C

__all__ = ['rasterize']


class RasterizeCuda(Function):
    """torch.autograd.Function for ``rasterize`` with backend 'cuda' (rasterization.py:243)."""

    @staticmethod
    def forward(ctx, height, width, face_vertices_z, face_vertices_image, face_features,
                valid_faces, multiplier, eps):
        face_vertices_z = face_vertices_z.contiguous()
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        interpolated_features, face_idx, output_weights, valid_u8 = \
            _C.render.mesh.rasterize_forward_fused(
                height, width, face_vertices_z, face_vertices_image, face_features,
                valid_faces, multiplier, eps)
        ctx.save_for_backward(face_idx, output_weights, face_vertices_image, face_features)
        ctx.mark_non_differentiable(face_idx)
        ctx.eps = eps
        ctx.multiplier = multiplier
        return interpolated_features, face_idx

    @staticmethod
    def backward(ctx, grad_interpolated_features, grad_face_idx):
        face_idx, output_weights, face_vertices_image, face_features = ctx.saved_tensors
        need_fvi, need_feat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        if not (need_fvi or need_feat):
            return None, None, None, None, None, None, None, None
        grad_fvi, grad_feat = _C.render.mesh.rasterize_backward_autograd(
            grad_interpolated_features.contiguous(), face_idx, output_weights,
            face_vertices_image, face_features, ctx.eps, need_feat=need_feat)
        return None, None, None, grad_fvi if need_fvi else None, grad_feat, None, None, None


def rasterize(height, width, face_vertices_z, face_vertices_image, face_features,
              valid_faces=None, multiplier=None, eps=None, backend='cuda'):
    r"""Fully differentiable rasterization (rasterization.py:390-506), HIP backend.

    Args and returns are the reference's: ``face_vertices_z`` (B, F, 3),
    ``face_vertices_image`` (B, F, 3, 2), ``face_features`` (B, F, 3, D) or a list of such,
    ``valid_faces`` (B, F) bool; returns (features (B, H, W, D) or tuple, face_idx (B, H, W)
    int64 with -1 for empty).  Defaults: multiplier 1000, eps 1e-8.  ``backend`` must be 'cuda'
    (the name is kept for drop-in compatibility; it runs the gfx950 kernels).  The nvdiffrast
    backends of the reference are not provided (NVIDIA-only OpenGL).
    """
    if multiplier is None:
        multiplier = 1000
    if eps is None:
        eps = 1e-8
    if backend != 'cuda':
        raise ValueError(f'"{backend}" is not a valid backend, valid choices are ["cuda"] '
                         '(nvdiffrast is not available on MI355X)')
    _face_features = torch.cat(face_features, dim=-1) \
        if isinstance(face_features, (list, tuple)) else face_features
    image_features, face_idx = RasterizeCuda.apply(
        height, width, face_vertices_z, face_vertices_image, _face_features, valid_faces,
        multiplier, eps)
    if isinstance(face_features, (list, tuple)):
        _image_features = []
        cur_idx = 0
        for face_feature in face_features:
            _image_features.append(image_features[..., cur_idx:cur_idx + face_feature.shape[-1]])
            cur_idx += face_feature.shape[-1]
        image_features = tuple(_image_features)
    return image_features, face_idx
