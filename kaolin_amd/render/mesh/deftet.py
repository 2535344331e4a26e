"""``deftet_sparse_render`` -- drop-in for kaolin/render/mesh/deftet.py:269-417.

Every intersection of each pixel's ray with the mesh, sorted by depth (DefTet, Gao et al. 2020).
The reference computes the face boxes in torch, runs one CUDA kernel that scans every face for
every pixel, then sorts / gathers / interpolates in torch (deftet.py:287-313).  Here the forward is
two HIP launches (64-face chunk boxes, then one wave per pixel that walks only the chunks whose
box holds the pixel, keeps the first knum hits, ranks them by depth and writes the sorted face
index, weights and interpolated features) and the backward is the rasterize backward kernel over
the (pixel, slot) samples (kaolin_amd/csrc/kd_deftet.hip).
"""
import torch
from torch.autograd import Function

from ... import _C

__all__ = ['deftet_sparse_render']


class DeftetSparseRenderer(Function):
    """torch.autograd.Function for :func:`deftet_sparse_render` (deftet.py:269-330)."""

    @staticmethod
    def forward(ctx, pixel_coords, render_ranges, face_vertices_z, face_vertices_image,
                face_features, knum, eps):
        face_vertices_image = face_vertices_image.contiguous()
        face_features = face_features.contiguous()
        interp, face_idx, weights = _C.render.mesh.deftet_sparse_render_forward(
            pixel_coords, render_ranges, face_vertices_z, face_vertices_image, face_features,
            knum, eps)
        ctx.save_for_backward(face_idx, weights, face_vertices_image, face_features)
        ctx.mark_non_differentiable(face_idx)
        ctx.eps = eps
        return interp, face_idx

    @staticmethod
    def backward(ctx, grad_interpolated_features, grad_face_idx):
        face_idx, weights, fvi, feat = ctx.saved_tensors
        need_fvi, need_feat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        if not (need_fvi or need_feat):
            return None, None, None, None, None, None, None
        gfvi, gfeat = _C.render.mesh.deftet_sparse_render_backward(
            grad_interpolated_features, face_idx, weights, fvi, feat, ctx.eps,
            need_feat=need_feat)
        return None, None, None, gfvi if need_fvi else None, gfeat, None, None


def deftet_sparse_render(pixel_coords, render_ranges, face_vertices_z, face_vertices_image,
                         face_features, knum=300, eps=1e-8):
    r"""Fully differentiable volumetric renderer of *Gao et al.* (deftet.py:333-417).

    Args are the reference's: pixel_coords (B, P, 2), render_ranges (B, P, 2) = [min, max) depth,
    face_vertices_z (B, F, 3), face_vertices_image (B, F, 3, 2), face_features (B, F, 3, D) or a
    list of such, knum, eps.  Returns (features (B, P, knum, D) or tuple, face_idx (B, P, knum)
    int64, -1 = void), sorted by depth, descending.  Not differentiable w.r.t. pixel_coords,
    render_ranges and face_vertices_z (as in the reference).
    """
    _face_features = torch.cat(face_features, dim=-1) \
        if isinstance(face_features, (list, tuple)) else face_features
    image_features, face_idx = DeftetSparseRenderer.apply(
        pixel_coords, render_ranges, face_vertices_z, face_vertices_image, _face_features, knum,
        eps)
    if isinstance(face_features, (list, tuple)):
        _image_features = []
        cur_idx = 0
        for face_feature in face_features:
            _image_features.append(image_features[..., cur_idx:cur_idx + face_feature.shape[-1]])
            cur_idx += face_feature.shape[-1]
        image_features = tuple(_image_features)
    return image_features, face_idx
