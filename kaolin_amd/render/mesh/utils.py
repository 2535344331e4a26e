"""``prepare_vertices`` -- drop-in for kaolin/render/mesh/utils.py:128-175, and
``texture_mapping`` -- drop-in for utils.py:23-76 (at the end of this file).

The reference moves the vertices to each camera (``pad(v, 1) @ camera_transform``, or
``(v - trans) @ rot^T`` via camera.rotate_translate_points, legacy.py:22-37), projects them
(camera.perspective_camera, legacy.py:120-139), gathers them per face (ops/mesh/mesh.py:24-45)
and computes unit face normals (ops/mesh/trianglemesh.py:313-336).  Here the forward is one HIP
kernel and the backward another (kaolin_amd/csrc/kd_prepare.hip) that walks each vertex's
incident face corners -- the face->vertex scatter of the reference's gather backward without
atomics.  ``vertices`` may have batch 1 with a batch of cameras (as in the reference, by
broadcasting); its gradient is then summed over the views inside the kernel.

Gradients w.r.t. the camera tensors are not produced by the fused kernels: when a camera tensor
requires grad, the reference's PyTorch composition is used instead (same results).
"""
import weakref

import torch
from torch.autograd import Function

from ... import _C

__all__ = ['prepare_vertices', 'texture_mapping']

_ADJ_CACHE = {}  # id(faces) -> (weakref(faces), version, num_vertices, adjacency)


def _adjacency(faces, num_vertices):
    """Vertex -> (face, corner) CSR for `faces`, built once per faces tensor (and version); the
    entry goes away with the tensor."""
    key = id(faces)
    ent = _ADJ_CACHE.get(key)
    if ent is not None and ent[0]() is faces and ent[1] == faces._version \
            and ent[2] == num_vertices:
        return ent[3]
    adj = _C.vertex_face_adjacency(faces, num_vertices)
    ref = weakref.ref(faces, lambda _r, k=key: _ADJ_CACHE.pop(k, None))
    _ADJ_CACHE[key] = (ref, faces._version, num_vertices, adj)
    return adj


class PrepareVerticesHip(Function):
    """torch.autograd.Function: fused prepare_vertices with a gather-form backward."""

    @staticmethod
    def forward(ctx, vertices, faces, camera_proj, camera_transform):
        vertices = vertices.contiguous()
        camera_proj = camera_proj.contiguous()
        camera_transform = camera_transform.contiguous()
        fvc, fvi, nrm = _C.prepare_vertices_forward(vertices, faces, camera_proj,
                                                    camera_transform)
        ctx.save_for_backward(faces, camera_proj, camera_transform, fvc)
        ctx.vertex_batch, ctx.num_vertices = vertices.shape[0], vertices.shape[1]
        ctx.adj = _adjacency(faces, vertices.shape[1]) if ctx.needs_input_grad[0] else None
        ctx.set_materialize_grads(False)
        return fvc, fvi, nrm

    @staticmethod
    def backward(ctx, grad_fvc, grad_fvi, grad_nrm):
        if not ctx.needs_input_grad[0] or (grad_fvc is None and grad_fvi is None
                                           and grad_nrm is None):
            return None, None, None, None
        faces, camera_proj, camera_transform, fvc = ctx.saved_tensors
        adj = ctx.adj
        c = (lambda t: None if t is None else t.contiguous())  # noqa: E731
        g = _C.prepare_vertices_backward(faces, camera_proj, camera_transform, fvc, c(grad_fvc),
                                         c(grad_fvi), c(grad_nrm), adj, ctx.vertex_batch,
                                         ctx.num_vertices)
        return g, None, None, None


def _transform_from_rot_trans(camera_rot, camera_trans):
    """(B,3,3) rotation and (B,3[,1]) translation -> the (B,4,3) transform of
    rotate_translate_points (legacy.py:35-36): p_cam = (p - t) @ R^T = [p, 1] @ [R^T; -t R^T]."""
    rt = camera_rot.permute(0, 2, 1)
    t = camera_trans.reshape(camera_rot.shape[0], 1, 3)
    return torch.cat([rt, -(t @ rt)], dim=1)


def _reference_composition(vertices, faces, camera_proj, camera_transform):
    padded = torch.nn.functional.pad(vertices, (0, 1), mode='constant', value=1.)
    vc = padded @ camera_transform
    pp = vc * camera_proj.view(-1, 1, 3)
    vi = pp[:, :, :2] / pp[:, :, 2:3]
    B = vc.shape[0]
    fvc = torch.index_select(vc, 1, faces.reshape(-1)).reshape(B, faces.shape[0], 3, 3)
    fvi = torch.index_select(vi, 1, faces.reshape(-1)).reshape(B, faces.shape[0], 3, 2)
    n = torch.cross(fvc[:, :, 1] - fvc[:, :, 0], fvc[:, :, 2] - fvc[:, :, 0], dim=2)
    n = n / (n.norm(dim=2, keepdim=True) + 1e-10)
    return fvc, fvi, n


def prepare_vertices(vertices, faces, camera_proj, camera_rot=None, camera_trans=None,
                     camera_transform=None):
    r"""Move and project vertices to the cameras, then index them with faces
    (kaolin/render/mesh/utils.py:128-175).

    Args are the reference's: vertices (B, V, 3) (B may be 1 with a batch of cameras), faces
    (F, 3) int64, camera_proj (3, 1), and either camera_rot (B, 3, 3) + camera_trans (B, 3)
    or camera_transform (B, 4, 3).  Returns (face_vertices_camera (B, F, 3, 3),
    face_vertices_image (B, F, 3, 2), face_normals (B, F, 3)).
    """
    if camera_transform is None:
        assert camera_trans is not None and camera_rot is not None, \
            "camera_transform or camera_trans and camera_rot must be defined"
        camera_transform = _transform_from_rot_trans(camera_rot, camera_trans)
    else:
        assert camera_trans is None and camera_rot is None, \
            "camera_trans and camera_rot must be None when camera_transform is defined"
    if faces.shape[-1] != 3:
        raise NotImplementedError('prepare_vertices is implemented for triangle meshes')
    if camera_transform.shape[0] != vertices.shape[0] and vertices.shape[0] != 1:
        raise RuntimeError('vertices batch must be 1 or the camera batch')
    if camera_proj.requires_grad or camera_transform.requires_grad:
        return _reference_composition(vertices, faces, camera_proj, camera_transform)
    return PrepareVerticesHip.apply(vertices, faces, camera_proj, camera_transform)


class TextureMappingHip(Function):
    """torch.autograd.Function over kd_texture_mapping_forward / _backward."""

    @staticmethod
    def forward(ctx, texture_coordinates, texture_maps, mode):
        out = _C.render.mesh.texture_mapping_forward(texture_coordinates, texture_maps, mode)
        ctx.save_for_backward(texture_coordinates, texture_maps)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, grad_out):
        coords, tex = ctx.saved_tensors
        gc, gt = _C.render.mesh.texture_mapping_backward(
            grad_out, coords, tex, ctx.mode, need_coords=ctx.needs_input_grad[0],
            need_tex=ctx.needs_input_grad[1])
        return gc, gt, None


def texture_mapping(texture_coordinates, texture_maps, mode='nearest'):
    r"""Interpolate texture_maps at texture_coordinates (kaolin/render/mesh/utils.py:23-76).

    Args:
        texture_coordinates (torch.Tensor): (batch_size, h, w, 2) dense image uvs or
            (batch_size, num_points, 2) sparse uvs, in [0, 1] (clamped), OpenGL convention
            (v from bottom to top).
        texture_maps (torch.Tensor): (batch_size, num_channels, h', w').  As an extension of the
            reference a batch of 1 is shared by every view (no ``repeat`` needed; its gradient
            is summed over the views).
        mode (str): 'nearest' or 'bilinear' (grid_sample, align_corners=False, border padding).

    Returns:
        (torch.Tensor): (batch_size, h, w, num_channels) or (batch_size, num_points,
        num_channels).
    """
    return TextureMappingHip.apply(texture_coordinates, texture_maps, mode)
