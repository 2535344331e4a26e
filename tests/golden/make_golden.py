"""Generate the golden fixtures under tests/golden/ from the reference (run ONCE, in the build
container, where /root/reference exists).  Never imported by the test suite or on the GPU box:
only the .npz files this script writes travel.

What is produced (all small, compressed):

* ``simple.npz``      -- the 2-mesh x 3-triangle case of
  ``tests/python/kaolin/render/mesh/test_dibr.py:43-62`` with the reference's soft-mask goldens
  (``tests/samples/dibr/simple/*.pt``, "From Kaolin V0.10.0") and its rasterize face_idx golden
  ``new_face_idx_35_31.pt``.
* ``sphere_inputs.npz`` -- the 960-face ``tests/samples/model.obj`` sphere seen by the 3 test
  cameras (``test_rasterization.py:50-117``), fp32 and fp64, flip in {0,1}: face_vertices_z,
  face_vertices_image, face_uvs, valid_faces (the "middle z" mask, ``test_rasterization.py:93-98``),
  face_normals_z (``test_dibr.py:454-458``).
* ``sphere_softmask.npz`` -- the reference's sphere soft-mask goldens (``tests/samples/dibr/sphere``).
* ``sphere_raster_naive.npz`` -- the reference's own rasterize oracle
  ``_naive_deftet_sparse_render(..., knum=1)`` (``kaolin/render/mesh/deftet.py:101-267``) run on the
  sphere inputs, forward (face_idx, interp) and autograd backward (grads of face_vertices_image and
  face_uvs for a seeded grad_out), exactly as ``test_rasterization.py:136-232`` uses it.
* ``soup_raster_naive.npz`` -- the same oracle on three seeded random triangle soups (overlaps,
  depth ordering, both windings).

The reference package is imported with four ``sys.modules`` stubs for its compiled / removed
dependencies: ``kaolin._C``, ``kaolin.ops.mesh.triangle_hash``,
``kaolin.ops.conversions.mise`` and ``torch._six``.  None of them is on the rasterize path.
"""
import math
import os
import sys
import types

import numpy as np
import torch

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    sys.path.insert(0, REF)
    c = types.ModuleType('kaolin._C')
    sys.modules['kaolin._C'] = c
    th = types.ModuleType('kaolin.ops.mesh.triangle_hash')
    th.TriangleHash = object
    sys.modules['kaolin.ops.mesh.triangle_hash'] = th
    mise = types.ModuleType('kaolin.ops.conversions.mise')
    mise.MISE = object
    sys.modules['kaolin.ops.conversions.mise'] = mise
    six = types.ModuleType('torch._six')
    six.string_classes = (str, bytes)
    sys.modules['torch._six'] = six
    import kaolin
    return kaolin


def load_pt(path):
    return torch.load(path, map_location='cpu', weights_only=True)


H, W = 35, 31


def simple_case(out):
    d = f'{REF}/tests/samples/dibr/simple'
    fvi = np.array(
        [[[[-0.7, 0.], [0., -0.7], [0., 0.7]],
          [[-0.7, 0.], [0., 0.7], [0., -0.7]],
          [[0., -0.7], [0., 0.7], [0.7, 0.]]],
         [[[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]],
          [[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]],
          [[-0.7, -0.7], [0.7, -0.7], [-0.7, 0.7]]]], dtype=np.float64)
    fvz = np.array(
        [[[-2., -1., -1.], [-2.5, -3., -3.], [-2., -2., -2.]],
         [[-2., -1., -3.], [-2., -2., -2.], [-2., -3., -1.]]], dtype=np.float64)
    out['simple_fvi'] = fvi
    out['simple_fvz'] = fvz
    out['simple_new_face_idx'] = load_pt(f'{d}/new_face_idx_{H}_{W}.pt').numpy().astype(np.int16)
    for sig in (7000, 70):
        for box in (0.02, 0.2):
            tag = f'{sig}_{box}'
            out[f'simple_soft_{tag}'] = load_pt(f'{d}/soft_mask_{H}_{W}_{tag}.pt').numpy()
            idx = load_pt(f'{d}/close_face_idx_{H}_{W}_{tag}.pt').long() - 1
            out[f'simple_close_idx_{tag}'] = idx.numpy().astype(np.int16)
            out[f'simple_close_prob_{tag}'] = load_pt(f'{d}/close_face_dist_{H}_{W}_{tag}.pt').numpy()
            out[f'simple_close_type_{tag}'] = load_pt(
                f'{d}/close_face_dist_type_{H}_{W}_{tag}.pt').numpy().astype(np.uint8)
            out[f'simple_grad_{tag}'] = load_pt(
                f'{d}/grad_face_vertices_image_{H}_{W}_{tag}.pt').numpy()


def sphere_inputs(kal, dtype, flip):
    """Restates the fixtures of test_rasterization.py:37-117 / test_dibr.py:404-458 on CPU."""
    mesh = kal.io.obj.import_mesh(f'{REF}/tests/samples/model.obj', with_materials=True)
    faces = mesh.faces
    if flip:
        faces = torch.flip(faces, dims=(-1,))
    B = 3
    camera_pos = torch.tensor([[0.5, 0.5, 3.], [2., 2., -2.], [3., 0.5, 0.5]], dtype=dtype)[:B]
    look_at = torch.full((B, 3), 0.5, dtype=dtype)
    camera_up = torch.tensor([[0., 1., 0.]], dtype=dtype).repeat(B, 1)
    camera_proj = kal.render.camera.generate_perspective_projection(
        fovyangle=math.pi / 4., dtype=dtype)
    vertices = mesh.vertices.to(dtype).unsqueeze(0)
    vmin = vertices.min(dim=1, keepdims=True)[0]
    vmax = vertices.max(dim=1, keepdims=True)[0]
    vertices = (vertices - vmin) / (vmax - vmin)
    rot, trans = kal.render.camera.generate_rotate_translate_matrices(camera_pos, look_at, camera_up)
    vcam = kal.render.camera.rotate_translate_points(vertices, rot, trans)
    vimg = kal.render.camera.perspective_camera(vcam, camera_proj)
    fvcam = kal.ops.mesh.index_vertices_by_faces(vcam, faces)
    fvz = fvcam[..., -1].contiguous()
    fvi = kal.ops.mesh.index_vertices_by_faces(vimg, faces)
    minz = fvz.reshape(B, -1).min(dim=1, keepdims=True)[0]
    maxz = fvz.reshape(B, -1).max(dim=1, keepdims=True)[0]
    valid = torch.all(fvz < ((minz + maxz) / 2.).unsqueeze(-1), dim=-1)
    uvidx = mesh.face_uvs_idx
    if flip:
        uvidx = torch.flip(uvidx, dims=(-1,))
    uvs = kal.ops.mesh.index_vertices_by_faces(mesh.uvs.unsqueeze(0).to(dtype), uvidx).repeat(B, 1, 1, 1)
    nz = kal.ops.mesh.face_normals(fvcam, unit=True)[..., -1]
    return dict(fvz=fvz, fvi=fvi, uvs=uvs, valid=valid, normals_z=nz, vcam=vcam)


def pixel_grid(B, h, w, dtype):
    """test_rasterization.py:119-126 / :128-134"""
    x = (2 * torch.arange(w, dtype=dtype) + 1 - w) / w
    y = (h - 2 * torch.arange(h, dtype=dtype) - 1.) / h
    return torch.stack([x.reshape(1, 1, -1).repeat(B, h, 1),
                        y.reshape(1, -1, 1).repeat(B, 1, w)], dim=-1).reshape(B, -1, 2)


def naive_raster(kal, fvz, fvi, feats, valid, h, w, with_grad, seed):
    from kaolin.render.mesh.deftet import _naive_deftet_sparse_render
    B = fvz.shape[0]
    dtype = fvz.dtype
    px = pixel_grid(B, h, w, dtype)
    zmin = fvz.reshape(B, -1).min(dim=1)[0]
    zmax = fvz.reshape(B, -1).max(dim=1)[0]
    rr = torch.stack([zmin - 1e-2, zmax + 1e-2], dim=-1).unsqueeze(1).repeat(1, h * w, 1)
    fvi = fvi.detach().clone().requires_grad_(with_grad)
    feats = feats.detach().clone().requires_grad_(with_grad)
    kw = {} if valid is None else {'valid_faces': valid}
    interp, fidx = _naive_deftet_sparse_render(px, rr, fvz, fvi, feats, 1, **kw)
    interp = interp.reshape(B, h, w, feats.shape[-1])
    res = dict(face_idx=fidx.reshape(B, h, w).numpy().astype(np.int32),
               interp=interp.detach().numpy())
    if with_grad:
        g = torch.Generator().manual_seed(seed)
        grad_out = torch.rand(interp.shape, generator=g, dtype=dtype)
        interp.backward(grad_out)
        res['grad_out'] = grad_out.numpy()
        res['grad_fvi'] = fvi.grad.numpy()
        res['grad_feat'] = feats.grad.numpy()
    return res


def soup(nf, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    B = 2
    centers = torch.rand(B, nf, 1, 2, generator=g, dtype=torch.float64) * 1.6 - 0.8
    size = 0.25
    fvi = centers + (torch.rand(B, nf, 3, 2, generator=g, dtype=torch.float64) - 0.5) * size
    fvz = -2. - torch.rand(B, nf, 1, generator=g, dtype=torch.float64) \
        + (torch.rand(B, nf, 3, generator=g, dtype=torch.float64) - 0.5) * 0.4
    feats = torch.rand(B, nf, 3, 3, generator=g, dtype=torch.float64)
    valid = torch.rand(B, nf, generator=g) > 0.3
    return fvz.to(dtype), fvi.to(dtype), feats.to(dtype), valid


def main():
    kal = import_reference()
    torch.set_num_threads(8)
    out = {}
    simple_case(out)
    np.savez_compressed(f'{OUT}/simple.npz', **out)
    print('simple.npz', len(out))

    inp, nai = {}, {}
    for dname, dtype in (('f32', torch.float32), ('f64', torch.float64)):
        for flip in (0, 1):
            s = sphere_inputs(kal, dtype, flip)
            key = f'{dname}_flip{flip}'
            for k in ('fvz', 'fvi', 'uvs', 'valid', 'normals_z'):
                inp[f'{k}_{key}'] = s[k].numpy()
            for v in (0, 1):
                r = naive_raster(kal, s['fvz'], s['fvi'], s['uvs'], s['valid'] if v else None,
                                 H, W, with_grad=True, seed=100 + 10 * flip + v)
                for k, a in r.items():
                    nai[f'{k}_{key}_valid{v}'] = a
            print('sphere', key)
    np.savez_compressed(f'{OUT}/sphere_inputs.npz', **inp)
    np.savez_compressed(f'{OUT}/sphere_raster_naive.npz', **nai)

    d = f'{REF}/tests/samples/dibr/sphere'
    sm = {}
    for sig in (7000, 70):
        for box in (0.02, 0.01):
            tag = f'{sig}_{box}'
            sm[f'soft_{tag}'] = load_pt(f'{d}/soft_mask_{H}_{W}_{tag}.pt').numpy()
            sm[f'close_idx_{tag}'] = (load_pt(f'{d}/close_face_idx_{H}_{W}_{tag}.pt').long() - 1
                                      ).numpy().astype(np.int16)
            sm[f'close_prob_{tag}'] = load_pt(f'{d}/close_face_dist_{H}_{W}_{tag}.pt').numpy()
            sm[f'close_type_{tag}'] = load_pt(
                f'{d}/close_face_dist_type_{H}_{W}_{tag}.pt').numpy().astype(np.uint8)
            sm[f'grad_{tag}'] = load_pt(f'{d}/grad_face_vertices_image_{H}_{W}_{tag}.pt').numpy()
    np.savez_compressed(f'{OUT}/sphere_softmask.npz', **sm)
    print('sphere_softmask.npz')

    so = {}
    for i, (nf, h, w) in enumerate(((60, 24, 20), (150, 40, 48), (200, 33, 17))):
        for dname, dtype in (('f32', torch.float32), ('f64', torch.float64)):
            fvz, fvi, feats, valid = soup(nf, 7 + i, dtype)
            key = f'soup{i}_{dname}'
            so[f'fvz_{key}'] = fvz.numpy()
            so[f'fvi_{key}'] = fvi.numpy()
            so[f'feat_{key}'] = feats.numpy()
            so[f'valid_{key}'] = valid.numpy()
            so[f'hw_{key}'] = np.array([h, w])
            for v in (0, 1):
                r = naive_raster(kal, fvz, fvi, feats, valid if v else None, h, w,
                                 with_grad=True, seed=200 + i)
                for k, a in r.items():
                    so[f'{k}_{key}_valid{v}'] = a
            print('soup', key)
    np.savez_compressed(f'{OUT}/soup_raster_naive.npz', **so)


if __name__ == '__main__':
    main()
