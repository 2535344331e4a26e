"""Generate tests/golden/f2.npz -- fixtures for SURVEY.md §8 f2 (mask_iou, texture_mapping) from
the reference itself (run ONCE, in the build container, where /root/reference exists; only the
.npz travels).

* the reference's own test cases, inputs and expected values:
  ``tests/python/kaolin/metrics/test_render.py:24-52`` (mask_iou = 0.3105) and
  ``tests/python/kaolin/render/mesh/test_utils.py:24-120`` (texture_mapping sparse 1-d / 3-d and
  dense 3-d, nearest and bilinear) -- the expected tensors are produced here by the reference
  functions and checked against the test's literals before being saved;
* seeded random cases run through the reference's ``kaolin.metrics.render.mask_iou``
  (render.py:18-40) and ``kaolin.render.mesh.utils.texture_mapping`` (utils.py:23-76) on the CPU,
  forward and autograd backward (seeded incoming gradients), fp32 and fp64, including
  coordinates outside [0, 1] and exactly on texel centres / borders.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import import_reference  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'f2.npz')
DT = {'f32': torch.float32, 'f64': torch.float64}


def reference_test_inputs():
    lhs = torch.tensor([[[0., 0.2, 0.1, 1.], [0.5, 0.5, 0.9, 0.9], [0., 1., 1., 0.9],
                         [0.8, 0.7, 0.2, 0.1]],
                        [[1., 1., 1., 1.], [1., 1., 1., 1.], [1., 1., 1., 1.],
                         [1., 1., 1., 1.]]], dtype=torch.float64)
    rhs = torch.tensor([[[0.1, 0.3, 0.3, 0.9], [0.5, 0.5, 1., 0.3], [0., 0.9, 0.9, 0.8],
                         [1., 1., 0., 0.]],
                        [[0.3, 0.6, 0.7, 0.7], [0.8, 0.9, 0.9, 1.], [1., 0.9, 0.9, 0.5],
                         [0.8, 0.7, 0.8, 0.5]]], dtype=torch.float64)
    l1 = torch.tensor([[11.0, 12.0, 13.0, 14.0, 15.0], [21.0, 22.0, 23.0, 24.0, 25.0],
                       [31.0, 32.0, 33.0, 34.0, 35.0], [41.0, 42.0, 43.0, 44.0, 45.0]],
                      dtype=torch.float64)
    tex1 = torch.stack((l1, l1 + 100)).unsqueeze(1)
    tex3 = torch.cat((tex1, -tex1, tex1), dim=1)
    sp = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0, 1.0], [0.5, 0.5]], dtype=torch.float64)
    sparse = torch.stack((sp, torch.flip(sp, dims=(0,))))
    de = torch.tensor([[[0.0, 0.0], [0.25, 0.0], [0.5, 0.0], [0.75, 0.0], [1.0, 0.0]],
                       [[0.0, 1 / 8], [0.25, 1 / 8], [0.5, 1 / 8], [0.75, 1 / 8],
                        [1.0, 1 / 8]]], dtype=torch.float64)
    dense = torch.stack((de, torch.flip(de, dims=(0,))))
    return lhs, rhs, tex1, tex3, sparse, dense


def main():
    kaolin = import_reference()
    from kaolin.metrics.render import mask_iou
    from kaolin.render.mesh.utils import texture_mapping
    out = {}
    lhs, rhs, tex1, tex3, sparse, dense = reference_test_inputs()
    out['t_lhs'], out['t_rhs'] = lhs.numpy(), rhs.numpy()
    out['t_tex1'], out['t_tex3'] = tex1.numpy(), tex3.numpy()
    out['t_sparse'], out['t_dense'] = sparse.numpy(), dense.numpy()
    for k, dt in DT.items():
        loss = mask_iou(lhs.to(dt), rhs.to(dt))
        assert torch.allclose(loss, torch.tensor([0.3105], dtype=dt))  # test_render.py:51-52
        out[f't_iou_{k}'] = loss.numpy()
    lit = {('sparse', 'nearest'): [[41, 15, 11, 33], [133, 111, 115, 141]],
           ('sparse', 'bilinear'): [[41, 15, 11, 28], [128, 111, 115, 141]]}
    for mode in ('nearest', 'bilinear'):
        for k, dt in DT.items():
            for tname, tex in (('tex1', tex1), ('tex3', tex3)):
                r = texture_mapping(sparse.to(dt), tex.to(dt), mode=mode)
                e = torch.tensor(lit[('sparse', mode)], dtype=dt)
                assert torch.equal(r[..., 0], e)  # test_utils.py:66-71, 78-90
                out[f't_sparse_{tname}_{mode}_{k}'] = r.numpy()
            r = texture_mapping(dense.to(dt), tex3.to(dt), mode=mode)
            base = [41., 42., 43., 44., 45.] if mode == 'nearest' else \
                [41., 41.75, 43., 44.25, 45.]
            assert torch.equal(r[0, 0, :, 0], torch.tensor(base, dtype=dt))  # :96-106
            out[f't_dense_tex3_{mode}_{k}'] = r.numpy()

    # seeded random cases, forward + autograd backward
    g = torch.Generator().manual_seed(20)
    for k, dt in DT.items():
        B, H, W = 3, 37, 29
        l = torch.rand((B, H, W), generator=g, dtype=torch.float64).to(dt)
        r = (torch.rand((B, H, W), generator=g, dtype=torch.float64) > 0.5).to(dt)
        l.requires_grad_(True)
        r.requires_grad_(True)
        loss = mask_iou(l, r)
        gl_in = torch.tensor(0.75, dtype=dt)
        gl, gr = torch.autograd.grad(loss, [l, r], gl_in)
        out[f'r_iou_l_{k}'], out[f'r_iou_r_{k}'] = l.detach().numpy(), r.detach().numpy()
        out[f'r_iou_loss_{k}'] = loss.detach().numpy()
        out[f'r_iou_gl_{k}'], out[f'r_iou_gr_{k}'] = gl.numpy(), gr.numpy()

        B, h, w, C, Ht, Wt = 2, 19, 23, 3, 13, 17
        uv = torch.rand((B, h, w, 2), generator=g, dtype=torch.float64) * 1.2 - 0.1
        # exact texel centres and borders: (i + 0.5) / Wt, 0, 1
        uv[:, 0, :Wt, 0] = (torch.arange(Wt, dtype=torch.float64) + 0.5) / Wt
        uv[:, 1, :, 0] = 0.
        uv[:, 2, :, 1] = 1.
        uv = uv.to(dt)
        tex = torch.rand((B, C, Ht, Wt), generator=g, dtype=torch.float64).to(dt)
        go = torch.rand((B, h, w, C), generator=g, dtype=torch.float64).to(dt)
        out[f'r_tex_uv_{k}'], out[f'r_tex_map_{k}'], out[f'r_tex_go_{k}'] = \
            uv.numpy(), tex.numpy(), go.numpy()
        for mode in ('nearest', 'bilinear'):
            u = uv.clone().requires_grad_(True)
            t = tex.clone().requires_grad_(True)
            res = texture_mapping(u, t, mode=mode)
            gu, gt = torch.autograd.grad(res, [u, t], go, allow_unused=True)
            out[f'r_tex_out_{mode}_{k}'] = res.detach().numpy()
            out[f'r_tex_guv_{mode}_{k}'] = (torch.zeros_like(uv) if gu is None else gu).numpy()
            out[f'r_tex_gmap_{mode}_{k}'] = gt.numpy()
    np.savez_compressed(OUT, **out)
    print(f'wrote {OUT}: {len(out)} arrays')


if __name__ == '__main__':
    main()
