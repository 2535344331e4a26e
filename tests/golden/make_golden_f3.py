"""Generate tests/golden/deftet.npz -- fixtures for SURVEY.md §8 f3 (deftet_sparse_render) from the
reference itself (run ONCE, in the build container, where /root/reference exists; only the .npz
travels).

The reference tests deftet_sparse_render against its own naive implementation
``_naive_deftet_sparse_render`` (kaolin/render/mesh/deftet.py:101-267) and against literals
(tests/python/kaolin/render/mesh/test_deftet.py).  Both are reproduced here on the CPU:

* ``simple_*``  -- the TestSimpleDeftetSparseRender case (test_deftet.py:33-165): its inputs, the
  literal expected face index (asserted here against the naive renderer's output) and the naive
  renderer's features and gradients (seeded incoming gradient);
* ``sphere_*``  -- the TestDeftetSparseRender case (test_deftet.py:330-520): the model.obj sphere seen
  by the 3 test cameras, seeded random pixel coordinates in [-1, 1], render ranges "up to the
  centre" or full, knum 20 / 30, fp32 / fp64: naive face index, features and gradients.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import import_reference, sphere_inputs  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'deftet.npz')
DT = {'f32': torch.float32, 'f64': torch.float64}

SIMPLE_FVI = [[[[-1., 0.], [0., -1.], [0., 1.]],
               [[-1., 0.], [0., 1.], [0., -1.]],
               [[0., -1.], [0., 1.], [1., 0.]]],
              [[[-1., -1.], [1., -1.], [-1., 1.]],
               [[-1., -1.], [1., -1.], [-1., 1.]],
               [[-1., -1.], [1., -1.], [-1., 1.]]]]
SIMPLE_FVZ = [[[-2., -1., -1.], [-2.5, -3., -3.], [-2., -2., -2.]],
              [[-2., -1., -3.], [-2., -2., -2.], [-2., -3., -1.]]]
SIMPLE_PX = [[[-0.999, 0.], [-0.001, -0.998], [0.001, 0.998], [0.999, 0.],
              [-0.45, 0.], [0.45, 0.], [-0.999, -0.999]],
             [[-0.998, -0.999], [0.998, -0.999], [-0.999, 0.998],
              [-0.001, -0.], [0., -0.999], [-0.999, 0.], [0.001, 0.001]]]
SIMPLE_GT = [[[0, 1, -1, -1, -1], [0, 1, -1, -1, -1], [2, -1, -1, -1, -1], [2, -1, -1, -1, -1],
              [0, 1, -1, -1, -1], [2, -1, -1, -1, -1], [-1, -1, -1, -1, -1]],
             [[0, 1, 2, -1, -1], [0, 1, 2, -1, -1], [2, 1, 0, -1, -1], [2, 1, 0, -1, -1],
              [0, 1, 2, -1, -1], [2, 1, 0, -1, -1], [-1, -1, -1, -1, -1]]]


def run(naive, px, rr, fvz, fvi, feat, knum, seed):
    fvi = fvi.detach().clone().requires_grad_(True)
    feat = feat.detach().clone().requires_grad_(True)
    interp, fidx = naive(px, rr, fvz, fvi, feat, knum)
    g = torch.Generator().manual_seed(seed)
    go = torch.rand(interp.shape, generator=g, dtype=interp.dtype)
    interp.backward(go)
    # the incoming gradient is not stored: tests regenerate it (torch CPU generator, `seed`)
    return dict(face_idx=fidx.numpy().astype(np.int16), interp=interp.detach().numpy(),
                grad_fvi=fvi.grad.numpy(), grad_feat=feat.grad.numpy())


def main():
    kal = import_reference()
    from kaolin.render.mesh.deftet import _naive_deftet_sparse_render as naive
    torch.set_num_threads(8)
    out = {}
    for k, dt in DT.items():
        fvi = torch.tensor(SIMPLE_FVI, dtype=dt)
        fvz = torch.tensor(SIMPLE_FVZ, dtype=dt)
        per_face = torch.arange(6, dtype=dt).reshape(2, 3, 1, 1).expand(2, 3, 3, 1)
        per_vert = torch.arange(18, dtype=dt).reshape(2, 3, 3, 1)
        feat = torch.cat([per_face, per_vert], dim=-1)  # test_deftet.py:72-89 (cat_features)
        px = torch.tensor(SIMPLE_PX, dtype=dt)
        rr = torch.tensor([[[-4., 0.]]], dtype=dt).repeat(2, 7, 1)
        r = run(naive, px, rr, fvz, fvi, feat, 5, 1)
        assert np.array_equal(r['face_idx'], np.array(SIMPLE_GT))  # test_deftet.py:118-135
        out[f'simple_fvi_{k}'], out[f'simple_fvz_{k}'] = fvi.numpy(), fvz.numpy()
        out[f'simple_feat_{k}'], out[f'simple_px_{k}'] = feat.numpy(), px.numpy()
        out[f'simple_rr_{k}'] = rr.numpy()
        for name, a in r.items():
            out[f'simple_{name}_{k}'] = a

        s = sphere_inputs(kal, dt, 0)
        B = 3
        zmin = s['vcam'][:, :, -1].min(dim=1)[0]
        zmax = s['vcam'][:, :, -1].max(dim=1)[0]
        out[f'sphere_fvz_{k}'], out[f'sphere_fvi_{k}'] = s['fvz'].numpy(), s['fvi'].numpy()
        out[f'sphere_uvs_{k}'] = s['uvs'].numpy()
        for P in (31, 1025):
            g = torch.Generator().manual_seed(P)
            px = torch.rand((B, P, 2), generator=g, dtype=torch.float64).to(dt) * 2. - 1.
            out[f'sphere_px_{P}_{k}'] = px.numpy()
            for center in (0, 1):
                lo = (zmin + zmax) / 2. if center else zmin
                rr = torch.nn.functional.pad(lo.unsqueeze(-1), (0, 1), value=0.)
                rr = rr.unsqueeze(1).repeat(1, P, 1)  # test_deftet.py:410-418
                out[f'sphere_rr_{P}_{center}_{k}'] = rr.numpy()
                for knum in (20, 30):
                    r = run(naive, px, rr, s['fvz'], s['fvi'], s['uvs'], knum,
                            1000 + P + 10 * center + knum)
                    for name, a in r.items():
                        out[f'sphere_{name}_{P}_{center}_{knum}_{k}'] = a
        print(k, 'done')
    np.savez_compressed(OUT, **out)
    print(f'wrote {OUT}: {len(out)} arrays')


if __name__ == '__main__':
    main()
