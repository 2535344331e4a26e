"""Generate tests/golden/f1.npz -- fixtures for SURVEY.md §8 f1 (prepare_vertices: camera
transform, perspective projection, face gather, unit face normals, and the gather backward) from
the reference itself (run ONCE, in the build container, where /root/reference exists; only the
.npz travels).

The reference function is ``kaolin.render.mesh.utils.prepare_vertices`` (utils.py:128-175), over
``camera.rotate_translate_points`` / ``camera.perspective_camera`` (render/camera/legacy.py:22-37,
120-139), ``ops.mesh.index_vertices_by_faces`` (ops/mesh/mesh.py:24-45) and
``ops.mesh.face_normals`` (ops/mesh/trianglemesh.py:313-336).  Cases (CPU, fp32 and fp64):
  * ``tf``:  shared vertices (1, V, 3) under camera_transform (B, 4, 3) -- the DIB-R training
    loop's form (examples/tutorial/ian_dibr.py);
  * ``tfb``: per-view vertices (B, V, 3) under camera_transform;
  * ``rt``:  per-view vertices under camera_rot (B, 3, 3) + camera_trans (B, 3).
For each: the three outputs, and the autograd gradient of the vertices for seeded incoming
gradients of all three outputs (``g_all``) and of face_vertices_image alone (``g_fvi``).
"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from make_golden import import_reference  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'f1.npz')
DT = {'f32': torch.float32, 'f64': torch.float64}
B = 3


def inputs():
    from kaolin_amd import workloads
    verts, faces, _ = workloads.uv_sphere(30, 17, seed=4, dtype=torch.float64)
    cam = workloads.orbit_cameras(B, 0.4, dtype=torch.float64)
    proj = workloads.generate_perspective_projection(math.pi / 4, dtype=torch.float64)
    g = torch.Generator().manual_seed(7)
    vb = verts.unsqueeze(0) + 0.01 * torch.randn((B,) + verts.shape, generator=g,
                                                  dtype=torch.float64)
    q, _ = torch.linalg.qr(torch.randn((B, 3, 3), generator=g, dtype=torch.float64))
    trans = torch.tensor([[0., 0., 4.], [0.5, -0.2, 5.], [-0.3, 0.1, 3.5]], dtype=torch.float64)
    F = faces.shape[0]
    grads = [torch.randn((B, F, 3, 3), generator=g, dtype=torch.float64),
             torch.randn((B, F, 3, 2), generator=g, dtype=torch.float64),
             torch.randn((B, F, 3), generator=g, dtype=torch.float64)]
    return verts, faces, cam, proj, vb, q, trans, grads


def main():
    import_reference()
    from kaolin.render.mesh.utils import prepare_vertices
    verts, faces, cam, proj, vb, rot, trans, grads = inputs()
    out = {'faces': faces.numpy(), 'verts': verts.numpy(), 'verts_b': vb.numpy(),
           'cam': cam.numpy(), 'proj': proj.numpy(), 'rot': rot.numpy(), 'trans': trans.numpy()}
    for i, gg in enumerate(grads):
        out[f'g{i}'] = gg.numpy()
    for k, dt in DT.items():
        cases = {'tf': (verts.unsqueeze(0), dict(camera_transform=cam)),
                 'tfb': (vb, dict(camera_transform=cam)),
                 'rt': (vb, dict(camera_rot=rot, camera_trans=trans))}
        for name, (v, kw) in cases.items():
            kw = {a: t.to(dt) for a, t in kw.items()}
            for which in ('all', 'fvi'):
                vv = v.to(dt).clone().requires_grad_(True)
                res = prepare_vertices(vv, faces, proj.to(dt), **kw)
                if which == 'all':
                    torch.autograd.backward(res, [x.to(dt) for x in grads])
                    for o, r in zip(('fvc', 'fvi', 'nrm'), res):
                        out[f'{name}_{k}_{o}'] = r.detach().numpy()
                else:
                    torch.autograd.backward(res[1], grads[1].to(dt))
                out[f'{name}_{k}_grad_{which}'] = vv.grad.numpy()
    np.savez_compressed(OUT, **out)
    print('wrote', OUT, len(out), 'arrays')


if __name__ == '__main__':
    main()
