"""Which op of the close-lists DIB-R step differs between a captured-graph replay and eager?
python tools/dbg_lists_graph.py -- each op (prepare_vertices, rasterize, dibr_soft_mask with
lists, and the three composed) captured alone in a HIP graph, replayed twice, and its input
gradients compared with an eager run (max abs difference, NaN count)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr, prepare_vertices  # noqa: E402
from kaolin_amd.render.mesh.rasterization import rasterize  # noqa: E402

_lib.load()
dev = torch.device('cuda')
h = 256
B = 2
verts, faces, face_uvs = workloads.uv_sphere(100, 51, seed=0)
vertices = verts.to(dev).requires_grad_(True)
faces = faces.to(dev)
cam = workloads.orbit_cameras(B, 0.3).to(dev)
proj = workloads.generate_perspective_projection(math.pi / 4).to(dev)
uvs = face_uvs.to(dev).unsqueeze(0).repeat(B, 1, 1, 1)
feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous().requires_grad_(True)
g_feat, g_soft = workloads.view_grads(0, B, h, h, 3)
g_feat, g_soft = g_feat.to(dev), g_soft.to(dev)
with torch.no_grad():
    fvc0, fvi0, nrm0 = prepare_vertices(vertices.unsqueeze(0), faces, proj, camera_transform=cam)
fvi_leaf = fvi0.clone().requires_grad_(True)


def op_prepare():
    fvc, fvi, nrm = prepare_vertices(vertices.unsqueeze(0), faces, proj, camera_transform=cam)
    torch.autograd.backward([fvi], [torch.ones_like(fvi)])


def op_raster():
    interp, fidx = rasterize(h, h, fvc0[..., 2], fvi_leaf, feats, nrm0[..., 2] >= 0)
    torch.autograd.backward([interp], [g_feat])


def op_soft():
    _, fidx = rasterize(h, h, fvc0[..., 2], fvi0, feats.detach(), nrm0[..., 2] >= 0)
    with dibr.close_lists(True):
        soft = dibr.dibr_soft_mask(fvi_leaf, fidx)
    torch.autograd.backward([soft], [g_soft])


def op_all():
    with dibr.close_lists(True):
        fvc, fvi, nrm = prepare_vertices(vertices.unsqueeze(0), faces, proj,
                                         camera_transform=cam)
        interp, soft, fidx = dibr.dibr_rasterization(h, h, fvc[..., 2], fvi, feats, nrm[..., 2])
    torch.autograd.backward([interp, soft], [g_feat, g_soft])


leaves = [vertices, feats, fvi_leaf]
for name, fn in [('prepare', op_prepare), ('raster', op_raster), ('soft', op_soft),
                 ('all', op_all)]:
    for p in leaves:
        p.grad = None
    fn()
    torch.cuda.synchronize()
    ref = [None if p.grad is None else p.grad.clone() for p in leaves]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for p in leaves:
                p.grad = None
            fn()
    torch.cuda.current_stream().wait_stream(s)
    for p in leaves:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for rep in range(2):
        for p in leaves:
            if p.grad is not None:
                p.grad.fill_(float('nan'))
        g.replay()
        torch.cuda.synchronize()
        out = []
        for p, r in zip(leaves, ref):
            if r is None:
                continue
            d = (p.grad - r).abs()
            out.append(f'max|d| {d.nan_to_num(float("inf")).max().item():.3g} '
                       f'nan {int(p.grad.isnan().sum())} scale {r.abs().max().item():.3g}')
        print(name, rep, ' | '.join(out), flush=True)
    del g

# the lists forward alone: outputs of each replay against an eager call
from kaolin_amd import _C  # noqa: E402
with torch.no_grad():
    _, fidx0 = rasterize(h, h, fvc0[..., 2], fvi0, feats.detach(), nrm0[..., 2] >= 0)


def fwd_lists():
    return _C.render.mesh.dibr_soft_mask_forward_fused(fvi0, fidx0, 7000., 0.02, 30, 1000.,
                                                       with_lists=True, want_grad=False)


ref = [t.clone() if t is not None else None for t in fwd_lists()]
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        fwd_lists()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    outs = fwd_lists()
for rep in range(3):
    for t in outs:
        if t is not None and t.dtype != torch.uint8:
            t.fill_(-3)
    g.replay()
    torch.cuda.synchronize()
    msg = []
    for name, t, r in zip(['soft', 'ws', 'prob', 'cidx', 'ctype'], outs, ref):
        if name == 'ws' or t is None:
            continue
        ne = (t != r)
        msg.append(f'{name} diff {int(ne.sum())}')
        if ne.any() and name == 'cidx':
            idx = ne.nonzero()[:3].tolist()
            msg.append(f'at {idx} got {[int(t[tuple(i)]) for i in idx]} want '
                       f'{[int(r[tuple(i)]) for i in idx]}')
    print('lists fwd', rep, ' | '.join(msg), flush=True)
