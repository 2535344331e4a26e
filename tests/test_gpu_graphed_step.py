"""GPU: the timed region of bench.py -- ``distributed.GraphedStep`` (the DIB-R training step
captured once in a HIP graph and replayed) -- against the eager step and the oracle.

Every replay must restart the library's device state: the pool counters and the record cursor
(zeroed by kd_bin_count, kd_binning.hip), the gradient buffers the forward zeroes on the side
(kd_softpair.hip soft_pairs_tile), the IoU accumulators.  So three consecutive replays must each
give the eager step's face_idx (bit-exact), and its vertex and feature gradients up to the float
atomics' summation order; view 0 of a replay is also checked against the oracle's brute-force
loops (face index, interpolated features, feature gradient).
"""
import math

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()


def _setup(n_lon, n_lat, h, B, iou):
    from kaolin_amd import workloads
    verts, faces, face_uvs = workloads.uv_sphere(n_lon, n_lat, seed=0)
    vertices = verts.to(DEV).requires_grad_(True)
    faces = faces.to(DEV)
    cam = workloads.orbit_cameras(B, 0.3).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    uvs = face_uvs.to(DEV).unsqueeze(0).repeat(B, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
    feats.requires_grad_(True)
    g_feat, g_soft = workloads.view_grads(0, B, h, h, 3)
    gt = None
    if iou:
        yy, xx = torch.meshgrid(torch.arange(h, dtype=torch.float32),
                                torch.arange(h, dtype=torch.float32), indexing='ij')
        gt = (((yy - h / 2) ** 2 + (xx - h / 2) ** 2) < (0.4 * h) ** 2).float()
        gt = gt.expand(B, h, h).contiguous().to(DEV)
    return dict(vertices=vertices, faces=faces, cam=cam, proj=proj, feats=feats,
                g_feat=g_feat.to(DEV), g_soft=g_soft.to(DEV), gt=gt, h=h)


def _fn(s):
    from kaolin_amd import distributed
    return lambda: distributed.dibr_forward_backward(
        s['vertices'], s['faces'], s['proj'], s['cam'], s['feats'], s['h'], s['h'], s['g_feat'],
        s['g_soft'], gt_mask=s['gt'], iou='fused')


def _eager(s):
    s['vertices'].grad = None
    s['feats'].grad = None
    fidx = _fn(s)()
    torch.cuda.synchronize()
    return fidx.clone(), s['vertices'].grad.clone(), s['feats'].grad.clone()


@pytest.mark.parametrize('cfg', [(100, 51, 256, 4), (250, 101, 512, 2)], ids=['c2', 'c3x2'])
@pytest.mark.parametrize('iou', [False, True], ids=['grad_soft', 'mask_iou'])
def test_graphed_step_replays_match_eager(cfg, iou):
    from kaolin_amd import distributed
    n_lon, n_lat, h, B = cfg
    s = _setup(n_lon, n_lat, h, B, iou)
    e_fidx, e_gv, e_gf = _eager(s)
    gs = distributed.GraphedStep([s['vertices'], s['feats']], _fn(s),
                                 params_to_reduce=[s['vertices']])
    for rep in range(3):
        # poison the outputs so a replay that skipped work cannot pass
        s['vertices'].grad.fill_(float('nan'))
        s['feats'].grad.fill_(float('nan'))
        gs.out.fill_(-7)
        fidx = gs()
        torch.cuda.synchronize()
        assert torch.equal(fidx, e_fidx), rep
        for x, y in ((s['vertices'].grad, e_gv), (s['feats'].grad, e_gf)):
            scale = y.abs().max().item()
            assert scale > 0
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * scale)
    # view 0 of the last replay against the oracle
    from kaolin_amd.render.mesh import prepare_vertices
    with torch.no_grad():
        fvc, fvi, nrm = prepare_vertices(s['vertices'].detach().unsqueeze(0), s['faces'],
                                         s['proj'], camera_transform=s['cam'])
    N = lambda t: np.ascontiguousarray(t[:1].detach().cpu().numpy())  # noqa: E731
    feats0 = N(s['feats'])
    ri, rf, rw = oracle.rasterize(h, h, N(fvc[..., 2]), N(fvi), feats0, N(nrm[..., 2]) >= 0)
    np.testing.assert_array_equal(N(gs.out), rf)
    _, gfeat = oracle.rasterize_backward(N(s['g_feat']), rf, rw, N(fvi), feats0, 1e-8)
    np.testing.assert_allclose(N(s['feats'].grad), gfeat, rtol=1e-4,
                               atol=1e-5 * np.abs(gfeat).max())


def test_graphed_step_with_close_lists_matches_eager():
    """the reference-structured path (the (B, H, W, K) close-face lists materialised by the
    forward and read by the backward, bench.py --lists) captured and replayed"""
    from kaolin_amd import distributed
    from kaolin_amd.render.mesh import dibr
    s = _setup(100, 51, 256, 2, False)
    with dibr.close_lists(True):
        e_fidx, e_gv, e_gf = _eager(s)
        gs = distributed.GraphedStep([s['vertices'], s['feats']], _fn(s),
                                     params_to_reduce=[s['vertices']])
        for rep in range(2):
            s['vertices'].grad.fill_(float('nan'))
            s['feats'].grad.fill_(float('nan'))
            gs.out.fill_(-7)
            fidx = gs()
            torch.cuda.synchronize()
            assert torch.equal(fidx, e_fidx), rep
            for x, y in ((s['vertices'].grad, e_gv), (s['feats'].grad, e_gf)):
                scale = y.abs().max().item()
                torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * scale)


def _two_rank_worker(rank, port, out_dir):
    """One rank of test_graphed_step_two_ranks: the eager dibr_step and the captured step (two
    reduced parameters: the vertices and a shared feature table, so GradBucket packs both into
    its flat buffer inside the graph) over a gloo group, both ranks on cuda:0."""
    import torch.distributed as dist
    from kaolin_amd import _lib, distributed, workloads
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                            world_size=2)
    try:
        _lib.load()
        h, total = 128, 2
        verts, faces, face_uvs = workloads.uv_sphere(40, 21, seed=0)
        vertices = verts.to(DEV).requires_grad_(True)
        faces = faces.to(DEV)
        cam = workloads.orbit_cameras(total, 0.3)[rank:rank + 1].to(DEV)
        proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
        uvs = face_uvs.to(DEV).unsqueeze(0)
        feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
        feats.requires_grad_(True)  # (1, F, 3, 3): shared by the views, reduced over the ranks
        g_feat, g_soft = workloads.view_grads(rank, 1, h, h, 3)
        g_feat, g_soft = g_feat.to(DEV), g_soft.to(DEV)
        distributed.dibr_step(vertices, faces, proj, cam, feats, h, h, g_feat, g_soft,
                              shared=[feats])
        torch.cuda.synchronize()
        e_gv, e_gf = vertices.grad.clone(), feats.grad.clone()
        fn = (lambda: distributed.dibr_forward_backward(vertices, faces, proj, cam, feats, h, h,
                                                        g_feat, g_soft))
        gs = distributed.GraphedStep([vertices, feats], fn, params_to_reduce=[vertices, feats])
        for rep in range(2):
            vertices.grad.fill_(float('nan'))
            feats.grad.fill_(float('nan'))
            gs()
            torch.cuda.synchronize()
            for x, y in ((vertices.grad, e_gv), (feats.grad, e_gf)):
                scale = y.abs().max().item()
                assert scale > 0
                torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * scale)
        torch.save({'gv': e_gv.cpu(), 'gf': e_gf.cpu()}, f'{out_dir}/rank{rank}.pt')
    finally:
        dist.destroy_process_group()


def test_graphed_step_two_ranks(tmp_path):
    """GraphedStep's captured GradBucket.pack() and its all-reduce after the replay, with a real
    process group: two gloo ranks on one GPU, each rendering its own view; the
    replayed gradients equal the eager dibr_step's, and the reduced gradients agree across ranks"""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    procs = [ctx.Process(target=_two_rank_worker, args=(r, port, str(tmp_path))) for r in (0, 1)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r0 = torch.load(tmp_path / 'rank0.pt', weights_only=True)
    r1 = torch.load(tmp_path / 'rank1.pt', weights_only=True)
    for k in ('gv', 'gf'):
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)


def test_bench_starts_its_own_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE launches its two ranks itself: with
    the gloo backend both share this box's one GPU; the JSON line reports n_gpus 2 and the
    all-reduce's own time."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env['KD_BENCH_BACKEND'] = 'gloo'
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2',
                        '--views-per-gpu', '1', '--steps', '3', '--warmup', '1', '--no-weak',
                        '--config', 'c2'], capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith('{')][-1]
    out = json.loads(line)
    assert out['n_gpus'] == 2
    assert out['config']['global_batch'] == 2
    assert out['allreduce_us'] is not None and out['allreduce_us'] > 0
