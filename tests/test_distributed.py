"""Multi-process (world size 2, gloo, CPU) tests of the view-sharded DIB-R step (SURVEY §8 e).

The per-view renderer here is the CPU oracle (tests may use it); the code under test is the
sharding and the one exchange step bench.py uses: ``distributed.shard_views`` +
``workloads.orbit_cameras(first_view=...)`` and ``distributed.allreduce_grads_`` of the shared
vertex gradient.  The summed vertex gradient of 2 ranks must equal the single-process gradient
over all views (up to fp32 summation order).
"""
import math
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaolin_amd import distributed, workloads  # noqa: E402

TOTAL_VIEWS, H, W = 5, 24, 28  # odd view count: uneven shards


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _vertex_grad(first, nviews, total):
    """Oracle DIB-R fwd+bwd for views [first, first+nviews) of `total`; returns vertices.grad."""
    import oracle
    verts, faces, face_uvs = workloads.uv_sphere(12, 9, seed=0)
    vertices = verts.clone().requires_grad_(True)
    cam = workloads.orbit_cameras(nviews, 0.3, first_view=first, total_views=total)
    proj = workloads.generate_perspective_projection(math.pi / 4)
    fvc, fvi, nrm = workloads.prepare_vertices(vertices.unsqueeze(0).expand(nviews, -1, -1),
                                               faces, proj, cam)
    uvs = face_uvs.unsqueeze(0).repeat(nviews, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1)
    n = lambda t: t.detach().numpy()  # noqa: E731
    interp, fidx, wts = oracle.rasterize(H, W, n(fvc[..., 2]), n(fvi), n(feats),
                                         n(nrm[..., 2]) >= 0)
    soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(n(fvi), fidx, 7000, 0.02, 30, 1000.)
    # per-view upstream grads seeded by the GLOBAL view index (same numbers however sharded)
    g_feat = np.stack([np.random.default_rng(100 + first + b).random((H, W, 3), np.float32)
                       for b in range(nviews)])
    g_soft = np.stack([np.random.default_rng(200 + first + b).random((H, W), np.float32)
                       for b in range(nviews)])
    gfvi_r, _ = oracle.rasterize_backward(g_feat, fidx, wts, n(fvi), n(feats), 1e-8)
    gfvi_s = oracle.soft_mask_backward(g_soft, soft, fidx, prob, cidx, ctype, sfvi, 7000, 1000.)
    torch.autograd.backward(fvi, torch.as_tensor(gfvi_r + gfvi_s))
    return vertices.grad.detach().clone()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, wsz, _ = distributed.init_from_env('gloo')
        first, nv = distributed.shard_views(TOTAL_VIEWS, r, wsz)
        g = _vertex_grad(first, nv, TOTAL_VIEWS)
        distributed.allreduce_grads_([g])
        q.put((r, first, nv, g.numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, 'error', repr(e), None))


@pytest.mark.parametrize('world', [2])
def test_sharded_step_matches_single_process(world):
    import oracle
    oracle.lib()  # build the checker once, before the workers load it
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if r[1] == 'error']
    assert not errs, errs
    res.sort(key=lambda r: r[0])
    # the shards tile the views exactly once
    spans = [(r[1], r[2]) for r in res]
    assert spans[0][0] == 0 and sum(s[1] for s in spans) == TOTAL_VIEWS
    assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    # every rank holds the same all-reduced gradient == the single-process full-batch gradient
    ref = _vertex_grad(0, TOTAL_VIEWS, TOTAL_VIEWS).numpy()
    for r in res:
        np.testing.assert_allclose(r[3], ref, rtol=1e-4, atol=1e-5)
    assert np.abs(ref).sum() > 0


def test_shard_views_partition():
    for total in range(0, 20):
        for world in range(1, 9):
            cover = []
            for r in range(world):
                first, n = distributed.shard_views(total, r, world)
                cover.extend(range(first, first + n))
            assert cover == list(range(total))


def test_allreduce_noop_without_process_group():
    t = torch.arange(6.)
    out = distributed.allreduce_grads_([t, None])
    assert len(out) == 1 and torch.equal(t, torch.arange(6.))
