"""Multi-process (world size 2, gloo, CPU) tests of the view-sharded DIB-R step (SURVEY §8 e).

The code under test is the product's step, ``kaolin_amd.distributed.dibr_step`` -- the function
bench.py times (prepare_vertices -> dibr_rasterization -> backward -> one bucketed all-reduce of
the shared gradients, with early asynchronous reduction of shared parameters) -- together with
``shard_views`` and ``workloads.orbit_cameras(first_view=...)``.  On CPU its two GPU stages are
swapped for test doubles with the same signatures: the reference's PyTorch prepare_vertices
composition and an autograd Function over the CPU oracle (tests may use it).  The summed
gradients of 2 ranks must equal the single-process gradients over all views (fp32 sum order).
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


def _prepare(vertices, faces, camera_proj, camera_transform):
    """The reference composition of prepare_vertices (utils.py:128-175), CPU."""
    B = camera_transform.shape[0]
    return workloads.prepare_vertices(vertices.expand(B, -1, -1), faces, camera_proj,
                                      camera_transform)


class _OracleDibr(torch.autograd.Function):
    """dibr_rasterization (dibr.py:119-209) forward / backward through the CPU oracle."""

    @staticmethod
    def forward(ctx, height, width, fvz, fvi, feats, nz, sigmainv, boxlen, knum):
        import oracle
        n = lambda t: np.ascontiguousarray(t.detach().numpy())  # noqa: E731
        interp, fidx, wts = oracle.rasterize(height, width, n(fvz), n(fvi), n(feats), n(nz) >= 0)
        soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(n(fvi), fidx, sigmainv, boxlen,
                                                                 knum, 1000.)
        ctx.state = (fidx, wts, n(fvi), n(feats), soft, prob, cidx, ctype, sfvi, sigmainv)
        fi = torch.as_tensor(fidx)
        ctx.mark_non_differentiable(fi)
        return torch.as_tensor(interp), torch.as_tensor(soft), fi

    @staticmethod
    def backward(ctx, g_interp, g_soft, _):
        import oracle
        fidx, wts, fvi, feats, soft, prob, cidx, ctype, sfvi, sigmainv = ctx.state
        gr, gfeat = oracle.rasterize_backward(g_interp.numpy(), fidx, wts, fvi, feats, 1e-8)
        gs = oracle.soft_mask_backward(g_soft.numpy(), soft, fidx, prob, cidx, ctype, sfvi,
                                       sigmainv, 1000.)
        return (None, None, None, torch.as_tensor(gr + gs), torch.as_tensor(gfeat), None, None,
                None, None)


def _render(height, width, fvz, fvi, feats, nz, sigmainv, boxlen, knum):
    return _OracleDibr.apply(height, width, fvz, fvi, feats, nz, sigmainv, boxlen, knum)


def _rank_step(first, nviews, total, shared):
    """dibr_step on views [first, first+nviews) of `total`; returns (vertices.grad, feature
    table grad or None)."""
    verts, faces, face_uvs = workloads.uv_sphere(12, 9, seed=0)
    vertices = verts.clone().requires_grad_(True)
    cam = workloads.orbit_cameras(nviews, 0.3, first_view=first, total_views=total)
    proj = workloads.generate_perspective_projection(math.pi / 4)
    table = torch.cat([face_uvs, torch.ones_like(face_uvs[..., :1])], dim=-1).unsqueeze(0)
    if shared:  # one feature table shared by every view: its gradient is reduced too
        feats = table.clone().requires_grad_(True)
        params = (feats,)
    else:
        feats = table.repeat(nviews, 1, 1, 1).requires_grad_(True)
        params = ()
    # per-view upstream grads seeded by the GLOBAL view index (same numbers however sharded)
    g_feat, g_soft = workloads.view_grads(first, nviews, H, W, 3)
    distributed.dibr_step(vertices, faces, proj, cam, feats, H, W, g_feat, g_soft,
                          shared=params, prepare=_prepare, render=_render)
    return vertices.grad.detach().clone(), (feats.grad.detach().clone() if shared else None)


def _worker(rank, world, port, shared, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, wsz, _ = distributed.init_from_env('gloo')
        first, nv = distributed.shard_views(TOTAL_VIEWS, r, wsz)
        gv, gf = _rank_step(first, nv, TOTAL_VIEWS, shared)
        q.put((r, first, nv, gv.numpy(), None if gf is None else gf.numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, 'error', repr(e), None, None))


@pytest.mark.parametrize('world', [2])
@pytest.mark.parametrize('shared', [False, True])
def test_sharded_step_matches_single_process(world, shared):
    import oracle
    oracle.lib()  # build the checker once, before the workers load it
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shared, q))
             for r in range(world)]
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
    # every rank holds the same all-reduced gradients == the single-process full-batch ones
    ref_v, ref_f = _rank_step(0, TOTAL_VIEWS, TOTAL_VIEWS, shared)
    for r in res:
        np.testing.assert_allclose(r[3], ref_v.numpy(), rtol=1e-4, atol=1e-5)
        if shared:
            np.testing.assert_allclose(r[4], ref_f.numpy(), rtol=1e-4, atol=1e-5)
    assert np.abs(ref_v.numpy()).sum() > 0


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


# --------------------------------------------------------------------------------------------
# the exchange of GraphedStep / dibr_step (GradBucket) and the ordered early reduction
# --------------------------------------------------------------------------------------------
def _bucket_worker(rank, world, port, q):
    """GradBucket over two shared parameters, one of which has no gradient on rank 1 (a rank
    that produced none contributes zeros); pack() then reduce(), the two calls GraphedStep makes
    (pack inside the captured graph, reduce after the replay)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, wsz, _ = distributed.init_from_env('gloo')
        a = torch.zeros(3, 4, requires_grad=True)
        b = torch.zeros(5, requires_grad=True)
        a.grad = torch.arange(12.).reshape(3, 4) * (r + 1)
        if r == 0:
            b.grad = torch.full((5,), 2.5)
        bucket = distributed.GradBucket([a, b])
        bucket.pack()
        bucket.reduce()
        # a second step reuses the flat buffer
        a.grad.fill_(1.)
        b.grad.fill_(float(r))
        bucket()
        q.put((r, a.grad.numpy().copy(), b.grad.numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, 'error', repr(e)))


def _early_worker(rank, world, port, q):
    """EarlyReduce with two shared parameters whose gradients are produced in OPPOSITE orders on
    the two ranks (separate backward calls): the all-reduces must still pair up."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, wsz, _ = distributed.init_from_env('gloo')
        p0 = torch.zeros(4, requires_grad=True)
        p1 = torch.zeros(7, requires_grad=True)
        early = distributed.EarlyReduce([p0, p1])
        x0 = torch.arange(4.) + 10 * r
        x1 = torch.arange(7.) - 3 * r
        order = [(p0, x0), (p1, x1)] if r == 0 else [(p1, x1), (p0, x0)]
        for p, x in order:
            (p * x).sum().backward()
        early.wait()
        early.remove()
        q.put((r, p0.grad.numpy().copy(), p1.grad.numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, 'error', repr(e)))


def _run_world(target, world=2):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if isinstance(r[1], str)]
    assert not errs, errs
    return sorted(res, key=lambda r: r[0])


def test_grad_bucket_world2():
    res = _run_world(_bucket_worker)
    for _, ga, gb in res:
        np.testing.assert_array_equal(ga, np.ones((3, 4)) * 2)
        np.testing.assert_array_equal(gb, np.full(5, 1.0))


def test_early_reduce_fixed_order_world2():
    res = _run_world(_early_worker)
    for _, g0, g1 in res:
        np.testing.assert_array_equal(g0, 2 * np.arange(4.) + 10)
        np.testing.assert_array_equal(g1, 2 * np.arange(7.) - 3)
