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


# --------------------------------------------------------------------------------------------
# dibr_step's collective order when one rank produces no shared gradient
# --------------------------------------------------------------------------------------------
def _no_shared_grad_worker(rank, world, port, q):
    """dibr_step with a shared feature table that only rank 0's render uses: rank 1's hook never
    fires, so its EarlyReduce issues the table's all-reduce (zeros) only at flush().  Both ranks
    must issue [table, vertices] in that order (different sizes: a mismatch fails under gloo or
    mixes up the sums).  The local gradients are computed first, with no process group."""
    import types
    verts, faces, face_uvs = workloads.uv_sphere(6, 5, seed=0)
    F = faces.shape[0]
    cam = workloads.orbit_cameras(2, 0.3, first_view=2 * rank, total_views=4)
    proj = workloads.generate_perspective_projection(math.pi / 4)
    g_feat, g_soft = workloads.view_grads(2 * rank, 2, 4, 5, 3)

    def render(height, width, fvz, fvi, feats, nz, sigmainv, boxlen, knum):
        base = (fvi * fvi).sum() + (feats.sum() if rank == 0 else 0.)
        B = fvi.shape[0]
        return (base * torch.ones(B, height, width, 3), base * torch.ones(B, height, width),
                torch.zeros(B, height, width, dtype=torch.long))

    def run():
        v = verts.clone().requires_grad_(True)
        table = torch.ones(1, F, 3, 3).requires_grad_(True)
        distributed.dibr_step(v, faces, proj, cam, table, 4, 5, g_feat, g_soft, shared=(table,),
                              prepare=_prepare, render=render)
        return types.SimpleNamespace(v=v.grad.detach().clone(),
                                     t=None if table.grad is None else table.grad.detach().clone())

    try:
        local = run()
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        distributed.init_from_env('gloo')
        red = run()
        q.put((rank, local.v.numpy(), None if local.t is None else local.t.numpy(),
               red.v.numpy(), red.t.numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, 'error', repr(e), None, None))


def test_dibr_step_rank_without_shared_grad_world2():
    res = _run_world(_no_shared_grad_worker)
    (_, v0, t0, rv0, rt0), (_, v1, t1, rv1, rt1) = res
    assert t0 is not None and t1 is None  # only rank 0 produced a table gradient
    for rv, rt in ((rv0, rt0), (rv1, rt1)):
        np.testing.assert_allclose(rv, v0 + v1, rtol=1e-6)
        np.testing.assert_allclose(rt, t0, rtol=1e-6)


# --------------------------------------------------------------------------------------------
# GradBucket keeps each gradient's dtype
# --------------------------------------------------------------------------------------------
def _mixed_dtype_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        distributed.init_from_env('gloo')
        a = torch.zeros(4, requires_grad=True)
        b = torch.zeros(3, dtype=torch.float64, requires_grad=True)
        c = torch.zeros(2, requires_grad=True)
        a.grad = torch.full((4,), 1. + rank)
        b.grad = torch.full((3,), 1. + 1e-12 * (rank + 1), dtype=torch.float64)
        c.grad = torch.full((2,), 3. * rank)
        bucket = distributed.GradBucket([a, b, c])
        bucket.pack()
        bucket.reduce()
        q.put((rank, a.grad.numpy().copy(), b.grad.numpy().copy(), c.grad.numpy().copy(),
               str(b.grad.dtype)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, 'error', repr(e), None, None))


def test_grad_bucket_mixed_dtypes_world2():
    for _, ga, gb, gc, dt in _run_world(_mixed_dtype_worker):
        assert dt == 'torch.float64'
        np.testing.assert_array_equal(ga, np.full(4, 3.))
        np.testing.assert_allclose(gb, np.full(3, 2. + 3e-12), rtol=1e-15)  # not through fp32
        assert np.all(gb - 2. > 2e-12)
        np.testing.assert_array_equal(gc, np.full(2, 3.))


# --------------------------------------------------------------------------------------------
# bench.py's workload through the product's sharded step (test doubles for the GPU stages)
# --------------------------------------------------------------------------------------------
def _bench_args():
    import types
    return types.SimpleNamespace(dtype='f32', config='c1', sigmainv=7000., boxlen=0.02,
                                 knum=30, iou=None, vertex_path='compose')


def _bench_rank_step(first, n, total):
    import bench
    wl = bench.Workload(_bench_args(), torch.device('cpu'), first, n, total)
    distributed.dibr_step(wl.vertices, wl.faces, wl.proj, wl.cam, wl.feats, wl.H, wl.W,
                          wl.g_feat, wl.g_soft, prepare=_prepare, render=_render, **wl.kw)
    return wl.vertices.grad.detach().clone().numpy()


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, wsz, _ = distributed.init_from_env('gloo')
        first, n = distributed.shard_views(3, r, wsz)
        q.put((r, _bench_rank_step(first, n, 3)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, 'error', repr(e)))


def test_bench_workload_sharded_world2():
    """bench.Workload (C1 shapes, 3 views over 2 ranks: uneven shards) through dibr_step: the
    all-reduced vertex gradient equals the single-process one over all views."""
    import oracle
    oracle.lib()
    res = _run_world(_bench_worker)
    ref = _bench_rank_step(0, 3, 3)
    assert np.abs(ref).sum() > 0
    for _, g in res:
        np.testing.assert_allclose(g, ref, rtol=1e-4, atol=1e-5)


def test_bench_launcher_cmd():
    """bench.py --gpus N without WORLD_SIZE starts its N ranks with the driver's own launch form
    (torch.distributed.run, one node, rendezvous on 127.0.0.1) and passes its arguments on."""
    import bench
    cmd = bench.launcher_cmd(4, ['--gpus', '4', '--steps', '5'], 29555)
    assert cmd[1:4] == ['-m', 'torch.distributed.run', '--nnodes=1']
    assert '--nproc-per-node=4' in cmd
    i = cmd.index('--master-addr')
    assert cmd[i + 1] == '127.0.0.1' and cmd[i + 2:i + 4] == ['--master-port', '29555']
    assert cmd[-5].endswith('bench.py') and cmd[-4:] == ['--gpus', '4', '--steps', '5']
    assert 0 < bench.free_port() < 65536
