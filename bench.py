#!/usr/bin/env python
"""DIB-R forward+backward throughput on MI355X (BASELINE.json metric).

One step = prepare_vertices (camera transform, projection, per-face gather, normals; fused HIP,
kaolin_amd/csrc/kd_prepare.hip) -> dibr_rasterization (HIP: rasterize + soft mask) -> torch.autograd.backward(
[interp, soft_mask], [g_feat, g_soft]) through the HIP backward kernels and the face->vertex
scatter -> (N > 1) one RCCL all-reduce of the shared vertex gradient.  Inputs are resident in HBM
before the timed region.  N GPUs: one process per GPU, each renders its own block of views of the
same mesh (weak scaling: views per GPU fixed).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--views-per-gpu B]
For N > 1 launch with torch.distributed.run (see README / the driver contract).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from kaolin_amd import _C, _lib, distributed, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr, dibr_rasterization, prepare_vertices  # noqa: E402

METRIC = 'Mpixels/s DIB-R fwd+bwd, 50k-face mesh @512² bs=8, 1/2/4/8 GPU'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# name -> (n_lon, n_lat, H, W, views per GPU, elevation); SURVEY.md §8(d) configs C2-C5
CONFIGS = {
    'c2': (100, 51, 256, 256, 4, 0.3),
    'c3': (250, 101, 512, 512, 8, 0.3),
    'c4': (250, 101, 1024, 1024, 8, 0.3),
    'c5': (500, 201, 512, 512, 16, 0.6),
}
# name -> (faces, H, W, views per GPU): the C5 stress soup (workloads.soup, seed 3); a step is
# dibr_rasterization fwd + bwd on per-view face soups (no shared mesh: no all-reduce)
SOUP_CONFIGS = {
    'c5soup': (200000, 512, 512, 16),
}


def algorithmic_bytes(kernel, P, F, Fv, D, K, lists, pairs=None, V=0, esize=4, fused=True):
    """Bytes each kernel must move at minimum per launch: every tensor of its contract read or
    written once (SURVEY.md §8(d) decomposed per kernel).  P pixels, F faces
    (all views), Fv valid (front) faces, D features, K knum, pairs = (pixel, close face) pairs of
    the soft mask, V vertices.  None where a term is unknown."""
    e = esize
    if kernel == 'kd_raster_fwd':      # out: face_idx, weights, interp; in: valid faces' rows
        return P * (8 + 3 * e + D * e) + Fv * (6 * e + 3 * e + 3 * D * e) + F * 1
    if kernel == 'kd_raster_bwd_tile':  # in: idx, weights, grad; face rows read + added once
        return P * (8 + 3 * e + D * e) + F * (6 * e + 3 * D * e) * 2
    if kernel == 'kd_bin_count':       # both face sets: corners (+ normal z) in, spans (+ cull) out
        return F * (6 * e + e + 8 + 32) + F * (6 * e + 8)
    if kernel == 'kd_bin_scatter':     # both sets: spans in, >= one bin entry out per face
        return 2 * F * (8 + 4)
    if kernel == 'kd_zero':
        return F * (6 + 3 * D) * e
    if kernel == 'kd_prepare_fwd':     # vertices + faces in; fvc, fvi, normals out
        return V * 3 * e + F * (9 + 6 + 3) * e
    if kernel == 'kd_prepare_bwd':     # fvc + grad_fvi in, vertex grads out
        return F * (9 + 6) * e + V * 3 * e
    if pairs is None:
        return None
    if kernel == 'kd_soft_pairs' and fused:  # whole soft mask: face_idx + corners in; records,
        # probabilities, types, counts, soft out
        return P * (8 + 4 + e) + F * 6 * e + pairs * (12 + e + 1)
    if kernel == 'kd_soft_pairs':      # face_idx in; records, counts, soft out
        return P * (8 + 4 + e) + pairs * 12
    if kernel == 'kd_soft_pair_math':  # records in; probabilities, types out
        return pairs * (12 + e + 1)
    if kernel == 'kd_soft_reduce':     # probabilities in, soft out
        return pairs * e
    if kernel == 'kd_soft_bwd_pairs':  # records + probabilities, grad/soft, corners in; face
        # grads added
        return pairs * (12 + e) + P * 2 * e + F * 6 * e * 3
    if kernel == 'kd_dibr_fwd':        # raster forward + whole soft mask in one launch
        return (algorithmic_bytes('kd_raster_fwd', P, F, Fv, D, K, lists, pairs, V, e) +
                algorithmic_bytes('kd_soft_pairs', P, F, Fv, D, K, lists, pairs, V, e))
    if kernel == 'kd_dibr_bwd':        # the two backwards above in one launch
        return (algorithmic_bytes('kd_raster_bwd_tile', P, F, Fv, D, K, lists, pairs, V, e) +
                algorithmic_bytes('kd_soft_bwd_pairs', P, F, Fv, D, K, lists, pairs, V, e))
    return None


def survey_step_bytes(P, F, D, K, esize=4):
    """SURVEY.md §8(d) whole-step formula (K-lists counted as the reference writes them, the
    N_read term omitted): bytes of one DIB-R fwd+bwd step."""
    e = esize
    pix = (8 + 3 * e + D * e) + (8 + e + 13 * K) + (D * e + 8 + 3 * e) + (e + e + 8)
    face = (e * (3 + 6 + 3 * D) + 4) + 24 + 2 * (24 + 12 * D) + 2 * 24
    return P * pix + F * face


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='c3', choices=sorted(CONFIGS) + sorted(SOUP_CONFIGS))
    ap.add_argument('--views-per-gpu', type=int, default=None)
    ap.add_argument('--knum', type=int, default=30)
    ap.add_argument('--sigmainv', type=float, default=7000.)
    ap.add_argument('--boxlen', type=float, default=0.02)
    ap.add_argument('--lists', action='store_true',
                    help='materialise the (B,H,W,K) close-face lists (reference structure)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample-views', type=int, default=8)
    ap.add_argument('--cpu-min-seconds', type=float, default=10.0,
                    help='repeat the CPU sample until at least this much CPU time has passed')
    ap.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'pmc_traffic.json'))
    args = ap.parse_args()

    # KD_BENCH_BACKEND=gloo rehearses the multi-rank path on a single GPU (ranks share cuda:0;
    # RCCL refuses two ranks on one device).  The default is RCCL ("nccl").
    backend = os.environ.get('KD_BENCH_BACKEND', 'nccl')
    rank, world, local = distributed.init_from_env(backend)
    if world != args.gpus and rank == 0:
        print(f'[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}', file=sys.stderr)
    dev = torch.device('cuda', local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    _lib.load()
    dibr.SAVE_CLOSE_LISTS = args.lists

    soup = args.config in SOUP_CONFIGS
    kw = dict(sigmainv=args.sigmainv, boxlen=args.boxlen, knum=args.knum)
    if soup:
        F, H, W, B_def = SOUP_CONFIGS[args.config]
        Bl = args.views_per_gpu or B_def
        first, _ = distributed.shard_views(Bl * world, rank, world)
        sz, si, sn = workloads.soup(F, seed=3, batch=Bl * world)
        sfvz = sz[first:first + Bl].to(dev).contiguous()
        sfvi = si[first:first + Bl].to(dev).contiguous().requires_grad_(True)
        snz = sn[first:first + Bl].to(dev).contiguous()
        g = torch.Generator().manual_seed(4)
        uvs = torch.rand((Bl, F, 3, 2), generator=g).to(dev)
        feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
        feats.requires_grad_(True)
        n_lon = n_lat = None
        verts = None
    else:
        n_lon, n_lat, H, W, B_def, elev = CONFIGS[args.config]
        Bl = args.views_per_gpu or B_def
        first, _ = distributed.shard_views(Bl * world, rank, world)
        verts, faces, face_uvs = workloads.uv_sphere(n_lon, n_lat, seed=0)
        F = faces.shape[0]
        vertices = verts.to(dev).requires_grad_(True)
        faces = faces.to(dev)
        cam = workloads.orbit_cameras(Bl, elev, first_view=first,
                                      total_views=Bl * world).to(dev)
        proj = workloads.generate_perspective_projection(math.pi / 4).to(dev)
        uvs = face_uvs.to(dev).unsqueeze(0).repeat(Bl, 1, 1, 1)
        feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
        feats.requires_grad_(True)  # learnable per-face-vertex features: grad_feat is computed
    D = feats.shape[-1]
    g = torch.Generator().manual_seed(1)
    g_feat = torch.rand((Bl, H, W, D), generator=g).to(dev)
    g = torch.Generator().manual_seed(2)
    g_soft = torch.rand((Bl, H, W), generator=g).to(dev)

    def inputs():
        if soup:
            return sfvz, sfvi, snz
        # one mesh, Bl cameras: vertices batch 1 broadcast over the views (utils.py:128-175)
        fvc, fvi, nrm = prepare_vertices(vertices.unsqueeze(0), faces, proj,
                                         camera_transform=cam)
        return fvc[..., 2], fvi, nrm[..., 2]

    def step():
        fvz, fvi, nz = inputs()
        interp, soft, face_idx = dibr_rasterization(H, W, fvz, fvi, feats, nz, **kw)
        torch.autograd.backward([interp, soft], [g_feat, g_soft])
        if soup:
            sfvi.grad = None
        else:
            distributed.allreduce_grads_([vertices.grad])
            vertices.grad = None
        feats.grad = None
        return face_idx

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---- timed region --------------------------------------------------------------------
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    pixels = Bl * world * H * W
    value = pixels * args.steps / elapsed / 1e6

    # ---- per-kernel durations: HIP events recorded on the launch stream, second pass ------
    _lib.profile_enable(True)
    face_idx = None
    for _ in range(args.steps):
        face_idx = step()
    torch.cuda.synchronize(dev)
    _lib.profile_enable(False)
    prof = _lib.profile_collect()
    fv = int((face_idx >= 0).sum().item())  # covered pixels (for the record)

    with torch.no_grad():
        fvz, fvi, nz = inputs()
        fvi = fvi.detach()
        Fv = int((nz >= 0).sum().item())
    P = Bl * H * W
    Ftot = Bl * F
    V = 0 if soup else vertices.shape[0]
    pairs = None
    if not args.lists:
        with torch.no_grad():
            _, _, _, _, ws = _C.render.mesh.dibr_rasterization_forward_fused(
                H, W, fvz, fvi, feats, nz, args.sigmainv, args.boxlen,
                args.knum, 1000., 1e-8, want_grad=True)
            pairs = int(_lib.load().kd_dibr_pair_count(ws.data_ptr(), Bl, H, W, F, args.knum, 0,
                                                       torch.cuda.current_stream(dev).cuda_stream))
            del ws
    fused = 'kd_soft_pair_math' not in prof  # the one-launch soft mask (kd_softpair.hip)
    kernels = {}
    for name, (ms, n) in prof.items():
        avg_us = ms * 1e3 / n
        ab = algorithmic_bytes(name, P, Ftot, Fv, D, args.knum, args.lists, pairs, V,
                               fused=fused)
        kernels[name] = {'avg_us': round(avg_us, 2), 'launches': n,
                         'share': round(ms / max(sum(v[0] for v in prof.values()), 1e-9), 3)}
        if ab is not None:
            kernels[name]['alg_bytes'] = ab
            kernels[name]['GB_s'] = round(ab / (avg_us * 1e-6) / 1e9, 1)
    dom = max(prof.items(), key=lambda kv: kv[1][0])[0] if prof else None
    roofline = None
    if dom is not None:
        ms, n = prof[dom]
        avg_s = ms / n / 1e3
        ab = algorithmic_bytes(dom, P, Ftot, Fv, D, args.knum, args.lists, pairs, V,
                               fused=fused)
        achieved = ab / avg_s / 1e9 if ab else None
        traffic = None
        if os.path.exists(args.pmc):
            try:
                with open(args.pmc) as f:
                    pm = json.load(f)
                ent = pm.get('kernels', {}).get(dom)
                if ent and pm.get('config') == args.config and bool(pm.get('lists')) == args.lists:
                    traffic = ent.get('hbm_bytes_per_launch')
            except (OSError, ValueError):
                traffic = None
        roofline = {'kernel': dom, 'bound': 'hbm',
                    'achieved': None if achieved is None else round(achieved, 1),
                    'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
                    'traffic': traffic,
                    'alg_bytes_per_launch': ab, 'avg_launch_us': round(avg_s * 1e6, 2)}

    sb = survey_step_bytes(P, Ftot, D, args.knum)
    step_roof = {'formula': 'SURVEY.md §8(d): 482 B/px + 268 B/face at D=3, K=30 (K-lists as '
                            'the reference writes them, N_read omitted)',
                 'bytes_per_step_per_gpu': sb,
                 'achieved': round(sb / (ms_per_step * 1e-3) / 1e9, 1), 'peak': HBM_PEAK_GBS,
                 'unit': 'GB/s', 'frac': round(sb / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 'pairs_per_step': pairs}

    # ---- CPU baseline: the oracle (C port of the reference kernels), rank 0, N == 1 -------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, fvz, fvi, nz, feats, g_feat, g_soft, H, W, kw)

    out = {
        'metric': METRIC, 'value': round(value, 2), 'unit': 'Mpixels/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (seeded uv-sphere, orbit cameras; no dataset)',
        'config': {'workload': f'{args.config.upper()}: ' +
                               (f'soup({F}, seed=3) per view' if soup else
                                f'uv_sphere({n_lon},{n_lat}) {F} faces') + ', '
                               f'{H}x{W}, {Bl} views/GPU, D={D}, knum={args.knum}, '
                               f'sigmainv={args.sigmainv:g}, boxlen={args.boxlen:g}',
                   'faces': F, 'height': H, 'width': W, 'views_per_gpu': Bl,
                   'global_batch': Bl * world,
                   'parallelism': f'view-sharded x{world}' +
                                  (' + RCCL vertex-grad all-reduce'
                                   if world > 1 and not soup else ''),
                   'close_lists': 'materialised' if args.lists else 'not materialised',
                   'covered_px_per_step': fv, 'front_faces': Fv},
        'roofline': roofline,
        'step_roofline': step_roof,
        'cpu_baseline': cpu,
        'kernels': kernels,
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(args, fvz, fvi, nz, feats, g_feat, g_soft, H, W, kw):
    """The CPU oracle (oracle/dibr_oracle.c, OpenMP) doing the same fwd+bwd on a bounded sample
    (the first `--cpu-sample-views` views of the workload)."""
    import numpy as np
    import oracle
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or os.cpu_count()
    oracle.set_num_threads(threads)
    nb = max(1, min(args.cpu_sample_views, fvi.shape[0]))
    n = lambda t: t[:nb].detach().cpu().numpy()  # noqa: E731
    fvz_, fvi_, nz_, ft_ = n(fvz), n(fvi), n(nz), n(feats)
    gf_, gs_ = n(g_feat), n(g_soft)
    reps = 0
    t0 = time.perf_counter()
    while True:
        interp, face_idx, weights = oracle.rasterize(H, W, fvz_, fvi_, ft_, nz_ >= 0)
        soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(
            fvi_, face_idx, kw['sigmainv'], kw['boxlen'], kw['knum'], 1000.)
        oracle.rasterize_backward(gf_, face_idx, weights, fvi_, ft_, 1e-8)
        oracle.soft_mask_backward(gs_, soft, face_idx, prob, cidx, ctype, sfvi, kw['sigmainv'],
                                  1000.)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_min_seconds:
            break
    px = nb * H * W * reps
    return {'value': round(px / dt / 1e6, 5), 'unit': 'Mpixels/s', 'cores': threads,
            'kind': 'port',
            'sample': f'{nb} view(s) of the same workload ({nb * H * W} px, {fvi.shape[1]} '
                      f'faces) x {reps} repetition(s), fwd+bwd, brute-force reference loops '
                      f'(oracle/dibr_oracle.c, OpenMP), {dt:.2f} s'}


if __name__ == '__main__':
    main()
