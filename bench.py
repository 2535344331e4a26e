#!/usr/bin/env python
"""DIB-R forward+backward throughput on MI355X (BASELINE.json metric).

One step = kaolin_amd.distributed.dibr_step: prepare_vertices (camera transform, projection,
per-face gather, normals; fused HIP, kd_prepare.hip) -> dibr_rasterization (HIP: rasterize + soft
mask) -> torch.autograd.backward([interp, soft_mask], [g_feat, g_soft]) through the HIP backward
kernels and the face->vertex scatter -> (N > 1) one RCCL all-reduce of the shared vertex
gradient.  Inputs are resident in HBM before the timed region.

Scaling: the headline config (C3) is a GLOBAL batch of 8 views split over the N GPUs (8/4/2/1
views per GPU at N = 1/2/4/8: "strong").  With N > 1 a second timed phase renders the config's
full batch on every GPU ("weak_scaling" field).  --views-per-gpu B makes the main line weak.

The GPU part of the step is captured once in a HIP graph and replayed (GraphedStep; --no-graph
runs it eagerly); the all-reduce stays an eager RCCL call.  Every kernel of the step runs in
every replay.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--dtype f32|f64]
For N > 1 the driver launches it with torch.distributed.run; without WORLD_SIZE in the
environment `--gpus N` starts the N ranks itself (the same torch.distributed.run command, as a
child process, before any GPU call).
"""
import argparse
import json
import math
import os
import statistics
import subprocess
import sys
import time

# HIP graph replays dispatched through the runtime's regular kernel path instead of its
# pre-recorded AQL packets (a launch-mode setting of the HIP runtime, read at its initialisation;
# results are unchanged).  Same-box A/B, profiles/r06/ab_graph_packet_env.txt: C3 8 views
# 0.2667 -> 0.2638 ms per step, 1 view 0.0898 -> 0.0869 ms.  Set KD_BENCH_KEEP_HIP_ENV=1 to
# leave the runtime's default.
if not os.environ.get('KD_BENCH_KEEP_HIP_ENV'):
    os.environ.setdefault('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '0')

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from kaolin_amd import _C, _lib, distributed, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr, dibr_rasterization  # noqa: E402

METRIC = 'Mpixels/s DIB-R fwd+bwd, 50k-face mesh @512² bs=8, 1/2/4/8 GPU'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU roof: 256 CUs x 4 SIMDs at the 2.4 GHz peak clock.  Issue cost per wave64 instruction on a
# SIMD with >= 2 waves (MI355X_MICROARCH.md, per-instruction cycle constants: v_fma_f32 2 cycles
# on SIMD-32, 4 for one wave alone; transcendentals twice an add): fp32 / int / other 2, fp32
# transcendental 4; fp64 add / mul / fma at half the fp32 rate 4, fp64 transcendental 8 (the
# MI355X's fp64 vector rate is half its fp32 rate).  The counts come from the per-type
# SQ_INSTS_VALU_* counters (tools/pmc_mix.sh); instructions of no listed type (moves, compares,
# selects, DPP, bit ops) are priced at 2.
VALU_SIMDS, CLOCK_HZ = 1024, 2.4e9
VALU_MIX_CYCLES = {'ADD_F32': 2, 'MUL_F32': 2, 'FMA_F32': 2, 'TRANS_F32': 4, 'ADD_F64': 4,
                   'MUL_F64': 4, 'FMA_F64': 4, 'TRANS_F64': 8, 'INT32': 2, 'INT64': 4, 'CVT': 2}
VALU_OTHER_CYCLES = 2


def valu_issue_cycles(ent):
    """Mix-weighted issue cycles of one launch (summed over its waves) from a pmc_traffic entry,
    and the per-type breakdown; None without the per-type counters."""
    total = ent.get('SQ_INSTS_VALU')
    if not total or not all(f'SQ_INSTS_VALU_{k}' in ent for k in VALU_MIX_CYCLES):
        return None, None
    mix = {k: ent[f'SQ_INSTS_VALU_{k}'] for k in VALU_MIX_CYCLES}
    other = max(total - sum(mix.values()), 0.0)
    cyc = sum(mix[k] * VALU_MIX_CYCLES[k] for k in mix) + other * VALU_OTHER_CYCLES
    return cyc, dict(mix, OTHER=other)

# name -> (n_lon, n_lat, H, W, global batch, elevation); SURVEY.md §8(d) configs C1-C5 (C1: the
# reference's CPU-runnable plumbing case, used by the CPU tests of the sharded step)
CONFIGS = {
    'c1': (25, 21, 128, 128, 1, 0.3),
    'c2': (100, 51, 256, 256, 4, 0.3),
    'c3': (250, 101, 512, 512, 8, 0.3),
    'c4': (250, 101, 1024, 1024, 8, 0.3),
    'c5': (500, 201, 512, 512, 16, 0.6),
}
# name -> (faces, H, W, global batch): the C5 stress soup (workloads.soup, seed 3); a step is
# dibr_rasterization fwd + bwd on per-view face soups (no shared mesh: no all-reduce)
SOUP_CONFIGS = {
    'c5soup': (200000, 512, 512, 16),
}
DTYPES = {'f32': torch.float32, 'f64': torch.float64}


def algorithmic_bytes(kernel, P, F, Fv, D, K, lists, pairs=None, V=0, esize=4, fused=True,
                      prep=None):
    """Bytes each kernel must move at minimum per launch: every tensor of its contract read or
    written once (SURVEY.md §8(d) decomposed per kernel).  P pixels, F faces
    (all views), Fv valid (front) faces, D features, K knum, pairs = (pixel, close face) pairs of
    the soft mask, V vertices.  prep = (vertices, faces of the mesh, views) when the count
    projects the mesh itself (kd_bin_count PREP: dibr_rasterization_from_vertices).  None where a
    term is unknown."""
    e = esize
    if kernel == 'kd_bin_count' and prep:  # PREP: vertices, faces, cameras in; prepare_vertices'
        # fvc / fvi / normals out; both sets' spans (+ the raster's cull coefficients) out
        Vm, Fm, nv = prep
        return (Vm * 3 * e + Fm * 3 * 8 + nv * (12 + 3) * e + F * (9 + 6 + 3) * e +
                F * (8 + 32) + F * 8)
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
    if kernel == 'kd_prepare_bwd' and prep:  # from the vertices (the node's backward): grad_fvi,
        # the vertices and the CSR (entry, vertex) pairs in, vertex grads out
        Vm, Fm, nv = prep
        return F * 6 * e + Vm * 3 * e * 2 + Fm * 3 * (4 + 4)
    if kernel == 'kd_prepare_bwd':     # fvc + grad_fvi in, vertex grads out
        return F * (9 + 6) * e + V * 3 * e
    if pairs is None:
        return None
    # soft-mask records (kd_soft.hpp SoftPairRec): 8 B {row, slot, pixel, type} + the
    # probability; work items 16 B per 256 records
    if kernel == 'kd_soft_pairs' and fused:  # whole soft mask: face_idx + corners in; records
        # (with their type), probabilities, soft out
        return P * (8 + e) + F * 6 * e + pairs * (8 + e)
    if kernel == 'kd_soft_pairs':      # face_idx in; records, per-pixel counts, soft out
        return P * (8 + 4 + e) + pairs * 8
    if kernel == 'kd_soft_pair_math':  # records in; probabilities, types out
        return pairs * (8 + e + 1)
    if kernel == 'kd_soft_reduce':     # probabilities in, soft out
        return pairs * e
    if kernel == 'kd_soft_bwd_pairs':  # records + probabilities, grad/soft, corners in; face
        # grads added
        return pairs * (8 + e) + P * 2 * e + F * 6 * e * 3
    if kernel == 'kd_dibr_fwd':        # raster forward + whole soft mask in one launch
        return (algorithmic_bytes('kd_raster_fwd', P, F, Fv, D, K, lists, pairs, V, e) +
                algorithmic_bytes('kd_soft_pairs', P, F, Fv, D, K, lists, pairs, V, e))
    if kernel == 'kd_dibr_bwd':        # the two backwards above in one launch
        return (algorithmic_bytes('kd_raster_bwd_tile', P, F, Fv, D, K, lists, pairs, V, e) +
                algorithmic_bytes('kd_soft_bwd_pairs', P, F, Fv, D, K, lists, pairs, V, e))
    return None


def survey_step_bytes(P, F, D, K, esize=4):
    """SURVEY.md §8(d) whole-step formula (K-lists counted as the reference writes them, the
    N_read term omitted): bytes of one DIB-R fwd+bwd step under the reference's op contract."""
    e = esize
    pix = (8 + 3 * e + D * e) + (8 + e + 13 * K) + (D * e + 8 + 3 * e) + (e + e + 8)
    face = (e * (3 + 6 + 3 * D) + 4) + 24 + 2 * (24 + 12 * D) + 2 * 24
    return P * pix + F * face


class Workload:
    """Inputs of one rank: views [first, first + n) of a global batch, resident on `dev`."""

    def __init__(self, args, dev, first, n, total):
        dt = DTYPES[args.dtype]
        self.soup = args.config in SOUP_CONFIGS
        self.n = n
        kw = dict(sigmainv=args.sigmainv, boxlen=args.boxlen, knum=args.knum)
        self.kw = kw
        if self.soup:
            F, H, W, _ = SOUP_CONFIGS[args.config]
            sz, si, sn = workloads.soup(F, seed=3, batch=total, dtype=dt)
            self.fvz = sz[first:first + n].to(dev).contiguous()
            self.fvi = si[first:first + n].to(dev).contiguous().requires_grad_(True)
            self.nz = sn[first:first + n].to(dev).contiguous()
            g = torch.Generator().manual_seed(4)
            uvs = torch.rand((total, F, 3, 2), generator=g, dtype=dt)[first:first + n].to(dev)
            self.vertices = None
            self.desc = f'soup({F}, seed=3) per view'
        else:
            n_lon, n_lat, H, W, _, elev = CONFIGS[args.config]
            verts, faces, face_uvs = workloads.uv_sphere(n_lon, n_lat, seed=0, dtype=dt)
            F = faces.shape[0]
            self.vertices = verts.to(dev).requires_grad_(True)
            self.faces = faces.to(dev)
            self.cam = workloads.orbit_cameras(n, elev, first_view=first, total_views=total,
                                               dtype=dt).to(dev)
            self.proj = workloads.generate_perspective_projection(math.pi / 4, dtype=dt).to(dev)
            uvs = face_uvs.to(dev).unsqueeze(0).repeat(n, 1, 1, 1)
            self.desc = f'uv_sphere({n_lon},{n_lat}) {F} faces'
        # learnable per-view, per-face-vertex features (uv + mask ones, ian_dibr.py:240-243)
        self.feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
        self.feats.requires_grad_(True)
        self.F, self.H, self.W, self.D = F, H, W, self.feats.shape[-1]
        g_feat, g_soft = workloads.view_grads(first, n, H, W, self.D, dtype=dt)
        self.g_feat, self.g_soft = g_feat.to(dev), g_soft.to(dev)
        self.iou = args.iou
        self.vertex_path = args.vertex_path
        if args.vertex_path != 'compose':
            dibr.FUSED_VERTEX_BACKWARD = args.vertex_path == 'node-vtx'
        self.gt = None
        if self.iou and not self.soup:  # a target silhouette: a disc in the middle of each view
            yy, xx = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt),
                                    indexing='ij')
            disc = (((yy - H / 2) ** 2 + (xx - W / 2) ** 2) < (0.4 * min(H, W)) ** 2).to(dt)
            self.gt = disc.expand(n, H, W).contiguous().to(dev)
        self.params = [self.fvi, self.feats] if self.soup else [self.vertices, self.feats]
        # --perturb LR: the step ends by moving the mesh with its own gradient -- the vertices
        # become v0 - LR * sign(grad), an Adam-sized step (ian_dibr.py:172-173, 288-290) from the
        # initial mesh v0, captured in the graph -- so every replay renders geometry the previous
        # step's tile history was not measured on, while the workload stays the C3 sphere
        # (anchored at v0: repeated sign steps would otherwise roughen it step after step)
        self.perturb = 0.0 if self.soup else float(getattr(args, 'perturb', 0.0) or 0.0)
        self.v0 = self.vertices.detach().clone() if self.perturb else None

    def forward_backward(self):
        """The GPU part of the step (no collective)."""
        if self.soup:
            interp, soft, face_idx = dibr_rasterization(self.H, self.W, self.fvz, self.fvi,
                                                        self.feats, self.nz, **self.kw)
            torch.autograd.backward([interp, soft], [self.g_feat, self.g_soft])
            return face_idx
        face_idx = distributed.dibr_forward_backward(
            self.vertices, self.faces, self.proj, self.cam, self.feats, self.H, self.W,
            self.g_feat, self.g_soft, gt_mask=self.gt, iou=self.iou or 'fused',
            fused_vertices=self.vertex_path != 'compose', **self.kw)
        if self.perturb:
            with torch.no_grad():
                torch.add(self.v0, self.vertices.grad.sign(), alpha=-self.perturb,
                          out=self.vertices)
        return face_idx

    def clear(self):
        for p in self.params:
            p.grad = None

    def exchange(self):
        """The step's one collective: the sum over ranks of the shared vertex gradient."""
        if not self.soup:
            distributed.allreduce_grads_([self.vertices.grad])

    def eager_step(self):
        self.clear()
        face_idx = self.forward_backward()
        self.exchange()
        return face_idx

    def inputs(self):
        """(fvz, fvi, normals_z) of the rank's views (detached)."""
        with torch.no_grad():
            if self.soup:
                return self.fvz, self.fvi.detach(), self.nz
            from kaolin_amd.render.mesh import prepare_vertices
            fvc, fvi, nrm = prepare_vertices(self.vertices.detach().unsqueeze(0), self.faces,
                                             self.proj, camera_transform=self.cam)
            return fvc[..., 2], fvi, nrm[..., 2]


def make_step(wl, use_graph):
    """(callable step, launch description).  The graph holds the GPU part; the all-reduce of the
    shared vertex gradient runs eagerly after each replay."""
    if use_graph:
        try:
            gs = distributed.GraphedStep(wl.params, wl.forward_backward,
                                         params_to_reduce=[] if wl.soup else [wl.vertices])
            return gs, 'hip graph replay (GPU part) + eager RCCL all-reduce'
        except Exception as e:  # noqa: BLE001 -- report and fall back to eager launches
            torch.cuda.synchronize()
            return wl.eager_step, f'eager (graph capture failed: {type(e).__name__}: {e})'[:200]
    return wl.eager_step, 'eager'


def timed(step, steps, warmup, dev, world, wl=None):
    """W untimed steps, then exactly K steps between barrier + synchronize on both sides; the
    wall time is the max over ranks (nothing else is enqueued in that region).  Then K more steps,
    each bracketed by HIP events on the current stream (the replay, and for a GraphedStep at N > 1
    the all-reduce after it), for the median step and the all-reduce's own time.  Returns
    (elapsed s, {'step_ms': [...], 'allreduce_ms': [...] or None})."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the per-step event pass (not part of the timed region)
    graphed = isinstance(step, distributed.GraphedStep)
    split = world > 1 and (graphed or wl is not None)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in ev:
        e[0].record()
        if split and graphed:
            step.replay()
            e[1].record()
            step.exchange()
        elif split:  # the eager step in its two parts: the render, then the all-reduce
            wl.clear()
            wl.forward_backward()
            e[1].record()
            wl.exchange()
        else:
            step()
        e[2].record()
    torch.cuda.synchronize(dev)
    step_ms = [e[0].elapsed_time(e[2]) for e in ev]
    ar_ms = [e[1].elapsed_time(e[2]) for e in ev] if split else None
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, {'step_ms': step_ms, 'allreduce_ms': ar_ms}


def _median_over_ranks(xs, dev, world):
    """The median of this rank's samples, max over the ranks (None without samples)."""
    if not xs:
        return None
    m = statistics.median(xs)
    if world > 1:
        t = torch.tensor([m], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        m = float(t.item())
    return m


def kernel_map(wl, steps, lists):
    """Per-kernel durations from the library's HIP events on the launch stream, over `steps`
    eager launches of the step (events cannot be recorded inside the captured graph on this
    stack: the capture leaves the context unusable).  The graph replays' own per-kernel
    durations are in the committed rocprofv3 kernel traces (tools/trace_steps.py).
    Returns ({name: (total ms, launches)}, source, face_idx)."""
    with dibr.close_lists(lists):
        _lib.profile_enable(True)
        for _ in range(steps):
            face_idx = wl.eager_step()
        torch.cuda.synchronize()
        _lib.profile_enable(False)
    return _lib.profile_collect(), 'eager launches (HIP events around each library launch)', \
        face_idx


def load_pmc(path, config, dtype, lists, views):
    """Per-launch HBM traffic of each kernel from a committed PMC summary of the same workload:
    FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md, HBM: gfx950's FETCH_SIZE reads half of a
    wide streaming read; WRITE_SIZE is exact)."""
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return {}, None
    if (pm.get('config') != config or bool(pm.get('lists')) != lists or
            pm.get('dtype', 'f32') != dtype or pm.get('views_per_gpu', views) != views):
        return {}, None
    out = {}
    for k, ent in pm.get('kernels', {}).items():
        if 'FETCH_SIZE_KiB' in ent and 'WRITE_SIZE_KiB' in ent:
            cyc, mix = valu_issue_cycles(ent)
            out[k] = {'traffic': round((2 * ent['FETCH_SIZE_KiB'] + ent['WRITE_SIZE_KiB']) * 1024),
                      'valu': ent.get('SQ_INSTS_VALU'), 'salu': ent.get('SQ_INSTS_SALU'),
                      'valu_cycles': cyc, 'valu_mix': mix,
                      'valu_active': ent.get('SQ_ACTIVE_INST_VALU'),
                      'device_kernel': ent.get('device_kernel')}
    return out, os.path.relpath(path, ROOT)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launcher_cmd(n, argv, port):
    """The torch.distributed.run command that starts `n` ranks of this script on one node (the
    driver's own form of the N > 1 launch; rendezvous on 127.0.0.1)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
            '--master-addr', '127.0.0.1', '--master-port', str(port),
            os.path.abspath(__file__), *argv]


def spawn_ranks(n, argv):
    """`python bench.py --gpus N` without WORLD_SIZE: launch N ranks (one per GPU; with
    KD_BENCH_BACKEND=gloo they may share one) as a child torch.distributed.run and return its
    exit status.  Nothing here initialises the GPU: torch.cuda.device_count() does not on this
    stack, and no HIP call is made before the children exit."""
    backend = os.environ.get('KD_BENCH_BACKEND', 'nccl')
    visible = torch.cuda.device_count()
    if backend == 'nccl' and visible < n:
        print(f'[bench] --gpus {n}: only {visible} GPU(s) visible (RCCL needs one per rank)',
              file=sys.stderr)
        return 2
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC (RCCL peer buffers)
    return subprocess.call(launcher_cmd(n, argv, free_port()), env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # defaults: a steady-state run (~25 ms timed at C3).  A run that starts from an idle GPU is
    # ~8% slower over its first few ms (profiles/r06/bench_steps_sweep.txt: K = 20 / 100 / 400
    # timed steps after 3 warmup steps gave 0.2537 / 0.2366 / 0.2323 ms per step), so 20 warmup
    # steps and 100 timed ones; the driver's --steps / --warmup are used as given
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='c3', choices=sorted(CONFIGS) + sorted(SOUP_CONFIGS))
    ap.add_argument('--dtype', default='f32', choices=sorted(DTYPES))
    ap.add_argument('--views-per-gpu', type=int, default=None,
                    help='weak scaling: this many views on every GPU (default: the global batch '
                         'of the config split over the GPUs)')
    ap.add_argument('--knum', type=int, default=30)
    ap.add_argument('--sigmainv', type=float, default=7000.)
    ap.add_argument('--boxlen', type=float, default=0.02)
    ap.add_argument('--lists', action='store_true',
                    help='materialise the (B,H,W,K) close-face lists (reference structure)')
    ap.add_argument('--no-graph', action='store_true', help='launch every kernel eagerly')
    ap.add_argument('--iou', default=None, choices=['fused', 'compose'],
                    help='the soft mask\'s gradient from the silhouette loss mask_iou(soft, gt) '
                         '(the training loop\'s), fused into the renderer or as the composition')
    ap.add_argument('--no-weak', action='store_true', help='skip the N > 1 weak-scaling phase')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--vertex-path', default='node', choices=['compose', 'node', 'node-vtx'],
                    help='prepare_vertices + dibr_rasterization as two nodes (compose), or as '
                         'dibr_rasterization_from_vertices (node: the projection inside the '
                         'binning launch, gather backward; node-vtx: its face -> vertex step '
                         'inside the DIB-R backward kernel)')
    ap.add_argument('--coarse-tile', type=int, default=0, choices=[0, 16, 32],
                    help='coarse bin edge of the DIB-R binning (kd_set_coarse_tile; 0: auto)')
    ap.add_argument('--tile-split', type=int, default=0, choices=[0, 1, 2, 4],
                    help='workgroups per tile of the fused forward (kd_set_tile_split; 0: auto)')
    ap.add_argument('--tile-history', type=int, default=1, choices=[0, 1],
                    help='dispatch the fused forward by the previous same-shape call\'s tile '
                         'durations (kd_set_tile_history; default on)')
    ap.add_argument('--perturb', type=float, default=0.0, metavar='LR',
                    help='move the mesh every step: vertices = v0 - LR * sign(grad) with the '
                         'step\'s own gradient, inside the timed step (1 GPU; tile history A/B '
                         'under motion)')
    ap.add_argument('--pmc', default=None,
                    help='PMC traffic summary (default profiles/r06, r05, r04, r03 or r02/pmc_traffic_<config>.json)')
    args = ap.parse_args()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # one process per GPU: started here, before anything touches the GPU (this process only
        # waits for them and exits with their status)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    # KD_BENCH_BACKEND=gloo rehearses the multi-rank path on a single GPU (ranks share cuda:0;
    # RCCL refuses two ranks on one device).  The default is RCCL ("nccl").
    backend = os.environ.get('KD_BENCH_BACKEND', 'nccl')
    rank, world, local = distributed.init_from_env(backend)
    if args.perturb and world > 1:
        raise SystemExit('--perturb: one GPU only (the update would use un-reduced gradients)')
    if world != args.gpus and rank == 0:
        print(f'[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}', file=sys.stderr)
    dev = torch.device('cuda', local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    _lib.load()
    _lib.set_tile_split(args.tile_split)
    _lib.set_coarse_tile(args.coarse_tile)
    _lib.set_tile_history(bool(args.tile_history))
    soup = args.config in SOUP_CONFIGS
    B_global = SOUP_CONFIGS[args.config][3] if soup else CONFIGS[args.config][4]
    weak_main = args.views_per_gpu is not None
    if weak_main:
        total = args.views_per_gpu * world
        first, n = rank * args.views_per_gpu, args.views_per_gpu
    else:
        total = B_global
        first, n = distributed.shard_views(B_global, rank, world)
    use_graph = not args.no_graph and not args.lists and backend == 'nccl'
    with dibr.close_lists(args.lists):
        wl = Workload(args, dev, first, n, total)
        covered0 = None
        if wl.perturb:  # the workload's coverage before the mesh moves
            covered0 = int((wl.eager_step() >= 0).sum().item())
        step, launch = make_step(wl, use_graph)
        elapsed, evt = timed(step, args.steps, args.warmup, dev, world,
                             wl if step == wl.eager_step else None)
    ms_per_step = elapsed * 1e3 / args.steps
    step_median = _median_over_ranks(evt['step_ms'], dev, world)
    ar_median = _median_over_ranks(evt['allreduce_ms'], dev, world) if world > 1 else None
    H, W = wl.H, wl.W
    pixels = total * H * W
    value = pixels * args.steps / elapsed / 1e6

    weak = None
    if world > 1 and not weak_main and not args.no_weak:
        del step
        with dibr.close_lists(args.lists):
            wl2 = Workload(args, dev, rank * B_global, B_global, B_global * world)
            step2, _ = make_step(wl2, use_graph)
            el2, _ = timed(step2, args.steps, args.warmup, dev, world)
        weak = {'value': round(B_global * world * H * W * args.steps / el2 / 1e6, 2),
                'ms_per_step': round(el2 * 1e3 / args.steps, 4), 'views_per_gpu': B_global,
                'global_batch': B_global * world}
        del step2, wl2

    # ---- per-kernel durations: HIP events recorded on the launch stream, eager pass ---------
    prof, prof_src, face_idx = kernel_map(wl, args.steps, args.lists)
    covered = int((face_idx >= 0).sum().item())

    fvz, fvi, nz = wl.inputs()
    Fv = int((nz >= 0).sum().item())
    P = n * H * W
    Ftot = n * wl.F
    V = 0 if soup else wl.vertices.shape[0]
    esize = 8 if args.dtype == 'f64' else 4
    pairs = None
    if not args.lists:
        with torch.no_grad():
            _, _, _, _, ws = _C.render.mesh.dibr_rasterization_forward_fused(
                H, W, fvz, fvi, wl.feats.detach(), nz, args.sigmainv, args.boxlen,
                args.knum, 1000., 1e-8, want_grad=True)
            pairs = int(_lib.load().kd_dibr_pair_count(
                ws.data_ptr(), n, H, W, wl.F, args.knum, 1 if args.dtype == 'f64' else 0,
                torch.cuda.current_stream(dev).cuda_stream))
            del ws
    fused = 'kd_soft_pair_math' not in prof  # the one-launch soft mask (kd_softpair.hip)
    # the step's count projects the mesh (dibr_rasterization_from_vertices, kd_bin_count PREP)
    prep = (V, wl.F, n) if (not soup and args.vertex_path != 'compose' and not args.iou) else None
    pmc, pmc_src = {}, None
    for rnd in ([args.pmc] if args.pmc else ['r06', 'r05', 'r04', 'r03', 'r02']):  # the newest committed summary
        pmc_path = rnd if args.pmc else os.path.join(ROOT, 'profiles', rnd,
                                                       f'pmc_traffic_{args.config}.json')
        pmc, pmc_src = load_pmc(pmc_path, args.config, args.dtype, args.lists, n)
        if pmc:
            break
    kernels = {}
    moved = 0
    for name, (ms, cnt) in prof.items():
        avg_us = ms * 1e3 / cnt
        ab = algorithmic_bytes(name, P, Ftot, Fv, wl.D, args.knum, args.lists, pairs, V, esize,
                               fused=fused, prep=prep)
        kernels[name] = {'avg_us': round(avg_us, 2), 'launches': cnt,
                         'share': round(ms / max(sum(v[0] for v in prof.values()), 1e-9), 3)}
        if ab is not None:
            kernels[name]['alg_bytes'] = ab
            kernels[name]['GB_s'] = round(ab / (avg_us * 1e-6) / 1e9, 1)
            moved += ab * cnt / args.steps
        if name in pmc:
            kernels[name]['traffic'] = pmc[name]['traffic']
            if ab:
                kernels[name]['traffic_ratio'] = round(pmc[name]['traffic'] / ab, 3)
            kernels[name]['pmc_kernel'] = pmc[name]['device_kernel']
            if pmc[name]['valu_cycles']:
                kernels[name]['valu_issue_frac'] = round(
                    pmc[name]['valu_cycles'] / (VALU_SIMDS * CLOCK_HZ) / (avg_us * 1e-6), 3)
            if pmc[name]['valu_active']:  # quad-cycles summed over waves
                kernels[name]['valu_busy_frac'] = round(
                    pmc[name]['valu_active'] * 4 / (VALU_SIMDS * CLOCK_HZ) / (avg_us * 1e-6), 3)
    dom = max(prof.items(), key=lambda kv: kv[1][0])[0] if prof else None
    roofline = None
    if dom is not None:
        ms, cnt = prof[dom]
        avg_s = ms / cnt / 1e3
        ab = kernels[dom].get('alg_bytes')
        achieved = ab / avg_s / 1e9 if ab else None
        traffic = pmc[dom]['traffic'] if dom in pmc else None
        hbm_frac = None if achieved is None else achieved / HBM_PEAK_GBS
        valu = None
        if dom in pmc and pmc[dom]['valu']:
            e = pmc[dom]
            issue_s = e['valu_cycles'] / (VALU_SIMDS * CLOCK_HZ) if e['valu_cycles'] else None
            busy_s = e['valu_active'] * 4 / (VALU_SIMDS * CLOCK_HZ) if e['valu_active'] else None
            valu = {'insts_per_launch': round(e['valu']),
                    'salu_insts_per_launch': round(e['salu'] or 0),
                    'mix_per_launch': {k: round(v) for k, v in (e['valu_mix'] or {}).items()},
                    'issue_us': None if issue_s is None else round(issue_s * 1e6, 2),
                    'frac': None if issue_s is None else round(issue_s / avg_s, 4),
                    'roof': f'{VALU_SIMDS} SIMDs at {CLOCK_HZ / 1e9:g} GHz, wave64 issue cycles '
                            f'per instruction type {VALU_MIX_CYCLES}, other {VALU_OTHER_CYCLES} '
                            f'(MI355X_MICROARCH.md: >= 2 waves per SIMD)',
                    'busy_us': None if busy_s is None else round(busy_s * 1e6, 2),
                    'busy_frac': None if busy_s is None else round(busy_s / avg_s, 4),
                    'busy': 'SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) x 4 / (SIMDs x '
                            'clock): the cycles the SIMDs measured executing VALU instructions',
                    'source': f'{pmc_src}: {e["device_kernel"]}, SQ_INSTS_VALU_* per launch'}
        # the contract's bound is "hbm" | "mfma": this path has no MFMA work, so "hbm" with the
        # byte fraction; `limiter` names the larger of the roof fractions (VALU issue here)
        vf = max(valu.get('frac') or 0, valu.get('busy_frac') or 0) if valu else 0
        limiter = 'valu_issue' if valu and hbm_frac is not None and vf > hbm_frac else 'hbm'
        roofline = {'kernel': dom, 'bound': 'hbm', 'limiter': limiter,
                    'achieved': None if achieved is None else round(achieved, 1),
                    'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': None if hbm_frac is None else round(hbm_frac, 4),
                    'traffic': traffic,
                    'traffic_ratio': round(traffic / ab, 3) if traffic and ab else None,
                    'traffic_source': pmc_src and f'{pmc_src}: FETCH_SIZE x 2 + WRITE_SIZE',
                    'valu_issue': valu,
                    'alg_bytes_per_launch': ab, 'avg_launch_us': round(avg_s * 1e6, 2)}
    ref_bytes = survey_step_bytes(P, Ftot, wl.D, args.knum, esize)
    step_roof = {
        'bytes_per_step_per_gpu': round(moved),
        'formula': 'sum over the step\'s kernels of their algorithmic bytes per launch '
                   '(the bytes this implementation must move)',
        'achieved': round(moved / (ms_per_step * 1e-3) / 1e9, 1) if moved else None,
        'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': round(moved / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if moved else None,
        'pairs_per_step': pairs,
        'reference_contract': {
            'formula': 'SURVEY.md §8(d): 482 B/px + 268 B/face at D=3, K=30, fp32 (the (B,H,W,K) '
                       'close lists counted as the reference op writes them; N_read omitted)',
            'bytes_per_step_per_gpu': ref_bytes,
            'equivalent_GB_s': round(ref_bytes / (ms_per_step * 1e-3) / 1e9, 1),
            'note': 'not HBM traffic of this path: the K-lists are ' +
                    ('written (--lists)' if args.lists else 'never materialised here')}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, fvz, fvi, nz)

    out = {
        'metric': METRIC, 'value': round(value, 2), 'unit': 'Mpixels/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
        'ms_per_step_median': None if step_median is None else round(step_median, 4),
        'allreduce_us': None if ar_median is None else round(ar_median * 1e3, 2),
        'timing': 'value and ms_per_step: K steps between barrier + synchronize, wall clock, max '
                  'over ranks, nothing else enqueued; ms_per_step_median: median of the per-step '
                  'HIP event times of K further steps (max over ranks); allreduce_us: median '
                  'per-step time of the RCCL all-reduce after the graph replay (N > 1)',
        'higher_is_better': True, 'scaling': 'weak' if weak_main else 'strong',
        'vs_baseline': None, 'dtype': args.dtype,
        'data': 'synthetic (seeded ' + ('triangle soup' if soup else 'uv-sphere, orbit cameras')
                + '; no dataset)',
        'config': {'workload': f'{args.config.upper()}: {wl.desc}, {H}x{W}, global batch '
                               f'{total} ({n} views/GPU), D={wl.D}, knum={args.knum}, '
                               f'sigmainv={args.sigmainv:g}, boxlen={args.boxlen:g}',
                   'faces': wl.F, 'height': H, 'width': W, 'views_per_gpu': n,
                   'global_batch': total,
                   'parallelism': f'view-sharded x{world}' +
                                  ((' + RCCL' if backend == 'nccl' else f' + {backend}') +
                                   ' vertex-grad all-reduce' if world > 1 and not soup else ''),
                   'launch': launch,
                   'hip_graph_packet_capture': os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE',
                                                              'runtime default'),
                   'vertex_path': {'compose': 'prepare_vertices + dibr_rasterization',
                                   'node': 'dibr_rasterization_from_vertices (projection in the '
                                           'binning launch; gather backward)',
                                   'node-vtx': 'dibr_rasterization_from_vertices (face -> vertex '
                                               'step in the DIB-R backward kernel)'}[
                                       args.vertex_path],
                   'tile_split': args.tile_split or 'auto',
                   'coarse_tile': args.coarse_tile or 'auto',
                   'tile_history': bool(args.tile_history),
                   'perturb': None if not wl.perturb else {
                       'lr': wl.perturb, 'update': 'vertices = v0 - lr * sign(vertices.grad) '
                                                   'inside every timed step (graph)',
                       'covered_px_first_step': covered0},
                   'close_lists': 'materialised' if args.lists else 'not materialised',
                   'soft_mask_grad': (f'mask_iou(soft, gt) ({args.iou})' if args.iou
                                      else 'fixed seeded grad_soft'),
                   'covered_px_per_step': covered, 'front_faces': Fv},
        'roofline': roofline,
        'step_roofline': step_roof,
        'weak_scaling': weak,
        'cpu_baseline': cpu,
        'kernels': kernels,
        'kernels_source': prof_src,
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _cpu_model():
    try:
        txt = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            if line.startswith('Model name'):
                return line.split(':', 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def cpu_baseline(wl, fvz, fvi, nz, runs=5):
    """The CPU oracle (oracle/dibr_oracle.c: the reference's brute-force loops in C, OpenMP) on a
    bounded sample of the same workload, SURVEY.md §8(d) protocol: median of `runs` after one
    warmup, on the box's host cores (OMP_NUM_THREADS) and on one thread.  Sample: the rank's
    first view, fwd+bwd (all threads); rows 3/8..5/8 of it (one thread)."""
    import numpy as np
    import oracle
    # the GPU box gives each GPU a 16-CPU share and sets OMP_NUM_THREADS to it (os.cpu_count()
    # shows the whole host); without that variable, every CPU this process may run on
    affinity = len(os.sched_getaffinity(0))
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or affinity
    H, W, kw = wl.H, wl.W, wl.kw
    n = lambda t: np.ascontiguousarray(t[:1].detach().cpu().numpy())  # noqa: E731
    fvz_, fvi_, nz_, ft_ = n(fvz), n(fvi), n(nz), n(wl.feats)
    gf_, gs_ = n(wl.g_feat), n(wl.g_soft)

    def once(rows):
        t0 = time.perf_counter()
        _, face_idx, weights = oracle.rasterize(H, W, fvz_, fvi_, ft_, nz_ >= 0, rows=rows)
        soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(
            fvi_, face_idx, kw['sigmainv'], kw['boxlen'], kw['knum'], 1000., rows=rows)
        oracle.rasterize_backward(gf_, face_idx, weights, fvi_, ft_, 1e-8)
        oracle.soft_mask_backward(gs_, soft, face_idx, prob, cidx, ctype, sfvi, kw['sigmainv'],
                                  1000.)
        return time.perf_counter() - t0

    def median_rate(px, rows):
        once(rows)  # warmup
        ts = [once(rows) for _ in range(runs)]
        med = statistics.median(ts)
        return px / med / 1e6, med, ts

    oracle.set_num_threads(threads)
    rate, med, ts = median_rate(H * W, None)
    r0, r1 = (3 * H) // 8, (5 * H) // 8
    oracle.set_num_threads(1)
    rate1, med1, _ = median_rate((r1 - r0) * W, (r0, r1))
    oracle.set_num_threads(threads)
    return {'value': round(rate, 5), 'unit': 'Mpixels/s', 'cores': threads, 'kind': 'port',
            'sample': f'1 view of the workload ({H}x{W} px, {fvi.shape[1]} faces), fwd+bwd, '
                      f'brute-force reference loops (oracle/dibr_oracle.c, OpenMP, {threads} '
                      f'threads): median of {runs} runs after 1 warmup = {med:.3f} s',
            'runs_s': [round(t, 3) for t in ts],
            'single_thread': {'value': round(rate1, 5), 'unit': 'Mpixels/s',
                              'sample': f'rows {r0}..{r1 - 1} of the same view, 1 thread, '
                                        f'median of {runs} after 1 warmup = {med1:.3f} s'},
            'host': {'lscpu_model': _cpu_model(), 'nproc': os.cpu_count(),
                     'affinity_cpus': affinity,
                     'omp_num_threads': os.environ.get('OMP_NUM_THREADS')},
            'cores_reason': ('OMP_NUM_THREADS: the GPU box\'s CPU share per GPU (the pool sets it '
                             'to 16; nproc shows every CPU of the host, which other GPUs\' jobs '
                             'share)') if os.environ.get('OMP_NUM_THREADS') else
                            'every CPU in this process\'s affinity mask'}


if __name__ == '__main__':
    main()
