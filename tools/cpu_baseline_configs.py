#!/usr/bin/env python
"""CPU baseline at every SURVEY.md §8(d) config (its protocol: the brute-force C restatement of the
reference kernels, oracle/dibr_oracle.c, on all host cores and on one thread, median of 5 runs
after 1 warmup; forward at C1-C5, forward + backward at C2-C3).

The reference has no CPU implementation of this path (SURVEY finding 3), so this is the port
(``kind: "port"``).  Each run covers a bounded band of rows of the config's first view (at least
4 rows per thread -- OpenMP runs over rows -- grown by a calibration run until one run takes about
`--target` seconds); Mpixels/s is over the
band's pixels.  The brute force costs O(pixels x faces), so the band is representative of the
whole view only up to the silhouette share in it: the band is centred on the image.

Usage: python tools/cpu_baseline_configs.py [--target 1.5] [--out profiles/r02/cpu_baseline.jsonl]
"""
import argparse
import json
import math
import os
import statistics
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from kaolin_amd import workloads  # noqa: E402

# name -> (mesh, H, W, elevation, fwd+bwd?)
CONFIGS = {
    'c1': (('sphere', 20, 26), 128, 128, 0.3, False),
    'c2': (('sphere', 100, 51), 256, 256, 0.3, True),
    'c3': (('sphere', 250, 101), 512, 512, 0.3, True),
    'c4': (('sphere', 250, 101), 1024, 1024, 0.3, False),
    'c5': (('sphere', 500, 201), 512, 512, 0.6, False),
    'c5soup': (('soup', 200000), 512, 512, 0.3, False),
}


def view0(mesh, H, W, elev):
    if mesh[0] == 'soup':
        fvz, fvi, nz = workloads.soup(mesh[1], seed=3, batch=1)
        F = mesh[1]
        uvs = torch.rand((1, F, 3, 2), generator=torch.Generator().manual_seed(4))
    else:
        verts, faces, face_uvs = workloads.uv_sphere(mesh[1], mesh[2], seed=0)
        cam = workloads.orbit_cameras(1, elev, first_view=0, total_views=8)
        proj = workloads.generate_perspective_projection(math.pi / 4)
        fvc, fvi, nrm = workloads.prepare_vertices(verts.unsqueeze(0), faces, proj, cam)
        fvz, nz = fvc[..., 2], nrm[..., 2]
        uvs = face_uvs.unsqueeze(0)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1)
    g_feat, g_soft = workloads.view_grads(0, 1, H, W, 3)
    n = lambda t: np.ascontiguousarray(t.detach().numpy().astype(np.float32))  # noqa: E731
    return n(fvz), n(fvi), n(nz), n(feats), n(g_feat), n(g_soft)


def run(inp, H, W, rows, bwd):
    fvz, fvi, nz, ft, gf, gs = inp
    t0 = time.perf_counter()
    _, face_idx, weights = oracle.rasterize(H, W, fvz, fvi, ft, nz >= 0, rows=rows)
    soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(fvi, face_idx, 7000., 0.02, 30,
                                                             1000., rows=rows)
    if bwd:
        oracle.rasterize_backward(gf, face_idx, weights, fvi, ft, 1e-8)
        oracle.soft_mask_backward(gs, soft, face_idx, prob, cidx, ctype, sfvi, 7000., 1000.)
    return time.perf_counter() - t0


def measure(inp, H, W, bwd, threads, target, runs=5):
    oracle.set_num_threads(threads)
    mid = H // 2
    band = lambda n: (max(0, mid - n // 2), min(H, max(0, mid - n // 2) + n))  # noqa: E731
    n = min(H, 4 * threads)  # OpenMP runs over rows: every thread gets rows
    while True:  # calibration: grow the band until a run is long enough to scale from
        t = run(inp, H, W, band(n), bwd)
        if t >= target / 8 or n >= H:
            break
        n = min(H, n * 4)
    n = int(max(min(H, 4 * threads), min(H, n * target / max(t, 1e-6))))
    r0 = band(n)[0]
    rows = (r0, min(H, r0 + n))
    run(inp, H, W, rows, bwd)  # warmup
    ts = [run(inp, H, W, rows, bwd) for _ in range(runs)]
    med = statistics.median(ts)
    px = (rows[1] - rows[0]) * W
    return {'value': round(px / med / 1e6, 6), 'unit': 'Mpixels/s', 'threads': threads,
            'rows': list(rows), 'median_s': round(med, 4), 'runs_s': [round(t, 4) for t in ts]}


def cpu_model():
    try:
        txt = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            if line.startswith('Model name'):
                return line.split(':', 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--target', type=float, default=1.5, help='seconds per timed run')
    ap.add_argument('--configs', default=','.join(CONFIGS))
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or os.cpu_count()
    host = {'lscpu_model': cpu_model(), 'nproc': os.cpu_count(),
            'omp_num_threads': os.environ.get('OMP_NUM_THREADS')}
    lines = []
    for name in args.configs.split(','):
        mesh, H, W, elev, fb = CONFIGS[name]
        inp = view0(mesh, H, W, elev)
        for bwd in ([False, True] if fb else [False]):
            rec = {'config': name, 'what': 'fwd+bwd' if bwd else 'fwd', 'H': H, 'W': W,
                   'faces': int(inp[1].shape[1]), 'kind': 'port',
                   'all_threads': measure(inp, H, W, bwd, threads, args.target),
                   'single_thread': measure(inp, H, W, bwd, 1, args.target), 'host': host}
            lines.append(rec)
            print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            for r in lines:
                f.write(json.dumps(r) + '\n')


if __name__ == '__main__':
    main()
