"""Is the bench step launch-bound?  python tools/launch_probe.py [--config c3] [--steps 40]

Times the bench step (bench.py's step) three ways on one GPU:
  eager   the wall time per step with one sync at the end, and the host time spent issuing it;
  graph   the whole step (forward, backward, gradient all-reduce) captured once in a HIP graph
          (torch.cuda.graph) and replayed -- no host work and no per-kernel launch overhead;
and checks that the graph replay produces the same vertex gradient as the eager step.
"""
import argparse
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization, prepare_vertices  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    ap.add_argument('--steps', type=int, default=40)
    args = ap.parse_args()
    _lib.load()
    dev = torch.device('cuda', 0)
    n_lon, n_lat, H, W, B, elev = bench.CONFIGS[args.config]
    verts, faces, face_uvs = workloads.uv_sphere(n_lon, n_lat, seed=0)
    vertices = verts.to(dev).requires_grad_(True)
    faces = faces.to(dev)
    cam = workloads.orbit_cameras(B, elev).to(dev)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(dev)
    uvs = face_uvs.to(dev).unsqueeze(0).repeat(B, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
    feats.requires_grad_(True)
    g = torch.Generator().manual_seed(1)
    g_feat = torch.rand((B, H, W, 3), generator=g).to(dev)
    g = torch.Generator().manual_seed(2)
    g_soft = torch.rand((B, H, W), generator=g).to(dev)

    def step():
        fvc, fvi, nrm = prepare_vertices(vertices.unsqueeze(0), faces, proj, camera_transform=cam)
        interp, soft, face_idx = dibr_rasterization(H, W, fvc[..., 2], fvi, feats, nrm[..., 2])
        torch.autograd.backward([interp, soft], [g_feat, g_soft])

    for _ in range(5):
        vertices.grad = None
        feats.grad = None
        step()
    torch.cuda.synchronize()
    ref = vertices.grad.clone()

    host = 0.
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vertices.grad = None
        feats.grad = None
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / args.steps
    print(f'eager: {eager * 1e3:.4f} ms/step, host issue {host / args.steps * 1e3:.4f} ms/step')

    # graph capture (grads accumulate into .grad inside the graph: zero them in the graph)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            vertices.grad = None
            feats.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    vertices.grad = None
    feats.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    graph.replay()
    torch.cuda.synchronize()
    diff = float((vertices.grad - ref).abs().max())
    scale = float(ref.abs().max())
    print(f'graph grad max |diff| {diff:.3e} (scale {scale:.3e})')
    for _ in range(5):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay()
    torch.cuda.synchronize()
    gt = (time.perf_counter() - t0) / args.steps
    print(f'graph: {gt * 1e3:.4f} ms/step')


if __name__ == '__main__':
    main()
