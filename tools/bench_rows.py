"""Throughput of the SURVEY §8 (f) rows on the GPU: python tools/bench_rows.py [--steps N]

For each row, the HIP kernels' average launch time (HIP events, kd_profile_*), their algorithmic
HBM bytes per launch (stated below) and the fraction of the 8 TB/s HBM peak; and, where the
reference's implementation of the row is plain torch (mask_iou: kaolin/metrics/render.py:32-41;
texture_mapping: kaolin/render/mesh/utils.py:59-76), that torch composition timed on the same GPU
as the reference number.  Prints one JSON line per row.

Workloads (the C3 training step's shapes: 8 views of 512 x 512, a 512 x 512 RGB texture as in
examples/tutorial/ian_dibr.py:38, the 50k-face uv-sphere):
  mask_iou         fwd + bwd on (8, 512, 512) fp32
  texture_mapping  bilinear fwd + bwd (texture and uv gradients), (8, 512, 512, 2) uvs
  rast_interpolate nvdiffrast-format buffer (8, 512, 512, 4) -> features D=3 + weights + index
  deftet           sparse render of the 50k-face sphere at 262144 pixel coords (one view), knum 30
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.metrics.render import mask_iou  # noqa: E402
from kaolin_amd.render.mesh import (deftet_sparse_render, prepare_vertices,  # noqa: E402
                                    rasterize_from_rast, texture_mapping)

PEAK = 8000.0  # GB/s
DEV = 'cuda'


def timed(fn, steps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.profile_collect()
    _lib.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    _lib.profile_enable(False)
    prof = _lib.profile_collect()
    return wall, {k: ms * 1e3 / n for k, (ms, n) in prof.items()}


def torch_time(fn, steps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def line(row, wall, kern, bytes_):
    out = {'row': row, 'wall_us': round(wall * 1e6, 1), 'kernels': {}}
    for k, us in kern.items():
        e = {'avg_us': round(us, 2)}
        if k in bytes_:
            e['alg_bytes'] = bytes_[k]
            e['GB_s'] = round(bytes_[k] / (us * 1e-6) / 1e9, 1)
            e['frac'] = round(e['GB_s'] / PEAK, 3)
        out['kernels'][k] = e
    return out


def torch_mask_iou(l, r):
    B = l.shape[0]
    mul = l * r
    add = l + r
    up = torch.sum(mul.reshape(B, -1), dim=1)
    down = torch.sum((add - mul).reshape(B, -1), dim=1)
    return 1.0 - torch.mean(up / (down + 1e-10))


def torch_texture_mapping(uv, tex, mode):
    B, C = uv.shape[0], tex.shape[1]
    t = uv.reshape(B, -1, 1, 2)
    t = torch.clamp(t, 0., 1.)
    t = t * 2 - 1
    t = torch.stack([t[..., 0], -t[..., 1]], dim=-1)
    r = torch.nn.functional.grid_sample(tex, t, mode=mode, align_corners=False,
                                        padding_mode='border')
    return r.permute(0, 2, 3, 1).reshape(B, *uv.shape[1:-1], C)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--rows', default='mask_iou,texture_mapping,rast_interpolate,deftet')
    ap.add_argument('--dt-fwd', action='store_true', help='deftet: the forward alone (no grad)')
    args = ap.parse_args()
    rows = args.rows.split(',')
    _lib.load()
    torch.manual_seed(0)
    B, H, W = 8, 512, 512
    P = B * H * W
    S = args.steps

    # mask_iou ------------------------------------------------------------------------------
    if 'mask_iou' in rows:
        soft = torch.rand((B, H, W), device=DEV).requires_grad_(True)
        gt = (torch.rand((B, H, W), device=DEV) > 0.5).float()

        def iou_step():
            mask_iou(soft, gt).backward()

        def iou_ref():
            torch_mask_iou(soft, gt).backward()
        wall, kern = timed(iou_step, S)
        r = line('mask_iou', wall, kern, {'kd_iou_partial': 8 * P, 'kd_iou_bwd': 12 * P})
        r['torch_reference_us'] = round(torch_time(iou_ref, S) * 1e6, 1)
        print(json.dumps(r))

    # the C3 render: interpolated uvs, face index, barycentrics of the real DIB-R forward
    from kaolin_amd.render.mesh import dibr_rasterization
    verts, faces, face_uvs = workloads.uv_sphere(250, 101, seed=0)
    F = faces.shape[0]
    cams = workloads.orbit_cameras(B, 0.3).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    with torch.no_grad():
        fvc, fvi_r, nrm = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                           camera_transform=cams)
        uvs_b = face_uvs.to(DEV).unsqueeze(0).repeat(B, 1, 1, 1)
        interp, _, face_idx = dibr_rasterization(H, W, fvc[..., 2], fvi_r, uvs_b, nrm[..., 2])
        _, _, weights, _, _ = __import__('kaolin_amd')._C.render.mesh \
            .dibr_rasterization_forward_fused(H, W, fvc[..., 2], fvi_r, uvs_b, nrm[..., 2],
                                              7000., 0.02, 30, 1000., 1e-8, want_grad=False)
    mask = (face_idx >= 0).float().unsqueeze(-1)

    # texture_mapping (ian_dibr.py:248-252: the rendered uvs, background uv = 0; the image loss
    # gradient is masked, so background samples carry a zero gradient) ----------------------
    if 'texture_mapping' in rows or 'rast_interpolate' in rows:
        uv = interp.detach().clone().requires_grad_(True)
        tex = torch.rand((B, 3, 512, 512), device=DEV).requires_grad_(True)
        go = torch.rand((B, H, W, 3), device=DEV) * mask
        texb = tex.numel() * 4

        def tex_step():
            torch.autograd.backward(texture_mapping(uv, tex, mode='bilinear'), go)

        def tex_ref():
            torch.autograd.backward(torch_texture_mapping(uv, tex, 'bilinear'), go)
        wall, kern = timed(tex_step, S)
        r = line('texture_mapping', wall, kern,
                 {'kd_tex_fwd': P * (8 + 12) + texb, 'kd_tex_bwd': P * (8 + 12 + 8) + 2 * texb})
        r['torch_reference_us'] = round(torch_time(tex_ref, S) * 1e6, 1)
        print(json.dumps(r))

        # rast_interpolate: a rast buffer holding the C3 render (u, v, 0, face + 1) ------------
        feat = uvs_b.clone().requires_grad_(True)
        fvi = fvi_r.clone().requires_grad_(True)
        rast = torch.cat([weights[..., :2], torch.zeros_like(weights[..., :1]),
                          (face_idx + 1).float().unsqueeze(-1)], dim=-1).contiguous()
        cov = int((face_idx >= 0).sum())
        go2 = torch.rand((B, H, W, 2), device=DEV)

        def ri_step():
            out, _ = rasterize_from_rast(rast, fvi, feat)
            out.backward(go2)
        wall, kern = timed(ri_step, S)
        print(json.dumps(line('rast_interpolate', wall, kern,
                              {'kd_rast_interp': P * (16 + 8 + 8 + 12) + cov * 24})))

    # deftet --------------------------------------------------------------------------------
    cam = cams[:1]
    with torch.no_grad():
        fvc, fvi1, _ = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                        camera_transform=cam)
    fvz1 = fvc[..., 2].contiguous()
    xs = (2 * torch.arange(W, device=DEV) + 1 - W) / W
    ys = (H - 2 * torch.arange(H, device=DEV) - 1.) / H
    px = torch.stack([xs.reshape(1, -1).expand(H, W), ys.reshape(-1, 1).expand(H, W)],
                     -1).reshape(1, -1, 2).contiguous()
    rr = torch.tensor([-1e9, 0.], device=DEV).expand(1, H * W, 2).contiguous()
    uvs1 = face_uvs.to(DEV).unsqueeze(0).contiguous().requires_grad_(True)
    fvi1 = fvi1.contiguous().requires_grad_(True)
    K = 30
    gdt = torch.rand((1, H * W, K, 2), device=DEV)

    def dt_step():
        if args.dt_fwd:
            with torch.no_grad():
                deftet_sparse_render(px, rr, fvz1, fvi1, uvs1, K)
            return
        interp, _ = deftet_sparse_render(px, rr, fvz1, fvi1, uvs1, K)
        interp.backward(gdt)
    wall, kern = timed(dt_step, S)
    with torch.no_grad():
        _, fidx = deftet_sparse_render(px, rr, fvz1, fvi1, uvs1, K)
    hits = int((fidx >= 0).sum())
    r = line('deftet', wall, kern,
             {'kd_dt_fwd': H * W * (16 + K * (8 + 2 * 4 + 3 * 4)) + F * 60 + hits * 24})
    r['hits'] = hits
    print(json.dumps(r))


if __name__ == '__main__':
    main()
