"""Per-workgroup timeline of the pooled DefTet forward at the bench_rows workload (diagnostic
build, flag 64): kernel span, workgroup start spread (dispatch), durations and the walk+test /
rank / store phases.   KAOLIN_AMD_DIAG=1 python tools/dt_timeline.py   (GPU)
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import deftet_sparse_render, prepare_vertices  # noqa: E402

DEV = 'cuda'
# DT_KERNEL=pool (flag 2048, 4 pixels per workgroup) or cell (the default kernel: one slot per
# work item, P / 64 + 64^2 of them; slot 2 holds the cell's list length instead of a phase end)
KERNEL = os.environ.get('DT_KERNEL', 'cell')


def main():
    H = W = 512
    verts, faces, face_uvs = workloads.uv_sphere(250, 101, seed=0)
    cams = workloads.orbit_cameras(8, 0.3).to(DEV)[:1]
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    with torch.no_grad():
        fvc, fvi, _ = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                       camera_transform=cams)
    fvz = fvc[..., 2].contiguous()
    xs = (2 * torch.arange(W, device=DEV) + 1 - W) / W
    ys = (H - 2 * torch.arange(H, device=DEV) - 1.) / H
    px = torch.stack([xs.reshape(1, -1).expand(H, W), ys.reshape(-1, 1).expand(H, W)],
                     -1).reshape(1, -1, 2).contiguous()
    rr = torch.tensor([-1e9, 0.], device=DEV).expand(1, H * W, 2).contiguous()
    uvs = face_uvs.to(DEV).unsqueeze(0).contiguous()
    fvi = fvi.contiguous()
    nwg = (H * W + 3) // 4 if KERNEL == 'pool' else (H * W + 63) // 64 + 64 * 64
    lib = _lib.load()
    buf = torch.zeros(5 * nwg, dtype=torch.int64, device=DEV)
    for _ in range(3):
        deftet_sparse_render(px, rr, fvz, fvi, uvs, 30)
    lib.kd_debug_buffer(buf.data_ptr())
    _lib.debug_set(64 | (2048 if KERNEL == "pool" else 1024))
    deftet_sparse_render(px, rr, fvz, fvi, uvs, 30)
    torch.cuda.synchronize()
    _lib.debug_set(0)
    lib.kd_debug_buffer(None)
    b = buf.reshape(5, nwg).double() / 100.  # 100 MHz ticks -> us
    dur, start, t_walk, t_rank, t_store = b
    t0 = start.min()
    end = start + dur
    print(f'span {float(end.max() - t0):.1f} us, workgroups {nwg}, '
          f'sum of durations {float(dur.sum()) / 1e3:.2f} ms')
    print(f'duration mean {float(dur.mean()):.2f} p50 {float(dur.median()):.2f} '
          f'p99 {float(dur.quantile(0.99)):.2f} max {float(dur.max()):.2f} us')
    if KERNEL == 'pool':
        print(f'phases mean: walk+test {float((t_walk - start).mean()):.2f} rank '
              f'{float((t_rank - t_walk).mean()):.2f} store {float((t_store - t_rank).mean()):.2f} '
              f'rest {float((end - t_store).mean()):.2f} us')
    else:
        nl = t_walk * 100.  # back to the raw value
        live = nl > 0
        for lo_, hi_ in ((1, 64), (65, 128), (129, 256), (257, 512), (513, 100000)):
            m = live & (nl >= lo_) & (nl <= hi_)
            if m.any():
                print(f'  list {lo_:4d}-{hi_:6d}: {int(m.sum()):5d} items, duration mean '
                      f'{float(dur[m].mean()):7.1f} max {float(dur[m].max()):7.1f} us')
    s = (start - t0).sort().values
    for f in (0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0):
        i = min(int(f * (nwg - 1)), nwg - 1)
        print(f'  {int(f * 100):3d}% of workgroups started by {float(s[i]):7.1f} us')
    top = dur.topk(5)
    print('slowest:', [(int(i), round(float(v), 1)) for v, i in zip(top.values, top.indices)])


if __name__ == '__main__':
    main()
