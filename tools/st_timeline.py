"""Per-workgroup timeline of the small-batch forward (kd_dibr_fwd_st<true>, debug flag 64): the
raster and soft phases of each (tile, quadrant), the slowest ones and their bin sizes.
python tools/st_timeline.py [c3:1]"""
import os
os.environ.setdefault('KAOLIN_AMD_DIAG', '1')  # the diagnostic build (per-tile clocks)
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3:1'
cfg, _, nv = cfg.partition(':')
n_lon, n_lat, H, W, B, elev = bench.CONFIGS[cfg]
B = int(nv) if nv else B
dev = torch.device('cuda')
v = workloads.sphere_views(n_lon, n_lat, H, W, B, dev, elevation=elev)
fvz, fvi, feats, nz = v['fvz'], v['fvi'].requires_grad_(True), v['feats'], v['normals_z']
ntx, nty = (W + 15) // 16, (H + 15) // 16
n = B * ntx * nty
nwg = 4 * ((n + 7) // 8 * 8)
buf = torch.zeros(5 * nwg, dtype=torch.int64, device=dev)
lib = _lib.load()
lib.kd_debug_buffer(buf.data_ptr())
lib.kd_debug_set(1 << 27)  # the small-batch form (the mode fixes the workspace layout: set first)
for _ in range(3):
    dibr_rasterization(H, W, fvz, fvi, feats, nz)
torch.cuda.synchronize()
lib.kd_debug_set(64 | (1 << 27))
_, _, fidx = dibr_rasterization(H, W, fvz, fvi, feats, nz)
torch.cuda.synchronize()
lib.kd_debug_set(0)
lib.kd_debug_buffer(None)
t = buf.view(5, nwg).cpu().numpy()
live = t[1] > 0
dur = t[1] / 100.0
start = (t[2] - t[2][live].min()) / 100.0
rdur = (t[3] - t[2]) / 100.0
sdur = dur - rdur
end = start + dur
print(f'kernel span {end[live].max():.1f} us, workgroups {live.sum()}, sum {dur.sum() / 1e3:.2f} ms '
      f'(raster {rdur[live].sum() / 1e3:.2f}, soft {sdur[live].sum() / 1e3:.2f})')
key = t[0] & 0xffffffff
rbin = t[0] >> 32
unc = (fidx < 0).reshape(B, nty, 2, 8, ntx, 2, 8).sum(dim=(3, 6))  # (B, ty, qy, tx, qx)
unc = unc.permute(0, 1, 3, 2, 4).reshape(-1, 4).cpu().numpy()   # (tile, quad = qy*2+qx)
order = np.argsort(end)[::-1]
print('slowest: slot start raster soft | tile quad raster_bin soft_bin unc')
for i in order[:16]:
    tq = int(key[i])
    print(f'  {i:5d} {start[i]:6.1f} {rdur[i]:6.1f} {sdur[i]:6.1f} | {tq // 4:5d} {tq % 4} '
          f'{int(rbin[i]):6d} {int(t[4][i]):6d} {int(unc[tq // 4, tq % 4]):3d}')
for q in range(10):
    sl = slice(q * nwg // 10, (q + 1) * nwg // 10)
    m = live[sl]
    print(f'  slots {sl.start:5d}: start [{start[sl][m].min():6.1f},{start[sl][m].max():6.1f}] '
          f'raster mean {rdur[sl][m].mean():5.1f} max {rdur[sl][m].max():5.1f}  soft mean '
          f'{sdur[sl][m].mean():5.1f} max {sdur[sl][m].max():5.1f}')
