"""Per-tile durations of the tile kernels (kd_debug_set flag 64): distribution and hot spots."""
import os
os.environ.setdefault('KAOLIN_AMD_DIAG', '1')  # the diagnostic build (ablation flags)
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
n_lon, n_lat, H, W, B, elev = bench.CONFIGS[cfg]
dev = torch.device('cuda')
v = workloads.sphere_views(n_lon, n_lat, H, W, B, dev, elevation=elev)
fvz, fvi, feats, nz = v['fvz'], v['fvi'].requires_grad_(True), v['feats'], v['normals_z']
g1 = torch.rand((B, H, W, feats.shape[-1]), device=dev)
g2 = torch.rand((B, H, W), device=dev)
ntx, nty = (W + 15) // 16, (H + 15) // 16
buf = torch.zeros(3 * B * ntx * nty, dtype=torch.int64, device=dev)
lib = _lib.load()
lib.kd_debug_buffer(buf.data_ptr())


def run():
    i, s, f = dibr_rasterization(H, W, fvz, fvi, feats, nz)
    torch.autograd.backward([i, s], [g1, g2])


extra = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for _ in range(3):
    run()
torch.cuda.synchronize()
_lib.debug_set(64 | extra)
run()
torch.cuda.synchronize()
_lib.debug_set(0)
lib.kd_debug_buffer(None)
t = buf.view(3, B, nty, ntx).cpu().numpy() / 100.0  # microseconds
for k, name in enumerate(['raster_fwd_pairs', 'soft_pairs', 'soft_bwd_pairs']):
    d = t[k].ravel()
    act = d[d > 2.0]
    hist = np.histogram(d[d > 0], bins=[0, 1, 2, 4, 8, 16, 32, 64, 128, 1e9])[0]
    print(f'{name}: histogram (us) <1:{hist[0]} 1-2:{hist[1]} 2-4:{hist[2]} 4-8:{hist[3]} '
          f'8-16:{hist[4]} 16-32:{hist[5]} 32-64:{hist[6]} 64-128:{hist[7]} >128:{hist[8]}')
    q = np.percentile(act, [50, 90, 99]) if len(act) else [0, 0, 0]
    print(f'{name:18s} tiles {d.size} active(>2us) {len(act)}  p50 {q[0]:.1f}  p90 {q[1]:.1f}  '
          f'p99 {q[2]:.1f}  max {d.max():.1f} us  sum {d.sum() / 1e3:.2f} ms')
    top = np.argsort(d)[::-1][:5]
    print('   slowest (view, ty, tx, us):',
          [(int(i // (nty * ntx)), int(i // ntx % nty), int(i % ntx), round(float(d[i]), 1))
           for i in top])
