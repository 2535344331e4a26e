"""Ablation timings of the forward kernels (diagnostics; kd_debug_set flags)."""
import os
os.environ.setdefault('KAOLIN_AMD_DIAG', '1')  # the diagnostic build (ablation flags)
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
n_lon, n_lat, H, W, B, elev = bench.CONFIGS[cfg]
if len(sys.argv) > 3:
    B = int(sys.argv[3])
dev = torch.device('cuda')
v = workloads.sphere_views(n_lon, n_lat, H, W, B, dev, elevation=elev)
fvz, fvi, feats, nz = v['fvz'], v['fvi'].requires_grad_(True), v['feats'], v['normals_z']
g1 = torch.rand((B, H, W, feats.shape[-1]), device=dev)
g2 = torch.rand((B, H, W), device=dev)


def run():
    i, s, f = dibr_rasterization(H, W, fvz, fvi, feats, nz)
    torch.autograd.backward([i, s], [g1, g2])


for flags in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "4", "8", "0"])]:
    _lib.debug_set(flags)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    prof = _lib.profile_collect()
    print(f'flags={flags}: ' + '  '.join(f'{k.replace("kd_", "")}={ms * 1e3 / n:7.1f}us'
                                         for k, (ms, n) in sorted(prof.items())))
_lib.debug_set(0)
