"""Debug: forward outputs of the small-batch / balanced / per-wave tile forms against the oracle."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import oracle
from kaolin_amd import _lib, workloads
from kaolin_amd.render.mesh import dibr_rasterization

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c2'
n_lon, n_lat, h, B = {'c2': (100, 51, 256, 4), 'c3': (250, 101, 512, 1)}[cfg]
v = workloads.sphere_views(n_lon, n_lat, h, h, B, 'cuda')
fvz, fvi, feats, nz = v['fvz'], v['fvi'], v['feats'].contiguous(), v['normals_z']
N = lambda t: t.detach().cpu().numpy()
ri, rf, rw = oracle.rasterize(h, h, N(fvz), N(fvi), N(feats), N(nz) >= 0)
osoft = oracle.soft_mask_forward(N(fvi), rf)[0]
for name, fl in (('st', 0), ('tiles_bal', 1 << 27), ('tiles_wave', (1 << 27) | (1 << 28))):
    _lib.load().kd_debug_set(fl)
    i, s, f = dibr_rasterization(h, h, fvz, fvi, feats, nz)
    torch.cuda.synchronize()
    _lib.load().kd_debug_set(0)
    fi = N(f)
    bad_f = np.argwhere(fi != rf)
    bad_s = np.argwhere(np.abs(N(s) - osoft) > 1e-6)
    print(name, 'face_idx mismatches', len(bad_f), 'interp', int((N(i) != ri).any(-1).sum()),
          'soft', len(bad_s))
    for b_ in bad_f[:5]:
        print('   px', b_, 'got', fi[tuple(b_)], 'ref', rf[tuple(b_)])
    for b_ in bad_s[:5]:
        print('   soft px', b_, 'got', N(s)[tuple(b_)], 'ref', osoft[tuple(b_)])
