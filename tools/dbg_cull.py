import sys, zlib, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import oracle
from test_gpu_parity import _cull_soup
from kaolin_amd import _lib
from kaolin_amd.render.mesh import rasterize
kind, multiplier, eps = 'grid', -1000, 1e-8
rng = np.random.default_rng(zlib.crc32(f'{kind}/{multiplier}/{eps}'.encode()))
h, w = 45, 53
fvi = _cull_soup(kind, rng, h, w); Fn = fvi.shape[1]
fvz = (-1 - rng.uniform(0, 1, (1, Fn, 3))).astype(np.float32)
fvz = np.round(fvz, 1).astype(np.float32)
feat = rng.random((1, Fn, 3, 2)).astype(np.float32)
ri, rf, rw = oracle.rasterize(h, w, fvz, fvi, feat, None, multiplier=multiplier, eps=eps)
for flags in (0, 8):
    _lib.load().kd_debug_set(flags)
    interp, fi = rasterize(h, w, torch.tensor(fvz).cuda(), torch.tensor(fvi).cuda(), torch.tensor(feat).cuda(), multiplier=multiplier, eps=eps)
    fi = fi.cpu().numpy()
    bad = np.argwhere(fi != rf)
    print('flags', flags, 'mismatch', len(bad))
    for b in bad[:6]:
        print(b, 'gpu', fi[tuple(b)], 'oracle', rf[tuple(b)])
# f64 path
interp, fi = rasterize(h, w, torch.tensor(fvz).double().cuda(), torch.tensor(fvi).double().cuda(), torch.tensor(feat).double().cuda(), multiplier=multiplier, eps=eps)
ri2, rf2, _ = oracle.rasterize(h, w, fvz.astype(np.float64), fvi.astype(np.float64), feat.astype(np.float64), None, multiplier=multiplier, eps=eps)
print('f64 mismatch', (fi.cpu().numpy() != rf2).sum())
