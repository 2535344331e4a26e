"""Diagnostics: coarse-bin occupancy and per-kernel times for a bench config (GPU)."""
import math, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kaolin_amd import _lib, workloads
from kaolin_amd import _C

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
import bench
n_lon, n_lat, H, W, B, elev = bench.CONFIGS[cfg]
dev = torch.device('cuda')
v = workloads.sphere_views(n_lon, n_lat, H, W, B, dev, elevation=elev)
fvz, fvi, feats, nz = v['fvz'], v['fvi'], v['feats'], v['normals_z']
F = fvz.shape[1]
valid = (nz >= 0).contiguous().view(torch.uint8)
nb = _lib.workspace_size(_lib.KD_WS_RASTER, B, H, W, B * F, F)
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
interp = torch.empty((B, H, W, feats.shape[-1]), device=dev)
fidx = torch.empty((B, H, W), device=dev, dtype=torch.long)
wts = torch.empty((B, H, W, 3), device=dev)
s = torch.cuda.current_stream().cuda_stream
def run():
    _lib.call('kd_rasterize_forward_f32', B, H, W, F, feats.shape[-1], fvz.data_ptr(), fvi.data_ptr(),
              feats.data_ptr(), valid.data_ptr(), 1000.0, 1e-8, interp.data_ptr(), fidx.data_ptr(),
              wts.data_ptr(), ws.data_ptr(), nb, s)
run(); torch.cuda.synchronize()
# layout: spans [N] (8B), counts [B][nchunk][nct], totals [B][nct]
N = B * F
def al(x): return (x + 255) // 256 * 256
ct = 64
while (max(H, W) + ct - 1) // ct > 32: ct *= 2
nct = ((W + ct - 1) // ct) * ((H + ct - 1) // ct)
nchunk = (F + 255) // 256
off = al(8 * N) + al(4 * B * nchunk * nct)
totals = ws[off: off + 4 * B * nct].view(torch.int32).reshape(B, nct)
print('raster bins: ctile', ct, 'nct', nct, 'totals mean/max', totals.float().mean().item(), totals.max().item())
spans = ws[:8 * N].view(torch.int16).reshape(N, 4).int()
w_ = (spans[:, 1] - spans[:, 0] + 1).clamp(min=0); h_ = (spans[:, 3] - spans[:, 2] + 1).clamp(min=0)
area = (w_ * h_).float()
print('raster spans: mean w %.2f h %.2f area %.1f max area %d nonempty %d' % (w_[area>0].float().mean(), h_[area>0].float().mean(), area[area>0].mean(), area.max(), (area>0).sum()))
_lib.profile_enable(True)
for _ in range(5): run()
torch.cuda.synchronize(); _lib.profile_enable(False)
for k, (ms, n) in _lib.profile_collect().items(): print(f'{k:24s} {ms*1e3/n:9.1f} us')
# exact spans by brute force for a sample of faces of view 0 (float32 centres like the kernel)
M = torch.tensor(1000.0, dtype=torch.float32)
ws_ = torch.arange(W, device=dev, dtype=torch.float32)
hs_ = torch.arange(H, device=dev, dtype=torch.float32)
cx = (M / W) * (2 * ws_ + 1 - W)
cy = (M / H) * (H - 2 * hs_ - 1)
sfvi = fvi[0] * 1000.0
bmin = sfvi.min(dim=1)[0]; bmax = sfvi.max(dim=1)[0]
bad = 0
for f in range(0, F, 97):
    if not bool(valid[0, f]): continue
    xs = torch.nonzero((cx >= bmin[f, 0]) & (cx < bmax[f, 0])).flatten()
    ys = torch.nonzero((cy >= bmin[f, 1]) & (cy < bmax[f, 1])).flatten()
    sp = spans[f].tolist()
    ex = [xs.min().item(), xs.max().item()] if len(xs) else None
    ey = [ys.min().item(), ys.max().item()] if len(ys) else None
    if ex is None or ey is None:
        if sp[0] <= sp[1] and sp[2] <= sp[3]: bad += 1
        continue
    if sp != ex + ey:
        bad += 1
        if bad < 6: print('face', f, 'kernel', sp, 'exact', ex + ey, 'box', bmin[f].tolist(), bmax[f].tolist())
print('span mismatches', bad)
