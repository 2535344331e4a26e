"""Dispatch-slot timeline of the forward tile kernel (kd_dibr_fwd_tiles, or kd_soft_pairs with
debug flag 1<<26; kd_debug_set flag 64): when do the heavy tiles start and end, and (fused) how
long is each tile's raster phase?
python tools/soft_timeline.py [config] [extra debug flags] [tile split 1|2|4, default 1]"""
import os
os.environ.setdefault('KAOLIN_AMD_DIAG', '1')  # the diagnostic build (ablation flags)
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kaolin_amd import _lib, workloads  # noqa: E402
from kaolin_amd.render.mesh import dibr_rasterization  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'   # 'c3' or 'c3:1' (views override)
cfg, _, nv = cfg.partition(':')
n_lon, n_lat, H, W, B, elev = bench.CONFIGS[cfg]
B = int(nv) if nv else B
dev = torch.device('cuda')
v = workloads.sphere_views(n_lon, n_lat, H, W, B, dev, elevation=elev)
fvz, fvi, feats, nz = v['fvz'], v['fvi'].requires_grad_(True), v['feats'], v['normals_z']
ntx, nty = (W + 15) // 16, (H + 15) // 16
split = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n = B * ntx * nty * split  # dispatch slots (parts of tiles)
buf = torch.zeros(24 * n, dtype=torch.int64, device=dev)
extra = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
lib = _lib.load()
_lib.set_tile_split(split)
lib.kd_debug_buffer(buf.data_ptr())
for _ in range(3):
    dibr_rasterization(H, W, fvz, fvi, feats, nz)
torch.cuda.synchronize()
_lib.debug_set(64 | extra)
dibr_rasterization(H, W, fvz, fvi, feats, nz)
torch.cuda.synchronize()
_lib.debug_set(0)
lib.kd_debug_buffer(None)
t = buf.view(24, n).cpu().numpy()
dur = t[1] / 100.0          # us (100 MHz wall clock)
start = (t[2] - t[2].min()) / 100.0
end = start + dur
print(f'kernel span {end.max():.1f} us, tiles {n}, sum {dur.sum() / 1e3:.2f} ms')
if t[3].any():
    rdur = (t[3] - t[2]) / 100.0
    print(f'raster phase: sum {rdur.sum() / 1e3:.2f} ms, soft phase: sum '
          f'{(dur - rdur).sum() / 1e3:.2f} ms')
    for q in range(10):
        sl = slice(q * n // 10, (q + 1) * n // 10)
        print(f'  slots {sl.start:5d}: raster mean {rdur[sl].mean():6.1f} max {rdur[sl].max():6.1f}'
              f'   soft mean {(dur - rdur)[sl].mean():6.1f} max {(dur - rdur)[sl].max():6.1f}')
for q in range(10):
    sl = slice(q * n // 10, (q + 1) * n // 10)
    print(f'  slots {sl.start:5d}-{sl.stop:5d}: mean dur {dur[sl].mean():6.1f}  max dur '
          f'{dur[sl].max():6.1f}  start [{start[sl].min():6.1f}, {start[sl].max():6.1f}]  '
          f'max end {end[sl].max():6.1f}')
tile = t[0] & 0xffffffff
nbin = t[0] >> 32
_, _, fidx = dibr_rasterization(H, W, fvz, fvi, feats, nz)
unc = (fidx < 0).reshape(B, nty, 16, ntx, 16).sum(dim=(2, 4)).reshape(-1).cpu().numpy()
u_slot = unc[tile]
print('slot deciles: mean uncovered px / mean coarse count (soft bins)')
for q in range(10):
    sl = slice(q * n // 10, (q + 1) * n // 10)
    heavy = dur[sl] > 30
    print(f'  {sl.start:5d}: unc {u_slot[sl].mean():6.1f}  nbin {nbin[sl].mean():7.1f}  heavy '
          f'{heavy.sum():4d}  heavy unc {u_slot[sl][heavy].mean() if heavy.any() else 0:6.1f} '
          f'heavy nbin {nbin[sl][heavy].mean() if heavy.any() else 0:7.1f}')
if t[3].any():  # per-slot table for offline study: slot, tile, raster / soft bin counts, unc, us
    out = os.path.join('gpurun_out', f'timeline_{cfg}_{B}.csv')
    os.makedirs('gpurun_out', exist_ok=True)
    with open(out, 'w') as fh:
        fh.write('slot,tile,raster_nbin,soft_nbin,unc,start,raster_us,soft_us\n')
        for i in range(n):
            fh.write(f'{i},{tile[i]},{nbin[i]},{t[4][i]},{u_slot[i]},{start[i]:.2f},'
                     f'{rdur[i]:.2f},{dur[i] - rdur[i]:.2f}\n')
    print('wrote', out)
if t[5].any():  # soft phase split: pass A (walk + records), pair math, product (+ IoU)
    rend = t[3]
    pa = np.where(t[5] > 0, (t[5] - rend) / 100.0, 0)
    pm = np.where((t[6] > 0) & (t[5] > 0), (t[6] - t[5]) / 100.0, 0)
    # raster split: walk + tests (start -> t[7]) and the epilogue (t[7] -> t[3])
    rw = np.where(t[7] > 0, (t[7] - t[2]) / 100.0, 0)
    print('slowest tiles: slot | raster us (walk+tests epilogue) | soft: passA pairmath rest | '
          'soft_nbin unc | raster_nbin | view tx ty')
    for i in np.argsort(end)[::-1][:15]:
        tv = int(tile[i]) // (ntx * nty)
        tt = int(tile[i]) % (ntx * nty)
        print(f'  {i:5d} | {rdur[i]:6.1f} ({rw[i]:5.1f} {rdur[i] - rw[i]:5.1f}) | {pa[i]:6.1f} {pm[i]:6.1f} '
              f'{dur[i] - rdur[i] - pa[i] - pm[i]:6.1f} | {t[4][i]:5d} {u_slot[i]:4d} | '
              f'{nbin[i]:5d} | {tv} {tt % ntx} {tt // ntx}')
    print(f'sums (ms): passA {pa.sum() / 1e3:.2f} pairmath {pm.sum() / 1e3:.2f}')
    # raster pass A / B split of wave 0 (core clock cycles; diag CLK counters)
    print('raster wave 0 (kcycles): rows+transpose place passB dense | chunks pairs dense batches')
    for i in np.argsort(rdur)[::-1][:8]:
        c = t[8:16, i]
        print(f'  slot {i:5d} raster {rdur[i]:5.1f} us: {c[0] / 1e3:7.1f} {c[1] / 1e3:7.1f} '
              f'{c[2] / 1e3:7.1f} {c[3] / 1e3:7.1f} | {c[4]:4d} {c[5]:6d} {c[6]:4d} {c[7]:3d}')
    # soft pass A of wave 0 (core clock cycles; diag CLK counters)
    print('soft pass A wave 0 (kcycles): passA round write done | batches chunks faces records')
    for i in np.argsort(pa)[::-1][:10]:
        c = t[16:24, i]
        print(f'  slot {i:5d} passA {pa[i]:5.1f} us: {c[7] / 1e3:7.1f} {c[0] / 1e3:7.1f} '
              f'{c[1] / 1e3:7.1f} {c[2] / 1e3:7.1f} | {c[3]:3d} {c[4]:4d} {c[5]:5d} {c[6]:5d}')
late = np.argsort(end)[::-1][:10]
print('latest ending (slot, start, dur):', [(int(i), round(float(start[i]), 1),
                                            round(float(dur[i]), 1)) for i in late])
