import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import load_golden
from helpers import sphere
from kaolin_amd.render.mesh import dibr_rasterization, dibr_soft_mask, rasterize
import oracle
s = sphere(load_golden('sphere_inputs.npz'), 'f32', 0)
T = lambda a: torch.as_tensor(a).cuda()
fvz, fvi, uvs, nz = T(s['fvz']), T(s['fvi']), T(s['uvs']), T(s['normals_z'])
H, W = 35, 31
gi, gf = rasterize(H, W, fvz, fvi, uvs, nz >= 0., 1000)
gs = dibr_soft_mask(fvi, gf, 7000, 0.02, 30, 1000)
gs2 = dibr_soft_mask(fvi, gf, 7000, 0.02, 30, 1000)
i, sm, f = dibr_rasterization(H, W, fvz, fvi, uvs, nz, 7000, 0.02, 30, 1000)
i2, sm2, f2 = dibr_rasterization(H, W, fvz, fvi, uvs, nz, 7000, 0.02, 30, 1000)
osoft = oracle.soft_mask_forward(s['fvi'], gf.cpu().numpy())[0]
for name, t in (('gs', gs), ('gs2', gs2), ('sm', sm), ('sm2', sm2)):
    d = np.abs(t.cpu().numpy() - osoft)
    print(name, 'max diff vs oracle', d.max(), 'n>1e-6', (d > 1e-6).sum(), np.argwhere(d > 1e-6)[:5].tolist())
from kaolin_amd import _lib
_lib.load().kd_debug_set(32768)
i, sm, f = dibr_rasterization(H, W, fvz, fvi, uvs, nz, 7000, 0.02, 30, 1000)
d = np.abs(sm.cpu().numpy() - osoft)
print('separate reduce: max diff', d.max(), (d > 1e-6).sum())
_lib.load().kd_debug_set(0)
fg = fvi.clone().requires_grad_(True)
gsg = dibr_soft_mask(fg, gf, 7000, 0.02, 30, 1000)
d = np.abs(gsg.detach().cpu().numpy() - osoft)
print('standalone grad path: max diff', d.max(), (d > 1e-6).sum())
i, smg, f = dibr_rasterization(H, W, fvz, fg, uvs, nz, 7000, 0.02, 30, 1000)
d = np.abs(smg.detach().cpu().numpy() - osoft)
print('dibr grad path: max diff', d.max(), (d > 1e-6).sum())
_, prob, cidx, ctype, _ = oracle.soft_mask_forward(s['fvi'], gf.cpu().numpy())
npx = (cidx >= 0).sum(-1)
bad = np.abs(sm.cpu().numpy() - osoft) > 1e-6
print('np of bad pixels', np.bincount(npx[bad])); print('np of all uncovered-with-faces', np.bincount(npx[(npx > 0)]))
print('sm bad', sm.cpu().numpy()[bad][:12]); print('oracle', osoft[bad][:12])
print('gs bad', gs.cpu().numpy()[bad][:12])
