"""GPU: the fused fp32 forward with helper workgroups (kd_dibr_fwd_help, kd_soft.hpp HelpJob:
silhouette tiles with more than 1024 records publish their pair math in 512-record chunks, claimed
by the owner and by helper workgroups launched after the tiles, on the owner's XCD; opt-in, debug
flag 256 -- measured slower) against the plain tile kernel and the oracle.

Bars: face_idx, weights, interpolated features and the soft mask bit-identical with and without
helpers (the same per-record arithmetic; only which workgroup runs a chunk differs), gradients at
the float atomics' summation-order bar (rtol 1e-4, absolute floor 1e-5 x the largest magnitude);
one view of C3 and a dense soup against the oracle's brute-force loops.  The soup cases at boxlen
0.1 publish more jobs than the job table / FIFO hold (the owner-only fallbacks).
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = 'cuda'
HELPERS = 256
OWNERS_ONLY = 512  # the helped kernel without helper workgroups


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    yield
    _lib.load().kd_debug_set(0)


def N(t):
    return t.detach().cpu().numpy()


def _run(fvz, fvi0, feats0, nz, H, W, flags=0, seed=1, gt=None, **kw):
    from kaolin_amd import _lib
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_rasterization_with_mask_iou
    _lib.load().kd_debug_set(flags)
    try:
        fvi = fvi0.clone().requires_grad_(True)
        feats = feats0.clone().requires_grad_(True)
        g = torch.Generator().manual_seed(seed)
        if gt is None:
            interp, soft, face_idx = dibr_rasterization(H, W, fvz, fvi, feats, nz, **kw)
            gi = torch.rand(interp.shape, generator=g, dtype=torch.float64).to(DEV, interp.dtype)
            gs = torch.rand(soft.shape, generator=g, dtype=torch.float64).to(DEV, soft.dtype)
            torch.autograd.backward([interp, soft], [gi, gs])
        else:
            interp, soft, face_idx, loss = dibr_rasterization_with_mask_iou(
                H, W, fvz, fvi, feats, nz, gt, **kw)
            gi = torch.rand(interp.shape, generator=g, dtype=torch.float64).to(DEV, interp.dtype)
            gs = None
            torch.autograd.backward([interp, loss], [gi, torch.ones_like(loss)])
        torch.cuda.synchronize()
        return interp, soft, face_idx, fvi.grad, feats.grad, gi, gs
    finally:
        _lib.load().kd_debug_set(0)


def _sphere(n_lon, n_lat, H, W, B, elevation=0.3, first_view=0, total_views=None):
    from kaolin_amd import workloads
    v = workloads.sphere_views(n_lon, n_lat, H, W, B, DEV, elevation=elevation,
                               first_view=first_view, total_views=total_views)
    return v['fvz'], v['fvi'].detach(), v['feats'].contiguous(), v['normals_z']


def _soup(F, B, seed=3):
    from kaolin_amd import workloads
    fvz, fvi, nz = workloads.soup(F, seed=seed, batch=B)
    g = torch.Generator().manual_seed(4)
    uvs = torch.rand((B, F, 3, 2), generator=g)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1)
    return fvz.to(DEV), fvi.to(DEV), feats.to(DEV), nz.to(DEV)


CASES = {
    'c3_1view': lambda: (_sphere(250, 101, 512, 512, 1), 512, 512, {}),
    'c3_2views': lambda: (_sphere(250, 101, 512, 512, 2, first_view=6, total_views=8), 512,
                          512, {}),
    'c3_8views': lambda: (_sphere(250, 101, 512, 512, 8), 512, 512, {}),
    'c3_1view_k32_wide': lambda: (_sphere(250, 101, 512, 512, 1), 512, 512,
                                  {'knum': 32, 'boxlen': 0.05}),
    'soup_1view_wide': lambda: (_soup(60000, 1), 512, 512, {'boxlen': 0.1}),
    'soup_4views_wide': lambda: (_soup(60000, 4), 512, 512, {'boxlen': 0.1}),
    'pole_ragged': lambda: (_sphere(120, 40, 197, 251, 3, elevation=0.9), 197, 251,
                            {'boxlen': 0.05}),
}


def _same(a, b):
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    for x, y in zip(a[3:5], b[3:5]):
        scale = y.abs().max().item()
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * max(scale, 1e-30))


@pytest.mark.parametrize('case', sorted(CASES))
def test_helpers_equal_tile_kernel(case):
    (fvz, fvi, feats, nz), H, W, kw = CASES[case]()
    a = _run(fvz, fvi, feats, nz, H, W, flags=HELPERS, **kw)
    b = _run(fvz, fvi, feats, nz, H, W, **kw)
    _same(a, b)
    _same(_run(fvz, fvi, feats, nz, H, W, flags=OWNERS_ONLY, **kw), b)


def test_helpers_repeatable():
    """Back-to-back forwards reuse the job table and FIFO (zeroed by the binning each call)."""
    (fvz, fvi, feats, nz), H, W, kw = CASES['c3_1view']()
    ref = _run(fvz, fvi, feats, nz, H, W)
    for _ in range(3):
        _same(_run(fvz, fvi, feats, nz, H, W, flags=HELPERS), ref)


def test_helpers_fused_iou():
    """mask_iou fused into the forward: the per-tile IoU terms of helped tiles."""
    (fvz, fvi, feats, nz), H, W, kw = CASES['c3_2views']()
    B = fvz.shape[0]
    yy, xx = torch.meshgrid(torch.arange(H, device=DEV), torch.arange(W, device=DEV),
                            indexing='ij')
    gt = (((xx - W / 2) ** 2 + (yy - H / 2) ** 2) < (0.3 * W) ** 2).float()
    gt = gt.expand(B, H, W).contiguous()
    a = _run(fvz, fvi, feats, nz, H, W, flags=HELPERS, gt=gt)
    b = _run(fvz, fvi, feats, nz, H, W, gt=gt)
    _same(a, b)


@pytest.mark.parametrize('case', ['c3_1view', 'soup_1view_wide'])
def test_helpers_vs_oracle(case):
    (fvz, fvi, feats, nz), H, W, kw = CASES[case]()
    boxlen = kw.get('boxlen', 0.02)
    interp, soft, face_idx, gfvi, gfeat, gi, gs = _run(fvz, fvi, feats, nz, H, W, flags=HELPERS,
                                                       **kw)
    ri, rf, rw = oracle.rasterize(H, W, N(fvz), N(fvi), N(feats), N(nz) >= 0)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), rf, boxlen=boxlen)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    gr, gfe = oracle.rasterize_backward(N(gi), rf, rw, N(fvi), N(feats), 1e-8)
    gsm = oracle.soft_mask_backward(N(gs), osoft, rf, oprob, ocidx, octype, sfvi, 7000., 1000.)
    ref = gr + gsm
    np.testing.assert_allclose(N(gfvi), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())
    np.testing.assert_allclose(N(gfeat), gfe, rtol=1e-4, atol=1e-5 * np.abs(gfe).max())
