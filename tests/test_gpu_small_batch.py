"""GPU: the small-batch forward of dibr_rasterization (kd_dibr_fwd_st: one workgroup per 8x8
quadrant over 16-pixel coarse bins, for B x 16x16 tiles <= 2048, enabled by debug flag 1 << 27;
measured no faster than the tile kernel at C3) against the tile kernel
(kd_dibr_fwd_tiles) and the oracle.

Bars: face_idx, weights, interpolated features and the soft mask bit-identical between the two
forms (the same per-pixel arithmetic; only the work split differs), gradients at the float
atomics' summation-order bar (rtol 1e-4, absolute floor 1e-5 x the largest magnitude); every
output and both gradients of the small-batch form against the oracle's brute-force loops.
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = 'cuda'
SMALL_BATCH = 1 << 27


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    yield
    _lib.load().kd_debug_set(0)


def N(t):
    return t.detach().cpu().numpy()


def _run(fvz, fvi0, feats0, nz, H, W, seed=1, flags=SMALL_BATCH, **kw):
    from kaolin_amd import _lib
    from kaolin_amd.render.mesh import dibr_rasterization
    _lib.load().kd_debug_set(flags)
    try:
        fvi = fvi0.clone().requires_grad_(True)
        feats = feats0.clone().requires_grad_(True)
        interp, soft, face_idx = dibr_rasterization(H, W, fvz, fvi, feats, nz, **kw)
        g = torch.Generator().manual_seed(seed)
        gi = torch.rand(interp.shape, generator=g, dtype=torch.float64).to(DEV, interp.dtype)
        gs = torch.rand(soft.shape, generator=g, dtype=torch.float64).to(DEV, soft.dtype)
        torch.autograd.backward([interp, soft], [gi, gs])
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
    'c3_1view': lambda: (_sphere(250, 101, 512, 512, 1, first_view=3, total_views=8), 512, 512),
    'c3_2views': lambda: (_sphere(250, 101, 512, 512, 2, first_view=6, total_views=8), 512, 512),
    'c2_4views': lambda: (_sphere(100, 51, 256, 256, 4), 256, 256),
    'pole_ragged': lambda: (_sphere(120, 40, 197, 251, 3, elevation=0.9), 197, 251),
    'soup_1view': lambda: (_soup(60000, 1), 512, 512),
    'tiny': lambda: (_sphere(12, 7, 9, 13, 2), 9, 13),
}


@pytest.mark.parametrize('case', sorted(CASES))
def test_small_batch_equals_tile_kernel(case):
    (fvz, fvi, feats, nz), H, W = CASES[case]()
    a = _run(fvz, fvi, feats, nz, H, W)
    b = _run(fvz, fvi, feats, nz, H, W, flags=0)
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    for x, y in zip(a[3:5], b[3:5]):
        scale = y.abs().max().item()
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * max(scale, 1e-30))


@pytest.mark.parametrize('case', ['c3_1view', 'pole_ragged', 'soup_1view'])
def test_small_batch_vs_oracle(case):
    (fvz, fvi, feats, nz), H, W = CASES[case]()
    interp, soft, face_idx, gfvi, gfeat, gi, gs = _run(fvz, fvi, feats, nz, H, W)
    ri, rf, rw = oracle.rasterize(H, W, N(fvz), N(fvi), N(feats), N(nz) >= 0)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), rf)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    gr, gfe = oracle.rasterize_backward(N(gi), rf, rw, N(fvi), N(feats), 1e-8)
    gsm = oracle.soft_mask_backward(N(gs), osoft, rf, oprob, ocidx, octype, sfvi, 7000., 1000.)
    ref = gr + gsm
    np.testing.assert_allclose(N(gfvi), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())
    np.testing.assert_allclose(N(gfeat), gfe, rtol=1e-4, atol=1e-5 * np.abs(gfe).max())


@pytest.mark.parametrize('limits', [(1.0, 0.3), (0.2, 1.0), (0.0, 0.0)])
def test_small_batch_pool_overflow(limits):
    """The overflow paths at a pool limit (quadrant entries of kd_soft_ovf_fwd / _bwd, bins walked
    in full): the same outputs as the unlimited run and the tile kernel's gradients."""
    from kaolin_amd import _lib
    (fvz, fvi, feats, nz), H, W = CASES['c3_1view']()
    ref = _run(fvz, fvi, feats, nz, H, W)
    _lib.set_pool_limits(*limits)
    try:
        a = _run(fvz, fvi, feats, nz, H, W)
    finally:
        _lib.set_pool_limits(1.0, 1.0)
    for x, y in zip(a[:3], ref[:3]):
        assert torch.equal(x, y)
    for x, y in zip(a[3:5], ref[3:5]):
        scale = y.abs().max().item()
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * scale)


def test_small_batch_knum_sweep():
    """knum 1, 7 and 32 (the fused bound) at the pole: first-K selection across the waves'
    chunks."""
    (fvz, fvi, feats, nz), H, W = CASES['pole_ragged']()
    for knum in (1, 7, 32):
        a = _run(fvz, fvi, feats, nz, H, W, knum=knum, boxlen=0.05)
        b = _run(fvz, fvi, feats, nz, H, W, flags=0, knum=knum, boxlen=0.05)
        for x, y in zip(a[:3], b[:3]):
            assert torch.equal(x, y), knum
