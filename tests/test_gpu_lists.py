"""GPU: the reference-structured close-face lists (the (B, H, W, K) prob / idx / type tensors of
dibr_soft_mask_forward_cuda, dibr_soft_mask.cpp:86-107, and DibrSoftMaskCuda's saved tensors,
dibr.py:40-54) as written row-coalesced by kd_soft_lists, and the op-form backward over given lists
(kd_soft_bwd_lists, dibr_soft_mask_cuda.cu:230-353) -- against the oracle.

Bars: close_face_idx and close_face_dist_type bit-exact (including the -1 / 0 / 0 padding),
probabilities and soft mask rtol 1e-6, gradients rtol 1e-4 (fp32, atomic summation order) with an
absolute floor of 1e-5 x the largest magnitude; 1e-9 in fp64.
"""
import numpy as np
import pytest
import torch

import oracle
from helpers import TORCH_DTYPES

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    yield
    _lib.load().kd_debug_set(0)


def N(t):
    return t.detach().cpu().numpy()


def _view(n_lon, n_lat, h, B, dt, elevation=0.3):
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import rasterize
    v = workloads.sphere_views(n_lon, n_lat, h, h, B, DEV, dtype=dt, elevation=elevation)
    _, face_idx = rasterize(h, h, v['fvz'], v['fvi'], v['feats'], v['normals_z'] >= 0)
    return v['fvi'].contiguous(), face_idx


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('knum', [30, 40, 70])
def test_lists_vs_oracle(dname, knum):
    """Whole views (C2 mesh, 256x256, 2 views, the pole in view): every list element, padding
    included; knum 40 and 70 take several 32-slot passes."""
    from kaolin_amd import _C
    dt = TORCH_DTYPES[dname]
    fvi, face_idx = _view(100, 51, 256, 2, dt, elevation=0.7)
    sig, box = 7000., 0.03
    soft, _, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_fused(
        fvi, face_idx, sig, box, knum, 1000., with_lists=True, want_grad=False)
    osoft, oprob, ocidx, octype, _ = oracle.soft_mask_forward(N(fvi), N(face_idx), sig, box, knum)
    np.testing.assert_array_equal(N(cidx), ocidx)
    np.testing.assert_array_equal(N(ctype), octype)
    np.testing.assert_allclose(N(prob), oprob, rtol=1e-6, atol=1e-37)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    assert (ocidx[..., knum - 1] >= 0).any()  # some rows are full


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('knum', [30, 40])
def test_op_backward_on_lists_with_holes(dname, knum):
    """The op backward reads given lists and stops at a row's first -1, whatever follows it
    (dibr_soft_mask_cuda.cu:273-276): rows with a -1 punched into slot 3 must drop their later
    entries."""
    from kaolin_amd import _C, _lib
    dt = TORCH_DTYPES[dname]
    fvi, face_idx = _view(100, 51, 256, 2, dt, elevation=0.7)
    sig, box, M = 7000., 0.03, 1000.
    soft, _, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_fused(
        fvi, face_idx, sig, box, knum, M, with_lists=True, want_grad=False)
    holes = cidx.clone()
    rows = holes[..., 5] >= 0
    holes[..., 3][rows & (torch.arange(rows.numel(), device=DEV).reshape(rows.shape) % 3 == 0)] = -1
    g = torch.Generator().manual_seed(5)
    gs = torch.rand(soft.shape, generator=g, dtype=torch.float64).to(DEV, dt)
    sfvi = (fvi * M).contiguous()
    osoft, oprob, _, octype, osfvi = oracle.soft_mask_forward(N(fvi), N(face_idx), sig, box, knum)
    ref = oracle.soft_mask_backward(N(gs), N(soft), N(face_idx), N(prob), N(holes), N(ctype),
                                    N(sfvi), sig, M)
    tol = 1e-4 if dname == 'f32' else 1e-9
    gop = _C.render.mesh.dibr_soft_mask_backward_cuda(gs, soft, face_idx, prob, holes, ctype,
                                                      sfvi, sig, M)
    torch.cuda.synchronize()
    np.testing.assert_allclose(N(gop), ref, rtol=tol, atol=tol * 0.1 * np.abs(ref).max())


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('knum', [30, 40])
def test_fused_forward_lists_vs_oracle(dname, knum):
    """kd_dibr_rasterization_forward_lists (dibr_rasterization inside close_lists()): the one
    binning pass and one launch of the fused forward, then the lists writer -- the lists and soft
    mask against the oracle, bit-exact indices / types, and the raster outputs equal to the op
    form's (rasterize)."""
    from kaolin_amd import _C, workloads
    from kaolin_amd.render.mesh import rasterize
    dt = TORCH_DTYPES[dname]
    v = workloads.sphere_views(100, 51, 256, 256, 2, DEV, dtype=dt, elevation=0.7)
    sig, box, M = 7000., 0.03, 1000.
    interp, face_idx, weights, soft, _, prob, cidx, ctype = \
        _C.render.mesh.dibr_rasterization_forward_fused(
            256, 256, v['fvz'], v['fvi'], v['feats'], v['normals_z'], sig, box, knum, M, 1e-8,
            want_grad=False, with_lists=True)
    ri, rf = rasterize(256, 256, v['fvz'], v['fvi'], v['feats'], v['normals_z'] >= 0)
    np.testing.assert_array_equal(N(face_idx), N(rf))
    np.testing.assert_array_equal(N(interp), N(ri))
    osoft, oprob, ocidx, octype, _ = oracle.soft_mask_forward(N(v['fvi']), N(face_idx), sig, box,
                                                              knum)
    np.testing.assert_array_equal(N(cidx), ocidx)
    np.testing.assert_array_equal(N(ctype), octype)
    np.testing.assert_allclose(N(prob), oprob, rtol=1e-6, atol=1e-37)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_close_lists_fused_matches_composition(dname):
    """dibr_rasterization inside close_lists(): the fused forward with lists
    (DibrRasterizationListsHip) against the reference composition (rasterize + dibr_soft_mask):
    equal outputs, and gradients equal up to the lists backward's atomic summation order."""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr, dibr_rasterization
    from kaolin_amd.render.mesh.dibr import close_lists
    dt = TORCH_DTYPES[dname]
    v = workloads.sphere_views(100, 51, 192, 192, 2, DEV, dtype=dt, elevation=0.5)
    g = torch.Generator().manual_seed(3)
    gi = torch.rand((2, 192, 192, v['feats'].shape[-1]), generator=g, dtype=torch.float64)
    gsft = torch.rand((2, 192, 192), generator=g, dtype=torch.float64)
    out = {}
    try:
        for fused in (True, False):
            dibr.LISTS_FUSED = fused
            fvi = v['fvi'].detach().clone().requires_grad_(True)
            feat = v['feats'].detach().clone().requires_grad_(True)
            with close_lists():
                interp, soft, fidx = dibr_rasterization(192, 192, v['fvz'], fvi, feat,
                                                        v['normals_z'], 7000., 0.02, 30)
            torch.autograd.backward([interp, soft], [gi.to(DEV, dt), gsft.to(DEV, dt)])
            out[fused] = [N(t) for t in (interp, soft, fidx, fvi.grad, feat.grad)]
    finally:
        dibr.LISTS_FUSED = True
    for a, b in zip(out[True][:3], out[False][:3]):
        np.testing.assert_array_equal(a, b)
    tol = 1e-4 if dname == 'f32' else 1e-9
    for a, b in zip(out[True][3:], out[False][3:]):
        np.testing.assert_allclose(a, b, rtol=tol, atol=tol * 0.1 * np.abs(b).max())


def test_op_backward_soft_zero_rows_keep_their_terms():
    """soft == 0 only says that every 1 - prob rounded to 1; with boxlen 0.05 and
    sigmainv 30000 many rows hold probabilities of ~1e-30..3e-8 under a soft mask of exactly 0,
    and their terms dLdz * geometry (dibr_soft_mask_cuda.cu:283-348) are nonzero.  The incoming
    gradient is nonzero on those pixels only, so a backward that skipped them would return 0."""
    from kaolin_amd import _C
    fvi, face_idx = _view(100, 51, 256, 2, torch.float32, elevation=0.7)
    sig, box, K, M = 30000., 0.05, 30, 1000.
    soft, _, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_fused(
        fvi, face_idx, sig, box, K, M, with_lists=True, want_grad=False)
    zero_rows = (soft == 0) & (prob[..., 0] > 0) & (face_idx < 0)
    assert int(zero_rows.sum()) > 100, 'the case needs soft == 0 rows with probabilities'
    gs = zero_rows.to(torch.float32)
    sfvi = (fvi * M).contiguous()
    ref = oracle.soft_mask_backward(N(gs), N(soft), N(face_idx), N(prob), N(cidx), N(ctype),
                                    N(sfvi), sig, M)
    gop = _C.render.mesh.dibr_soft_mask_backward_cuda(gs, soft, face_idx, prob, cidx, ctype,
                                                      sfvi, sig, M)
    torch.cuda.synchronize()
    assert np.abs(ref).max() > 0
    np.testing.assert_allclose(N(gop), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


def test_fused_lists_backward_keeps_soft_zero_rows():
    """The fused lists path's backward skips only the rows without listed faces (the forward's
    row lengths; kd_dibr_rasterization_soft_backward_lists): on soft == 0 rows with
    probabilities (boxlen 0.05, sigmainv 30000) its gradient equals the op-form backward's,
    which reads every row."""
    from kaolin_amd import _C, workloads
    v = workloads.sphere_views(100, 51, 256, 256, 2, DEV, elevation=0.7)
    sig, box, K, M = 30000., 0.05, 30, 1000.
    out = _C.render.mesh.dibr_rasterization_forward_fused(
        256, 256, v['fvz'], v['fvi'], v['feats'], v['normals_z'], sig, box, K, M, 1e-8,
        want_grad=False, with_lists=True)
    _, face_idx, _, soft, ws, prob, cidx, ctype = out
    zero_rows = (soft == 0) & (prob[..., 0] > 0) & (face_idx < 0)
    assert int(zero_rows.sum()) > 100
    g = torch.Generator().manual_seed(11)
    gs = torch.rand(soft.shape, generator=g).to(DEV) * (zero_rows | (soft < 1)).float()
    sfvi = (v['fvi'] * M).contiguous()
    ref = _C.render.mesh.dibr_soft_mask_backward_cuda(gs, soft, face_idx, prob, cidx, ctype, sfvi,
                                                      sig, M)
    new = _C.render.mesh.dibr_soft_mask_backward_lists_ws(gs, soft, face_idx, prob, cidx, ctype,
                                                          sfvi, sig, M, ws)
    torch.cuda.synchronize()
    np.testing.assert_allclose(N(new), N(ref), rtol=1e-4, atol=1e-5 * N(ref).__abs__().max())
    # and on the soft == 0 rows alone
    gz = zero_rows.float()
    ref = _C.render.mesh.dibr_soft_mask_backward_cuda(gz, soft, face_idx, prob, cidx, ctype, sfvi,
                                                      sig, M)
    new = _C.render.mesh.dibr_soft_mask_backward_lists_ws(gz, soft, face_idx, prob, cidx, ctype,
                                                          sfvi, sig, M, ws)
    torch.cuda.synchronize()
    assert N(ref).__abs__().max() > 0
    np.testing.assert_allclose(N(new), N(ref), rtol=1e-4, atol=1e-5 * N(ref).__abs__().max())
