"""GPU parity breadth: whole images, every view of a batch.

- all 8 views of the C3 bench batch (50k-face uv-sphere, 512x512, knum 30), rendered in the one
  batched call the bench makes: face_idx / interpolated features bit-exact, soft mask at 1e-6,
  both gradients at the float atomics' bar, per view against the oracle's brute-force loops
  (oracle/dibr_oracle.c, the reference's per-pixel loops: rasterization_cuda.cu:62-171,
  dibr_soft_mask_cuda.cu:27-353);
- the C4 sigma / boxlen pairs (7000, 0.02) and (17000, 0.02) on one whole 1024x1024 view,
  forward and backward (the row tests of test_gpu_parity.py cover the other pairs' rows);
- one whole C3 view in fp64 (the benched size; the fp64 tile kernels' LDS layouts and term passes
  differ from fp32): face_idx / features bit-exact, soft mask at 1e-12, gradients at 1e-9, also
  with both pools limited (every overflow path: bins walking their view, tiles without records).
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def N(t):
    return t.detach().cpu().numpy()


def _fwd_bwd(h, w, v, sigmainv=7000., boxlen=0.02):
    dt = v['fvi'].dtype
    from kaolin_amd.render.mesh import dibr_rasterization
    fvz, feats, nz = v['fvz'], v['feats'].contiguous().clone(), v['normals_z']
    fvi = v['fvi'].detach().clone().requires_grad_(True)
    feats.requires_grad_(True)
    interp, soft, face_idx = dibr_rasterization(h, w, fvz, fvi, feats, nz, sigmainv, boxlen)
    g = torch.Generator().manual_seed(7)
    g_feat = torch.rand(interp.shape, generator=g).to(DEV, dt)
    g_soft = torch.rand(soft.shape, generator=g).to(DEV, dt)
    torch.autograd.backward([interp, soft], [g_feat, g_soft])
    torch.cuda.synchronize()
    return fvz, fvi, feats, nz, interp, soft, face_idx, g_feat, g_soft


def _check_view(h, w, b, out, sigmainv=7000., boxlen=0.02):
    fvz, fvi, feats, nz, interp, soft, face_idx, g_feat, g_soft = out
    f64 = fvi.dtype == torch.float64
    stol = 1e-12 if f64 else 1e-6  # device exp against glibc's
    gtol = 1e-9 if f64 else 1e-4   # float atomics' summation order
    s = slice(b, b + 1)
    valid = N(nz[s]) >= 0
    ri, rf, rw = oracle.rasterize(h, w, N(fvz[s]), N(fvi[s]), N(feats[s]), valid)
    np.testing.assert_array_equal(N(face_idx[s]), rf)
    np.testing.assert_array_equal(N(interp[s]), ri)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi[s]), rf, sigmainv, boxlen)
    np.testing.assert_allclose(N(soft[s]), osoft, rtol=stol, atol=stol * 0.1)
    gr, gfeat = oracle.rasterize_backward(N(g_feat[s]), rf, rw, N(fvi[s]), N(feats[s]), 1e-8)
    gs = oracle.soft_mask_backward(N(g_soft[s]), osoft, rf, oprob, ocidx, octype, sfvi, sigmainv,
                                   1000.)
    ref = gr + gs
    np.testing.assert_allclose(N(fvi.grad[s]), ref, rtol=gtol,
                               atol=gtol * 0.1 * np.abs(ref).max())
    np.testing.assert_allclose(N(feats.grad[s]), gfeat, rtol=gtol,
                               atol=gtol * 0.1 * np.abs(gfeat).max())


def test_c3_all_views_full_fwd_bwd_vs_oracle():
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, 8, DEV)
    out = _fwd_bwd(h, w, v)
    for b in range(8):
        _check_view(h, w, b, out)


@pytest.mark.parametrize('sweep', [(7000., 0.02), (17000., 0.02)])
def test_c4_view_full_fwd_bwd_vs_oracle(sweep):
    from kaolin_amd import workloads
    sig, box = sweep
    h = w = 1024
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, first_view=5, total_views=8)
    out = _fwd_bwd(h, w, v, sig, box)
    _check_view(h, w, 0, out, sig, box)


@pytest.mark.parametrize('limits', [(1.0, 1.0), (0.3, 0.05)])
def test_c3_view_full_fwd_bwd_f64_vs_oracle(limits):
    """One whole C3 view (50k faces, 512x512, knum 30) in fp64 through dibr_rasterization fwd +
    bwd against the oracle; (0.3, 0.05) limits both pools (kd_set_pool_limits)."""
    from kaolin_amd import _lib, workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, dtype=torch.float64, first_view=6,
                               total_views=8)
    _lib.set_pool_limits(*limits)
    try:
        out = _fwd_bwd(h, w, v)
    finally:
        _lib.set_pool_limits(1.0, 1.0)
    _check_view(h, w, 0, out)


def test_tiny_face_soup_single_record_runs_vs_oracle():
    """Thousands of tiny scattered faces on a mostly empty image: a face is close to one or two
    uncovered pixels, so most soft-backward runs are a single record and a wave's 64 lanes are
    often all run ends -- the row-repacked atomics' case with no spare lane for the push
    (kd_softpair.hip soft_bwd_items_body) -- forward and backward against the oracle."""
    g = torch.Generator().manual_seed(21)
    F, h, w = 4000, 96, 96
    centre = torch.rand((1, F, 1, 2), generator=g) * 2 - 1
    offs = (torch.rand((1, F, 3, 2), generator=g) - 0.5) * 0.03  # about one pixel across
    v = dict(fvi=(centre + offs).to(DEV),
             fvz=(-1 - torch.rand((1, F, 3), generator=g)).to(DEV),
             feats=torch.rand((1, F, 3, 3), generator=g).to(DEV),
             normals_z=torch.ones((1, F), device=DEV))
    out = _fwd_bwd(h, w, v)
    assert (out[5] < 1).any() and (out[6] >= 0).any()
    _check_view(h, w, 0, out)
