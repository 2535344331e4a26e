"""GPU: the autograd contract of dibr_soft_mask / dibr_rasterization and whole-image gradient
parity at the SURVEY §8(d) configs C2, C4 and C5.

- A second backward over a retained graph (``retain_graph=True``, ``torch.autograd.grad`` twice)
  must give the same gradients as the first: the reference keeps its K-lists in
  ``save_for_backward`` (kaolin/render/mesh/dibr.py:51-54), so its backward is repeatable.
- Non-contiguous inputs (an expanded feature tensor, a permuted face_vertices_image) must give
  the same outputs and gradients as their contiguous copies.
- C2 / C4 / C5: every output and both gradients of whole images against the oracle's brute-force
  loops (oracle/dibr_oracle.c), at the bars of test_gpu_parity.py (integer outputs and
  interpolated features bit-exact, soft mask 1e-6, gradients rtol 1e-4 with an absolute floor of
  1e-5 x the gradient's largest magnitude).
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


def N(t):
    return t.detach().cpu().numpy()


def _views(n_lon, n_lat, h, B, dt=torch.float32, elevation=0.3, first_view=0, total_views=None,
           seed=0):
    from kaolin_amd import workloads
    v = workloads.sphere_views(n_lon, n_lat, h, h, B, DEV, dtype=dt, seed=seed,
                               elevation=elevation, first_view=first_view,
                               total_views=total_views)
    return v['fvz'], v['fvi'].detach(), v['feats'].contiguous(), v['normals_z']


def _grads(shape_feat, shape_soft, dt, seed=1):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape_feat, generator=g, dtype=torch.float64).to(DEV, dt),
            torch.rand(shape_soft, generator=g, dtype=torch.float64).to(DEV, dt))


# --------------------------------------------------------------------------------------------
# retained graph
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_dibr_rasterization_retained_graph_twice(dname):
    from kaolin_amd.render.mesh import dibr_rasterization
    dt = TORCH_DTYPES[dname]
    h = 96
    fvz, fvi0, feats0, nz = _views(40, 21, h, 2, dt, elevation=0.5)
    fvi = fvi0.clone().requires_grad_(True)
    feats = feats0.clone().requires_grad_(True)
    interp, soft, face_idx = dibr_rasterization(h, h, fvz, fvi, feats, nz)
    g1, g2 = _grads(interp.shape, soft.shape, dt)
    a = torch.autograd.grad([interp, soft], [fvi, feats], [g1, g2], retain_graph=True)
    b = torch.autograd.grad([interp, soft], [fvi, feats], [g1, g2], retain_graph=True)
    # backward() twice accumulates: 2x the single gradient
    torch.autograd.backward([interp, soft], [g1, g2], retain_graph=True)
    torch.autograd.backward([interp, soft], [g1, g2])
    # equal up to the float atomics' summation order
    for x, y in ((a[0], b[0]), (a[1], b[1]), (fvi.grad, 2 * a[0]), (feats.grad, 2 * a[1])):
        scale = y.abs().max().item()
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6 * scale)
    # and both gradients are the oracle's
    valid = N(nz) >= 0
    _, rf, rw = oracle.rasterize(h, h, N(fvz), N(fvi), N(feats), valid)
    np.testing.assert_array_equal(N(face_idx), rf)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), rf)
    gr, gfeat = oracle.rasterize_backward(N(g1), rf, rw, N(fvi), N(feats), 1e-8)
    gs = oracle.soft_mask_backward(N(g2), osoft, rf, oprob, ocidx, octype, sfvi, 7000, 1000.)
    tol = 1e-4 if dname == 'f32' else 1e-9
    ref = gr + gs
    for x in (a, b):
        np.testing.assert_allclose(N(x[0]), ref, rtol=tol, atol=tol * 0.1 * np.abs(ref).max())
        np.testing.assert_allclose(N(x[1]), gfeat, rtol=tol,
                                   atol=tol * 0.1 * np.abs(gfeat).max())


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('lists', [False, True])
def test_dibr_soft_mask_retained_graph_twice(dname, lists):
    from kaolin_amd.render.mesh import dibr, dibr_soft_mask, rasterize
    dt = TORCH_DTYPES[dname]
    h = 80
    fvz, fvi0, feats, nz = _views(30, 16, h, 2, dt)
    _, face_idx = rasterize(h, h, fvz, fvi0, feats, nz >= 0)
    fvi = fvi0.clone().requires_grad_(True)
    with dibr.close_lists(lists):
        soft = dibr_soft_mask(fvi, face_idx)
    _, g = _grads((1,), soft.shape, dt)
    a = torch.autograd.grad(soft, fvi, g, retain_graph=True)[0]
    b = torch.autograd.grad(soft, fvi, g, retain_graph=True)[0]
    c = torch.autograd.grad(soft, fvi, g)[0]  # frees the graph
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * a.abs().max().item())
    torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6 * a.abs().max().item())
    with pytest.raises(RuntimeError):
        torch.autograd.grad(soft, fvi, g)  # freed like any PyTorch graph
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), N(face_idx))
    ref = oracle.soft_mask_backward(N(g), osoft, N(face_idx), oprob, ocidx, octype, sfvi, 7000,
                                    1000.)
    tol = 1e-4 if dname == 'f32' else 1e-9
    np.testing.assert_allclose(N(a), ref, rtol=tol, atol=tol * 0.1 * np.abs(ref).max())


# --------------------------------------------------------------------------------------------
# non-contiguous inputs
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_dibr_rasterization_noncontiguous_inputs(dname):
    """face_features = uvs.expand(B, ...) (batch stride 0) and a permuted face_vertices_image:
    same outputs and gradients as contiguous copies through rasterize + dibr_soft_mask."""
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_soft_mask, rasterize
    dt = TORCH_DTYPES[dname]
    B, h = 3, 88
    fvz, fvi0, feats0, nz = _views(36, 19, h, B, dt, elevation=0.4)
    g1, g2 = _grads(feats0.shape[:1] + (h, h, feats0.shape[-1]), (B, h, h), dt, seed=7)
    # shared (expanded) features: one per-face-vertex table for all views
    base = feats0[:1].clone().requires_grad_(True)
    feats_x = base.expand(B, -1, -1, -1)
    assert feats_x.stride(0) == 0
    # permuted storage: (B, F, 2, 3) -> transpose to (B, F, 3, 2)
    fvi_store = fvi0.transpose(-1, -2).contiguous().clone().requires_grad_(True)
    fvi_x = fvi_store.transpose(-1, -2)
    assert not fvi_x.is_contiguous()
    i_a, s_a, f_a = dibr_rasterization(h, h, fvz, fvi_x, feats_x, nz)
    torch.autograd.backward([i_a, s_a], [g1, g2])
    # contiguous reference composition
    fvi_b = fvi0.clone().requires_grad_(True)
    feats_b = feats0[:1].expand(B, -1, -1, -1).contiguous().requires_grad_(True)
    i_b, f_b = rasterize(h, h, fvz, fvi_b, feats_b, nz >= 0)
    s_b = dibr_soft_mask(fvi_b, f_b)
    torch.autograd.backward([i_b, s_b], [g1, g2])
    assert torch.equal(f_a, f_b) and torch.equal(i_a, i_b) and torch.equal(s_a, s_b)
    tol = dict(rtol=1e-4, atol=1e-5) if dname == 'f32' else dict(rtol=1e-9, atol=1e-10)
    torch.testing.assert_close(fvi_store.grad.transpose(-1, -2), fvi_b.grad, **tol)
    torch.testing.assert_close(base.grad, feats_b.grad.sum(0, keepdim=True), **tol)


# --------------------------------------------------------------------------------------------
# whole-image gradient parity at C2 / C4 / C5
# --------------------------------------------------------------------------------------------
def _full_vs_oracle(fvz, fvi0, feats0, nz, h, sig, box, knum=30, seed=1):
    from kaolin_amd.render.mesh import dibr_rasterization
    fvi = fvi0.clone().requires_grad_(True)
    feats = feats0.clone().requires_grad_(True)
    interp, soft, face_idx = dibr_rasterization(h, h, fvz, fvi, feats, nz, sig, box, knum)
    g_feat, g_soft = _grads(interp.shape, soft.shape, fvi.dtype, seed)
    torch.autograd.backward([interp, soft], [g_feat, g_soft])
    valid = N(nz) >= 0
    ri, rf, rw = oracle.rasterize(h, h, N(fvz), N(fvi), N(feats), valid)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), rf, sig, box, knum)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    gr, gfeat = oracle.rasterize_backward(N(g_feat), rf, rw, N(fvi), N(feats), 1e-8)
    gs = oracle.soft_mask_backward(N(g_soft), osoft, rf, oprob, ocidx, octype, sfvi, sig, 1000.)
    ref = gr + gs
    np.testing.assert_allclose(N(fvi.grad), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())
    np.testing.assert_allclose(N(feats.grad), gfeat, rtol=1e-4, atol=1e-5 * np.abs(gfeat).max())
    return int((ocidx >= 0).sum())


def test_c2_full_fwd_bwd_vs_oracle():
    """C2: uv_sphere(100,51) 10k faces, 256x256, all 4 views."""
    fvz, fvi, feats, nz = _views(100, 51, 256, 4)
    assert _full_vs_oracle(fvz, fvi, feats, nz, 256, 7000., 0.02) > 0


@pytest.mark.parametrize('sweep', [(3000., 0.05), (30000., 0.01)])
def test_c4_view_full_fwd_bwd_vs_oracle(sweep):
    """C4: one whole 1024x1024 view of the 50k-face sphere at the heaviest (3000 / 0.05) and
    the lightest (30000 / 0.01) point of the sigma / boxlen sweep."""
    sig, box = sweep
    fvz, fvi, feats, nz = _views(250, 101, 1024, 1, first_view=5, total_views=8)
    assert _full_vs_oracle(fvz, fvi, feats, nz, 1024, sig, box) > 0


def test_c5_sphere_view_full_fwd_bwd_vs_oracle():
    """C5: one whole view of uv_sphere(500,201) (200k faces) at elevation 0.6 (the dense pole fan
    in view), 512x512."""
    fvz, fvi, feats, nz = _views(500, 201, 512, 1, elevation=0.6, first_view=2, total_views=16)
    assert _full_vs_oracle(fvz, fvi, feats, nz, 512, 7000., 0.02) > 0
