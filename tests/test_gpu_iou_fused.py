"""GPU: dibr_rasterization with the silhouette loss fused in against the
composition it replaces -- ``dibr_rasterization`` followed by ``mask_iou(soft_mask, gt_mask)``
(kaolin/metrics/render.py:18-40), the DIB-R training loop's form
(examples/tutorial/ian_dibr.py:264-265) -- both on the HIP kernels, whose parity with the
reference is pinned elsewhere (test_gpu_parity.py, test_gpu_f2.py).

Bars: interpolated features, soft mask and face_idx bit-identical (the same kernels); the loss to
1e-6 relative in fp32 / 1e-12 in fp64 (its fp64 view sums are accumulated by atomics in tile order
instead of the standalone kernel's fixed order); gradients at the atomic-summation-order bars of
test_gpu_autograd.py (rtol 1e-4 with an absolute floor of 1e-5 x the largest magnitude in fp32;
1e-9 in fp64).
"""
import numpy as np
import pytest
import torch

from helpers import TORCH_DTYPES

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def N(t):
    return t.detach().cpu().numpy()


def _views(n_lon, n_lat, h, B, dt, seed=0):
    from kaolin_amd import workloads
    v = workloads.sphere_views(n_lon, n_lat, h, h, B, DEV, dtype=dt, seed=seed)
    return v['fvz'], v['fvi'].detach(), v['feats'].contiguous(), v['normals_z']


def _gt(face_idx, dt):
    """A target silhouette: the covered mask shifted by 5 pixels (test_dibr.py:176-179)."""
    mask = (face_idx != -1).to(dt)
    return torch.nn.functional.pad(mask, (0, 5))[..., 5:].contiguous()


def _run(fused, fvz, fvi0, feats0, nz, h, gt, knum, outputs, seed=3):
    from kaolin_amd.metrics.render import mask_iou
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_rasterization_with_mask_iou
    fvi = fvi0.clone().requires_grad_(True)
    feats = feats0.clone().requires_grad_(True)
    if fused:
        interp, soft, face_idx, loss = dibr_rasterization_with_mask_iou(
            h, h, fvz, fvi, feats, nz, gt, knum=knum)
    else:
        interp, soft, face_idx = dibr_rasterization(h, h, fvz, fvi, feats, nz, knum=knum)
        loss = mask_iou(soft, gt)
    g = torch.Generator().manual_seed(seed)
    gi = torch.rand(interp.shape, generator=g, dtype=torch.float64).to(DEV, interp.dtype)
    gs = torch.rand(soft.shape, generator=g, dtype=torch.float64).to(DEV, soft.dtype)
    terms = {'loss': [loss], 'all': [loss, interp, soft]}[outputs]
    grads = {'loss': [torch.tensor(0.75, device=DEV, dtype=loss.dtype)],
             'all': [torch.tensor(0.75, device=DEV, dtype=loss.dtype), gi, gs]}[outputs]
    torch.autograd.backward(terms, grads)
    return interp, soft, face_idx, loss, fvi.grad, feats.grad


def _compare(a, b, dname):
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    rt = 1e-6 if dname == 'f32' else 1e-12
    np.testing.assert_allclose(N(a[3]), N(b[3]), rtol=rt, atol=rt)
    for x, y in zip(a[4:], b[4:]):
        if y is None:
            assert x is None
            continue
        ref = N(y)
        if dname == 'f32':
            np.testing.assert_allclose(N(x), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())
        else:
            np.testing.assert_allclose(N(x), ref, rtol=1e-9, atol=1e-9 * np.abs(ref).max())


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('outputs', ['loss', 'all'])
def test_fused_iou_matches_composition(dname, outputs):
    dt = TORCH_DTYPES[dname]
    fvz, fvi, feats, nz = _views(40, 21, 96, 3, dt)
    from kaolin_amd.render.mesh import rasterize
    _, fidx = rasterize(96, 96, fvz, fvi, feats, nz >= 0)
    gt = _gt(fidx, dt)
    a = _run(True, fvz, fvi, feats, nz, 96, gt, 30, outputs)
    b = _run(False, fvz, fvi, feats, nz, 96, gt, 30, outputs)
    _compare(a, b, dname)
    assert float(N(a[3])) > 0.0


def test_fused_iou_c3_view():
    """Two whole C3 views (50k faces, 512x512), all three outputs' gradients."""
    fvz, fvi, feats, nz = _views(250, 101, 512, 2, torch.float32)
    from kaolin_amd.render.mesh import rasterize
    _, fidx = rasterize(512, 512, fvz, fvi, feats, nz >= 0)
    gt = _gt(fidx, torch.float32)
    a = _run(True, fvz, fvi, feats, nz, 512, gt, 30, 'all')
    b = _run(False, fvz, fvi, feats, nz, 512, gt, 30, 'all')
    _compare(a, b, 'f32')


def test_fused_iou_fallback_and_retained_graph():
    """knum > 32 runs the composition; a second backward over a retained graph repeats the
    first."""
    from kaolin_amd.render.mesh import dibr_rasterization_with_mask_iou
    fvz, fvi, feats, nz = _views(30, 17, 64, 2, torch.float32)
    gt = torch.rand((2, 64, 64), generator=torch.Generator().manual_seed(5)).to(DEV)
    a = _run(True, fvz, fvi, feats, nz, 64, gt, 40, 'all')
    b = _run(False, fvz, fvi, feats, nz, 64, gt, 40, 'all')
    _compare(a, b, 'f32')
    x = fvi.clone().requires_grad_(True)
    *_, loss = dibr_rasterization_with_mask_iou(64, 64, fvz, x, feats, nz, gt)
    g1, = torch.autograd.grad(loss, x, retain_graph=True)
    g2, = torch.autograd.grad(loss, x)
    np.testing.assert_allclose(N(g1), N(g2), rtol=1e-5, atol=1e-6 * float(N(g1.abs().max())))


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_gt_mask_requiring_grad_gets_its_gradient(dname):
    """mask_iou differentiates its right-hand mask too (metrics/render.py:18-40): a gt_mask that
    requires grad must receive d loss / d gt (the fused kernels produce none, so the composition
    runs) -- equal to the composition's, and the renderer's gradients unchanged."""
    from kaolin_amd.metrics.render import mask_iou
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_rasterization_with_mask_iou
    dt = TORCH_DTYPES[dname]
    h = 64
    fvz, fvi0, feats, nz = _views(30, 16, h, 2, dt)
    _, _, fidx = dibr_rasterization(h, h, fvz, fvi0, feats, nz)
    gt0 = _gt(fidx, dt)
    res = []
    for fused in (True, False):
        fvi = fvi0.clone().requires_grad_(True)
        gt = gt0.clone().requires_grad_(True)
        if fused:
            _, soft, _, loss = dibr_rasterization_with_mask_iou(h, h, fvz, fvi, feats, nz, gt)
        else:
            _, soft, _ = dibr_rasterization(h, h, fvz, fvi, feats, nz)
            loss = mask_iou(soft, gt)
        loss.backward()
        assert gt.grad is not None and gt.grad.abs().max() > 0
        res.append((loss.detach(), fvi.grad, gt.grad))
    tol = dict(rtol=1e-5, atol=1e-7) if dname == 'f32' else dict(rtol=1e-12, atol=1e-14)
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(a, b, **tol)
