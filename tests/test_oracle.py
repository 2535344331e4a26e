"""Pins the CPU oracle (oracle/) against the reference's own golden vectors (CPU-only).

Mirrors the reference tests:
  tests/python/kaolin/render/mesh/test_rasterization.py:136-232 (naive-oracle parity)
  tests/python/kaolin/render/mesh/test_dibr.py:109-191, 309-394 (soft-mask goldens)
"""
import numpy as np
import pytest

import oracle
from helpers import DTYPES, iou_grad_soft, sphere

H, W = 35, 31


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_simple_raster_face_idx(simple_golden, dname):
    dt = DTYPES[dname]
    fvz = simple_golden['simple_fvz'].astype(dt)
    fvi = simple_golden['simple_fvi'].astype(dt)
    feat = np.zeros(fvz.shape + (1,), dt)
    _, face_idx, _ = oracle.rasterize(H, W, fvz, fvi, feat)
    np.testing.assert_array_equal(face_idx, simple_golden['simple_new_face_idx'])


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('sigmainv', [7000, 70])
@pytest.mark.parametrize('boxlen', [0.02, 0.2])
@pytest.mark.parametrize('multiplier', [1000, 100, 1])
@pytest.mark.parametrize('knum', [30, 20])
def test_simple_soft_mask(simple_golden, dname, sigmainv, boxlen, multiplier, knum):
    dt = DTYPES[dname]
    g = simple_golden
    tag = f'{sigmainv}_{boxlen}'
    fvi = g['simple_fvi'].astype(dt)
    face_idx = g['simple_new_face_idx'].astype(np.int64)
    soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(fvi, face_idx, sigmainv, boxlen,
                                                             knum, multiplier)
    np.testing.assert_allclose(soft, g[f'simple_soft_{tag}'], atol=1e-5, rtol=1e-5)
    np.testing.assert_array_equal(cidx, g[f'simple_close_idx_{tag}'][..., :knum])
    np.testing.assert_allclose(prob, g[f'simple_close_prob_{tag}'][..., :knum], atol=1e-5,
                               rtol=1e-5)
    np.testing.assert_array_equal(ctype, g[f'simple_close_type_{tag}'][..., :knum])
    # backward through mask_iou against a 5-px shifted mask (test_dibr.py:167-191)
    gsoft = iou_grad_soft(soft, face_idx)
    grad = oracle.soft_mask_backward(gsoft, soft, face_idx, prob, cidx, ctype, sfvi, sigmainv,
                                     multiplier)
    np.testing.assert_allclose(grad, g[f'simple_grad_{tag}'], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('sigmainv', [7000, 70])
@pytest.mark.parametrize('boxlen', [0.02, 0.01])
@pytest.mark.parametrize('knum', [30, 40])
def test_sphere_soft_mask(sphere_inputs, sphere_softmask, dname, sigmainv, boxlen, knum):
    s = sphere(sphere_inputs, dname, 0)
    g = sphere_softmask
    tag = f'{sigmainv}_{boxlen}'
    feat = np.zeros(s['fvz'].shape + (1,), s['fvz'].dtype)
    _, face_idx, _ = oracle.rasterize(H, W, s['fvz'], s['fvi'], feat)
    assert np.all(g[f'soft_{tag}'][face_idx >= 0] == 1.)  # covered => soft == 1 (:68-70)
    for multiplier in (1000, 100):
        soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(s['fvi'], face_idx, sigmainv,
                                                                 boxlen, knum, multiplier)
        np.testing.assert_allclose(soft, g[f'soft_{tag}'], atol=1e-5, rtol=1e-5)
        np.testing.assert_array_equal(cidx, g[f'close_idx_{tag}'][..., :knum])
        np.testing.assert_allclose(prob, g[f'close_prob_{tag}'][..., :knum], atol=1e-5,
                                   rtol=1e-5)
        assert np.mean(ctype != g[f'close_type_{tag}'][..., :knum]) <= 0.01
    for multiplier in (1000, 100, 1):
        soft, prob, cidx, ctype, sfvi = oracle.soft_mask_forward(s['fvi'], face_idx, sigmainv,
                                                                 boxlen, knum, multiplier)
        gsoft = iou_grad_soft(soft, face_idx)
        grad = oracle.soft_mask_backward(gsoft, soft, face_idx, prob, cidx, ctype, sfvi,
                                         sigmainv, multiplier)
        np.testing.assert_allclose(grad, g[f'grad_{tag}'], atol=1e-1, rtol=1e-1)


def _check_naive(fvz, fvi, feat, valid, h, w, ref, key):
    interp, face_idx, weights = oracle.rasterize(h, w, fvz, fvi, feat, valid)
    np.testing.assert_array_equal(face_idx, ref[f'face_idx_{key}'])
    np.testing.assert_allclose(interp, ref[f'interp_{key}'], atol=1e-5, rtol=1e-5)
    gfvi, gfeat = oracle.rasterize_backward(ref[f'grad_out_{key}'], face_idx, weights, fvi, feat,
                                            1e-8)
    np.testing.assert_allclose(gfvi, ref[f'grad_fvi_{key}'], atol=1e-2, rtol=1e-3)
    np.testing.assert_allclose(gfeat, ref[f'grad_feat_{key}'], atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('with_valid', [0, 1])
def test_sphere_raster_vs_naive(sphere_inputs, sphere_naive, dname, flip, with_valid):
    s = sphere(sphere_inputs, dname, flip)
    _check_naive(s['fvz'], s['fvi'], s['uvs'], s['valid'] if with_valid else None, H, W,
                 sphere_naive, f'{dname}_flip{flip}_valid{with_valid}')


@pytest.mark.parametrize('i', [0, 1, 2])
@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('with_valid', [0, 1])
def test_soup_raster_vs_naive(soup_naive, i, dname, with_valid):
    z = soup_naive
    key = f'soup{i}_{dname}'
    h, w = (int(v) for v in z[f'hw_{key}'])
    _check_naive(z[f'fvz_{key}'], z[f'fvi_{key}'], z[f'feat_{key}'],
                 z[f'valid_{key}'] if with_valid else None, h, w, z, f'{key}_valid{with_valid}')
