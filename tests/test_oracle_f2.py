"""Pins the f2 oracle (oracle/f2.py: mask_iou, texture_mapping) against the reference's own test
literals and against the reference functions' outputs on seeded inputs (tests/golden/f2.npz,
written by tests/golden/make_golden_f2.py).  CPU only.

Mirrors tests/python/kaolin/metrics/test_render.py:49-52 and
tests/python/kaolin/render/mesh/test_utils.py:59-107.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import f2

DT = {'f32': np.float32, 'f64': np.float64}
MODES = ['nearest', 'bilinear']


@pytest.fixture(scope='module')
def g():
    return load_golden('f2.npz')


def tol(k):
    return dict(rtol=1e-5, atol=1e-6) if k == 'f32' else dict(rtol=1e-12, atol=1e-13)


@pytest.mark.parametrize('k', ['f32', 'f64'])
def test_mask_iou_reference_case(g, k):
    loss, _ = f2.mask_iou(g['t_lhs'].astype(DT[k]), g['t_rhs'].astype(DT[k]))
    np.testing.assert_allclose(loss, 0.3105, rtol=1e-5, atol=1e-8)  # test_render.py:51-52
    np.testing.assert_allclose(loss, g[f't_iou_{k}'], **tol(k))


@pytest.mark.parametrize('k', ['f32', 'f64'])
def test_mask_iou_random(g, k):
    l, r = g[f'r_iou_l_{k}'], g[f'r_iou_r_{k}']
    loss, stats = f2.mask_iou(l, r)
    np.testing.assert_allclose(loss, g[f'r_iou_loss_{k}'], **tol(k))
    gl, gr = f2.mask_iou_backward(0.75, l, r, stats)
    np.testing.assert_allclose(gl, g[f'r_iou_gl_{k}'], **tol(k))
    np.testing.assert_allclose(gr, g[f'r_iou_gr_{k}'], **tol(k))


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_reference_cases(g, k, mode):
    dt = DT[k]
    for tname in ('tex1', 'tex3'):
        out = f2.texture_mapping(g['t_sparse'].astype(dt), g[f't_{tname}'].astype(dt), mode)
        np.testing.assert_array_equal(out, g[f't_sparse_{tname}_{mode}_{k}'])  # torch.equal
    out = f2.texture_mapping(g['t_dense'].astype(dt), g['t_tex3'].astype(dt), mode)
    np.testing.assert_array_equal(out, g[f't_dense_tex3_{mode}_{k}'])


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('mode', MODES)
def test_texture_random(g, k, mode):
    uv, tex, go = g[f'r_tex_uv_{k}'], g[f'r_tex_map_{k}'], g[f'r_tex_go_{k}']
    out = f2.texture_mapping(uv, tex, mode)
    np.testing.assert_allclose(out, g[f'r_tex_out_{mode}_{k}'], **tol(k))
    guv, gt = f2.texture_mapping_backward(go, uv, tex, mode)
    np.testing.assert_allclose(gt, g[f'r_tex_gmap_{mode}_{k}'], **tol(k))
    # the uv gradient is a 4-tap sum with cancellation, scaled by 2 * size / 2 (~17 here); ATen's
    # CPU kernel factors it differently, so fp32 agrees to a few ulp of that scale
    gtol = dict(rtol=1e-4, atol=2e-5) if k == 'f32' else tol(k)
    np.testing.assert_allclose(guv, g[f'r_tex_guv_{mode}_{k}'], **gtol)


def test_texture_shared_map_sums_views(g):
    uv, tex, go = g['r_tex_uv_f64'], g['r_tex_map_f64'][:1], g['r_tex_go_f64']
    out = f2.texture_mapping(uv, tex, 'bilinear')
    rep = np.repeat(tex, uv.shape[0], axis=0)
    np.testing.assert_array_equal(out, f2.texture_mapping(uv, rep, 'bilinear'))
    _, gt = f2.texture_mapping_backward(go, uv, tex, 'bilinear')
    _, gr = f2.texture_mapping_backward(go, uv, rep, 'bilinear')
    np.testing.assert_allclose(gt[0], gr.sum(0), rtol=1e-12)
