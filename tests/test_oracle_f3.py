"""Pins the f3 oracle (oracle/f3.py, deftet_sparse_render) against the reference's literals and its
naive renderer (tests/golden/deftet.npz, written by tests/golden/make_golden_f3.py).  CPU only.

Mirrors tests/python/kaolin/render/mesh/test_deftet.py:105-165 (simple case, exact face index)
and :420-520 (model.obj sphere vs the naive renderer: face index exact, features rtol 1e-4,
gradients 5e-3 / 1e-3).
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden
from oracle import f3


@pytest.fixture(scope='module')
def g():
    return load_golden('deftet.npz')


def grad_out(shape, dtype, seed):
    """The incoming gradient make_golden_f3.py used (torch CPU generator)."""
    gen = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=gen, dtype=torch.float32 if dtype == np.float32
                      else torch.float64).numpy()


@pytest.mark.parametrize('k', ['f32', 'f64'])
def test_simple_case(g, k):
    interp, fidx, w = f3.deftet_forward(g[f'simple_px_{k}'], g[f'simple_rr_{k}'],
                                        g[f'simple_fvz_{k}'], g[f'simple_fvi_{k}'],
                                        g[f'simple_feat_{k}'], 5)
    np.testing.assert_array_equal(fidx, g[f'simple_face_idx_{k}'])
    np.testing.assert_allclose(interp, g[f'simple_interp_{k}'], rtol=1e-5, atol=1e-5)
    go = grad_out(interp.shape, interp.dtype, 1)
    gfvi, gfeat = oracle.rasterize_backward(go, fidx, w, g[f'simple_fvi_{k}'],
                                            g[f'simple_feat_{k}'], 1e-8)
    np.testing.assert_allclose(gfvi, g[f'simple_grad_fvi_{k}'], rtol=5e-3, atol=5e-3)
    np.testing.assert_allclose(gfeat, g[f'simple_grad_feat_{k}'], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('P', [31, 1025])
@pytest.mark.parametrize('center', [0, 1])
@pytest.mark.parametrize('knum', [20, 30])
def test_sphere_vs_naive(g, k, P, center, knum):
    key = f'{P}_{center}_{knum}_{k}'
    fvi, uvs = g[f'sphere_fvi_{k}'], g[f'sphere_uvs_{k}']
    interp, fidx, w = f3.deftet_forward(g[f'sphere_px_{P}_{k}'], g[f'sphere_rr_{P}_{center}_{k}'],
                                        g[f'sphere_fvz_{k}'], fvi, uvs, knum)
    np.testing.assert_array_equal(fidx, g[f'sphere_face_idx_{key}'])
    np.testing.assert_allclose(interp, g[f'sphere_interp_{key}'], rtol=1e-4, atol=1e-4)
    go = grad_out(interp.shape, interp.dtype, 1000 + P + 10 * center + knum)
    gfvi, gfeat = oracle.rasterize_backward(go, fidx, w, fvi, uvs, 1e-8)
    np.testing.assert_allclose(gfvi, g[f'sphere_grad_fvi_{key}'], rtol=5e-3, atol=5e-3)
    np.testing.assert_allclose(gfeat, g[f'sphere_grad_feat_{key}'], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize('k', ['f32', 'f64'])
@pytest.mark.parametrize('knum', [20, 30])
def test_raw_op_oracle_sorts_to_the_goldens(g, k, knum):
    """The op-form oracle (deftet_forward_raw: the reference kernel's unsorted first-knum hits,
    deftet_sparse_render_forward_cuda) sorted by depth like deftet.py:300-303 gives the golden
    face indices."""
    P, center = 1025, 1
    fvi = g[f'sphere_fvi_{k}']
    bbox = np.concatenate([fvi.min(2), fvi.max(2)], -1)  # deftet.py:287-289
    fidx, depth, w0, w1 = f3.deftet_forward_raw(g[f'sphere_px_{P}_{k}'],
                                                g[f'sphere_rr_{P}_{center}_{k}'],
                                                g[f'sphere_fvz_{k}'], fvi, bbox, knum)
    m = fidx >= 0  # hits first (ascending face index), padding last
    assert (m[..., 1:] <= m[..., :-1]).all()
    assert (np.diff(fidx, axis=-1)[m[..., 1:]] > 0).all()
    assert np.isneginf(depth[fidx < 0]).all() and (w0[fidx < 0] == 0).all()
    order = np.argsort(-depth, axis=-1, kind='stable')
    np.testing.assert_array_equal(np.take_along_axis(fidx, order, -1),
                                  g[f'sphere_face_idx_{P}_{center}_{knum}_{k}'])
