"""Pins the f4 oracle (oracle/f4.py, the nvdiffrast_fwd data path) through the reference's
rasterize goldens (CPU only): a rast buffer (u, v, 0, face_idx + 1) holding the barycentrics of
the reference forward reproduces the reference's face index exactly, its features to rounding and,
through rasterize_backward on the derived weights, its gradients -- the same bars as
test_oracle.py's naive-oracle parity (test_rasterization.py:136-232).
"""
import numpy as np
import pytest

import oracle
from helpers import sphere
from oracle import f4

H, W = 35, 31


def rast_from(face_idx, weights):
    r = np.zeros(face_idx.shape + (4,), weights.dtype)
    r[..., :2] = weights[..., :2]
    r[..., 3] = (face_idx + 1).astype(weights.dtype)
    return r


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('with_valid', [0, 1])
def test_rast_path_reproduces_reference(sphere_inputs, sphere_naive, dname, flip, with_valid):
    s = sphere(sphere_inputs, dname, flip)
    key = f'{dname}_flip{flip}_valid{with_valid}'
    valid = s['valid'] if with_valid else None
    _, face_idx, weights = oracle.rasterize(H, W, s['fvz'], s['fvi'], s['uvs'], valid)
    interp, fidx, w = f4.rast_interpolate(rast_from(face_idx, weights), s['uvs'])
    np.testing.assert_array_equal(fidx, sphere_naive[f'face_idx_{key}'])
    np.testing.assert_allclose(interp, sphere_naive[f'interp_{key}'], atol=1e-5, rtol=1e-5)
    cov = fidx >= 0  # empty pixels: (0, 0, 1) here, (0, 0, 0) in the cuda backend; unused
    # the cuda backend's weights sum to S / (S + eps) (eps-normalised), rast's to exactly 1
    np.testing.assert_allclose(w[cov], weights[cov], atol=1e-6 if dname == 'f32' else 1e-9)
    gfvi, gfeat = oracle.rasterize_backward(sphere_naive[f'grad_out_{key}'], fidx, w, s['fvi'],
                                            s['uvs'], 1e-8)
    np.testing.assert_allclose(gfvi, sphere_naive[f'grad_fvi_{key}'], atol=1e-2, rtol=1e-3)
    np.testing.assert_allclose(gfeat, sphere_naive[f'grad_feat_{key}'], atol=1e-3, rtol=1e-3)


def test_rast_empty_and_out_of_range_ids():
    feat = np.arange(2 * 4 * 3 * 2, dtype=np.float32).reshape(2, 4, 3, 2)
    rast = np.zeros((2, 2, 3, 4), np.float32)
    rast[0, 0, 0] = [0.25, 0.5, 0.3, 3]      # face 2
    rast[1, 1, 2] = [0.1, 0.2, 0.9, 9]       # id beyond F -> empty
    rast[1, 0, 1] = [0.1, 0.2, 0.9, -2]      # negative -> empty
    interp, fidx, w = f4.rast_interpolate(rast, feat)
    assert fidx[0, 0, 0] == 2 and (fidx.reshape(-1)[1:] == -1).all()
    a = feat[0, 2]
    np.testing.assert_array_equal(interp[0, 0, 0],
                                  np.float32(0.25) * a[0] + np.float32(0.5) * a[1] +
                                  np.float32(0.25) * a[2])
    assert (interp.reshape(-1, 2)[1:] == 0).all()
    np.testing.assert_array_equal(w[0, 0, 1], [0, 0, 1])
