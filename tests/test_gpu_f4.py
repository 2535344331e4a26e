"""GPU parity for SURVEY.md §8 f4 (nvdiffrast_fwd compatibility): kd_rast_interpolate and the
rasterize backward behind ``rasterize_from_rast`` against the oracle (oracle/f4.py +
oracle.rasterize_backward).  Bars: interp / face_idx / weights bit-exact (same op sequence);
gradients to the grad tolerance of test_gpu_parity.py.
"""
import numpy as np
import pytest
import torch

import oracle
from helpers import sphere
from oracle import f4

pytestmark = pytest.mark.gpu

DEV = 'cuda'
H, W = 35, 31


@pytest.fixture(scope='module', autouse=True)
def _native():
    import kaolin_amd  # noqa: F401
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV)


def N(t):
    return t.detach().cpu().numpy()


def grad_tol(dname):
    return dict(rtol=1e-4, atol=1e-5) if dname == 'f32' else dict(rtol=1e-9, atol=1e-10)


def rast_from(face_idx, weights):
    r = np.zeros(face_idx.shape + (4,), weights.dtype)
    r[..., :2] = weights[..., :2]
    r[..., 3] = (face_idx + 1).astype(weights.dtype)
    return r


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
def test_rast_path_sphere(sphere_inputs, dname, flip):
    from kaolin_amd.render.mesh import rasterize_from_rast
    s = sphere(sphere_inputs, dname, flip)
    _, face_idx, weights = oracle.rasterize(H, W, s['fvz'], s['fvi'], s['uvs'], s['valid'])
    rast = rast_from(face_idx, weights)
    oi, of, ow = f4.rast_interpolate(rast, s['uvs'])
    fvi, feat = T(s['fvi']).requires_grad_(True), T(s['uvs']).requires_grad_(True)
    interp, fidx = rasterize_from_rast(T(rast), fvi, feat)
    np.testing.assert_array_equal(N(fidx), of)
    np.testing.assert_array_equal(N(interp), oi)
    g = np.random.default_rng(3).random(oi.shape).astype(oi.dtype)
    gfvi, gfeat = torch.autograd.grad(interp, [fvi, feat], T(g))
    rfvi, rfeat = oracle.rasterize_backward(g, of, ow, s['fvi'], s['uvs'], 1e-8)
    np.testing.assert_allclose(N(gfvi), rfvi, **grad_tol(dname))
    np.testing.assert_allclose(N(gfeat), rfeat, **grad_tol(dname))


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_rast_random_buffers(dname):
    """Random barycentrics and ids, including empty, out-of-range and negative ids; C3 size."""
    from kaolin_amd import _C
    dt = np.float32 if dname == 'f32' else np.float64
    rng = np.random.default_rng(11)
    B, h, w, F, D = 8, 512, 512, 5000, 3
    rast = rng.random((B, h, w, 4)).astype(dt)
    rast[..., 3] = rng.integers(-2, F + 3, size=(B, h, w)).astype(dt)
    feat = rng.standard_normal((B, F, 3, D)).astype(dt)
    oi, of, ow = f4.rast_interpolate(rast, feat)
    interp, fidx, weights = _C.render.mesh.rast_interpolate(T(rast), T(feat))
    np.testing.assert_array_equal(N(fidx), of)
    np.testing.assert_array_equal(N(weights), ow)
    np.testing.assert_array_equal(N(interp), oi)


def test_backends_without_nvdiffrast():
    from kaolin_amd.render.mesh import dibr_rasterization, rasterize
    from kaolin_amd.render.mesh import rasterization as r
    fvz = torch.zeros((1, 2, 3), device=DEV)
    fvi = torch.zeros((1, 2, 3, 2), device=DEV)
    feat = torch.zeros((1, 2, 3, 1), device=DEV)
    if not r._has_nvdiffrast:
        for backend in ('nvdiffrast', 'nvdiffrast_fwd'):
            with pytest.raises(ValueError, match='nvdiffrast must be installed'):
                rasterize(8, 8, fvz, fvi, feat, backend=backend)
            with pytest.raises(ValueError, match='nvdiffrast must be installed'):
                dibr_rasterization(8, 8, fvz, fvi, feat, torch.ones((1, 2), device=DEV),
                                   rast_backend=backend)
    with pytest.raises(ValueError, match='not a valid backend'):
        rasterize(8, 8, fvz, fvi, feat, backend='opengl')


def test_legacy_to_opengl_layout():
    """_legacy_to_opengl (rasterization.py:41-79): positions and triangles nvdiffrast consumes."""
    from kaolin_amd.render.mesh.rasterization import _legacy_to_opengl
    rng = np.random.default_rng(2)
    fvi = T(rng.random((2, 4, 3, 2)).astype(np.float32))
    fvz = T(-rng.random((2, 4, 3)).astype(np.float32) - 1)
    valid = T(rng.random((2, 4)) > 0.5)
    pos, tri = _legacy_to_opengl(fvi, fvz, valid)
    assert pos.shape == (2, 12, 4) and tri.shape == (4, 3)
    assert torch.equal(tri.reshape(-1).long().cpu(), torch.arange(12))
    np.testing.assert_array_equal(N(pos[..., 0]), N(fvi[..., 0]).reshape(2, 12))
    np.testing.assert_array_equal(N(pos[..., 1]), -N(fvi[..., 1]).reshape(2, 12))
    z = -N(fvz) / (np.abs(N(fvz)).max() + np.float32(1e-6))
    np.testing.assert_allclose(N(pos[..., 2]), z.reshape(2, 12), rtol=1e-6)
    np.testing.assert_array_equal(N(pos[..., 3]),
                                  np.repeat(np.where(N(valid), 1., -1.), 3, axis=1))
