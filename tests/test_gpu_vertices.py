"""GPU: dibr_rasterization_from_vertices -- prepare_vertices + dibr_rasterization as one node
whose forward projects the vertices inside the binning launch (kd_dibr_rasterization_forward_
vertices) and whose backward is either the DIB-R backward + prepare_vertices' gather kernel or the
face -> vertex step fused into the DIB-R backward kernel (SURVEY.md §8 f1,
kd_dibr_rasterization_backward_vertices).

Its outputs must be the composition's bit for bit (the same forward kernels), and its vertex and
feature gradients the composition's (prepare_vertices' gather-form backward over the fused
backward's grad_fvi) up to float-atomic summation order: rtol 1e-4 in fp32, 1e-9 in fp64, with an
absolute floor at that fraction of the gradient's largest magnitude.  The composition's vertex
gradient is itself pinned against the reference's PyTorch composition in test_gpu_parity.py
(test_prepare_vertices_vs_torch) and its grad_fvi against the oracle.
"""
import math

import pytest
import torch

from helpers import TORCH_DTYPES

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()


@pytest.fixture(autouse=True, params=['gather', 'fused'])
def vertex_backward(request):
    """both backwards of the from-vertices node: the DIB-R backward + prepare_vertices' gather
    kernel (default) and the face -> vertex step inside the DIB-R backward kernel"""
    from kaolin_amd.render.mesh import dibr
    old = dibr.FUSED_VERTEX_BACKWARD
    dibr.FUSED_VERTEX_BACKWARD = request.param == 'fused'
    yield request.param
    dibr.FUSED_VERTEX_BACKWARD = old


def _scene(n_lon, n_lat, B, dt, elevation=0.3, shared=True, seed=0):
    from kaolin_amd import workloads
    verts, faces, face_uvs = workloads.uv_sphere(n_lon, n_lat, seed=seed, dtype=dt)
    cam = workloads.orbit_cameras(B, elevation, dtype=dt).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4, dtype=dt).to(DEV)
    v = verts.to(DEV).unsqueeze(0)
    if not shared:
        g = torch.Generator().manual_seed(seed + 5)
        v = v.repeat(B, 1, 1) + 0.01 * torch.randn((B,) + tuple(v.shape[1:]), generator=g,
                                                    dtype=dt).to(DEV)
    uvs = face_uvs.to(DEV).unsqueeze(0).repeat(B, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
    return v.contiguous(), faces.to(DEV), proj, cam, feats


def _grads(h, B, D, dt, seed=1):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand((B, h, h, D), generator=g, dtype=torch.float64).to(DEV, dt),
            torch.rand((B, h, h), generator=g, dtype=torch.float64).to(DEV, dt))


def _close(a, b, dt):
    tol = 1e-4 if dt == torch.float32 else 1e-9
    torch.testing.assert_close(a, b, rtol=tol, atol=tol * 0.1 * b.abs().max().item())


def _both(h, v0, faces, proj, cam, feats0, dt, which=('interp', 'soft'), sig=7000., box=0.02):
    from kaolin_amd.render.mesh import (dibr_rasterization, dibr_rasterization_from_vertices,
                                        prepare_vertices)
    B, D = cam.shape[0], feats0.shape[-1]
    g1, g2 = _grads(h, B, D, dt)
    res = []
    for fused in (True, False):
        v = v0.clone().requires_grad_(True)
        feats = feats0.clone().requires_grad_(True)
        if fused:
            interp, soft, fi = dibr_rasterization_from_vertices(h, h, v, faces, proj, cam, feats,
                                                                sig, box)
        else:
            fvc, fvi, nrm = prepare_vertices(v, faces, proj, camera_transform=cam)
            interp, soft, fi = dibr_rasterization(h, h, fvc[..., 2], fvi, feats, nrm[..., 2],
                                                  sig, box)
        outs = [t for t, k in ((interp, 'interp'), (soft, 'soft')) if k in which]
        grads = [g for g, k in ((g1, 'interp'), (g2, 'soft')) if k in which]
        torch.autograd.backward(outs, grads)
        res.append((interp.detach(), soft.detach(), fi, v.grad, feats.grad))
    return res


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('shared', [True, False])
def test_fused_vertex_backward_matches_composition(dname, shared):
    dt = TORCH_DTYPES[dname]
    h, B = 192, 3
    v0, faces, proj, cam, feats = _scene(60, 31, B, dt, shared=shared)
    (i1, s1, f1, gv1, gf1), (i2, s2, f2, gv2, gf2) = _both(h, v0, faces, proj, cam, feats, dt)
    assert torch.equal(i1, i2) and torch.equal(s1, s2) and torch.equal(f1, f2)
    assert gv1.shape == v0.shape
    _close(gv1, gv2, dt)
    _close(gf1, gf2, dt)


@pytest.mark.parametrize('which', [('interp',), ('soft',)])
def test_fused_vertex_backward_one_output(which):
    """Only one of the two outputs carries a gradient (the other's kernel half is skipped)."""
    dt = torch.float32
    h, B = 128, 2
    v0, faces, proj, cam, feats = _scene(40, 21, B, dt, elevation=0.5)
    (_, _, _, gv1, gf1), (_, _, _, gv2, gf2) = _both(h, v0, faces, proj, cam, feats, dt, which)
    _close(gv1, gv2, dt)
    if 'interp' in which:
        _close(gf1, gf2, dt)


def test_fused_vertex_backward_c3_view_and_overflow():
    """Two views of the C3 sphere at 512x512 (the bench workload), and the same with the record
    pool limited so every tile takes the overflow path (kd_soft_ovf_bwd with vertex output)."""
    from kaolin_amd import _lib
    dt = torch.float32
    h = 512
    v0, faces, proj, cam, feats = _scene(250, 101, 2, dt)
    (i1, s1, _, gv1, gf1), (i2, s2, _, gv2, gf2) = _both(h, v0, faces, proj, cam, feats, dt)
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
    _close(gv1, gv2, dt)
    _close(gf1, gf2, dt)
    _lib.set_pool_limits(1.0, 0.0)
    try:
        (i3, s3, _, gv3, gf3), _ = _both(h, v0, faces, proj, cam, feats, dt)
        torch.cuda.synchronize()
    finally:
        _lib.set_pool_limits(1.0, 1.0)
    assert torch.equal(s3, s1)
    _close(gv3, gv2, dt)
    _close(gf3, gf2, dt)


def test_fused_vertex_backward_retained_graph():
    from kaolin_amd.render.mesh import dibr_rasterization_from_vertices
    dt = torch.float32
    h, B = 96, 2
    v0, faces, proj, cam, feats0 = _scene(30, 16, B, dt)
    v = v0.clone().requires_grad_(True)
    feats = feats0.clone().requires_grad_(True)
    interp, soft, _ = dibr_rasterization_from_vertices(h, h, v, faces, proj, cam, feats)
    g1, g2 = _grads(h, B, 3, dt)
    a = torch.autograd.grad([interp, soft], [v, feats], [g1, g2], retain_graph=True)
    b = torch.autograd.grad([interp, soft], [v, feats], [g1, g2])
    _close(a[0], b[0], dt)
    _close(a[1], b[1], dt)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_from_vertices_forward_outputs_match_prepare(dname):
    """the binning launch's prepare_vertices outputs equal kd_prepare_vertices_forward's bit for
    bit, and the render equals dibr_rasterization of them (C3 views, shared and per-view
    vertices)"""
    from kaolin_amd import _C
    from kaolin_amd.render.mesh import dibr_rasterization
    dt = TORCH_DTYPES[dname]
    h = 256
    for shared in (True, False):
        v, faces, proj, cam, feats = _scene(250, 101, 2, dt, shared=shared)
        fvc, fvi, nrm, interp, face_idx, weights, soft, _ = \
            _C.render.mesh.dibr_rasterization_forward_vertices(
                h, h, v, faces, proj, cam, feats, 7000., 0.02, 30, 1000., 1e-8, want_grad=False)
        c2, i2, n2 = _C.prepare_vertices_forward(v, faces, proj, cam)
        assert torch.equal(fvc, c2) and torch.equal(fvi, i2) and torch.equal(nrm, n2)
        ri, rs, rf = dibr_rasterization(h, h, c2[..., 2], i2, feats, n2[..., 2])
        assert torch.equal(interp, ri) and torch.equal(soft, rs) and torch.equal(face_idx, rf)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('shared', [True, False])
def test_prepare_backward_from_vertices_bit_identical(dname, shared, vertex_backward):
    """kd_prepare_vertices_backward_vertices (the node's gather backward, each corner's
    camera-space point recomputed from the vertex per view: the bits of fvc) equals
    kd_prepare_vertices_backward over the forward's fvc for a random grad_fvi (C3 mesh, 3 views,
    shared and per-view vertices) -- to the summation order of a vertex's entries, which both
    kernels add in LDS with float atomics (their order is not fixed)"""
    if vertex_backward != 'gather':
        pytest.skip('a prepare-kernel test (one backward form suffices)')
    from kaolin_amd import _C
    from kaolin_amd.render.mesh.utils import _adjacency
    dt = TORCH_DTYPES[dname]
    B = 3
    v, faces, proj, cam, _ = _scene(250, 101, B, dt, shared=shared)
    fvc, fvi, _ = _C.prepare_vertices_forward(v, faces, proj, cam)
    g = torch.Generator().manual_seed(7)
    gfvi = (torch.rand(fvi.shape, generator=g, dtype=torch.float64) - 0.5).to(DEV, dt)
    adj = _adjacency(faces, v.shape[1])
    ref = _C.prepare_vertices_backward(faces, proj, cam, fvc, None, gfvi, None, adj,
                                       v.shape[0], v.shape[1])
    new = _C.prepare_vertices_backward_from_vertices(v, faces, proj, cam, gfvi, adj)
    torch.cuda.synchronize()
    tol = 1e-5 if dname == 'f32' else 1e-12
    torch.testing.assert_close(new, ref, rtol=tol, atol=tol * ref.abs().max().item())
