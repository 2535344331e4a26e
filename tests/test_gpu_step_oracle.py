"""GPU: the exact timed product of bench.py -- ``distributed.GraphedStep`` replaying
``dibr_rasterization_from_vertices`` (the projection inside the binning launch, the fused forward
with split tiles / the tile history, the DIB-R backward and the face -> vertex gather) -- checked
at the headline config against the oracle chain, not against another HIP path.

The oracle chain for the vertex gradient (what the reference's training loop computes,
examples/tutorial/ian_dibr.py:214-291):
  grad_fvi = rasterize backward + soft-mask backward of the C oracle (oracle/dibr_oracle.c, the
             reference kernels rasterization_cuda.cu:238-442 and dibr_soft_mask_cuda.cu:230-353
             restated), run on the oracle's own forward (face index bit-exact against the
             replay's);
  vertices.grad = that grad_fvi pushed through the PyTorch restatement of prepare_vertices
             (kaolin/render/mesh/utils.py:128-175, ops/mesh/mesh.py:24-45) in fp64 autograd --
             the restatement tests/test_f1_golden.py pins to the reference's own fixtures.

The tile history is made stale on purpose: the replays render vertices moved in place after the
capture (as an optimizer step would between training iterations), so each replay is dispatched by
durations measured on other geometry.  Bars: face_idx bit-exact; vertex and feature gradients
rtol 1e-4 with atol 1e-5 of the gradient's scale (fp32 float-atomic summation order), as every
other gradient test of the suite.
"""
import math

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _native():
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()
    _lib.set_tile_history(True)
    _lib.set_tile_split(0)
    yield
    _lib.set_tile_history(True)


def _oracle_step(vertices, faces, proj, cam, feats, g_feat, g_soft, h):
    """(face_idx, vertices.grad, feats.grad) of one step by the oracle chain."""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import prepare_vertices
    with torch.no_grad():  # the corners the step rendered (kd_prep.hpp arithmetic, bit-identical)
        fvc, fvi, nrm = prepare_vertices(vertices.detach().unsqueeze(0), faces, proj,
                                         camera_transform=cam)
    N = lambda t: np.ascontiguousarray(t.detach().cpu().numpy())  # noqa: E731
    fvi_, ft_ = N(fvi), N(feats)
    _, rf, rw = oracle.rasterize(h, h, N(fvc[..., 2]), fvi_, ft_, N(nrm[..., 2]) >= 0)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(fvi_, rf)
    gr, gfeat = oracle.rasterize_backward(N(g_feat), rf, rw, fvi_, ft_, 1e-8)
    gs = oracle.soft_mask_backward(N(g_soft), osoft, rf, oprob, ocidx, octype, sfvi, 7000, 1000.)
    grad_fvi = torch.from_numpy(np.asarray(gr, np.float64) + np.asarray(gs, np.float64))
    v64 = vertices.detach().cpu().double().unsqueeze(0).requires_grad_(True)
    out = workloads.prepare_vertices(v64, faces.cpu(), proj.cpu().double(), cam.cpu().double())
    out[1].backward(grad_fvi)
    return rf, v64.grad[0].numpy(), gfeat


def _close(ours, ref, what):
    ours = ours.detach().cpu().numpy().astype(np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).max()
    assert scale > 0, what
    np.testing.assert_allclose(ours, ref, rtol=1e-4, atol=1e-5 * scale, err_msg=what)


@pytest.mark.parametrize('B', [8, 1], ids=['c3x8', 'c3x1_split'])
def test_bench_step_gradients_vs_oracle_chain(B):
    from kaolin_amd import distributed, workloads
    h = 512
    verts, faces, face_uvs = workloads.uv_sphere(250, 101, seed=0)
    vertices = verts.to(DEV).requires_grad_(True)
    faces = faces.to(DEV)
    cam = workloads.orbit_cameras(B, 0.3).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    uvs = face_uvs.to(DEV).unsqueeze(0).repeat(B, 1, 1, 1)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], dim=-1).contiguous()
    feats.requires_grad_(True)
    g_feat, g_soft = workloads.view_grads(0, B, h, h, 3)
    g_feat, g_soft = g_feat.to(DEV), g_soft.to(DEV)
    fn = lambda: distributed.dibr_forward_backward(  # noqa: E731 -- bench.py's step
        vertices, faces, proj, cam, feats, h, h, g_feat, g_soft)
    # a prior call of the same shape on other geometry leaves its tile history behind
    with torch.no_grad():
        v0 = vertices.detach().clone()
        vertices.mul_(0.8)
    fn()
    torch.cuda.synchronize()
    with torch.no_grad():
        vertices.copy_(v0)
    gs = distributed.GraphedStep([vertices, feats], fn, params_to_reduce=[vertices])
    gen = torch.Generator().manual_seed(11)
    for rep in range(2):
        # move the mesh in place (static graph input): the history recorded by the previous
        # call describes other geometry
        with torch.no_grad():
            vertices.add_((0.01 * torch.randn(vertices.shape, generator=gen)).to(DEV))
        vertices.grad.fill_(float('nan'))
        feats.grad.fill_(float('nan'))
        gs.out.fill_(-7)
        fidx = gs()
        torch.cuda.synchronize()
        rf, gv, gf = _oracle_step(vertices, faces, proj, cam, feats.detach(), g_feat, g_soft, h)
        np.testing.assert_array_equal(fidx.cpu().numpy(), rf, err_msg=f'face_idx, replay {rep}')
        _close(vertices.grad, gv, f'vertices.grad, replay {rep}')
        _close(feats.grad, gf, f'feats.grad, replay {rep}')
