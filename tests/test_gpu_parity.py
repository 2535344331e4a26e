"""GPU parity: the gfx950 HIP path (through the C ABI) against the CPU oracle and the reference's
golden vectors.  Run with ``pytest -m gpu`` on an MI355X.

Bars (north_star): integer outputs (face_idx, close_face_idx, close_face_dist_type) bit-exact vs
the oracle; the forward floats are also checked bit-exact where the arithmetic is the same
IEEE-basic-op sequence (weights, interpolated features) and to 1e-6 relative where a
transcendental is involved (close_face_prob, soft mask: device expf vs glibc expf); gradients
(summed in a different order than the oracle) to rtol 1e-4 / atol 1e-5 in fp32 and 1e-10 in fp64.
The reference's own test tolerances are used against its goldens.
"""
import zlib

import numpy as np
import pytest
import torch

import oracle
from helpers import DTYPES, TORCH_DTYPES, iou_grad_soft, mask_iou, shifted_mask, sphere

pytestmark = pytest.mark.gpu

H, W = 35, 31
DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _native():
    import kaolin_amd  # noqa: F401  (fails loudly when the library is missing)
    from kaolin_amd import _lib
    _lib.load()
    assert torch.cuda.is_available()


def T(a, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def N(t):
    return t.detach().cpu().numpy()


def grad_tol(dname):
    return dict(rtol=1e-4, atol=1e-5) if dname == 'f32' else dict(rtol=1e-9, atol=1e-10)


# --------------------------------------------------------------------------------------------
# rasterize
# --------------------------------------------------------------------------------------------
def _raster_case(fvz, fvi, feat, valid, h, w, dname, multiplier=1000, rows=None):
    from kaolin_amd.render.mesh import rasterize
    ri, rf, rw = oracle.rasterize(h, w, fvz, fvi, feat, valid, multiplier=multiplier, rows=rows)
    tfvz, tfvi, tfeat = T(fvz), T(fvi), T(feat)
    tfvi.requires_grad_(True)
    tfeat.requires_grad_(True)
    interp, face_idx = rasterize(h, w, tfvz, tfvi, tfeat,
                                 None if valid is None else T(valid), multiplier=multiplier)
    sl = slice(None) if rows is None else slice(rows[0], rows[1])
    np.testing.assert_array_equal(N(face_idx)[:, sl], rf[:, sl])
    np.testing.assert_array_equal(N(interp)[:, sl], ri[:, sl])
    return tfvi, tfeat, interp, face_idx, rw


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
@pytest.mark.parametrize('with_valid', [0, 1])
def test_rasterize_sphere_fwd_bwd(sphere_inputs, sphere_naive, dname, flip, with_valid):
    s = sphere(sphere_inputs, dname, flip)
    valid = s['valid'] if with_valid else None
    tfvi, tfeat, interp, face_idx, rw = _raster_case(s['fvz'], s['fvi'], s['uvs'], valid, H, W,
                                                     dname)
    key = f'{dname}_flip{flip}_valid{with_valid}'
    # the reference's own oracle test (test_rasterization.py:136-157)
    np.testing.assert_array_equal(N(face_idx), sphere_naive[f'face_idx_{key}'])
    np.testing.assert_allclose(N(interp), sphere_naive[f'interp_{key}'], rtol=1e-5, atol=1e-5)
    grad_out = sphere_naive[f'grad_out_{key}']
    interp.backward(T(grad_out))
    gfvi, gfeat = oracle.rasterize_backward(grad_out, N(face_idx), rw, s['fvi'], s['uvs'], 1e-8)
    np.testing.assert_allclose(N(tfvi.grad), gfvi, **grad_tol(dname))
    np.testing.assert_allclose(N(tfeat.grad), gfeat, **grad_tol(dname))
    # and the reference test's tolerances against autograd through the naive oracle
    np.testing.assert_allclose(N(tfvi.grad), sphere_naive[f'grad_fvi_{key}'], rtol=1e-3,
                               atol=1e-2)
    np.testing.assert_allclose(N(tfeat.grad), sphere_naive[f'grad_feat_{key}'], rtol=1e-3,
                               atol=1e-3)


@pytest.mark.parametrize('i', [0, 1, 2])
@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('with_valid', [0, 1])
def test_rasterize_soup(soup_naive, i, dname, with_valid):
    z = soup_naive
    key = f'soup{i}_{dname}'
    h, w = (int(v) for v in z[f'hw_{key}'])
    valid = z[f'valid_{key}'] if with_valid else None
    tfvi, tfeat, interp, face_idx, rw = _raster_case(z[f'fvz_{key}'], z[f'fvi_{key}'],
                                                     z[f'feat_{key}'], valid, h, w, dname)
    np.testing.assert_array_equal(N(face_idx), z[f'face_idx_{key}_valid{with_valid}'])
    g = z[f'grad_out_{key}_valid{with_valid}']
    interp.backward(T(g))
    gfvi, gfeat = oracle.rasterize_backward(g, N(face_idx), rw, z[f'fvi_{key}'],
                                            z[f'feat_{key}'], 1e-8)
    np.testing.assert_allclose(N(tfvi.grad), gfvi, **grad_tol(dname))
    np.testing.assert_allclose(N(tfeat.grad), gfeat, **grad_tol(dname))


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_packed_op_vs_oracle(sphere_inputs, dname):
    """_C.render.mesh.packed_rasterize_forward_cuda on the reference's packed inputs."""
    from kaolin_amd import _C
    s = sphere(sphere_inputs, dname, 0)
    valid = s['valid']
    bi, fi = np.nonzero(valid)
    counts = valid.sum(1)
    first = np.zeros(len(counts) + 1, np.int64)
    first[1:] = np.cumsum(counts)
    pfvi = (s['fvi'][bi, fi] * 1000).astype(s['fvi'].dtype)
    bbox = np.concatenate([pfvi.min(1), pfvi.max(1)], 1)
    pfvz, pfeat = s['fvz'][bi, fi], s['uvs'][bi, fi]
    ri, rf, rw = oracle.packed_rasterize_forward(H, W, pfvz, pfvi, bbox, pfeat, first, 1000, 1e-8)
    interp, sel, weights = _C.render.mesh.packed_rasterize_forward_cuda(
        H, W, T(pfvz), T(pfvi), T(bbox), T(pfeat), T(first), 1000, 1e-8)
    np.testing.assert_array_equal(N(sel), rf)
    np.testing.assert_array_equal(N(weights), rw)
    np.testing.assert_array_equal(N(interp), ri)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_rasterize_backward_op_vs_oracle(sphere_inputs, dname):
    """_C.render.mesh.rasterize_backward_cuda (general atomic form)."""
    from kaolin_amd import _C
    s = sphere(sphere_inputs, dname, 0)
    ri, rf, rw = oracle.rasterize(H, W, s['fvz'], s['fvi'], s['uvs'])
    g = np.random.default_rng(0).random(ri.shape).astype(ri.dtype)
    gfvi, gfeat = _C.render.mesh.rasterize_backward_cuda(T(g), T(ri), T(rf), T(rw), T(s['fvi']),
                                                         T(s['uvs']), 1e-8)
    ofvi, ofeat = oracle.rasterize_backward(g, rf, rw, s['fvi'], s['uvs'], 1e-8)
    np.testing.assert_allclose(N(gfvi), ofvi, **grad_tol(dname))
    np.testing.assert_allclose(N(gfeat), ofeat, **grad_tol(dname))


def test_rasterize_list_features(sphere_inputs):
    """test_rasterization.py:159-187: list of features is concatenated then split."""
    from kaolin_amd.render.mesh import rasterize
    s = sphere(sphere_inputs, 'f32', 0)
    uvs = T(s['uvs'])
    (a, m), fi = rasterize(H, W, T(s['fvz']), T(s['fvi']), [uvs, torch.ones_like(uvs[..., :1])])
    full, fi2 = rasterize(H, W, T(s['fvz']), T(s['fvi']),
                          torch.cat([uvs, torch.ones_like(uvs[..., :1])], -1))
    assert torch.equal(fi, fi2)
    assert torch.equal(a, full[..., :2]) and torch.equal(m, full[..., 2:])
    assert torch.allclose(m[..., 0], (fi >= 0).to(m.dtype), rtol=1e-5, atol=1e-5)


def test_face_vertices_z_gets_no_grad(sphere_inputs):
    from kaolin_amd.render.mesh import rasterize
    s = sphere(sphere_inputs, 'f32', 0)
    fvz = T(s['fvz']).requires_grad_(True)
    fvi = T(s['fvi']).requires_grad_(True)
    interp, _ = rasterize(H, W, fvz, fvi, T(s['uvs']))
    interp.sum().backward()
    assert fvz.grad is None or torch.all(fvz.grad == 0)
    assert fvi.grad is not None


# --------------------------------------------------------------------------------------------
# soft mask
# --------------------------------------------------------------------------------------------
def _large_bbox(fvi_scaled, boxlen, multiplier):
    pmin, pmax = fvi_scaled.min(-2), fvi_scaled.max(-2)
    bl = boxlen * multiplier
    return np.concatenate([pmin - bl, pmax + bl], -1).astype(fvi_scaled.dtype)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('sigmainv', [7000, 70])
@pytest.mark.parametrize('boxlen', [0.02, 0.2])
@pytest.mark.parametrize('multiplier', [1000, 100, 1])
@pytest.mark.parametrize('knum', [30, 20])
def test_simple_soft_mask_op(simple_golden, dname, sigmainv, boxlen, multiplier, knum):
    """test_dibr.py:109-140 on the _C op, plus bit-exact vs the oracle."""
    from kaolin_amd import _C
    g = simple_golden
    tag = f'{sigmainv}_{boxlen}'
    fvi = g['simple_fvi'].astype(DTYPES[dname])
    sfvi = (fvi * multiplier).astype(fvi.dtype)
    bbox = _large_bbox(sfvi, boxlen, multiplier)
    face_idx = g['simple_new_face_idx'].astype(np.int64)
    soft, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_cuda(
        T(sfvi), T(bbox), T(face_idx), sigmainv, knum, multiplier)
    np.testing.assert_allclose(N(soft), g[f'simple_soft_{tag}'], atol=1e-5, rtol=1e-5)
    np.testing.assert_array_equal(N(cidx), g[f'simple_close_idx_{tag}'][..., :knum])
    np.testing.assert_allclose(N(prob), g[f'simple_close_prob_{tag}'][..., :knum], atol=1e-5,
                               rtol=1e-5)
    np.testing.assert_array_equal(N(ctype), g[f'simple_close_type_{tag}'][..., :knum])
    osoft, oprob, ocidx, octype = oracle.soft_mask_forward_raw(sfvi, bbox, face_idx, sigmainv,
                                                               knum, multiplier)
    np.testing.assert_array_equal(N(cidx), ocidx)
    np.testing.assert_array_equal(N(ctype), octype)
    np.testing.assert_allclose(N(prob), oprob, rtol=1e-6, atol=1e-37)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('sigmainv', [7000, 70])
@pytest.mark.parametrize('boxlen', [0.02, 0.2])
@pytest.mark.parametrize('multiplier', [1000, 100, 1])
@pytest.mark.parametrize('knum', [30, 20])
@pytest.mark.parametrize('lists', [False, True])
def test_simple_soft_mask_backward(simple_golden, dname, sigmainv, boxlen, multiplier, knum,
                                   lists):
    """test_dibr.py:167-191 through the autograd API (both saved-state modes)."""
    from kaolin_amd.render.mesh import dibr, dibr_soft_mask
    g = simple_golden
    tag = f'{sigmainv}_{boxlen}'
    fvi = T(g['simple_fvi'].astype(DTYPES[dname])).requires_grad_(True)
    face_idx = T(g['simple_new_face_idx'].astype(np.int64))
    with dibr.close_lists(lists):
        soft = dibr_soft_mask(fvi, face_idx, sigmainv, boxlen, knum, multiplier)
        loss = mask_iou(soft, shifted_mask(face_idx))
        loss.backward()
    np.testing.assert_allclose(N(soft), g[f'simple_soft_{tag}'], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(N(fvi.grad), g[f'simple_grad_{tag}'], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('sigmainv', [7000, 70])
@pytest.mark.parametrize('boxlen', [0.02, 0.01])
@pytest.mark.parametrize('knum', [30, 40])
@pytest.mark.parametrize('multiplier', [1000, 100])
def test_sphere_soft_mask(sphere_inputs, sphere_softmask, dname, sigmainv, boxlen, knum,
                          multiplier):
    """test_dibr.py:309-394 plus bit-exact vs the oracle, forward (op + API) and backward."""
    from kaolin_amd import _C
    from kaolin_amd.render.mesh import dibr_soft_mask, rasterize
    s = sphere(sphere_inputs, dname, 0)
    gz = sphere_softmask
    tag = f'{sigmainv}_{boxlen}'
    feat = T(np.zeros(s['fvz'].shape + (1,), s['fvz'].dtype))
    _, face_idx = rasterize(H, W, T(s['fvz']), T(s['fvi']), feat)
    fi = N(face_idx)
    sfvi = (s['fvi'] * multiplier).astype(s['fvi'].dtype)
    bbox = _large_bbox(sfvi, boxlen, multiplier)
    soft, prob, cidx, ctype = _C.render.mesh.dibr_soft_mask_forward_cuda(
        T(sfvi), T(bbox), face_idx, sigmainv, knum, multiplier)
    np.testing.assert_allclose(N(soft), gz[f'soft_{tag}'], atol=1e-5, rtol=1e-5)
    np.testing.assert_array_equal(N(cidx), gz[f'close_idx_{tag}'][..., :knum])
    np.testing.assert_allclose(N(prob), gz[f'close_prob_{tag}'][..., :knum], atol=1e-5,
                               rtol=1e-5)
    assert np.mean(N(ctype) != gz[f'close_type_{tag}'][..., :knum]) <= 0.01
    osoft, oprob, ocidx, octype = oracle.soft_mask_forward_raw(sfvi, bbox, fi, sigmainv, knum,
                                                               multiplier)
    np.testing.assert_array_equal(N(cidx), ocidx)
    np.testing.assert_array_equal(N(ctype), octype)
    np.testing.assert_allclose(N(prob), oprob, rtol=1e-6, atol=1e-37)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    # autograd API (fused forward, face-gather backward)
    tfvi = T(s['fvi']).requires_grad_(True)
    asoft = dibr_soft_mask(tfvi, face_idx, sigmainv, boxlen, knum, multiplier)
    np.testing.assert_allclose(N(asoft), osoft, rtol=1e-6, atol=1e-7)
    gsoft = iou_grad_soft(N(asoft), fi)
    asoft.backward(T(gsoft))
    ograd = oracle.soft_mask_backward(gsoft, osoft, fi, oprob, ocidx, octype, sfvi, sigmainv,
                                      multiplier)
    np.testing.assert_allclose(N(tfvi.grad), ograd, **grad_tol(dname))
    np.testing.assert_allclose(N(tfvi.grad), gz[f'grad_{tag}'], rtol=1e-1, atol=1e-1)
    # general op backward on the op's own lists
    gop = _C.render.mesh.dibr_soft_mask_backward_cuda(T(gsoft), soft, face_idx, prob, cidx, ctype,
                                                      T(sfvi), sigmainv, multiplier)
    np.testing.assert_allclose(N(gop), ograd, **grad_tol(dname))


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('flip', [0, 1])
def test_dibr_rasterization_composition(sphere_inputs, dname, flip):
    """test_dibr.py:482-529: dibr_rasterization == rasterize(normals_z >= 0) + dibr_soft_mask."""
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_soft_mask, rasterize
    s = sphere(sphere_inputs, dname, flip)
    fvz, fvi, uvs, nz = T(s['fvz']), T(s['fvi']), T(s['uvs']), T(s['normals_z'])
    for sig, box, knum, mult in ((7000, 0.02, 30, 1000), (70, 0.01, 40, 100)):
        gi, gf = rasterize(H, W, fvz, fvi, uvs, nz >= 0., mult)
        gs = dibr_soft_mask(fvi, gf, sig, box, knum, mult)
        i, sm, f = dibr_rasterization(H, W, fvz, fvi, uvs, nz, sig, box, knum, mult)
        assert torch.equal(i, gi) and torch.equal(sm, gs) and torch.equal(f, gf)


# --------------------------------------------------------------------------------------------
# larger scale: bit-exact rows of full-size images, determinism, edge cases
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize('cfg', [(20, 26, 128, 128, 1), (100, 51, 256, 256, 2),
                                 (250, 101, 512, 512, 2)])
def test_uv_sphere_rows_vs_oracle(cfg):
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization
    n_lon, n_lat, h, w, B = cfg
    v = workloads.sphere_views(n_lon, n_lat, h, w, B, DEV)
    fvz, fvi, feats, nz = v['fvz'], v['fvi'], v['feats'], v['normals_z']
    interp, soft, face_idx = dibr_rasterization(h, w, fvz, fvi, feats, nz)
    interp2, soft2, face_idx2 = dibr_rasterization(h, w, fvz, fvi, feats, nz)
    assert torch.equal(interp, interp2) and torch.equal(soft, soft2)  # deterministic
    assert torch.equal(face_idx, face_idx2)
    # rows through the silhouette band and the centre
    rows = sorted({h // 2, h // 2 + 1, int(h * 0.12), int(h * 0.88), int(h * 0.3)})
    valid = (N(nz) >= 0)
    for r in rows:
        ri, rf, _ = oracle.rasterize(h, w, N(fvz), N(fvi), N(feats), valid, rows=(r, r + 1))
        np.testing.assert_array_equal(N(face_idx)[:, r], rf[:, r])
        np.testing.assert_array_equal(N(interp)[:, r], ri[:, r])
        osoft, _, _, _, _ = oracle.soft_mask_forward(N(fvi), N(face_idx), rows=(r, r + 1))
        np.testing.assert_allclose(N(soft)[:, r], osoft[:, r], rtol=1e-6, atol=1e-7)


def test_c3_view_full_fwd_bwd_vs_oracle():
    """One whole C3 view (50k-face uv-sphere, 512x512, knum 30): every output and both
    gradients of the fused dibr_rasterization against the oracle's brute-force loops."""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, first_view=3, total_views=8)
    fvz, feats, nz = v['fvz'], v['feats'].contiguous(), v['normals_z']
    fvi = v['fvi'].detach().clone().requires_grad_(True)
    feats.requires_grad_(True)
    interp, soft, face_idx = dibr_rasterization(h, w, fvz, fvi, feats, nz)
    g = torch.Generator().manual_seed(1)
    g_feat = torch.rand(interp.shape, generator=g).to(DEV)
    g_soft = torch.rand(soft.shape, generator=g).to(DEV)
    torch.autograd.backward([interp, soft], [g_feat, g_soft])
    valid = N(nz) >= 0
    ri, rf, rw = oracle.rasterize(h, w, N(fvz), N(fvi), N(feats), valid)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    osoft, oprob, ocidx, octype, sfvi = oracle.soft_mask_forward(N(fvi), rf)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)
    gr, gfeat = oracle.rasterize_backward(N(g_feat), rf, rw, N(fvi), N(feats), 1e-8)
    gs = oracle.soft_mask_backward(N(g_soft), osoft, rf, oprob, ocidx, octype, sfvi, 7000, 1000.)
    np.testing.assert_allclose(N(fvi.grad), gr + gs, rtol=1e-4, atol=1e-5 * np.abs(gr + gs).max())
    np.testing.assert_allclose(N(feats.grad), gfeat, rtol=1e-4, atol=1e-5 * np.abs(gfeat).max())


@pytest.mark.parametrize('sweep', [(3000., 0.05), (7000., 0.02), (17000., 0.02), (30000., 0.01)])
def test_c4_rows_sigma_sweep(sweep):
    """C4 shapes (50k faces at 1024x1024) across SURVEY §8(d)'s (sigmainv, boxlen) sweep: rows
    through the silhouette band bit-exact / 1e-6 vs the oracle; the fused path equals the
    reference composition with materialised close-face lists (op-form kernels) everywhere."""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_soft_mask
    sig, box = sweep
    h = w = 1024
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, first_view=1, total_views=8)
    fvz, fvi, feats, nz = v['fvz'], v['fvi'], v['feats'], v['normals_z']
    interp, soft, face_idx = dibr_rasterization(h, w, fvz, fvi, feats, nz, sig, box)
    soft_op = dibr_soft_mask(fvi, face_idx, sig, box)
    assert torch.equal(soft, soft_op)
    valid = N(nz) >= 0
    for r in (int(h * 0.1), int(h * 0.12), h // 2, int(h * 0.88)):
        ri, rf, _ = oracle.rasterize(h, w, N(fvz), N(fvi), N(feats), valid, rows=(r, r + 1))
        np.testing.assert_array_equal(N(face_idx)[:, r], rf[:, r])
        np.testing.assert_array_equal(N(interp)[:, r], ri[:, r])
        osoft, _, _, _, _ = oracle.soft_mask_forward(N(fvi), N(face_idx), sig, box,
                                                     rows=(r, r + 1))
        np.testing.assert_allclose(N(soft)[:, r], osoft[:, r], rtol=1e-6, atol=1e-7)


def test_c5_soup_rows_and_grad_consistency():
    """C5 stress soup (200k clustered faces, 512x512): dense central tiles far past the LDS list
    capacity.  Rows vs the oracle; gradients of the fused pair pipeline vs the op-form
    (materialised K-lists, atomic) kernels on the whole image."""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr, dibr_rasterization
    h = w = 512
    sz, si, sn = workloads.soup(200000, seed=3, batch=1)
    fvz, fvi0, nz = T(sz), T(si), T(sn)
    gen = torch.Generator().manual_seed(4)
    feats = torch.rand((1, 200000, 3, 3), generator=gen).to(DEV)
    g = torch.Generator().manual_seed(1)
    g_feat = torch.rand((1, h, w, 3), generator=g).to(DEV)
    g_soft = torch.rand((1, h, w), generator=g).to(DEV)
    grads = []
    for lists in (False, True):
        fvi = fvi0.clone().requires_grad_(True)
        with dibr.close_lists(lists):
            interp, soft, face_idx = dibr_rasterization(h, w, fvz, fvi, feats, nz)
            torch.autograd.backward([interp, soft], [g_feat, g_soft])
        grads.append(fvi.grad)
        if not lists:
            out = (interp, soft, face_idx)
    interp, soft, face_idx = out
    scale = grads[1].abs().max().item()
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-4, atol=1e-5 * scale)
    valid = N(nz) >= 0
    for r in (h // 2, h // 2 + 7, int(h * 0.3), int(h * 0.05)):
        ri, rf, _ = oracle.rasterize(h, w, sz.numpy(), si.numpy(), N(feats), valid,
                                     rows=(r, r + 1))
        np.testing.assert_array_equal(N(face_idx)[:, r], rf[:, r])
        np.testing.assert_array_equal(N(interp)[:, r], ri[:, r])
        osoft, _, _, _, _ = oracle.soft_mask_forward(si.numpy(), N(face_idx), rows=(r, r + 1))
        np.testing.assert_allclose(N(soft)[:, r], osoft[:, r], rtol=1e-6, atol=1e-7)


def test_dense_tile_overflow():
    """More faces on one tile than the LDS list holds (the CAP overflow path): 3000 large
    overlapping triangles on a 48x40 image."""
    from kaolin_amd.render.mesh import dibr_soft_mask, rasterize
    rng = np.random.default_rng(5)
    Fn, h, w = 3000, 48, 40
    c = rng.normal(0, 0.2, (1, Fn, 1, 2))
    fvi = (c + rng.uniform(-0.6, 0.6, (1, Fn, 3, 2))).astype(np.float32)
    fvz = (-2 - rng.uniform(0, 1, (1, Fn, 3))).astype(np.float32)
    feat = rng.random((1, Fn, 3, 2)).astype(np.float32)
    interp, face_idx = rasterize(h, w, T(fvz), T(fvi), T(feat))
    ri, rf, _ = oracle.rasterize(h, w, fvz, fvi, feat)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    empty = T(np.full((1, h, w), -1, np.int64))
    soft = dibr_soft_mask(T(fvi), empty, 7000, 0.05, 100, 1000.)
    osoft, _, _, _, _ = oracle.soft_mask_forward(fvi, np.full((1, h, w), -1, np.int64), 7000,
                                                 0.05, 100, 1000.)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)


def test_edge_cases():
    from kaolin_amd.render.mesh import dibr_rasterization, rasterize
    # no faces at all
    z = torch.zeros((2, 0, 3), device=DEV)
    i, f = rasterize(17, 13, z, torch.zeros((2, 0, 3, 2), device=DEV),
                     torch.zeros((2, 0, 3, 4), device=DEV))
    assert torch.all(f == -1) and torch.all(i == 0) and i.shape == (2, 17, 13, 4)
    # all faces culled, odd sizes, degenerate (zero area) and NaN faces
    fvi = np.array([[[[-0.5, -0.5], [0.5, -0.5], [0., 0.5]],
                     [[0.1, 0.1], [0.1, 0.1], [0.1, 0.1]],
                     [[np.nan, 0.], [0.5, 0.5], [0.2, 0.9]],
                     [[-0.9, -0.9], [0.9, -0.9], [0.9, 0.9]]]], np.float32)
    fvz = np.array([[[-2., -2., -2.], [-1., -1., -1.], [-3., -3., -3.], [-2.5, -2.5, -2.5]]],
                   np.float32)
    feat = np.random.default_rng(1).random((1, 4, 3, 3)).astype(np.float32)
    for valid in (None, np.array([[True, True, True, True]]), np.array([[0, 0, 0, 0]], bool),
                  np.array([[1, 0, 1, 0]], bool)):
        ti, tf = rasterize(19, 23, T(fvz), T(fvi), T(feat), None if valid is None else T(valid))
        ri, rf, _ = oracle.rasterize(19, 23, fvz, fvi, feat, valid)
        np.testing.assert_array_equal(N(tf), rf)
        np.testing.assert_array_equal(N(ti), ri)
    nz = T(np.array([[1., 1., 1., -1.]], np.float32))
    dibr_rasterization(19, 23, T(fvz), T(fvi), T(feat), nz)


# --------------------------------------------------------------------------------------------
# fp32 edge culling (kd_binning.hip raster_cull_coefs): cases aimed at its error margins --
# vertices on pixel centres (edge functions exactly 0 at many centres), slivers, huge and tiny
# coordinates, odd multipliers and eps.  Every output must stay bit-identical to the oracle.
# --------------------------------------------------------------------------------------------
def _cull_soup(kind, rng, h, w, Fn=400):
    if kind == 'grid':
        px = rng.integers(0, w, (1, Fn, 3))
        py = rng.integers(0, h, (1, Fn, 3))
        x = (2 * px + 1 - w) / w
        y = (h - 2 * py - 1) / h
        return np.stack([x, y], -1).astype(np.float32)
    if kind == 'grid_half':  # corners on pixel borders / half-way points
        px = rng.integers(0, 2 * w + 1, (1, Fn, 3))
        py = rng.integers(0, 2 * h + 1, (1, Fn, 3))
        return np.stack([(px - w) / w, (h - py) / h], -1).astype(np.float32)
    if kind == 'sliver':
        a = rng.uniform(-1, 1, (1, Fn, 1, 2))
        d = rng.normal(0, 0.6, (1, Fn, 1, 2))
        t = rng.uniform(0, 1, (1, Fn, 1, 1))
        n = rng.normal(0, 1, (1, Fn, 1, 2)) * 10.0 ** rng.uniform(-9, -2, (1, Fn, 1, 1))
        return np.concatenate([a, a + d, a + t * d + n], 2).astype(np.float32)
    if kind == 'tiny':
        c = rng.uniform(-1, 1, (1, Fn, 1, 2))
        return (c + rng.normal(0, 1, (1, Fn, 3, 2)) * 10.0 **
                rng.uniform(-7, -2, (1, Fn, 1, 1))).astype(np.float32)
    if kind == 'huge':
        c = rng.uniform(-1, 1, (1, Fn, 1, 2))
        s = 10.0 ** rng.uniform(0, 12, (1, Fn, 1, 1))
        return (c + rng.normal(0, 1, (1, Fn, 3, 2)) * s).astype(np.float32)
    raise ValueError(kind)


@pytest.mark.parametrize('kind', ['grid', 'grid_half', 'sliver', 'tiny', 'huge'])
@pytest.mark.parametrize('mult_eps', [(1000, 1e-8), (1, 1e-8), (1e-3, 1e-8), (1000, 1e3),
                                      (-1000, 1e-8), (1e6, 0.0), (7.5, 1e30)])
def test_raster_cull_margins(kind, mult_eps):
    from kaolin_amd.render.mesh import rasterize
    multiplier, eps = mult_eps
    rng = np.random.default_rng(zlib.crc32(f'{kind}/{multiplier}/{eps}'.encode()))
    h, w = 45, 53
    fvi = _cull_soup(kind, rng, h, w)
    Fn = fvi.shape[1]
    fvz = (-1 - rng.uniform(0, 1, (1, Fn, 3))).astype(np.float32)
    if kind == 'grid':  # many exact depth ties too
        fvz = np.round(fvz, 1).astype(np.float32)
    feat = rng.random((1, Fn, 3, 2)).astype(np.float32)
    interp, face_idx = rasterize(h, w, T(fvz), T(fvi), T(feat), multiplier=multiplier, eps=eps)
    ri, rf, rw = oracle.rasterize(h, w, fvz, fvi, feat, None, multiplier=multiplier, eps=eps)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)


@pytest.mark.parametrize('multiplier', [-1000., -1., 0.])
@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_nonpositive_multiplier(multiplier, dname):
    """Pixel centres run right-to-left / bottom-to-top (or collapse to 0): spans by exact search."""
    from kaolin_amd.render.mesh import dibr_soft_mask, rasterize
    dt = DTYPES[dname]
    rng = np.random.default_rng(11)
    h, w, Fn = 29, 37, 300
    c = rng.uniform(-1, 1, (1, Fn, 1, 2))
    fvi = (c + rng.normal(0, 0.15, (1, Fn, 3, 2))).astype(dt)
    fvz = (-1 - rng.uniform(0, 1, (1, Fn, 3))).astype(dt)
    feat = rng.random((1, Fn, 3, 2)).astype(dt)
    interp, face_idx = rasterize(h, w, T(fvz), T(fvi), T(feat), multiplier=multiplier)
    ri, rf, _ = oracle.rasterize(h, w, fvz, fvi, feat, None, multiplier=multiplier)
    np.testing.assert_array_equal(N(face_idx), rf)
    np.testing.assert_array_equal(N(interp), ri)
    soft = dibr_soft_mask(T(fvi), face_idx, 7000, 0.05, 30, multiplier)
    osoft, _, _, _, _ = oracle.soft_mask_forward(fvi, rf, 7000, 0.05, 30, multiplier)
    np.testing.assert_allclose(N(soft), osoft, rtol=1e-6, atol=1e-7)


def test_nonfinite_multiplier_rejected():
    from kaolin_amd.render.mesh import rasterize
    z = torch.zeros((1, 2, 3), device=DEV)
    with pytest.raises((RuntimeError, ValueError)):
        rasterize(8, 8, z, torch.zeros((1, 2, 3, 2), device=DEV),
                  torch.zeros((1, 2, 3, 1), device=DEV), multiplier=float('inf'))


# --------------------------------------------------------------------------------------------
# prepare_vertices: fused projection / gather / normals and the gather-form
# backward vs the reference's PyTorch composition in fp64 (tolerances: fp32 1e-5 relative,
# fp64 1e-10)
# --------------------------------------------------------------------------------------------
def _torch_prepare(vertices, faces, proj, tf):
    padded = torch.nn.functional.pad(vertices, (0, 1), mode='constant', value=1.)
    vc = padded @ tf
    pp = vc * proj.view(-1, 1, 3)
    vi = pp[:, :, :2] / pp[:, :, 2:3]
    B = vc.shape[0]
    fvc = vc[:, faces.reshape(-1)].reshape(B, faces.shape[0], 3, 3)
    fvi = vi[:, faces.reshape(-1)].reshape(B, faces.shape[0], 3, 2)
    n = torch.cross(fvc[:, :, 1] - fvc[:, :, 0], fvc[:, :, 2] - fvc[:, :, 0], dim=2)
    return fvc, fvi, n / (n.norm(dim=2, keepdim=True) + 1e-10)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('shared', [True, False])
@pytest.mark.parametrize('which', ['all', 'fvi'])
def test_prepare_vertices_vs_torch(dname, shared, which):
    import math

    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import prepare_vertices
    dt = TORCH_DTYPES[dname]
    verts, faces, _ = workloads.uv_sphere(30, 17, seed=4)
    B = 3
    cam = workloads.orbit_cameras(B, 0.4).to(DEV, dt)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV, dt)
    faces = faces.to(DEV)
    v = verts.to(DEV, dt)
    gen = torch.Generator().manual_seed(7)
    if not shared:
        v = v.unsqueeze(0) + 0.01 * torch.randn((B,) + v.shape, generator=gen).to(DEV, dt)
    else:
        v = v.unsqueeze(0)
    v1 = v.clone().requires_grad_(True)
    v2 = v.detach().double().clone().requires_grad_(True)
    out1 = prepare_vertices(v1, faces, proj, camera_transform=cam)
    out2 = _torch_prepare(v2, faces, proj.double(), cam.double())
    rtol = 1e-5 if dname == 'f32' else 1e-10
    if dname == 'f64':
        for a, b in zip(out1, out2):
            torch.testing.assert_close(a, b, rtol=rtol, atol=rtol)
    else:  # fp32: within 4x the reference composition's own fp32 error (thin-triangle normals)
        out32 = _torch_prepare(v.detach(), faces, proj, cam)
        for a, b, r in zip(out1, out2, out32):
            err = (a.double() - b).abs().max().item()
            err_ref = (r.double() - b).abs().max().item()
            assert err <= 4 * err_ref + 1e-6, (err, err_ref)
    g = [torch.randn(o.shape, generator=gen, dtype=torch.float64).to(DEV) for o in out2]
    if which == 'fvi':
        torch.autograd.backward(out1[1], g[1].to(dt))
        torch.autograd.backward(out2[1], g[1])
    else:
        torch.autograd.backward(out1, [x.to(dt) for x in g])
        torch.autograd.backward(out2, g)
    if dname == 'f64':
        torch.testing.assert_close(v1.grad, v2.grad, rtol=1e-9, atol=1e-9)
    else:
        # fp32 bar: no worse than 4x the reference composition's own fp32 error (the unit-normal
        # gradient is ill-conditioned on thin pole triangles) and 1e-5 of the gradient's scale
        v3 = v.detach().clone().requires_grad_(True)
        out3 = _torch_prepare(v3, faces, proj, cam)
        if which == 'fvi':
            torch.autograd.backward(out3[1], g[1].to(dt))
        else:
            torch.autograd.backward(out3, [x.to(dt) for x in g])
        err = (v1.grad.double() - v2.grad).abs().max().item()
        err_ref = (v3.grad.double() - v2.grad).abs().max().item()
        assert err <= 4 * err_ref + 1e-5 * v2.grad.abs().max().item(), (err, err_ref)


@pytest.mark.parametrize('dname', ['f32', 'f64'])
@pytest.mark.parametrize('shared', [True, False])
def test_prepare_vertices_high_degree_and_isolated(dname, shared):
    """Owner-workgroup vertex sums: a hub vertex in 900 faces (its CSR run spans four 256-entry
    workgroups), runs crossing workgroup boundaries, and vertices without faces (zero)."""
    import math

    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import prepare_vertices
    dt = TORCH_DTYPES[dname]
    gen = torch.Generator().manual_seed(11)
    n_rim, B = 900, 2
    ang = torch.arange(n_rim, dtype=torch.float64) * (2 * math.pi / n_rim)
    rim = torch.stack([torch.cos(ang), torch.sin(ang), 0.1 * torch.sin(3 * ang)], -1)
    # vertex 0 hub, 1..900 rim, 901..909 isolated
    verts = torch.cat([torch.tensor([[0., 0., 0.3]], dtype=torch.float64), rim,
                       torch.randn((9, 3), generator=gen, dtype=torch.float64)])
    i = torch.arange(n_rim)
    faces = torch.stack([torch.zeros_like(i), 1 + i, 1 + (i + 1) % n_rim], -1)
    # a second strip so runs of other vertices cross workgroup boundaries too
    faces = torch.cat([faces, torch.stack([1 + i, 1 + (i + 2) % n_rim, 1 + (i + 1) % n_rim], -1)])
    faces = faces[torch.randperm(faces.shape[0], generator=gen)].to(DEV)
    cam = workloads.orbit_cameras(B, 0.5).to(DEV, torch.float64)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV, torch.float64)
    v = verts.unsqueeze(0).to(DEV)
    if not shared:
        v = v + 0.01 * torch.randn((B,) + verts.shape, generator=gen, dtype=torch.float64).to(DEV)
    v1 = v.to(dt).clone().requires_grad_(True)
    v2 = v.to(dt).double().clone().requires_grad_(True)
    out1 = prepare_vertices(v1, faces, proj.to(dt), camera_transform=cam.to(dt))
    out2 = _torch_prepare(v2, faces, proj, cam)
    g = [torch.randn(o.shape, generator=gen, dtype=torch.float64).to(DEV) for o in out2]
    torch.autograd.backward(out1[1], g[1].to(dt))
    torch.autograd.backward(out2[1], g[1])
    assert torch.all(v1.grad[:, 901:] == 0)
    tol = 1e-9 if dname == 'f64' else 2e-4 * v2.grad.abs().max().item()
    torch.testing.assert_close(v1.grad.double(), v2.grad, rtol=tol, atol=tol)


def test_prepare_vertices_rot_trans_and_camera_grad():
    from kaolin_amd.render.mesh import prepare_vertices
    rng = torch.Generator().manual_seed(3)
    v = torch.randn((2, 50, 3), generator=rng).to(DEV)
    faces = torch.randint(0, 50, (80, 3), generator=rng).to(DEV)
    q, _ = torch.linalg.qr(torch.randn((2, 3, 3), generator=rng))
    rot = q.to(DEV)
    trans = torch.tensor([[0., 0., 4.], [0.5, -0.2, 5.]], device=DEV)
    proj = torch.tensor([[1.7], [1.7], [-1.]], device=DEV)
    fvc, fvi, n = prepare_vertices(v, faces, proj, camera_rot=rot, camera_trans=trans)
    vc = torch.matmul(v - trans.view(-1, 1, 3), rot.permute(0, 2, 1))
    torch.testing.assert_close(fvc, vc[:, faces.reshape(-1)].reshape(2, 80, 3, 3),
                               rtol=1e-5, atol=1e-5)
    tf = torch.randn((2, 4, 3), device=DEV, requires_grad=True)  # camera grads: composition
    fvc, fvi, n = prepare_vertices(v, faces, proj, camera_transform=tf)
    fvi.sum().backward()
    assert tf.grad is not None


@pytest.mark.parametrize('dname', ['f32', 'f64'])
def test_dibr_rasterization_fused_matches_composition(dname):
    """The fused dibr_rasterization (one binning pass, one backward buffer) against rasterize +
    dibr_soft_mask run separately: identical forward, gradients to summation-order tolerance."""
    import math

    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization, dibr_soft_mask, prepare_vertices, \
        rasterize
    dt = TORCH_DTYPES[dname]
    verts, faces, uvs = workloads.uv_sphere(40, 21, seed=2)
    B, h, w = 2, 96, 80
    cam = workloads.orbit_cameras(B, 0.5).to(DEV, dt)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV, dt)
    v = verts.to(DEV, dt).unsqueeze(0)
    fvc, fvi, nrm = prepare_vertices(v, faces.to(DEV), proj, camera_transform=cam)
    feats = torch.cat([uvs, torch.ones_like(uvs[..., :1])], -1).to(DEV, dt)
    feats = feats.unsqueeze(0).repeat(B, 1, 1, 1)
    gen = torch.Generator().manual_seed(5)
    g1 = torch.rand((B, h, w, 3), generator=gen, dtype=torch.float64).to(DEV, dt)
    g2 = torch.rand((B, h, w), generator=gen, dtype=torch.float64).to(DEV, dt)
    fvi_a = fvi.detach().clone().requires_grad_(True)
    ft_a = feats.clone().requires_grad_(True)
    i_a, s_a, f_a = dibr_rasterization(h, w, fvc[..., 2], fvi_a, ft_a, nrm[..., 2])
    torch.autograd.backward([i_a, s_a], [g1, g2])
    fvi_b = fvi.detach().clone().requires_grad_(True)
    ft_b = feats.clone().requires_grad_(True)
    i_b, f_b = rasterize(h, w, fvc[..., 2].contiguous(), fvi_b, ft_b, nrm[..., 2] >= 0)
    s_b = dibr_soft_mask(fvi_b, f_b)
    torch.autograd.backward([i_b, s_b], [g1, g2])
    assert torch.equal(f_a, f_b) and torch.equal(i_a, i_b) and torch.equal(s_a, s_b)
    tol = dict(rtol=1e-4, atol=1e-5) if dname == 'f32' else dict(rtol=1e-9, atol=1e-10)
    torch.testing.assert_close(fvi_a.grad, fvi_b.grad, **tol)
    torch.testing.assert_close(ft_a.grad, ft_b.grad, **tol)


@pytest.mark.parametrize('D', [3, 5])
def test_dibr_fused_launches_match_split_launches(D):
    """dibr_rasterization's one-launch forward (kd_dibr_fwd_tiles) and backward (kd_dibr_bwd)
    against the same tile bodies as separate launches (kd_set_test_forms) on a 50k-face
    mesh: identical forward outputs, gradients to summation-order tolerance.  (D = 5 keeps the
    fused forward and the split backward.)"""
    import math

    from kaolin_amd import _lib, workloads
    from kaolin_amd.render.mesh import dibr_rasterization, prepare_vertices
    verts, faces, uvs = workloads.uv_sphere(250, 101, seed=0)
    B, h, w = 3, 256, 192
    cam = workloads.orbit_cameras(B, 0.4).to(DEV)
    proj = workloads.generate_perspective_projection(math.pi / 4).to(DEV)
    fvc, fvi, nrm = prepare_vertices(verts.to(DEV).unsqueeze(0), faces.to(DEV), proj,
                                     camera_transform=cam)
    F = faces.shape[0]
    gen = torch.Generator().manual_seed(11)
    feats = torch.rand((B, F, 3, D), generator=gen).to(DEV)
    g1 = torch.rand((B, h, w, D), generator=gen).to(DEV)
    g2 = torch.rand((B, h, w), generator=gen).to(DEV)
    out = []
    try:
        for forms in (0, _lib.FORM_SPLIT_FWD | _lib.FORM_SPLIT_BWD):
            _lib.set_test_forms(forms)
            fa = fvi.detach().clone().requires_grad_(True)
            ft = feats.clone().requires_grad_(True)
            i, s, f = dibr_rasterization(h, w, fvc[..., 2], fa, ft, nrm[..., 2])
            torch.autograd.backward([i, s], [g1, g2])
            torch.cuda.synchronize()
            out.append((i, s, f, fa.grad, ft.grad))
    finally:
        _lib.set_test_forms(0)
    (i0, s0, f0, ga0, gf0), (i1, s1, f1, ga1, gf1) = out
    assert (s0 < 1).any() and (f0 >= 0).any()
    assert torch.equal(f0, f1) and torch.equal(i0, i1) and torch.equal(s0, s1)
    torch.testing.assert_close(ga0, ga1, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gf0, gf1, rtol=1e-4, atol=1e-5)
