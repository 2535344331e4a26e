"""GPU: split tiles of the fused fp32 DIB-R forward (kd_dibr_fwd_tiles SPLIT, kd_set_tile_split)
and the 16-px coarse bins of small batches (kd_set_coarse_tile).

With 2 or 4 workgroups per 16x16 tile (half / quarter tiles, several waves per 8x8 sub-tile
sharing its face chunks), the forward must produce exactly what the one-workgroup tile produces:
face_idx, interpolated features and the soft mask bit-identical (the raster winner is a key
maximum; pass A keeps each pixel's first K close faces in face order across the roles'
chunks; the probabilities and the ordered product are the same expressions), gradients at the
float atomics' bar (the records sit in other places, so the backward's sums run in another
order).  Also against the oracle (the reference's brute-force loops, oracle/dibr_oracle.c) on
whole views, with image sides that are not multiples of 16 (parts beyond the image), and with
the fused mask_iou.
"""
import numpy as np
import pytest
import torch

from test_gpu_breadth import _check_view, _fwd_bwd

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def N(t):
    return t.detach().cpu().numpy()


@pytest.fixture(autouse=True)
def _restore_split():
    yield
    from kaolin_amd import _lib
    _lib.set_tile_split(0)
    _lib.set_coarse_tile(0)


def _with_split(split, fn):
    from kaolin_amd import _lib
    _lib.set_tile_split(split)
    try:
        return fn()
    finally:
        _lib.set_tile_split(0)


def _same(a, b):
    """(fvz, fvi, feats, nz, interp, soft, face_idx, g_feat, g_soft) of two runs"""
    for x, y in zip(a[4:7], b[4:7]):
        assert torch.equal(x, y)
    for x, y in ((a[1].grad, b[1].grad), (a[2].grad, b[2].grad)):
        ref = N(y)
        np.testing.assert_allclose(N(x), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


@pytest.mark.parametrize('views', [1, 2])
@pytest.mark.parametrize('split', [2, 4])
def test_split_matches_whole_tiles_c3(views, split):
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, views, DEV)
    one = _with_split(1, lambda: _fwd_bwd(h, w, v))
    many = _with_split(split, lambda: _fwd_bwd(h, w, v))
    _same(many, one)


@pytest.mark.parametrize('split', [2, 4])
def test_split_c3_view_vs_oracle(split):
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, first_view=3, total_views=8)
    out = _with_split(split, lambda: _fwd_bwd(h, w, v))
    _check_view(h, w, 0, out)


@pytest.mark.parametrize('split', [2, 4])
@pytest.mark.parametrize('hw', [(136, 200), (72, 40), (9, 300)])
def test_split_ragged_image_vs_oracle(split, hw):
    """sides not multiples of 16 or 8: parts and sub-tiles partly or wholly beyond the image"""
    from kaolin_amd import workloads
    h, w = hw
    v = workloads.sphere_views(60, 31, h, w, 2, DEV)
    out = _with_split(split, lambda: _fwd_bwd(h, w, v))
    for b in range(2):
        _check_view(h, w, b, out)
    one = _with_split(1, lambda: _fwd_bwd(h, w, v))
    _same(out, one)


@pytest.mark.parametrize('knum', [1, 7, 32])
def test_split_knum(knum):
    """first-K across the roles' chunks: K reached inside a group of chunks"""
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization
    h = w = 256
    v = workloads.sphere_views(250, 101, h, w, 1, DEV)

    def run():
        fvi = v['fvi'].detach().clone().requires_grad_(True)
        feats = v['feats'].contiguous().clone().requires_grad_(True)
        interp, soft, face_idx = dibr_rasterization(h, w, v['fvz'], fvi, feats, v['normals_z'],
                                                    7000., 0.05, knum)
        g = torch.Generator().manual_seed(5)
        gs = torch.rand(soft.shape, generator=g).to(DEV)
        torch.autograd.backward([soft], [gs])
        torch.cuda.synchronize()
        return interp, soft, face_idx, fvi.grad

    ref = _with_split(1, run)
    for split in (2, 4):
        got = _with_split(split, run)
        for x, y in zip(got[:3], ref[:3]):
            assert torch.equal(x, y)
        r = N(ref[3])
        np.testing.assert_allclose(N(got[3]), r, rtol=1e-4, atol=1e-5 * np.abs(r).max())


@pytest.mark.parametrize('split', [2, 4])
def test_split_fused_iou(split):
    from kaolin_amd import workloads
    from kaolin_amd.render.mesh import dibr_rasterization_with_mask_iou
    h = w = 256
    v = workloads.sphere_views(100, 51, h, w, 2, DEV)
    gt = torch.zeros((2, h, w), device=DEV)
    gt[:, 60:200, 50:190] = 1.

    def run():
        fvi = v['fvi'].detach().clone().requires_grad_(True)
        feats = v['feats'].contiguous().clone().requires_grad_(True)
        interp, soft, face_idx, loss = dibr_rasterization_with_mask_iou(
            h, w, v['fvz'], fvi, feats, v['normals_z'], gt)
        loss.backward()
        torch.cuda.synchronize()
        return interp, soft, face_idx, loss, fvi.grad

    ref = _with_split(1, run)
    got = _with_split(split, run)
    for x, y in zip(got[:3], ref[:3]):
        assert torch.equal(x, y)
    np.testing.assert_allclose(N(got[3]), N(ref[3]), rtol=1e-6)
    r = N(ref[4])
    np.testing.assert_allclose(N(got[4]), r, rtol=1e-4, atol=1e-5 * np.abs(r).max())


def test_split_hook_rejects_bad_values():
    from kaolin_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.set_tile_split(3)


def _with_ct(px, fn):
    from kaolin_amd import _lib
    _lib.set_coarse_tile(px)
    try:
        return fn()
    finally:
        _lib.set_coarse_tile(0)


@pytest.mark.parametrize('views', [1, 8])
def test_coarse_tile_16_matches_32_c3(views):
    """16-px coarse bins (each fine tile's own bin) against the 32-px bins: the walks keep the
    same faces in the same order, so every output is bit-identical"""
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, views, DEV)
    a = _with_ct(32, lambda: _fwd_bwd(h, w, v))
    b = _with_ct(16, lambda: _fwd_bwd(h, w, v))
    _same(b, a)


@pytest.mark.parametrize('hw', [(136, 200), (520, 72)])
def test_coarse_tile_16_ragged_vs_oracle(hw):
    """16-px bins on sides that are not multiples of 16 (and one side past 32 bins: 32-px bins)"""
    from kaolin_amd import workloads
    h, w = hw
    v = workloads.sphere_views(60, 31, h, w, 2, DEV)
    out = _with_ct(16, lambda: _fwd_bwd(h, w, v))
    for b in range(2):
        _check_view(h, w, b, out)


def test_coarse_tile_changed_between_forward_and_backward():
    """the backward finds its forward's records whatever coarse tile it would choose (the pair
    buffers lead the workspace)"""
    from kaolin_amd import _lib, workloads
    from kaolin_amd.render.mesh import dibr_rasterization
    h = w = 256
    v = workloads.sphere_views(100, 51, h, w, 2, DEV)
    ref = _with_ct(16, lambda: _fwd_bwd(h, w, v))
    fvi = v['fvi'].detach().clone().requires_grad_(True)
    feats = v['feats'].contiguous().clone().requires_grad_(True)
    _lib.set_coarse_tile(16)
    try:
        interp, soft, face_idx = dibr_rasterization(h, w, v['fvz'], fvi, feats, v['normals_z'])
        _lib.set_coarse_tile(32)
        torch.autograd.backward([interp, soft], [ref[7], ref[8]])
        torch.cuda.synchronize()
    finally:
        _lib.set_coarse_tile(0)
    assert torch.equal(face_idx, ref[6]) and torch.equal(soft, ref[5])
    for x, y in ((fvi.grad, ref[1].grad), (feats.grad, ref[2].grad)):
        r = N(y)
        np.testing.assert_allclose(N(x), r, rtol=1e-4, atol=1e-5 * np.abs(r).max())


def test_coarse_tile_hook_rejects_bad_values():
    from kaolin_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.set_coarse_tile(8)
