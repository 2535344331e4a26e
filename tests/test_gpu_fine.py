"""GPU: the raster fine lists of the one-launch fp32 DIB-R forward (kd_binning.hpp FineLists).

The binning count writes each chunk's valid faces as 80-byte records grouped by the 16x16 tile
they touch, and the forward's raster phase reads its tile's records instead of walking the raster
set's ordered coarse bin (kd_set_test_forms KD_FORM_COARSE_RASTER keeps the coarse walk, for
these comparisons).  The raster's winner is a maximum of (depth, ~face) keys, so the order of a
tile's records cannot change it: every output must be bit-identical to the coarse walk and to the
oracle (the reference's brute-force loops), gradients at the float atomics' bar.  Covered: C3 at
1 and 8 views, split tiles, ragged images, a chunk whose records overflow its segment (faces
spanning many tiles) and the pool-limit hook that shrinks every segment (the overflowed rows walk
all faces of their view with the exact span filter), NaN depths (the sequential replay walks the
view's faces in order).
"""
import numpy as np
import pytest
import torch

from test_gpu_breadth import _check_view, _fwd_bwd
from test_gpu_split import _same

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(autouse=True)
def _restore():
    yield
    from kaolin_amd import _lib
    _lib.set_test_forms(0)
    _lib.set_tile_split(0)
    _lib.set_pool_limits(1.0, 1.0)


def _coarse(fn):
    from kaolin_amd import _lib
    _lib.set_test_forms(_lib.FORM_COARSE_RASTER)
    try:
        return fn()
    finally:
        _lib.set_test_forms(0)


@pytest.mark.parametrize('views', [1, 8])
def test_fine_lists_match_coarse_walk_c3(views):
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, views, DEV)
    fine = _fwd_bwd(h, w, v)
    coarse = _coarse(lambda: _fwd_bwd(h, w, v))
    _same(fine, coarse)


@pytest.mark.parametrize('split', [1, 2, 4])
def test_fine_lists_split_tiles_vs_oracle(split):
    from kaolin_amd import _lib, workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, 1, DEV, first_view=6, total_views=8)
    _lib.set_tile_split(split)
    out = _fwd_bwd(h, w, v)
    _check_view(h, w, 0, out)


@pytest.mark.parametrize('hw', [(136, 200), (72, 40), (9, 300), (250, 17)])
def test_fine_lists_ragged_vs_oracle(hw):
    from kaolin_amd import workloads
    h, w = hw
    v = workloads.sphere_views(60, 31, h, w, 2, DEV)
    out = _fwd_bwd(h, w, v)
    for b in range(2):
        _check_view(h, w, b, out)
    _same(out, _coarse(lambda: _fwd_bwd(h, w, v)))


def _big_faces(h, nface, seed=5):
    """nface random large triangles (each spanning most of the image: ~h^2/256 tiles), all front
    facing, random depths -- a chunk's records exceed kRecPerFace per face"""
    g = torch.Generator().manual_seed(seed)
    c = torch.rand((1, nface, 3, 2), generator=g) * 2.4 - 1.2
    # counter-clockwise winding (normal z >= 0) for every face
    a = (c[..., 1, 0] - c[..., 0, 0]) * (c[..., 2, 1] - c[..., 0, 1]) - \
        (c[..., 1, 1] - c[..., 0, 1]) * (c[..., 2, 0] - c[..., 0, 0])
    flip = a < 0
    c[flip] = c[flip][:, [0, 2, 1]]
    fvz = -2.0 - torch.rand((1, nface, 3), generator=g)
    feats = torch.rand((1, nface, 3, 3), generator=g)
    nz = torch.ones((1, nface))
    return dict(fvz=fvz.to(DEV), fvi=c.to(DEV), feats=feats.to(DEV), normals_z=nz.to(DEV))


def test_fine_segment_overflow_vs_oracle():
    h = w = 256
    v = _big_faces(h, 40)
    out = _fwd_bwd(h, w, v)
    _check_view(h, w, 0, out)
    _same(out, _coarse(lambda: _fwd_bwd(h, w, v)))


@pytest.mark.parametrize('lim', [0.0, 0.2])
def test_fine_pool_limit_overflow(lim):
    """kd_set_pool_limits shrinks every segment: (some or all) rows overflow and their tiles walk
    the view's faces; the outputs stay those of the default run"""
    from kaolin_amd import _lib, workloads
    h = w = 256
    v = workloads.sphere_views(100, 51, h, w, 2, DEV)
    ref = _fwd_bwd(h, w, v)
    _lib.set_pool_limits(lim, 1.0)
    got = _fwd_bwd(h, w, v)
    _lib.set_pool_limits(1.0, 1.0)
    _same(got, ref)
    _check_view(h, w, 1, got)


def test_fine_lists_nan_depth_replay():
    """a NaN depth makes its pixels replay the reference's sequential loop, which with fine
    lists walks every face of the view in order"""
    from kaolin_amd import workloads
    h = w = 128
    v = workloads.sphere_views(40, 21, h, w, 2, DEV)
    fvz = v['fvz'].clone()
    fvz[0, ::7, 1] = float('nan')
    v = dict(v, fvz=fvz)
    out = _fwd_bwd(h, w, v)
    for b in range(2):
        _check_view(h, w, b, out)
    coarse = _coarse(lambda: _fwd_bwd(h, w, v))
    for x, y in zip(out[4:7], coarse[4:7]):
        assert torch.equal(torch.nan_to_num(x, 7.), torch.nan_to_num(y, 7.))
