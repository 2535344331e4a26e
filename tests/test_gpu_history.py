"""GPU: the tile cost history of the fused fp32 DIB-R forward (kd_set_tile_history).

Each call of the one-launch forward records its tiles' durations in a caller-owned buffer
(kd_tile_history_attach; kaolin_amd._C attaches one per device from the caching allocator), and
the next call of the same shape dispatches its tiles heaviest-first by them (tile_order) instead
of by the coarse bins' face counts.  Only the dispatch order changes, so the outputs must be
bit-identical to a call without history -- also when the history comes from another mesh of the
same shape (stale costs), with split tiles, and on images whose sides are not multiples of 16 --
and the gradients stay at the float atomics' bar.
"""
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
    _lib.set_tile_history(True)
    _lib.set_tile_split(0)


def _run(h, w, v, history):
    from kaolin_amd import _lib
    _lib.set_tile_history(history)
    try:
        return _fwd_bwd(h, w, v)
    finally:
        _lib.set_tile_history(True)


@pytest.mark.parametrize('views', [1, 8])
def test_history_matches_bin_count_order_c3(views):
    from kaolin_amd import workloads
    h = w = 512
    v = workloads.sphere_views(250, 101, h, w, views, DEV)
    ref = _run(h, w, v, False)
    _run(h, w, v, True)            # records the durations
    again = _run(h, w, v, True)    # dispatched by them
    _same(again, ref)


def test_stale_history_from_another_mesh():
    """same shape, other geometry: the recorded order is wrong for it, the results are not"""
    from kaolin_amd import workloads
    h = w = 512
    a = workloads.sphere_views(250, 101, h, w, 2, DEV)
    b = workloads.sphere_views(250, 101, h, w, 2, DEV, first_view=5, total_views=8)
    _run(h, w, a, True)
    stale = _run(h, w, b, True)
    _same(stale, _run(h, w, b, False))


@pytest.mark.parametrize('split', [1, 2])
@pytest.mark.parametrize('hw', [(136, 200), (9, 300)])
def test_history_ragged_vs_oracle(split, hw):
    from kaolin_amd import _lib, workloads
    h, w = hw
    v = workloads.sphere_views(120, 50, h, w, 1, DEV)
    _lib.set_tile_split(split)
    _run(h, w, v, True)
    out = _run(h, w, v, True)
    _check_view(h, w, 0, out)


def test_history_buffer_is_the_callers():
    """the forward records into the buffer the caller attached (the library allocates nothing),
    and with the buffer detached (no history) the outputs are the same"""
    from kaolin_amd import _lib, workloads
    h = w = 256
    v = workloads.sphere_views(100, 51, h, w, 2, DEV)
    buf = _lib.tile_history_buffer(torch.device(DEV))
    out = _run(h, w, v, True)
    torch.cuda.synchronize()
    assert buf.numel() == _lib.load().kd_tile_history_bytes()
    assert int((buf != 0).sum().item()) > 0, 'the forward did not record into the attached buffer'
    lib = _lib.load()
    stream = torch.cuda.current_stream(buf.device).cuda_stream
    assert lib.kd_tile_history_attach(stream, None, 0) == 0
    try:
        buf.zero_()
        none = _run(h, w, v, True)
        torch.cuda.synchronize()
        assert int((buf != 0).sum().item()) == 0, 'a detached buffer was written'
    finally:
        assert lib.kd_tile_history_attach(stream, buf.data_ptr(), buf.numel()) == 0
    _same(none, out)
    # too small a buffer is refused
    assert lib.kd_tile_history_attach(stream, buf.data_ptr(), 16) != 0


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason='needs two visible GPUs')
def test_history_on_a_device_other_than_the_current_one():
    """the forward's tensors (and stream) on cuda:1 while cuda:0 is current: the tile history
    and the CU count belong to the stream's device, so the outputs equal those of
    the same call made with cuda:1 current and no history"""
    from kaolin_amd import _lib, workloads
    from kaolin_amd.render.mesh import dibr_rasterization
    h = w = 256
    v = workloads.sphere_views(100, 51, h, w, 2, 'cuda:1')

    def run(current, history):
        _lib.set_tile_history(history)
        with torch.cuda.device(current):
            fvi = v['fvi'].detach().clone().requires_grad_(True)
            interp, soft, face_idx = dibr_rasterization(h, w, v['fvz'], fvi, v['feats'],
                                                        v['normals_z'])
            torch.autograd.backward([interp, soft], [torch.ones_like(interp),
                                                     torch.ones_like(soft)])
            torch.cuda.synchronize('cuda:1')
        return face_idx, interp, soft, fvi.grad

    run(0, True)
    other = run(0, True)   # dispatched by a history that must live on cuda:1
    ref = run(1, False)
    for x, y in zip(other[:3], ref[:3]):
        assert torch.equal(x, y)
    torch.testing.assert_close(other[3], ref[3], rtol=1e-4, atol=1e-5 * ref[3].abs().max().item())


def test_stream_device_resolution():
    """per-device state is keyed by the stream's device -- the null stream resolves to
    the current device, a stream to its own device, and the CU count is that device's"""
    import ctypes
    from kaolin_amd import _lib
    lib = _lib.load()
    cus = ctypes.c_int(0)
    assert lib.kd_stream_device(None, ctypes.byref(cus)) == torch.cuda.current_device()
    assert cus.value == torch.cuda.get_device_properties(0).multi_processor_count
    s = torch.cuda.Stream(device=0)
    assert lib.kd_stream_device(s.cuda_stream, None) == 0
    if torch.cuda.device_count() > 1:
        s1 = torch.cuda.Stream(device=1)
        assert lib.kd_stream_device(s1.cuda_stream, None) == 1
