"""CPU-only checks of the native boundary: the C-ABI library loads and exports every symbol
declared in include/kaolin_dibr.h; host-side argument validation of the torch shim."""
import ctypes

import pytest
import torch

from kaolin_amd import _lib


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = _lib.declared_symbols()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(lib, name), name
    # also visible to a plain dlopen (what a cgo / ctypes / N-API binding would use)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert getattr(raw, name) is not None


def test_version_and_workspace_size():
    lib = _lib.load()
    assert lib.kd_version() >= 1
    n = _lib.workspace_size(_lib.KD_WS_RASTER, 8, 512, 512, 8 * 50000, 50000)
    assert n > 8 * 50000 * 8  # spans + bins at least
    assert _lib.workspace_size(_lib.KD_WS_RASTER, -1, 1, 1, 1, 1) == 0


def test_shim_rejects_cpu_tensors_like_the_reference():
    from kaolin_amd import _C
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError):
        _C.render.mesh.packed_rasterize_forward_cuda(
            8, 8, x, torch.zeros(4, 3, 2), torch.zeros(4, 4), torch.zeros(4, 3, 1),
            torch.tensor([0, 4]), 1000, 1e-8)


def test_shim_rejects_bad_dtype_and_sizes():
    from kaolin_amd import _C
    with pytest.raises(RuntimeError):
        _C._sfx(torch.zeros(1, dtype=torch.float16), 'x')
    with pytest.raises(RuntimeError):
        _C._check_size('f', 'a', torch.zeros(2, 3), (2, 4))


def test_prepare_vertices_ranges_partition():
    """kd_prepare_vertices_ranges (host): ranges tile all entries, never split a vertex, hold at
    most `cap` entries unless a single vertex has more."""
    import numpy as np
    from kaolin_amd import _lib
    rng = np.random.default_rng(0)
    for cap in (1, 7, 256):
        deg = rng.integers(0, 12, 3000)
        deg[[5, 900, 2999]] = [0, 700, 300]  # isolated, hubs past the cap
        off = np.zeros(deg.size + 1, np.int64)
        np.cumsum(deg, out=off[1:])
        out = np.empty(deg.size + 2, np.int32)
        n = int(_lib.load().kd_prepare_vertices_ranges(off.ctypes.data, deg.size, cap,
                                                       out.ctypes.data))
        r = out[:n + 1].astype(np.int64)
        assert r[0] == 0 and r[-1] == off[-1] and np.all(np.diff(r) > 0)
        assert np.all(np.isin(r, off))  # boundaries fall between vertices
        for a, b in zip(r[:-1], r[1:]):
            if b - a > cap:  # only a single vertex may exceed the cap
                assert np.count_nonzero((off[:-1] >= a) & (off[:-1] < b) & (deg > 0)) == 1
    empty = np.zeros(4, np.int64)
    out = np.empty(5, np.int32)
    assert _lib.load().kd_prepare_vertices_ranges(empty.ctypes.data, 3, 256, out.ctypes.data) == 0


def test_production_library_reads_no_debug_flags():
    """The production library selects no kernel from debug flags (diagnostic build only); the
    launch-form test hook accepts only its KD_FORM_* bits."""
    lib = _lib.load()
    assert lib.kd_debug_set(0) == _lib.KD_OK
    assert lib.kd_debug_set(256) != _lib.KD_OK
    assert b'diagnostic' in lib.kd_last_error()
    assert lib.kd_set_test_forms(8) != _lib.KD_OK
    _lib.set_test_forms(_lib.FORM_SPLIT_FWD | _lib.FORM_SPLIT_BWD | _lib.FORM_SOFT_SPLIT)
    _lib.set_test_forms(0)


def test_tuning_hooks_reject_bad_values():
    """host-only setters: no GPU needed"""
    from kaolin_amd import _lib
    for fn, bad in ((_lib.load().kd_set_tile_history, 2), (_lib.load().kd_set_tile_split, 3),
                    (_lib.load().kd_set_coarse_tile, 8)):
        assert fn(bad) != 0
    _lib.set_tile_history(False)
    _lib.set_tile_history(True)
