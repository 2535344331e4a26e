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
