"""kaolin_amd -- MI355X-native (gfx950) DIB-R differentiable rasterization hot path.

Drop-in for the reference's ``kaolin.render.mesh`` rasterize / dibr_soft_mask /
dibr_rasterization (ian287913/kaolin 0.12.0) and its native ops ``kaolin._C.render.mesh.*``.
Kernels: hand-written HIP in kaolin_amd/csrc, exported through the C ABI in
include/kaolin_dibr.h and bound here with ctypes (kaolin_amd/_lib.py).
"""
from . import _C  # noqa: F401
from . import render  # noqa: F401
from . import metrics  # noqa: F401

__version__ = '0.1.0'
