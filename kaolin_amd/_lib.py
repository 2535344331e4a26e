"""ctypes binding of the C ABI in include/kaolin_dibr.h (kaolin_amd/lib/libkaolin_dibr.so).

The library is loaded from the package tree (never from site-packages).  There is no fallback:
if the library is missing or a call fails, a RuntimeError is raised.
"""
import ctypes
import os
import re
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
# KAOLIN_AMD_DIAG=1 (tools/ only): the diagnostic build with the device ablation switches
LIB_PATH = os.path.join(_PKG, 'lib', 'libkaolin_dibr_diag.so'
                        if os.environ.get('KAOLIN_AMD_DIAG') == '1' else 'libkaolin_dibr.so')
HEADER = os.path.join(os.path.dirname(_PKG), 'include', 'kaolin_dibr.h')

KD_OK = 0
KD_WS_RASTER_PACKED = 1
KD_WS_RASTER = 2
KD_WS_SOFT_MASK = 3

_lib = None
_lock = threading.Lock()

c_int, c_float, c_double, c_i64, c_size, c_p = (ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                                ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p)

# argument signatures (everything pointer-like is c_void_p)
_SIGS = {
    'kd_packed_rasterize_forward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p, c_p,
                                    c_float, c_float, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_rasterize_forward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p, c_double,
                             c_float, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_rasterize_backward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p, c_p,
                              c_float, c_p, c_p, c_p],
    'kd_dibr_soft_mask_forward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_float,
                                  c_float, c_p, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_dibr_soft_mask_forward_fused': [c_int, c_int, c_int, c_i64, c_int, c_p, c_double,
                                        c_double, c_p, c_float, c_p, c_p, c_p, c_p, c_p, c_int,
                                        c_p, c_size, c_p],
    'kd_dibr_soft_mask_backward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p, c_p,
                                   c_p, c_p, c_float, c_float, c_p, c_p],
    'kd_dibr_rasterization_forward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_i64, c_i64, c_p,
                                      c_p, c_p, c_i64, c_double, c_float, c_float, c_double,
                                      c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_p, c_p, c_size,
                                      c_p],
    'kd_dibr_rasterization_forward_lists': [c_int, c_int, c_int, c_i64, c_int, c_p, c_i64, c_i64,
                                            c_p, c_p, c_p, c_i64, c_double, c_float, c_float,
                                            c_double, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                            c_p, c_size, c_p],
    'kd_dibr_rasterization_forward_vertices': [c_int, c_int, c_int, c_int, c_i64, c_i64, c_int,
                                               c_p, c_p, c_p, c_p, c_p, c_double, c_float,
                                               c_float, c_double, c_int, c_p, c_p, c_p, c_p, c_p,
                                               c_p, c_p, c_int, c_p, c_p, c_p, c_size, c_p],
    'kd_dibr_rasterization_backward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p,
                                       c_p, c_p, c_p, c_float, c_double, c_double, c_float,
                                       c_int, c_p, c_p, c_int, c_p, c_size, c_p],
    'kd_dibr_rasterization_iou_forward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_i64, c_i64,
                                          c_p, c_p, c_p, c_i64, c_double, c_float, c_float,
                                          c_double, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                          c_int, c_p, c_p, c_p, c_size, c_p],
    'kd_dibr_rasterization_iou_backward': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p,
                                           c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_float, c_double,
                                           c_double, c_float, c_int, c_p, c_p, c_int, c_p,
                                           c_size, c_p],
    'kd_dibr_rasterization_backward_vertices': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p,
                                                c_p, c_p, c_p, c_p, c_p, c_float, c_double,
                                                c_double, c_float, c_int, c_int, c_i64, c_p,
                                                c_p, c_p, c_p, c_p, c_p, c_int, c_p, c_size,
                                                c_p],
    'kd_prepare_vertices_forward': [c_int, c_int, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p,
                                    c_p, c_p],
    'kd_prepare_vertices_backward': [c_int, c_int, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p,
                                     c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    'kd_dibr_rasterization_soft_backward_lists': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p,
                                                  c_p, c_p, c_p, c_p, c_p, c_float, c_float, c_p,
                                                  c_p, c_size, c_p],
    'kd_prepare_vertices_backward_vertices': [c_int, c_int, c_i64, c_i64, c_p, c_p, c_p, c_p,
                                              c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p],
    'kd_dibr_soft_mask_backward_binned': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p,
                                          c_double, c_double, c_float, c_p, c_p, c_size, c_int,
                                          c_p],
    'kd_mask_iou_forward': [c_int, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_mask_iou_backward': [c_int, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    'kd_texture_mapping_forward': [c_int, c_i64, c_int, c_int, c_int, c_p, c_p, c_i64, c_int,
                                   c_p, c_p],
    'kd_rast_interpolate': [c_int, c_int, c_int, c_i64, c_int, c_p, c_p, c_p, c_p, c_p, c_p],
    'kd_deftet_sparse_render_forward': [c_int, c_i64, c_i64, c_int, c_int, c_p, c_p, c_p, c_p,
                                        c_p, c_float, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_deftet_sparse_render_forward_raw': [c_int, c_i64, c_i64, c_int, c_p, c_p, c_p, c_p, c_p,
                                            c_float, c_p, c_p, c_p, c_p, c_p, c_size, c_p],
    'kd_deftet_sparse_render_backward': [c_int, c_i64, c_i64, c_int, c_int, c_p, c_p, c_p, c_p,
                                         c_p, c_float, c_p, c_p, c_p],
    'kd_texture_mapping_backward': [c_int, c_i64, c_int, c_int, c_int, c_p, c_p, c_i64, c_int,
                                    c_i64, c_p, c_p, c_p, c_p],
    'kd_texture_mapping_backward_tiled': [c_int, c_i64, c_int, c_int, c_int, c_p, c_p, c_i64,
                                          c_int, c_p, c_p, c_p, c_p, c_size, c_p],
}


def load():
    """Load (once) and return the ctypes library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f'kaolin_amd: native library {LIB_PATH} is missing; build it with '
                    f'`python -c "import __graft_entry__ as g; g.build()"` (hipcc, gfx950)')
            lib = ctypes.CDLL(LIB_PATH)
            lib.kd_workspace_size.argtypes = [c_int, c_int, c_int, c_int, c_i64, c_i64]
            lib.kd_workspace_size.restype = c_size
            lib.kd_soft_mask_workspace_size.argtypes = [c_int, c_int, c_int, c_i64, c_int, c_int]
            lib.kd_soft_mask_workspace_size.restype = c_size
            lib.kd_dibr_workspace_size.argtypes = [c_int, c_int, c_int, c_i64, c_int, c_int]
            lib.kd_dibr_workspace_size.restype = c_size
            lib.kd_dibr_pair_count.argtypes = [c_p, c_int, c_int, c_int, c_i64, c_int, c_int, c_p]
            lib.kd_dibr_pair_count.restype = c_i64
            lib.kd_mask_iou_workspace_size.argtypes = [c_int, c_i64, c_int]
            lib.kd_mask_iou_workspace_size.restype = c_size
            lib.kd_deftet_workspace_size.argtypes = [c_int, c_i64, c_int]
            lib.kd_deftet_workspace_size.restype = c_size
            lib.kd_texture_mapping_backward_workspace_size.argtypes = [c_int, c_i64, c_int, c_int,
                                                                       c_int]
            lib.kd_texture_mapping_backward_workspace_size.restype = c_size
            lib.kd_last_error.argtypes = []
            lib.kd_last_error.restype = ctypes.c_char_p
            lib.kd_version.restype = c_int
            lib.kd_profile_enable.argtypes = [c_int]
            lib.kd_profile_enable.restype = None
            lib.kd_profile_collect.argtypes = [c_p, c_p, c_int]
            lib.kd_profile_collect.restype = c_int
            lib.kd_profile_kernel_name.argtypes = [c_int]
            lib.kd_profile_kernel_name.restype = ctypes.c_char_p
            lib.kd_debug_set.argtypes = [c_int]
            lib.kd_debug_set.restype = c_int
            lib.kd_debug_buffer.argtypes = [c_p]
            lib.kd_debug_buffer.restype = c_int
            lib.kd_set_pool_limits.argtypes = [ctypes.c_double, ctypes.c_double]
            lib.kd_set_pool_limits.restype = c_int
            lib.kd_set_test_forms.argtypes = [c_int]
            lib.kd_set_test_forms.restype = c_int
            lib.kd_set_tile_split.argtypes = [c_int]
            lib.kd_set_tile_split.restype = c_int
            lib.kd_set_coarse_tile.argtypes = [c_int]
            lib.kd_set_coarse_tile.restype = c_int
            lib.kd_set_tile_history.argtypes = [c_int]
            lib.kd_set_tile_history.restype = c_int
            lib.kd_stream_device.argtypes = [c_p, c_p]
            lib.kd_stream_device.restype = c_int
            lib.kd_tile_history_bytes.argtypes = []
            lib.kd_tile_history_bytes.restype = c_size
            lib.kd_tile_history_attach.argtypes = [c_p, c_p, c_size]
            lib.kd_tile_history_attach.restype = c_int
            lib.kd_prepare_vertices_ranges.argtypes = [c_p, c_i64, ctypes.c_int32, c_p]
            lib.kd_prepare_vertices_ranges.restype = c_i64
            # diagnostic build only (A/B of kernel variants under the test suite): KD_DEBUG_FLAGS
            if os.environ.get('KD_DEBUG_FLAGS') and LIB_PATH.endswith('_diag.so'):
                lib.kd_debug_set(int(os.environ['KD_DEBUG_FLAGS'], 0))
            for base, sig in _SIGS.items():
                for sfx in ('f32', 'f64'):
                    fn = getattr(lib, f'{base}_{sfx}')
                    fn.argtypes = sig
                    fn.restype = c_int
            _lib = lib
    return _lib


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != KD_OK:
        msg = load().kd_last_error().decode(errors='replace')
        raise RuntimeError(f'{name} failed ({rc}): {msg}')


def workspace_size(kind, B, H, W, n_total, max_per_view):
    return int(load().kd_workspace_size(kind, B, H, W, n_total, max_per_view))


def soft_mask_workspace_size(B, H, W, F, knum, double_precision):
    return int(load().kd_soft_mask_workspace_size(B, H, W, F, knum, 1 if double_precision else 0))


def texture_backward_workspace_size(B, N, Ht, Wt, shared_texture):
    return int(load().kd_texture_mapping_backward_workspace_size(B, N, Ht, Wt,
                                                                 1 if shared_texture else 0))


def set_pool_limits(bins=1.0, pairs=1.0):
    """Fractions of the bin and record pools a forward may use (kd_set_pool_limits): a test
    hook that forces the overflow paths; 1, 1 restores the default."""
    global _pool_limited
    call_plain = load().kd_set_pool_limits(float(bins), float(pairs))
    if call_plain != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))
    _pool_limited = float(bins) < 1.0 or float(pairs) < 1.0


_pool_limited = False

# kd_set_test_forms bits (include/kaolin_dibr.h KD_FORM_*)
FORM_SPLIT_FWD, FORM_SPLIT_BWD, FORM_SOFT_SPLIT = 1, 2, 4


def set_test_forms(forms=0):
    """Run dibr_rasterization through the separate launches its one-launch kernels fuse
    (kd_set_test_forms, a test hook); 0 restores the default."""
    if load().kd_set_test_forms(int(forms)) != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))


def set_tile_split(split=0):
    """Workgroups per tile of the fused fp32 forward (kd_set_tile_split, a test and tuning hook):
    1, 2 or 4; 0 restores the automatic choice."""
    if load().kd_set_tile_split(int(split)) != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))


def set_coarse_tile(px=0):
    """dibr_rasterization's coarse bin edge (kd_set_coarse_tile, a test and tuning hook): 16 or
    32 pixels; 0 restores the default (32).  Hold it between a forward and its backward."""
    if load().kd_set_coarse_tile(int(px)) != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))


def set_tile_history(on=True):
    """Dispatch the fused fp32 forward's tiles by the previous same-shape call's tile durations
    (kd_set_tile_history, a tuning hook; on by default).  Results never depend on it."""
    if load().kd_set_tile_history(1 if on else 0) != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))


_history = {}  # device index -> the caller-owned tile history buffer (kd_tile_history_attach)


def tile_history_buffer(dev):
    """The tile history buffer attached for `dev` (a torch.device), allocating and attaching it
    on first use -- caller-owned memory from the caching allocator, held for the process so that
    captured graphs keep a valid address.  None inside a stream capture before one exists (no
    allocation there; that call runs without history)."""
    import torch
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    buf = _history.get(idx)
    if buf is not None:
        return buf
    if torch.cuda.is_current_stream_capturing():
        return None
    lib = load()
    with _lock:
        buf = _history.get(idx)
        if buf is None:
            nb = int(lib.kd_tile_history_bytes())
            d = torch.device('cuda', idx)
            buf = torch.zeros((nb,), dtype=torch.uint8, device=d)
            rc = lib.kd_tile_history_attach(torch.cuda.current_stream(d).cuda_stream,
                                            buf.data_ptr(), nb)
            if rc != KD_OK:
                raise RuntimeError(lib.kd_last_error().decode(errors='replace'))
            _history[idx] = buf
    return buf


def debug_set(flags):
    """Diagnostic ablation flags (kd_debug_set): the diagnostic library only (KAOLIN_AMD_DIAG=1,
    tools/); the production library refuses nonzero flags, and that refusal is raised here."""
    if load().kd_debug_set(int(flags)) != KD_OK:
        raise RuntimeError(load().kd_last_error().decode(errors='replace'))


def pool_limits_active():
    """True while set_pool_limits holds a pool below its full size (the test hook)."""
    return _pool_limited


def split_soft_mask_forced():
    """True when a diagnostic flag (KD_DEBUG_FLAGS bit 4096) forces the split soft-mask
    pipeline, which the fused mask_iou cannot use."""
    return bool(int(os.environ.get('KD_DEBUG_FLAGS', '0'), 0) & 4096)


def profile_enable(on=True):
    """Record HIP events around every library launch (see kd_profile_enable)."""
    load().kd_profile_enable(1 if on else 0)


def profile_collect():
    """{kernel name: (total ms, launches)} for the launches recorded since the last collect."""
    lib = load()
    n = 64
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    k = lib.kd_profile_collect(ctypes.cast(ms, c_p), ctypes.cast(cnt, c_p), n)
    return {lib.kd_profile_kernel_name(i).decode(): (ms[i], cnt[i]) for i in range(k) if cnt[i]}


def declared_symbols():
    """Every function name declared in include/kaolin_dibr.h."""
    with open(HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r'\b(kd_[a-z0-9_]+)\s*\(', text)))
