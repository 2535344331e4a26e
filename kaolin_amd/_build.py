"""Builds kaolin_amd/lib/libkaolin_dibr.so (the C-ABI library, HIP for gfx950) in-tree.

hipcc cross-compiles for gfx950 without a GPU.  Flags that are part of the numerics contract:
  -ffp-contract=off  no FMA contraction (the reference expressions are evaluated as written)
  no -ffast-math, no -fgpu-flush-denormals-to-zero
and one code-generation guard:
  -mllvm -disable-promote-alloca-to-lds  the AMDGPU pass that moves small private arrays into LDS
      (256 lanes x the array) fires or not depending on register pressure; in kd_bin_count it
      turned the 8-float cull array into 8 KB of LDS traffic per workgroup (30 -> 51 us)
"""
import concurrent.futures
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
LIBDIR = os.path.join(PKG, 'lib')
LIB = os.path.join(LIBDIR, 'libkaolin_dibr.so')
OBJDIR = os.path.join(PKG, 'build')
# the diagnostic variant (-DKD_DIAG=1: device ablation switches, per-tile clocks) for tools/ only
LIB_DIAG = os.path.join(LIBDIR, 'libkaolin_dibr_diag.so')
OBJDIR_DIAG = os.path.join(PKG, 'build_diag')

SOURCES = ['kd_capi.cpp', 'kd_binning.hip', 'kd_raster.hip', 'kd_softmask.hip', 'kd_softpair.hip',
           'kd_prepare.hip', 'kd_dibr.hip', 'kd_metrics.hip', 'kd_texture.hip',
           'kd_rastcompat.hip', 'kd_deftet.hip']
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith('.hpp'))  # every source depends on all
ARCH = os.environ.get('KAOLIN_AMD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', f'--offload-arch={ARCH}',
         '-mllvm', '-disable-promote-alloca-to-lds',
         '-Wall', '-Wno-unused-function', '-Wno-unused-result']

# per-source flags, each measured on one box against the default scheduler (tools/ab_variant.sh +
# tools/rocprof_flags.sh, alternating runs): the ILP scheduler takes kd_bin_count from 20.7 to
# 18.7-19.2 us at C3 and leaves the scan / scatter unchanged; on the tile kernels it changes
# nothing (kd_dibr_fwd_tiles) or loses (kd_dibr_bwd +2.7 us)
SOURCE_FLAGS = {'kd_binning.hip': ['-mllvm', '-amdgpu-sched-strategy=max-ilp']}


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, diag=False):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJDIR_DIAG if diag else OBJDIR, src + '.o')
    deps = [path, os.path.join(ROOT, 'include', 'kaolin_dibr.h'), __file__] + \
        [os.path.join(CSRC, h) for h in HEADERS]
    if _stale(obj, deps):
        lang = ['-x', 'hip'] if src.endswith('.cpp') else []
        extra = (['-DKD_DIAG=1'] if diag else []) + SOURCE_FLAGS.get(src, [])
        cmd = [HIPCC, *FLAGS, *extra, *lang, '-c', path, '-o', obj + '.tmp']
        subprocess.check_call(cmd)
        os.replace(obj + '.tmp', obj)
    return obj


def build(force=False, verbose=True, diag=False):
    """The production library (diag=False) or the diagnostic one (tools/ only)."""
    objdir, lib = (OBJDIR_DIAG, LIB_DIAG) if diag else (OBJDIR, LIB)
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    if force:
        for s in SOURCES:
            o = os.path.join(objdir, s + '.o')
            if os.path.exists(o):
                os.remove(o)
    with concurrent.futures.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, diag), SOURCES))
    if force or _stale(lib, objs):
        tmp = lib + f'.{os.getpid()}.tmp'
        subprocess.check_call([HIPCC, '-shared', f'--offload-arch={ARCH}', *objs, '-Wl,--no-undefined',
                               '-o', tmp])
        os.replace(tmp, lib)
        if verbose:
            print(f'[kaolin_amd] built {lib}', file=sys.stderr)
    return lib


if __name__ == '__main__':
    build(force='--force' in sys.argv, diag='--diag' in sys.argv)
