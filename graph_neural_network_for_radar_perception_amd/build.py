"""Build libradargnn.so (the HIP library behind the C ABI in include/radar_gnn.h).

Compiles every ``csrc/*.hip`` for gfx950 only with ``hipcc`` and links one
shared library in-tree at ``graph_neural_network_for_radar_perception_amd/lib/``
(so it travels with the repository snapshot to the GPU box).  Objects are
rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
LIBDIR = os.path.join(PKG, 'lib')
OBJDIR = os.path.join(PKG, 'lib', 'obj')
LIB = os.path.join(LIBDIR, 'libradargnn.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
FLAGS = ['-O3', '-std=c++17', f'--offload-arch={ARCH}', '-fPIC', '-Wall',
         '-Wno-unused-function', '-Wno-unused-variable', '-I', os.path.join(REPO, 'include')]
# per-source flags: the fused conv keeps its epilogue in scalar f32 (a packed v_pk_*_f32
# beside MFMAs costs far more than two scalar ops, MI355X_MICROARCH.md "price of one
# filler"); measured 3.5 % faster per conv layer than the packed build
FILE_FLAGS = {'conv_fused.hip': ['-DRG_NO_PK', '-fno-slp-vectorize'],
              'conv_x3.hip': ['-fno-slp-vectorize', '-mllvm', '-amdgpu-mfma-vgpr-form']}


def _headers():
    return glob.glob(os.path.join(CSRC, '*.h')) + [os.path.join(REPO, 'include', 'radar_gnn.h')]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, extra, objdir=OBJDIR):
    obj = os.path.join(objdir, os.path.basename(src) + '.o')
    if _stale(obj, [src] + _headers()):
        cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + extra + [
            '-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {src}:\n{r.stdout}\n{r.stderr}')
        if r.stderr.strip():
            sys.stderr.write(r.stderr)
    return obj


def build_library(verbose: bool = False, extra_flags=None) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    extra = list(extra_flags or [])
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra), srcs))
    if _stale(LIB, objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
    if verbose:
        print('built', LIB)
    return LIB


def build_variant(name: str, defines, only=None) -> str:
    """A copy of the library built with extra -D flags (kernel experiments), at
    lib/variants/libradargnn_<name>.so; load it with RG_LIBRARY=<path>."""
    vdir = os.path.join(LIBDIR, 'variants', name)
    os.makedirs(vdir, exist_ok=True)
    extra = [d if d.startswith('-') else f'-D{d}' for d in defines]
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    objs = []
    for s in srcs:
        if only is None or os.path.basename(s) in only:
            objs.append(_compile(s, extra, vdir))
        else:
            objs.append(_compile(s, []))
    out = os.path.join(LIBDIR, 'variants', f'libradargnn_{name}.so')
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', out] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
    return out


SAN_FLAGS = ['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined',
             '-Xarch_host', '-fno-sanitize-recover=undefined', '-Xarch_host',
             '-fno-omit-frame-pointer']


def build_sanitized_driver(driver: str) -> str:
    """The library's HOST code under AddressSanitizer + UndefinedBehaviorSanitizer, linked
    with a C++ driver into an executable at lib/asan/<driver name> (device code is compiled
    as usual: every -fsanitize= sits behind -Xarch_host, and the link line keeps the GPU side
    unsanitised with -fno-gpu-sanitize).  Run by tests/test_native_lib.py on the CPU; objects
    are rebuilt only when a source or header is newer."""
    adir = os.path.join(LIBDIR, 'asan')
    os.makedirs(adir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, SAN_FLAGS + ['-O1'], adir), srcs))
    exe = os.path.join(adir, os.path.splitext(os.path.basename(driver))[0])
    if _stale(exe, objs + [driver] + _headers()):
        dobj = exe + '.o'
        steps = [[HIPCC, '-std=c++17', '-O1', '-g', '-fPIC', '-fsanitize=address,undefined',
                  '-fno-omit-frame-pointer', '-I', os.path.join(REPO, 'include'), '-c', driver,
                  '-o', dobj],
                 [HIPCC, f'--offload-arch={ARCH}', '-fsanitize=address,undefined',
                  '-fno-gpu-sanitize', '-o', exe, dobj] + objs]
        for cmd in steps:
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f'sanitized build failed: {" ".join(cmd[:4])}...\n'
                                   f'{r.stdout}\n{r.stderr[-4000:]}')
    return exe


if __name__ == '__main__':
    build_library(verbose=True)
