"""Builds every native component of blendtorch in-tree.

Targets (all outputs live next to the Python sources so they travel with the
repository snapshot):

* ``blendtorch/_native*.so``   -- ZMTP transport + pickle codec (g++, C++17, no HIP)
* ``blendtorch/_hip*.so``      -- gfx950 kernels + GPU stream loader (hipcc)
* ``blendtorch/bin/cubesim``   -- headless Cube-scene producer (C++)
* ``blendtorch/bin/cartpolesim`` -- headless cart-pole REP environment (C++)

The build is incremental (mtime based) and compiles independent objects in
parallel.  ``python -m blendtorch._build`` builds everything.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent.parent
CSRC = ROOT / 'csrc'
BUILD = ROOT / 'build' / 'native'
BIN = PKG / 'bin'
HIP_ARCH = os.environ.get('BLENDTORCH_HIP_ARCH', 'gfx950')
ROCM = Path(os.environ.get('ROCM_PATH', '/opt/rocm'))

# -ffp-contract=off: host float code (e.g. codec/xform_fit.cpp) rounds every operation on its own
CXXFLAGS = ['-std=c++17', '-O3', '-fPIC', '-Wall', '-Wno-unused-parameter', '-pthread', '-ffp-contract=off']

TRANSPORT = ['transport/zmtp.cpp', 'transport/shmring.cpp']
CODEC = ['codec/pickle_codec.cpp', 'codec/xform_fit.cpp']
RASTER = ['sim/raster.cpp', 'sim/physics.cpp']


def _ext_suffix():
    return sysconfig.get_config_var('EXT_SUFFIX') or '.so'


def _py_includes():
    import pybind11
    return [f'-I{pybind11.get_include()}', f'-I{sysconfig.get_paths()["include"]}']


def _torch_lib():
    import importlib.util
    spec = importlib.util.find_spec('torch')
    if spec is None or spec.origin is None:
        return None
    return Path(spec.origin).parent / 'lib'


# what the last build_all() did per target: 'compiled' (objects recompiled
# and/or relinked) or 'up to date' -- build() prints it so a driver's build on
# another machine is observable (prebuilt .so files travel with the tree)
REPORT = {}


def _note(target: Path, changed: bool):
    REPORT[str(target)] = 'compiled' if changed else 'up to date'


def _newer(target: Path, deps):
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _headers():
    return [p for p in CSRC.rglob('*.h')]


def _run(cmd, verbose):
    if verbose:
        print(' '.join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'build failed: {" ".join(map(str, cmd))}\n{r.stdout}\n{r.stderr}')
    return r


def _compile(compiler, src: Path, obj: Path, flags, verbose):
    deps = [src] + _headers()
    # the command line is part of the object's identity: a flag change rebuilds
    stamp = obj.with_suffix('.cmd')
    cmd = ' '.join(str(a) for a in [compiler, *flags])
    if not _newer(obj, deps) and stamp.exists() and stamp.read_text() == cmd:
        return obj, False
    obj.parent.mkdir(parents=True, exist_ok=True)
    _run([compiler, *flags, '-c', src, '-o', obj], verbose)
    stamp.write_text(cmd)
    return obj, True


def _obj_path(src: Path, tag: str):
    rel = src.relative_to(CSRC)
    return BUILD / tag / (str(rel).replace('/', '__') + '.o')


def build_native(verbose=False, jobs=8):
    """Build `_native` Python module and the C++ simulator executables."""
    cxx = os.environ.get('CXX', 'g++')
    srcs = [CSRC / s for s in TRANSPORT + CODEC + RASTER]
    py_src = CSRC / 'python' / 'py_native.cpp'
    flags = CXXFLAGS + _py_includes()
    with ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, cxx, s, _obj_path(s, 'cpu'), flags, verbose) for s in srcs + [py_src]]
        sim_srcs = [CSRC / 'sim' / n for n in ('cubesim.cpp', 'cartpolesim.cpp', 'supershapesim.cpp')]
        sim_srcs = [s for s in sim_srcs if s.exists()]
        futs += [ex.submit(_compile, cxx, s, _obj_path(s, 'cpu'), CXXFLAGS, verbose) for s in sim_srcs]
        res = [f.result() for f in futs]
    objs = [r[0] for r in res]
    fresh = [r[1] for r in res]
    core = objs[:len(srcs)]
    py_obj = objs[len(srcs)]
    target = PKG / f'_native{_ext_suffix()}'
    link = _newer(target, core + [py_obj])
    if link:
        _run([cxx, '-shared', '-pthread', '-Wl,-Bsymbolic', *core, py_obj, '-o', target], verbose)
    _note(target, link or any(fresh[:len(srcs) + 1]))
    BIN.mkdir(exist_ok=True)
    for s, o, f in zip(sim_srcs, objs[len(srcs) + 1:], fresh[len(srcs) + 1:]):
        exe = BIN / s.stem
        deps = core + [o]
        link = _newer(exe, deps)
        if link:
            _run([cxx, '-pthread', '-O3', *deps, '-o', exe, '-lrt'], verbose)
        _note(exe, link or f)
    return target


def hip_available():
    return (ROCM / 'bin' / 'hipcc').exists()


def build_hip(verbose=False, jobs=8):
    """Build the `_hip` extension (gfx950 kernels + GPU stream loader)."""
    hipcc = ROCM / 'bin' / 'hipcc'
    if not hipcc.exists():
        raise RuntimeError('hipcc not found; cannot build the HIP extension')
    tl = _torch_lib()
    gpu_srcs = sorted((CSRC / 'gpu').glob('*.hip')) + sorted((CSRC / 'gpu').glob('*.cpp'))
    if not gpu_srcs:
        return None
    # MFMA accumulators in VGPRs (gfx950 allows either file): in the unrolled
    # MFMA loops the AGPR form left accumulator copies between the files
    hflags = ['-std=c++17', '-O3', '-fPIC', f'--offload-arch={HIP_ARCH}', '-Wall',
              '-Wno-unused-parameter', '-Wno-unused-result', '-mcode-object-version=5',
              '-mllvm', '-amdgpu-mfma-vgpr-form=1'] + _py_includes()
    cxx = os.environ.get('CXX', 'g++')
    cflags = CXXFLAGS
    with ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, hipcc, s, _obj_path(s, 'hip'), hflags, verbose) for s in gpu_srcs]
        futs += [ex.submit(_compile, cxx, CSRC / s, _obj_path(CSRC / s, 'cpu'), cflags + _py_includes(), verbose)
                 for s in TRANSPORT + CODEC]
        res = [f.result() for f in futs]
    objs = [r[0] for r in res]
    target = PKG / f'_hip{_ext_suffix()}'
    relink = _newer(target, objs)
    _note(target, relink or any(r[1] for r in res))
    if relink:
        link = [hipcc, '-shared', '-fPIC', f'--offload-arch={HIP_ARCH}', '-Wl,-Bsymbolic', *objs, '-o', target, '-ldl']
        if tl is not None:
            # resolve libamdhip64 to the runtime torch already loaded
            link += [f'-L{tl}', f'-Wl,-rpath,{tl}']
        _run(link, verbose)
    return target


def build_all(verbose=False, hip=True):
    REPORT.clear()
    out = [build_native(verbose)]
    if hip and hip_available():
        out.append(build_hip(verbose))
    return out


if __name__ == '__main__':
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--no-hip', action='store_true')
    ap.add_argument('-v', '--verbose', action='store_true')
    a = ap.parse_args()
    build_all(verbose=a.verbose, hip=not a.no_hip)
    for t, st in REPORT.items():
        print(f'{st}: {t}')
