"""Build libsbeacon_hip.so in-tree with hipcc for gfx950 (no CMake needed).

Objects go to ``build/`` next to this file; the shared library lands beside
the ``sbeacon`` package so ``sbeacon._lib`` finds it and it travels to the GPU
box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, 'build')
LIB = os.path.join(HERE, 'libsbeacon_hip.so')
SYNTH_LIB = os.path.join(HERE, 'libsbeacon_synth.so')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')
ARCH = os.environ.get('SBEACON_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')

SOURCES = ['api.cpp', 'requests.cpp', 'summarise.cpp', 'results.cpp', 'ingest.cpp', 'index.cpp', 'wire.cpp', 'routes.cpp', 'persist.cpp', 'query_kernels.hip', 'dedup_kernels.hip']
FLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-Wall', '-Wextra', '-Wno-unused-parameter',
         f'-I{INCLUDE}']


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hpp')]
    return hdrs + [os.path.join(INCLUDE, 'sbeacon.h')]


def _stale(out, inputs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(i) > t for i in inputs)


def build(verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    deps = _deps()
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src + '.o')
        if _stale(o, [s] + deps):
            cmd = [HIPCC] + FLAGS + ['-c', s, '-o', o]
            if src.endswith('.cpp'):
                cmd[1:1] = ['-x', 'hip']
            jobs.append(cmd)

    def run(cmd):
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f'compile failed: {" ".join(cmd)}\n{r.stdout}\n{r.stderr}')
        return r.stderr

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        for err in ex.map(run, jobs):
            if err.strip() and verbose:
                print(err, file=sys.stderr)
    objs = [os.path.join(BUILD, s + '.o') for s in SOURCES]
    if _stale(LIB, objs):
        run([HIPCC, f'--offload-arch={ARCH}', '-shared', '-o', LIB] + objs + ['-lz', '-lpthread'])
    # synthetic-data generator (bench / tests input only; host C++)
    syn = os.path.join(CSRC, 'synth.cpp')
    if _stale(SYNTH_LIB, [syn]):
        run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-pthread', '-Wall', '-o', SYNTH_LIB, syn, '-lz'])
    return LIB


ASAN_DIR = os.path.join(BUILD, 'asan')
ASAN_LIB = os.path.join(ASAN_DIR, 'libsbeacon_hip_asan.so')
HOST_SOURCES = ['api.cpp', 'requests.cpp', 'summarise.cpp', 'results.cpp', 'ingest.cpp', 'index.cpp', 'wire.cpp', 'routes.cpp', 'persist.cpp']
# host code only (-Xarch_host): device code is never instrumented; the kernel
# objects of build() are linked as they are.  SBEACON_CHECKS turns on the
# request-plan invariant checks (api.cpp check_request_plan).
SAN = ['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined', '-Xarch_host',
       '-fno-sanitize-recover=undefined', '-Xarch_host', '-fno-omit-frame-pointer', '-DSBEACON_CHECKS', '-g1']


def asan_runtime() -> str:
    """The clang AddressSanitizer runtime a Python process preloads to load ASAN_LIB."""
    import glob
    hits = sorted(glob.glob('/opt/rocm/lib/llvm/lib/clang/*/lib/*/libclang_rt.asan-x86_64.so') +
                  glob.glob('/opt/rocm/lib/llvm/lib/clang/*/lib/*/libclang_rt.asan.so'))
    if not hits:
        raise RuntimeError('no clang AddressSanitizer runtime under /opt/rocm/lib/llvm')
    return hits[0]


def build_sanitized(verbose: bool = False) -> str:
    """libsbeacon_hip with its host code under AddressSanitizer + UBSan
    (tests/test_host_sanitizers.py runs ingest, index writing, request planning
    and the wire parser through it on the CPU)."""
    build(verbose)
    os.makedirs(ASAN_DIR, exist_ok=True)
    deps = _deps()
    jobs = []
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(ASAN_DIR, src + '.o')
        if _stale(o, [s] + deps + [os.path.abspath(__file__)]):
            jobs.append([HIPCC, '-x', 'hip'] + FLAGS + SAN + ['-c', s, '-o', o])

    def run(cmd):
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f'compile failed: {" ".join(cmd)}\n{r.stdout}\n{r.stderr}')

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(ASAN_DIR, s + '.o') for s in HOST_SOURCES] + \
           [os.path.join(BUILD, s + '.o') for s in SOURCES if s.endswith('.hip')]
    if _stale(ASAN_LIB, objs):
        run([HIPCC, f'--offload-arch={ARCH}', '-shared', '-Xarch_host', '-fsanitize=address', '-Xarch_host',
             '-fsanitize=undefined', '-shared-libasan', '-o', ASAN_LIB] + objs + ['-lz', '-lpthread'])
    return ASAN_LIB


if __name__ == '__main__':
    print(build(verbose=True))
    if '--sanitized' in sys.argv:
        print(build_sanitized(verbose=True))
