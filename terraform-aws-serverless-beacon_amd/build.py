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

SOURCES = ['api.cpp', 'ingest.cpp', 'index.cpp', 'wire.cpp', 'query_kernels.hip', 'dedup_kernels.hip']
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


if __name__ == '__main__':
    print(build(verbose=True))
