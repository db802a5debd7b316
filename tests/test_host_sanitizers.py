"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).

build.build_sanitized() compiles api.cpp / ingest.cpp / index.cpp / wire.cpp
with -fsanitize=address,undefined on the host side only (device code is never
instrumented) and SBEACON_CHECKS (request-plan invariants: every chain's
range and staging capacity, runs of up to 64 chains); tests/asan_driver.py
then drives ingest, index writing, request planning (fixtures + a 240 k-record
genome shape with runs of 64 whole-contig chains) and the wire parser through
it in a child process with the ASan runtime preloaded.  Any report fails the
test.  Reference bar: lambda/summariseSlice/source/CMakeLists.txt:22-27 only
turns warnings on."""
import os
import subprocess
import sys

from conftest import PKG, REPO


def test_host_code_clean_under_asan_and_ubsan():
    sys.path.insert(0, PKG)
    import build
    lib = build.build_sanitized()
    env = dict(os.environ)
    env.update(LD_PRELOAD=build.asan_runtime(), SBEACON_LIB=lib,
               ASAN_OPTIONS='detect_leaks=0:abort_on_error=0:halt_on_error=1:exitcode=97',
               UBSAN_OPTIONS='halt_on_error=1:print_stacktrace=1:exitcode=98', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'tests', 'asan_driver.py')], env=env, capture_output=True,
                       text=True, timeout=1500)
    report = r.stderr[-6000:]
    assert 'ERROR: AddressSanitizer' not in r.stderr, report
    assert 'runtime error:' not in r.stderr, report
    assert r.returncode == 0, report
    assert 'asan driver ok' in r.stdout, (r.stdout[-2000:], report)
