"""ctypes view of oracle/_ref/libsbref.so (oracle/ref_harness.cpp): the
reference's AWS-free C++ compiled where it lies (oracle/Makefile.ref).

TEST INFRASTRUCTURE ONLY -- imported by tests/ to pin the oracle and the
engine's region-file / dedup paths to the reference's own code.  ``lib()``
builds the library when /root/reference is present and returns None when it
cannot (the GPU box, which has no reference sources)."""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, '_ref', 'libsbref.so')
REF = os.environ.get('SBEACON_REFERENCE', '/root/reference')
_lib = None


def build() -> bool:
    if not os.path.isdir(REF):
        return os.path.exists(PATH)
    subprocess.check_call(['make', '-s', '-C', HERE, '-f', 'Makefile.ref', f'REF={REF}'])
    return True


def lib():
    global _lib
    if _lib is None:
        if not build() or not os.path.exists(PATH):
            return None
        L = C.CDLL(PATH)
        L.ref_seq_code.restype = C.c_int
        L.ref_seq_code.argtypes = [C.c_int]
        L.ref_atoui64_len.restype = C.c_uint64
        L.ref_atoui64_len.argtypes = [C.c_char_p, C.c_uint8]
        L.ref_fast_atoi_u64.restype = C.c_uint64
        L.ref_fast_atoi_u64.argtypes = [C.c_char_p, C.c_size_t]
        L.ref_gzip_deflate.restype = C.c_int64
        L.ref_gzip_deflate.argtypes = [C.c_char_p, C.c_uint32, C.c_int, C.c_char_p, C.c_int64]
        L.ref_region_keys.restype = C.c_int64
        L.ref_region_keys.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_char_p, C.c_int64,
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        _lib = L
    return _lib


def gzip_deflate(data: bytes, level: int = 9) -> bytes:
    """gzip.cpp:19-59 deflateFile(level) of one buffer."""
    cap = len(data) + len(data) // 8 + 1024
    out = C.create_string_buffer(cap)
    n = lib().ref_gzip_deflate(data, len(data), level, out, cap)
    if n < 0:
        raise RuntimeError(f'ref_gzip_deflate failed ({n})')
    return out.raw[:n]


def region_keys(gz: bytes, range_start: int, range_end: int):
    """readVcfData.cpp:3-71 getVcfData over one region file's bytes (the
    real gzip reader): list of key strings (bytes), or RuntimeError where
    the reference throws."""
    cap = max(4096, 8 * len(gz) + 65536)
    while True:
        out = C.create_string_buffer(cap)
        ol = C.c_int64()
        what = C.c_int()
        n = lib().ref_region_keys(gz, len(gz), range_start, range_end, out, cap, C.byref(ol), C.byref(what))
        if n == -2:
            cap *= 4
            continue
        if n < 0:
            return RuntimeError(f'reference getVcfData throws (kind {what.value})')
        keys, at, raw = [], 0, out.raw[:ol.value]
        for _ in range(n):
            (k,) = struct.unpack_from('<I', raw, at)
            keys.append(raw[at + 4:at + 4 + k])
            at += 4 + k
        return keys
