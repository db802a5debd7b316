"""CPU-side checks of the C ABI: the library loads, exports every symbol
include/sbeacon.h declares, and the host ingest rejects what the store cannot
represent exactly (no GPU needed: ingest runs on the host)."""
import ctypes as C
import os
import re

import pytest

from conftest import REPO


def header_functions():
    src = open(os.path.join(REPO, 'include', 'sbeacon.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(sb_[a-z_]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    from sbeacon import _lib
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    assert L.sb_abi_version() == 2


def test_library_is_gfx950_code_object():
    from sbeacon import _lib
    blob = open(_lib.LIB_PATH, 'rb').read()
    assert b'gfx950' in blob


def _builder():
    from sbeacon import _lib
    L = _lib.lib()
    b = C.c_void_p()
    opts = _lib.BuildOpts(1, 2)
    assert L.sb_builder_new(C.byref(opts), C.byref(b)) == 0
    vid = C.c_uint32()
    assert L.sb_builder_begin_vcf(b, b'x.vcf', 5, C.byref(vid)) == 0
    return L, b, vid.value


HDR = b'##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n'


@pytest.mark.parametrize('body,ok', [
    (b'22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\n22\t101\t.\tC\tT\t.\t.\tAC=0;AN=2\tGT\t0|0\n', True),
    (b'22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\n22\t99\t.\tC\tT\t.\t.\tAC=0;AN=2\tGT\t0|0\n', False),
    (b'22\t0100\t.\tA\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\n', False),
    (b'22\t100\t.\t\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\n', False),
    (b'22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2\tGT\n', False),
    (b'22\t100\t.\tA\tG\t.\t.\tAC=1\tGT\t0|1|1|1\n', True),  # ploidy 4 fallback: a general record
    (b'22\t100\t.\tA\tG\t.\t.\tAC=1;AN=' + b'9' * 4300 + b'\tGT\t0|1\n', True),  # AN past int64: general
    (b'22\t100\t.\tA\t' + b','.join([b'C'] * 300) + b'\t.\t.\tAN=2\tGT\t0|299\n', True),  # 300 ALTs, no AC
])
def test_ingest_validation(body, ok):
    from sbeacon import _lib
    L, b, vid = _builder()
    try:
        rc = L.sb_builder_add_text(b, vid, HDR + body, len(HDR + body))
        if ok:
            assert rc == 0, L.sb_last_error()
        else:
            assert rc == -5, (rc, L.sb_last_error())
            assert L.sb_last_error()
    finally:
        L.sb_builder_free(b)


def test_finish_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('a device is present')
    L, b, vid = _builder()
    try:
        assert L.sb_builder_add_text(b, vid, HDR, len(HDR)) == 0
        s = C.c_void_p()
        rc = L.sb_builder_finish(b, 0, C.byref(s))
        assert rc == -3  # SB_EHIP: no CPU fallback
    finally:
        L.sb_builder_free(b)
