"""The oracle pinned to the reference's own C++ (oracle/_ref: gzip.cpp,
generalutils.*, fast_atoi.h compiled where they lie, oracle/Makefile.ref).

* sequenceToBinary (generalutils.hpp:19-36) for every byte value against the
  oracle's compressSeq table (summarise_oracle.c seq_code);
* atoui64(str, len) (fast_atoi.h:54-80) against the oracle's restatement on
  digit strings of every length 1..20 and on non-digit bytes;
* gzip members: the deflate payload of gzip.cpp:19-59 deflateFile(9) equals
  zlib level 9 / windowBits 31 / memLevel 9 -- the parameters the engine's
  region-file writer uses -- on region-file bytes the oracle builds;
* ReadVcfData::getVcfData (readVcfData.cpp:3-71) restated over the REAL gzip
  reader: the reference's range semantics on crafted region files (the read
  past rangeEnd while the stream has more data, the stop after the first
  entry past rangeEnd in the last window, the throw when an entry skipped
  below rangeStart straddles a 1 KiB window).

The reference gzip header carries uninitialised fields (gzip.cpp:23-26:
flags, mtime and OS come from the stack), so members are compared from the
deflate payload on.  Skipped when oracle/_ref cannot be built (no
/root/reference and no prebuilt library)."""
import random
import struct
import zlib

import pytest

from conftest import REPO  # noqa: F401


@pytest.fixture(scope='module')
def ref():
    from oracle import ref as R
    if R.lib() is None:
        pytest.skip('oracle/_ref not buildable here (no /root/reference)')
    return R


@pytest.fixture(scope='module')
def orc():
    import ctypes as C
    from oracle.oracle import lib
    L = lib()
    L.orc_seq_code.restype = C.c_int
    L.orc_seq_code.argtypes = [C.c_int]
    L.orc_atoui64_len.restype = C.c_int
    L.orc_atoui64_len.argtypes = [C.c_char_p, C.c_uint8, C.POINTER(C.c_uint64)]
    return L


def gzip_payload(member: bytes) -> bytes:
    """The deflate data + CRC32 + ISIZE of one gzip member (RFC 1952 header skipped)."""
    assert member[:3] == b'\x1f\x8b\x08'
    flg = member[3]
    at = 10
    if flg & 4:  # FEXTRA
        (xlen,) = struct.unpack_from('<H', member, at)
        at += 2 + xlen
    if flg & 8:  # FNAME
        at = member.index(b'\0', at) + 1
    if flg & 16:  # FCOMMENT
        at = member.index(b'\0', at) + 1
    if flg & 2:  # FHCRC
        at += 2
    return member[at:]


def deflate9(data: bytes) -> bytes:
    c = zlib.compressobj(9, zlib.DEFLATED, 16 + zlib.MAX_WBITS, 9, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(data) + c.flush()


def test_sequence_to_binary_table(ref, orc):
    for c in range(256):
        assert orc.orc_seq_code(c) == ref.lib().ref_seq_code(c), chr(c)
    assert ref.lib().ref_seq_code(ord('R')) == -1  # IUPAC codes throw (std::map::at)


def test_atoui64_len(ref, orc):
    import ctypes as C
    rng = random.Random(7)
    cases = [b'0', b'5008', b'152312', b'18446744073709551615', b'99999999999999999999', b'0000000001']
    for n in range(1, 21):
        for _ in range(30):
            cases.append(''.join(rng.choice('0123456789') for _ in range(n)).encode())
    cases += [b'12a', b'-5', b'4 2', b'.', b'1e5']  # non-digits: the reference's arithmetic as it is
    for s in cases:
        v = C.c_uint64()
        assert orc.orc_atoui64_len(s, len(s), C.byref(v)) == 0
        assert v.value == ref.lib().ref_atoui64_len(s, len(s)), s


def _entries(rng, n, pos0=1000, gap=(0, 40), long_p=0.05):
    """Region-file entries {pos u64, len u16, ref'_alt'} (write_data_to_s3.h:30-37,56-58)."""
    out, pos, poss = [], pos0, []
    for _ in range(n):
        pos += rng.randint(*gap)
        tail = bytes([rng.randint(1, 7)]) + b'_' + bytes([rng.randint(1, 7)])
        if rng.random() < long_p:
            tail = bytes(rng.randint(17, 119) for _ in range(rng.randint(2, 60))) + b'_' + bytes([3])
        out.append(struct.pack('<QH', pos, len(tail)) + tail)
        poss.append(pos)
    return out, poss


def test_gzip_member_payload(ref):
    rng = random.Random(3)
    for n in (1, 17, 400, 5000):
        ents, _ = _entries(rng, n)
        data = b''.join(ents)
        member = ref.gzip_deflate(data, 9)
        assert zlib.decompress(member, 16 + zlib.MAX_WBITS) == data
        assert gzip_payload(member) == gzip_payload(deflate9(data))


def test_region_reader_range_semantics(ref):
    rng = random.Random(11)
    ents, poss = _entries(rng, 3000, gap=(1, 30), long_p=0.0)
    gz = ref.gzip_deflate(b''.join(ents), 9)
    # the whole file in range: every entry
    all_keys = ref.region_keys(gz, 0, 1 << 62)
    assert [k for k in all_keys] == [str(p).encode() + e[10:] for p, e in zip(poss, ents)]
    # rangeEnd in the middle: the reader keeps going while the stream has
    # more data, so every entry up to the last window is returned, and inside
    # the last window the first entry past rangeEnd is the last one read
    re_ = poss[len(poss) // 2]
    got = ref.region_keys(gz, 0, re_)
    assert len(got) > len(poss) // 2 + 100  # far past rangeEnd
    assert got == all_keys[:len(got)]
    # a rangeEnd inside the last ~1 KiB window stops right after the first entry past it
    re2 = poss[-5]
    got2 = ref.region_keys(gz, 0, re2)
    assert got2 == all_keys[:len(poss) - 3]
    # rangeStart in the middle of 13-byte entries: a skipped entry's tail soon
    # crosses a 1 KiB window and the reference throws (next test)
    assert isinstance(ref.region_keys(gz, poss[1000], 1 << 62), RuntimeError)
    # 16-byte entries tile the 1 KiB windows exactly: nothing straddles, and
    # entries below rangeStart are skipped, not returned
    ents16 = [struct.pack('<QH', 500 + 3 * i, 6) + bytes([1, 2, 3]) + b'_' + bytes([4, 5]) for i in range(4000)]
    gz16 = ref.gzip_deflate(b''.join(ents16), 9)
    rs = 500 + 3 * 1500
    got3 = ref.region_keys(gz16, rs, 1 << 62)
    assert got3 == [str(500 + 3 * i).encode() + e[10:] for i, e in enumerate(ents16) if 500 + 3 * i >= rs]


def test_region_reader_skip_straddle_throws(ref):
    """An entry below rangeStart whose string crosses the 1 KiB window is
    skipped with no availability check (readVcfData.cpp:27-30): the next
    refill gets bufferPos > dataLength and gzip::proccesData throws."""
    ents = []
    pos = 100
    for i in range(40):
        tail = b'\x01_' + bytes(range(40, 40 + 60))  # 62-byte tails: entries straddle 1 KiB
        ents.append(struct.pack('<QH', pos + i, len(tail)) + tail)
    gz = ref.gzip_deflate(b''.join(ents), 9)
    assert isinstance(ref.region_keys(gz, 1000, 2000), RuntimeError)  # everything skipped
    assert len(ref.region_keys(gz, 0, 2000)) == 40  # nothing skipped: fine
