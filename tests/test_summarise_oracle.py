"""summariseSlice oracle (oracle/summarise_oracle.c) on hand-derived cases.

The reference C++ (lambda/summariseSlice/source) needs AWS SDK C++ and cannot
be built here, so these cases pin the restatement to values worked out by
hand from main.cpp:52-109,195-245 and vcf_chunk_reader.h (parity unpinned
against reference output)."""
import os
import random

import pytest

from bgzf_util import blocks, random_slices, record_starts, text
from conftest import FIXTURES


def rs(t):
    from oracle.oracle import region_stats
    return region_stats(t)


def rec(pos, info, gt='0|1'):
    return b'22\t%d\t.\tA\tG\t.\tPASS\t%s\tGT\t%s\n' % (pos, info.encode(), gt.encode())


def test_counts_first_ac_an_and_multiallelic():
    # numVariants = 1 + commas in AC; numCalls = AN (main.cpp:68-89)
    t = b'22\t1\t.\tA\tG,T,C\t.\tPASS\tAC=1,2,0;AN=10\tGT\t0|1\n'
    assert rs(t) == {'numVariants': 3, 'numCalls': 10, 'records': 1}


def test_scan_stops_once_both_tags_seen():
    # a second AC= after both were found is never read
    assert rs(rec(1, 'AC=1;AN=4;AC=5,5'))['numVariants'] == 1
    # but a repeated AC= before AN= is counted twice (reference quirk)
    assert rs(rec(1, 'AC=1;AC=2;AN=4')) == {'numVariants': 2, 'numCalls': 4, 'records': 1}


def test_missing_tags_and_short_fields():
    assert rs(rec(1, 'AN=7;X=1')) == {'numVariants': 0, 'numCalls': 7, 'records': 1}
    assert rs(rec(1, 'AC=;AN=2'))['numVariants'] == 0  # 'AC=' is shorter than 4 chars
    assert rs(rec(1, 'AC_AFR=3;AC=2;AN=2'))['numVariants'] == 1


def test_skip_heuristic_swallows_short_records():
    long1 = rec(1, 'AC=1;AN=2;' + ';'.join(f'K{i}=1' for i in range(30)))
    # skip = 2 * (29 ';' + 2 tab + 1 '|') = 64 >= rest of a short record
    short = [rec(p, f'AC={p};AN=2') for p in range(2, 6)]
    r = rs(long1 + b''.join(short))
    # r1, r2 visited; r2 overshoots into r4 -> resumes at r5, which overshoots past the end
    assert r == {'numVariants': 3, 'numCalls': 6, 'records': 3}


def test_no_skip_when_records_are_long_enough():
    t = b''.join(rec(p, 'AC=1;AN=2;X=1') for p in range(1, 8))
    assert rs(t) == {'numVariants': 7, 'numCalls': 14, 'records': 7}


def test_cut_mid_record_drops_unterminated_fields():
    t = rec(1, 'AC=1;AN=2;X=1') + rec(2, 'AC=1;AN=2;X=1')
    cut = t.index(b'AN=2', 30)  # inside the second record, before its AN
    assert rs(t[:cut]) == {'numVariants': 2, 'numCalls': 2, 'records': 2}


def test_atoui64_quirk_on_non_digits():
    # atoui64 arithmetic on 'x' (fast_atoi.h:73-99): ('x' - '0') = 72
    assert rs(rec(1, 'AC=1;AN=1x'))['numCalls'] == 1 * 10 + 72


@pytest.fixture(scope='module')
def tiny_bgzf(tmp_path_factory):
    from sbeacon.workload import write_bgzf
    p = str(tmp_path_factory.mktemp('bgzf') / 'tiny22.vcf.gz')
    write_bgzf(p, [open(os.path.join(FIXTURES, 'tiny22.vcf'), 'rb').read()])
    return p


def test_bgzf_slices_agree_with_stream_restatement(tiny_bgzf):
    from oracle.oracle import OracleBgzf
    o = OracleBgzf(tiny_bgzf)
    blk = blocks(tiny_bgzf)
    txt = text(tiny_bgzf)
    assert o.ulen == len(txt) and len(blk) > 3
    rng = random.Random(4)
    for vs, ve in random_slices(txt, blk, rng, 60):
        got = o.summarise_slice(vs, ve)
        u0, u1 = o.voff_to_u(vs), o.voff_to_u(ve)
        assert got == rs(txt[u0:u1])
    # whole file from the first record: every record visited (no overshoots here)
    starts = record_starts(txt)
    whole = o.summarise_slice((blk[0][0] << 16) | starts[0], (blk[-1][0] << 16))
    assert whole['records'] == len(starts)


def test_partition_chunks_and_split_model():
    from sbeacon.summarise_vcf import find_best_split, partition_chunks
    b = {'1': [0, 5 << 16, (9 << 16) | 7, 20 << 16, 21 << 16], '2': [30 << 16, 31 << 16]}
    # a slice closes at the first boundary >= 8 blocks-bytes past its start block
    assert partition_chunks(b, 8) == [(0, (9 << 16) | 7), ((9 << 16) | 7, 20 << 16), (20 << 16, 21 << 16),
                                      (30 << 16, 31 << 16)]
    # the Newton model converges to a positive size that grows with the file
    s1, s2 = find_best_split(1e7, 1000), find_best_split(5e9, 1000)
    assert 0 < s1 < s2


def test_region_files_split_on_gaps_and_count_bytes(tmp_path):
    """write_data_to_s3.h: one entry {pos u64, len u16, ref'_alt'} per ALT,
    a new file when POS jumps more than MAX_SLICE_GAP (100,000) past the last
    entry; file length = sum of 8 + 2 + |ref'| + 1 + |alt'|."""
    import struct

    from bgzf_util import blocks, record_starts, text
    from oracle.oracle import OracleBgzf
    from sbeacon.workload import write_bgzf
    hdr = b'##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n'
    recs = [(100, 'A', 'G'), (200, 'C', 'T,G'), (100200, 'GA', 'G'), (200300, 'A', '<DEL>'), (300301, 'T', 'C')]
    body = b''.join(f'5\t{p}\t.\t{r}\t{a}\t.\tPASS\tAC=1;AN=2;DP=5\n'.encode() for p, r, a in recs)
    path = write_bgzf(str(tmp_path / 'gaps.vcf.gz'), [hdr + body])
    o = OracleBgzf(path)
    blk, txt = blocks(path), text(path)
    starts = record_starts(txt)
    vs, ve = (blk[0][0] << 16) | starts[0], blk[-1][0] << 16
    files, data = o.region_files(vs, ve, with_data=True)
    # 100, 200 (x2) | 100200 (gap 100000: same file) ... 200300 (gap 100100: new) | 300301 (gap 100001: new)
    assert [(f[0], f[1], f[3]) for f in files] == [(100, 100200, 4), (200300, 200300, 1), (300301, 300301, 1)]
    # entry bytes: SNV 10+3; GA->G: ref' 1 packed byte + '_' + 1 = 13; <DEL> -> 'DEL' : 10+1+1+3
    assert [f[2] for f in files] == [13 * 4, 15, 13]
    p, ln = struct.unpack_from('<QH', data, 0)
    assert (p, ln) == (100, 3) and data[10:13] == b'\x01_\x03'
