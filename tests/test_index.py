"""CSI / TBI indexes and summariseVcf's slice plan (CPU).

Goldens (tests/golden/index_golden.json, make_index_goldens.py) come from
running the reference summariseVcf handler (lambda/summariseVcf/
lambda_function.py:253-304 with index_reader.py) over the indexes
sb_index_vcf writes for the fixtures of tests/golden/index_fixtures.py: the
SNS slice messages, the toUpdate strings, the sampleCount, the reference's
get_chunk_boundaries dict and partition_chunks at finer slice sizes.

* the writer reproduces the committed index bytes (deterministic);
* read_index / index_chunk_boundaries / slices_from_boundaries /
  partition_chunks / header_sample_count equal the reference's outputs;
* the index answers region lookups: every record is reachable from a chunk
  of a bin overlapping its interval (SAMv1 §5.3 reg2bins), and every chunk
  boundary is a record start or the end of the data;
* TBI refuses positions past 2^29, an unsorted VCF is refused."""
import json
import os
import struct
import zlib

import pytest

from conftest import REPO

GOLD = os.path.join(REPO, 'tests', 'golden')


@pytest.fixture(scope='module')
def golden():
    return json.load(open(os.path.join(GOLD, 'index_golden.json')))['cases']


@pytest.fixture(scope='module')
def fixture_files(tmp_path_factory):
    import sys
    sys.path.insert(0, GOLD)
    from index_fixtures import FIXTURES, write_fixture
    d = tmp_path_factory.mktemp('idx')
    return {name: write_fixture(name, str(d)) for name in FIXTURES}


def _committed(name, fmt):
    return open(os.path.join(GOLD, 'index', f'{name}.{fmt}'), 'rb').read()


def test_writer_reproduces_committed_indexes(golden, fixture_files):
    from sbeacon.summarise_vcf import write_index
    for c in golden:
        got = write_index(fixture_files[c['fixture']], c['format'])
        assert got == _committed(c['fixture'], c['format']), (c['fixture'], c['format'])


def test_slice_plan_matches_reference(golden):
    from sbeacon.summarise_vcf import index_chunk_boundaries, partition_chunks, slices_from_boundaries
    for c in golden:
        idx = _committed(c['fixture'], c['format'])
        cb = index_chunk_boundaries(idx)
        assert cb == c['boundaries'], (c['fixture'], c['format'])
        assert list(cb) == list(c['boundaries'])  # reference name order
        slices = slices_from_boundaries(cb)
        assert [list(s) for s in slices] == c['slices']
        assert sorted(f'{a}-{b}' for a, b in slices) == sorted(c['to_update'])
        for sz, exp in c['partitions'].items():
            assert [list(s) for s in partition_chunks(cb, int(sz))] == exp, sz


def test_sample_count_matches_reference(golden, fixture_files):
    from sbeacon.summarise_vcf import vcf_sample_count
    for c in golden:
        first = min(a for a, _ in c['slices']) >> 16
        assert vcf_sample_count(fixture_files[c['fixture']], first) == c['sample_count']


def _bgzf_blocks(path):
    """[(coffset, uncompressed bytes)] of a BGZF file."""
    data = open(path, 'rb').read()
    out, at = [], 0
    while at < len(data):
        xlen = struct.unpack_from('<H', data, at + 10)[0]
        bsize = struct.unpack_from('<H', data, at + 16)[0] + 1
        out.append((at, zlib.decompress(data[at + 12 + xlen:at + bsize - 8], -15)))
        at += bsize
    return out


def _records(path):
    """(contig, beg, end, voff) per data line, by the tabix VCF preset."""
    blocks = _bgzf_blocks(path)
    text = b''.join(b for _, b in blocks)
    starts = []
    u = 0
    for coff, b in blocks:
        starts.append((u, coff, len(b)))
        u += len(b)

    def voff(x):
        for u0, coff, n in starts:
            if u0 <= x < u0 + n:
                return (coff << 16) | (x - u0)
        return starts[-1][1] << 16

    out, at = [], 0
    for line in text.split(b'\n')[:-1]:
        if not line.startswith(b'#'):
            f = line.split(b'\t')
            beg = int(f[1]) - 1
            end = beg + len(f[3])
            for kv in f[7].split(b';'):
                if kv.startswith(b'END=') and int(kv[4:]) > beg:
                    end = int(kv[4:])
            out.append((f[0].decode(), beg, end, voff(at)))
        at += len(line) + 1
    return out, voff(len(text))


def _reg2bins(beg, end, min_shift, depth):
    end -= 1
    bins, s, t = [], min_shift + 3 * depth, 0
    for level in range(depth + 1):
        b, e = t + (beg >> s), t + (end >> s)
        bins.extend(range(b, e + 1))
        t += 1 << (3 * level)
        s -= 3
    return bins


@pytest.mark.parametrize('fmt', ['csi', 'tbi'])
def test_index_reaches_every_record(fixture_files, fmt):
    from sbeacon.summarise_vcf import index_chunk_boundaries, read_index, write_index
    for name, path in fixture_files.items():
        if fmt == 'tbi' and name == 'far_csi':
            continue
        data = write_index(path, fmt)
        idx = read_index(data)
        recs, data_end = _records(path)
        starts = {v for *_, v in recs} | {data_end}
        for bounds in index_chunk_boundaries(data).values():
            assert set(bounds) <= starts  # boundaries are record starts or the end
        by_ref = {n: dict(bins) for n, bins in zip(idx['names'], idx['refs'])}
        assert list(by_ref) == list(dict.fromkeys(r[0] for r in recs))
        for contig, beg, end, v in recs[::7]:
            bins = by_ref[contig]
            cand = [ch for b in _reg2bins(beg, end, idx['min_shift'], idx['depth']) for ch in bins.get(b, [])]
            assert any(u <= v < w for u, w in cand), (name, contig, beg, end, v)


def test_tbi_range_and_sorting(fixture_files, tmp_path):
    from sbeacon._lib import SbError
    from sbeacon.summarise_vcf import read_index, write_index
    with pytest.raises(SbError):
        write_index(fixture_files['far_csi'], 'tbi')
    assert read_index(write_index(fixture_files['far_csi'], 'csi'))['depth'] == 6
    from sbeacon.workload import write_bgzf
    bad = write_bgzf(str(tmp_path / 'unsorted.vcf.gz'),
                     [b'#CHROM\tPOS\tID\tREF\tALT\n1\t100\t.\tA\tC\n1\t50\t.\tA\tC\n'])
    with pytest.raises(SbError):
        write_index(bad, 'csi')
    split = write_bgzf(str(tmp_path / 'split.vcf.gz'),
                       [b'#CHROM\tPOS\tID\tREF\tALT\n1\t100\t.\tA\tC\n2\t5\t.\tA\tC\n1\t200\t.\tA\tC\n'])
    with pytest.raises(SbError):
        write_index(split, 'tbi')
    # save=True writes <path>.csi, which find_index then prefers
    from sbeacon.summarise_vcf import find_index
    data = write_index(fixture_files['multi3'], 'tbi', save=False)
    assert find_index(str(tmp_path / 'none.vcf.gz')) is None
    p = str(tmp_path / 'm.vcf.gz')
    open(p, 'wb').write(open(fixture_files['multi3'], 'rb').read())
    write_index(p, 'tbi', save=True)
    assert find_index(p) == data
    csi = write_index(p, 'csi', save=True)
    assert find_index(p) == csi
