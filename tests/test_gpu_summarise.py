"""Device summariseSlice vs the C restatement (oracle/summarise_oracle.c) on
BGZF files: random record-aligned slices (both spellings of a block-boundary
virtual offset), including a fixture built so the reference's skip heuristic
swallows records."""
import json
import os
import sys
import random

import pytest

from bgzf_util import blocks, random_slices, record_starts, text
from conftest import FIXTURES, REPO
from payload_gen import random_payload, read_records

pytestmark = pytest.mark.gpu


def skip_quirk_vcf(n=3000, seed=5):
    """Records whose INFO tails vary a lot: a slice that starts on a long-tail
    record gets a large skipSize and swallows the records after short ones."""
    rng = random.Random(seed)
    out = [b'##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\tB\tC\n']
    pos = 1000
    for i in range(n):
        pos += rng.randrange(0, 40)
        k = rng.choice([0, 0, 0, 1, 2, 40])
        tail = ''.join(f';T{j}={rng.randrange(100)}' for j in range(k))
        info = f'AC={rng.randrange(0, 9)};AN={rng.randrange(6, 7)}{tail}'
        if rng.random() < 0.1:
            info = f'AN={rng.randrange(10)};AC=1,{rng.randrange(3)}'
        alt = 'G' if rng.random() < 0.9 else 'G,T'
        gts = '\t'.join(rng.choice(['0|0', '0|1', '1|1', '0/1']) for _ in range(3))
        out.append(f'7\t{pos}\t.\tA\t{alt}\t.\tPASS\t{info}\tGT\t{gts}\n'.encode())
    return b''.join(out)


def gap_vcf(n=2500, seed=9):
    """Records with occasional POS jumps above MAX_SLICE_GAP (region-file
    splits), multiallelic and indel ALTs."""
    rng = random.Random(seed)
    out = [b'##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\n']
    pos = 500
    for i in range(n):
        pos += rng.choice([1, 5, 40, 300, 99999, 100000, 100001, 250000]) if rng.random() < 0.05 else rng.randrange(0, 60)
        ref = rng.choice(['A', 'C', 'GT', 'TTA'])
        alt = rng.choice(['G', 'T,C', 'A', '<DEL>', 'GTT'])
        out.append(f'3\t{pos}\t.\t{ref}\t{alt}\t.\tPASS\tAC=1;AN=2;DP=9\tGT\t0|1\n'.encode())
    return b''.join(out)


@pytest.fixture(scope='module')
def bgzf_files(tmp_path_factory):
    from sbeacon.workload import SyntheticVcf, write_bgzf
    d = tmp_path_factory.mktemp('bgzf')
    files = {}
    for name in ('tiny22', 'quirk22'):
        files[name] = write_bgzf(str(d / f'{name}.vcf.gz'), [open(os.path.join(FIXTURES, name + '.vcf'), 'rb').read()])
    files['skip7'] = write_bgzf(str(d / 'skip7.vcf.gz'), [skip_quirk_vcf()])
    files['gaps3'] = write_bgzf(str(d / 'gaps3.vcf.gz'), [gap_vcf()])
    g = SyntheticVcf(n_records=30000, n_samples=24, seed=99)
    files['synth'] = write_bgzf(str(d / 'synth.vcf.gz'), g.chunks(threads=4), threads=4)
    return files


@pytest.fixture(scope='module')
def bgzf_store(bgzf_files):
    from sbeacon.engine import Store
    return Store.build([(n + '.vcf.gz', p) for n, p in bgzf_files.items()], device=0)


@pytest.mark.parametrize('name', ['tiny22', 'quirk22', 'skip7', 'synth'])
def test_summarise_slices_vs_oracle(bgzf_files, bgzf_store, name):
    from oracle.oracle import OracleBgzf
    path = bgzf_files[name]
    o = OracleBgzf(path)
    blk, txt = blocks(path), text(path)
    rng = random.Random(len(name))
    slices = random_slices(txt, blk, rng, 300, max_records=2000)
    starts = record_starts(txt)
    slices.append(((blk[0][0] << 16) | starts[0], blk[-1][0] << 16))  # whole file
    got = bgzf_store.summarise_slices([(name + '.vcf.gz', vs, ve) for vs, ve in slices])
    n_skipped = 0
    for (vs, ve), g in zip(slices, got):
        e = o.summarise_slice(vs, ve)
        assert g == e, (name, vs, ve, g, e)
        u0, u1 = o.voff_to_u(vs), o.voff_to_u(ve)
        n_recs = sum(1 for s in starts if u0 <= s < u1)
        n_skipped += n_recs - e['records'] if n_recs else 0
    if name == 'skip7':
        assert n_skipped > 0  # the fixture really exercises the skip heuristic


def test_summarise_rejects_unaligned_slices(bgzf_files, bgzf_store):
    path = bgzf_files['tiny22']
    blk, txt = blocks(path), text(path)
    starts = record_starts(txt)
    from bgzf_util import voff
    mid = voff(blk, starts[10] + 3)
    got = bgzf_store.summarise_slices([('tiny22.vcf.gz', mid, voff(blk, starts[20]))])
    assert isinstance(got[0], NotImplementedError)


def test_bgzf_ingest_matches_text_ingest_for_queries(bgzf_files, bgzf_store):
    """The same VCF ingested from BGZF answers performQuery identically."""
    from oracle.oracle import OracleVcf
    plain = os.path.join(FIXTURES, 'tiny22.vcf')
    orc = OracleVcf(plain)
    recs, names = read_records(plain)
    rng = random.Random(77)
    payloads = [random_payload(rng, recs, names, 'tiny22.vcf.gz') for _ in range(800)]
    got = bgzf_store.query(payloads).responses()
    exp = orc.perform_query_batch(payloads, patched=True)
    for p, g, e in zip(payloads, got, exp):
        if isinstance(e, type):
            assert isinstance(g, e), p
        else:
            d = g.dump()
            d['sample_indices'] = sorted(d['sample_indices'])
            e['sample_indices'] = sorted(e['sample_indices'])
            assert d == e, p


def test_summarise_handler(bgzf_files, bgzf_store):
    import json

    from sbeacon import engine, summarise
    engine.registry.register(bgzf_store)
    path = bgzf_files['synth']
    blk, txt = blocks(path), text(path)
    starts = record_starts(txt)
    msg = {'location': 'synth.vcf.gz', 'virtual_start': (blk[0][0] << 16) | starts[0],
           'virtual_end': blk[-1][0] << 16}
    r = summarise.lambda_handler({'Records': [{'Sns': {'Message': json.dumps(msg)}}]})
    assert r['numVariants'] >= 30000 and r['numCalls'] == 48 * 30000
    engine.registry.clear()


def test_summarise_vcf_partition(bgzf_files, bgzf_store):
    """summariseVcf's partition over store chunk boundaries: slices tile each
    contig, and every slice agrees with the oracle."""
    from oracle.oracle import OracleBgzf
    from sbeacon.summarise_vcf import chunk_boundaries, plan_slices, summarise_vcf
    for name in ('synth', 'tiny22'):
        loc = name + '.vcf.gz'
        cb = chunk_boundaries(bgzf_store, loc)
        slices = plan_slices(bgzf_store, loc)
        assert slices and slices[0][0] == next(iter(cb.values()))[0]
        for (a, b), (c, d) in zip(slices, slices[1:]):
            assert b == c or any(b == v[-1] and c == w[0] for v, w in zip(cb.values(), list(cb.values())[1:]))
        o = OracleBgzf(bgzf_files[name])
        _, stats, tot = summarise_vcf(bgzf_store, loc)
        exp = [o.summarise_slice(a, b) for a, b in slices]
        assert stats == exp
        assert tot['variantCount'] == sum(e['numVariants'] for e in exp)
    # a small stride still covers every record
    assert plan_slices(bgzf_store, 'synth.vcf.gz', stride=7)


@pytest.mark.parametrize('name', ['tiny22', 'skip7', 'gaps3', 'synth'])
def test_region_files_vs_oracle(bgzf_files, bgzf_store, name):
    """summariseSlice's region files (write_data_to_s3.h): visited records
    only, gap splits, file lengths and bytes, against the C restatement."""
    from oracle.oracle import OracleBgzf
    path = bgzf_files[name]
    o = OracleBgzf(path)
    blk, txt = blocks(path), text(path)
    rng = random.Random(3 + len(name))
    slices = random_slices(txt, blk, rng, 120, max_records=3000)
    starts = record_starts(txt)
    slices.append(((blk[0][0] << 16) | starts[0], blk[-1][0] << 16))
    got = bgzf_store.region_files([(name + '.vcf.gz', vs, ve) for vs, ve in slices], with_data=True)
    n_files = 0
    for (vs, ve), g in zip(slices, got):
        try:
            exp, data = o.region_files(vs, ve, with_data=True)
        except ValueError:
            assert isinstance(g, Exception), (name, vs, ve)
            continue
        assert not isinstance(g, Exception), (name, vs, ve, g)
        assert [(f['first_pos'], f['last_pos'], f['bytes'], f['entries']) for f in g] == exp, (name, vs, ve)
        assert b''.join(f['data'] for f in g) == data
        n_files += len(g)
    if name == 'gaps3':
        assert n_files > len(slices)  # the fixture really splits files on gaps


@pytest.fixture(scope='module')
def index_files(tmp_path_factory):
    sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))
    from index_fixtures import FIXTURES, write_fixture
    d = tmp_path_factory.mktemp('idxvcf')
    return {name: write_fixture(name, str(d)) for name in FIXTURES}


def test_summarise_vcf_over_reference_index_slices(index_files):
    """summariseVcf over the CSI / TBI index (tests/golden/index_golden.json,
    the reference handler's own slices): the plan equals the reference's, and
    every slice's counts -- also at the finer partitions -- equal the
    oracle's summariseSlice; sampleCount equals get_sample_count's."""
    from oracle.oracle import OracleBgzf
    from sbeacon.engine import Store
    from sbeacon.summarise_vcf import index_chunk_boundaries, partition_chunks, summarise_vcf
    gold = json.load(open(os.path.join(REPO, 'tests', 'golden', 'index_golden.json')))['cases']
    store = Store.build([(n + '.vcf.gz', p) for n, p in index_files.items()], device=0)
    for c in gold:
        loc = c['fixture'] + '.vcf.gz'
        idx = open(os.path.join(REPO, 'tests', 'golden', 'index', f'{c["fixture"]}.{c["format"]}'), 'rb').read()
        slices, stats, tot = summarise_vcf(store, loc, index=idx)
        assert [list(s) for s in slices] == c['slices']
        assert tot['sampleCount'] == c['sample_count']
        o = OracleBgzf(index_files[c['fixture']])
        assert stats == [o.summarise_slice(a, b) for a, b in slices]
        fine = partition_chunks(index_chunk_boundaries(idx), 20000)
        assert [list(s) for s in fine] == c['partitions']['20000']
        got = store.summarise_slices([(loc, a, b) for a, b in fine])
        assert got == [o.summarise_slice(a, b) for a, b in fine]
        assert sum(s['numVariants'] for s in got) == tot['variantCount']
    # 'auto': no index next to the file, so the ingest writes one (CSI)
    slices, _, _ = summarise_vcf(store, 'multi3.vcf.gz')
    assert [list(s) for s in slices] == next(c['slices'] for c in gold if c['fixture'] == 'multi3'
                                                 and c['format'] == 'csi')
