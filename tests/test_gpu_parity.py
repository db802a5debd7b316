"""Device parity: libsbeacon_hip.so (HIP kernels on an MI355X) against the
reference goldens and the C oracle.  Bit-exact: integer and string work."""
import os
import random

import pytest

from conftest import FIXTURES, normalise
from payload_gen import random_payload, read_records

pytestmark = pytest.mark.gpu


def _cmp(got, c):
    """got: response object or exception; c: golden case."""
    if c['error']:
        assert isinstance(got, Exception) and type(got).__name__ == c['error'], (c['payload'], got)
    else:
        assert not isinstance(got, Exception), (c['payload'], got)
        assert normalise(got.dump()) == normalise(c['response']), c['payload']


@pytest.fixture(scope='module')
def fixture_stores():
    from sbeacon.engine import Store
    return {n: Store.build([(n + '.vcf', os.path.join(FIXTURES, n + '.vcf'))], device=0)
            for n in ('tiny22', 'quirk22')}


@pytest.mark.parametrize('fixture', ['tiny22', 'quirk22'])
def test_reference_goldens(goldens, fixture_stores, fixture):
    cases = [c for c in goldens if c['fixture'] == fixture and c['oracle'] == 'reference']
    rs = fixture_stores[fixture].query([c['payload'] for c in cases], strict_variant_type=True)
    got = rs.responses()
    for g, c in zip(got, cases):
        _cmp(g, c)


@pytest.mark.parametrize('fixture', ['tiny22', 'quirk22'])
def test_patched_variant_type_goldens(goldens, fixture_stores, fixture):
    cases = [c for c in goldens if c['fixture'] == fixture and c['oracle'] == 'patched-oracle']
    assert cases
    got = fixture_stores[fixture].query([c['payload'] for c in cases]).responses()
    for g, c in zip(got, cases):
        _cmp(g, c)


@pytest.mark.parametrize('fixture', ['tiny22', 'quirk22'])
@pytest.mark.parametrize('wrap', ['sync', 'sns'])
def test_handler_goldens(goldens, fixture_stores, fixture, wrap, monkeypatch):
    """performQuery lambda_handler (lambda/performQuery/lambda_function.py:
    23-49) against the reference goldens, invoked directly and as an SNS
    record (the payload JSON in Records[0].Sns.Message): the returned dict
    equals the reference response.dump(), and the reference's exception class
    is raised where it raised one (strict variantType, as generated)."""
    import json
    from sbeacon import engine, perform_query
    monkeypatch.setattr(perform_query, 'STRICT_VARIANT_TYPE', True)
    engine.registry.register(fixture_stores[fixture])
    try:
        for c in [c for c in goldens if c['fixture'] == fixture and c['oracle'] == 'reference']:
            ev = c['payload'] if wrap == 'sync' else {'Records': [{'Sns': {'Message': json.dumps(c['payload'])}}]}
            try:
                got = perform_query.lambda_handler(ev, None)
            except Exception as e:  # noqa: BLE001
                got = e
            if c['error']:
                assert type(got).__name__ == c['error'], (c['payload'], got)
            else:
                assert not isinstance(got, Exception), (c['payload'], got)
                assert normalise(got) == normalise(c['response']), c['payload']
    finally:
        engine.registry.clear()


def _vs_oracle(store, orc, payloads):
    got = store.query(payloads).responses()
    exp = orc.perform_query_batch(payloads, patched=True)
    for p, g, e in zip(payloads, got, exp):
        if isinstance(e, type):
            assert isinstance(g, e), (p, g)
        else:
            assert not isinstance(g, Exception), (p, g)
            assert normalise(g.dump()) == normalise(e), p


def wide_vcf(path, n_rec, n_samp, seed):
    """A cohort VCF too wide for make_fixture's pace: random phased GTs over
    1-3 ALTs (allele numbers within the record's ALTs), INFO AC / AN."""
    import numpy as np
    rng = np.random.default_rng(seed)
    gts = [np.array(['0|0', '0|1', '1|0', '1|1', '.|.']), np.array(['0|0', '0|1', '2|1', '0|2', '.|.']),
           np.array(['0|0', '3|1', '0|2', '0/3', '.|.'])]
    with open(path, 'w') as f:
        f.write('##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t')
        f.write('\t'.join(f'S{i}' for i in range(n_samp)) + '\n')
        pos = 16050000
        for r in range(n_rec):
            pos += int(rng.integers(1, 400))
            na = int(rng.integers(1, 4))
            alts = ','.join(rng.choice(['A', 'C', 'T', 'AT', '<DEL>'], size=na, replace=False))
            col = gts[na - 1][rng.choice(5, size=n_samp, p=[0.9, 0.04, 0.03, 0.02, 0.01])]
            ac = ','.join(str(int(x)) for x in rng.integers(0, 50, size=na))
            f.write(f'22\t{pos}\t.\tG\t{alts}\t50\tPASS\tAC={ac};AN={2 * n_samp}\tGT\t' + '\t'.join(col) + '\n')


def test_wide_cohort_samples(tmp_path):
    """66,000 samples = 1,032 bitset words, past the largest register window
    (1,024 words): carriers in the last words must come back.
    includeSamples over every record and selectedSamplesOnly subsets drawn
    from the whole cohort, each against the oracle."""
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    path = str(tmp_path / 'wide.vcf')
    n = 66000
    wide_vcf(path, 24, n, 15)
    store = Store.build([('w.vcf', path)], device=0)
    orc = OracleVcf(path)
    rng = random.Random(3)
    base = dict(dataset_id='ds', query_id='w', reference_bases='N', end_min=0, end_max=10**9, variant_type=None,
                include_details=True, requested_granularity='record', variant_min_length=0, variant_max_length=-1,
                vcf_location='w.vcf')
    payloads = []
    for alt in ('N', 'A', 'C', 'T'):
        payloads.append(dict(base, passthrough={'includeSamples': True}, region='22:16050000-16070000',
                             alternate_bases=alt))
    for k in (3, 50, 4000):
        names = [f'S{i}' for i in rng.sample(range(n), k)] + [f'S{n - 1}', f'S{n - 65}']
        payloads.append(dict(base, passthrough={'sampleNames': names, 'selectedSamplesOnly': True,
                                                'includeSamples': True},
                             region='22:16050000-16070000', alternate_bases='N'))
    _vs_oracle(store, orc, payloads)
    got = store.query(payloads[:1]).responses()[0].dump()
    assert any(int(x[1:]) >= 65536 for x in got['sample_names'])


@pytest.mark.parametrize('seed,quirks,n_rec,n_samp,spw', [(11, False, 20000, 40, '0'), (12, True, 6000, 70, '0'),
                                                            (13, False, 3000, 130, '0'), (11, False, 20000, 40, '8'),
                                                            (12, True, 6000, 70, '3'),
                                                            (14, False, 1500, 4500, 'nacc1')])
def test_random_vs_oracle(tmp_path, monkeypatch, seed, quirks, n_rec, n_samp, spw):
    """spw: slices per wave ('0' = the launch's own choice, one per wave for
    batches this small; '8' / '3' = slice runs with lane-parallel bounds;
    'nacc1' = a 64-word sample register window, so 4,500 samples (71 words)
    take the words-beyond-the-window path)."""
    if spw == 'nacc1':
        monkeypatch.setenv('SBEACON_MAX_NACC', '1')
    elif spw != '0':
        monkeypatch.setenv('SBEACON_SLICES_PER_WAVE', spw)
    from oracle.oracle import OracleVcf
    from sbeacon import synth
    from sbeacon.engine import Store
    path = str(tmp_path / f'r{seed}.vcf')
    synth.make_fixture(path, n_records=n_rec, n_samples=n_samp, seed=seed, quirks=quirks)
    store = Store.build([('r.vcf', path)], device=0)
    orc = OracleVcf(path)
    recs, names = read_records(path)
    rng = random.Random(seed)
    payloads = [random_payload(rng, recs, names, 'r.vcf') for _ in range(3000)]
    _vs_oracle(store, orc, payloads)


def test_multi_vcf_store_and_unknown_contig():
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    locs = {n: os.path.join(FIXTURES, n + '.vcf') for n in ('tiny22', 'quirk22')}
    store = Store.build(list(locs.items()), device=0)
    rng = random.Random(3)
    payloads = []
    for n, path in locs.items():
        recs, names = read_records(path)
        payloads += [random_payload(rng, recs, names, n) for _ in range(400)]
    rng.shuffle(payloads)
    payloads[0] = dict(payloads[0], region='7:1-100000000')  # contig absent -> empty slice
    got = store.query(payloads).responses()
    orcs = {n: OracleVcf(p) for n, p in locs.items()}
    for p, g in zip(payloads, got):
        try:
            e = orcs[p['vcf_location']].perform_query(p, patched=True)
        except Exception as ex:  # noqa: BLE001
            assert type(g) is type(ex), p
            continue
        assert normalise(g.dump()) == normalise(e), p


def test_prepared_batch_is_repeatable():
    from sbeacon.engine import Store
    path = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('t.vcf', path)], device=0)
    recs, names = read_records(path)
    rng = random.Random(9)
    payloads = [random_payload(rng, recs, names, 't.vcf', alt_none_p=0.0) for _ in range(500)]
    b = store.prepare(payloads)
    outs = []
    for _ in range(3):
        b.run()
        b.sync()
        t = b.timing()
        assert t['total_ms'] > 0 and t['scan_ms'] > 0
        outs.append([r.dump() if not isinstance(r, Exception) else type(r) for r in b.fetch().responses()])
    assert outs[0] == outs[1] == outs[2]
    one = [r.dump() if not isinstance(r, Exception) else type(r) for r in store.query(payloads).responses()]
    assert one == outs[0]


def test_handlers_through_registry():
    from sbeacon import engine, perform_query, split_query
    from sbeacon.engine import Store
    path = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('s3://bucket/tiny22.vcf.gz', path)], device=0)
    engine.registry.register(store)
    out = split_query.lambda_handler(dict(passthrough={}, dataset_id='d', query_id='q', reference_bases='N',
                                          start_min=16050000, start_max=16080000, end_min=16050000,
                                          end_max=16080000, alternate_bases='N', variant_type=None,
                                          include_datasets='HIT', vcf_locations={'s3://bucket/tiny22.vcf.gz': '22'},
                                          vcf_groups=[], requested_granularity='record', variant_min_length=0,
                                          variant_max_length=-1), None)
    assert len(out) == 4 and all(o['exists'] for o in out[:3])
    ev = {'Records': [{'Sns': {'Message': __import__('json').dumps(dict(
        region='22:16050000-16059999', reference_bases='N', end_min=0, end_max=10**9, alternate_bases='N',
        include_details=True, requested_granularity='count', variant_min_length=0, variant_max_length=-1,
        vcf_location='s3://bucket/tiny22.vcf.gz', dataset_id='d'))}}]}
    r = perform_query.lambda_handler(ev, None)
    assert r['exists'] and r['call_count'] > 0 and r['variants']
    engine.registry.clear()


@pytest.mark.parametrize('no_range8,spw', [('0', '0'), ('1', '0'), ('0', '8')])
def test_range_words_vs_oracle(tmp_path, monkeypatch, no_range8, spw):
    """ref=alt='N' range requests over a 1000G-shape VCF (one AN at every
    site): RangeHot8 words by default, RangeHot with SBEACON_NO_RANGE8=1;
    both must match the oracle.  Boolean / count granularities exercise the
    early exits, record granularity the hit lists."""
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    from sbeacon.workload import SyntheticVcf, config2_requests, requests_to_payloads
    monkeypatch.setenv('SBEACON_NO_RANGE8', no_range8)
    if spw != '0':
        monkeypatch.setenv('SBEACON_SLICES_PER_WAVE', spw)
    gen = SyntheticVcf(seed=31, n_records=40000, n_samples=8, mean_gap=60.0)
    path = str(tmp_path / 'shape.vcf')
    gen.write(path, sites_only=False)
    store = Store.build([('s.vcf', path)], device=0)
    reqs = config2_requests(gen, n_range=300, n_point=0, seed=77)
    payloads, _ = requests_to_payloads(reqs, vcf_location='s.vcf', chrom='22')
    rng = random.Random(5)
    for p in payloads:
        p['requested_granularity'] = rng.choice(['record', 'record', 'count', 'boolean'])
        p['include_details'] = p['requested_granularity'] == 'record' or rng.random() < 0.3
    _vs_oracle(store, OracleVcf(path), payloads)


def test_general_records_vs_oracle(tmp_path):
    """Records beyond the packed device words (> 64 ALTs, AC beyond int32, a
    GT fallback with ploidy 4) are general records answered by
    general_slice_kernel: every query over them equals the oracle (which is
    pinned to the reference on tests/golden/general_golden.json)."""
    from oracle.oracle import OracleVcf
    from sbeacon.engine import Store
    alts70 = ','.join('A' + 'C' * i for i in range(1, 71))
    lines = ['##fileformat=VCFv4.2', '#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS0\tS1',
             '22\t1000\t.\tA\tG\t50\tPASS\tAC=1;AN=4\tGT\t0|1\t0|0',
             f'22\t2000\t.\tA\t{alts70}\t50\tPASS\tAC={",".join(["1"] * 70)};AN=4\tGT\t0|1\t0|70',
             '22\t3000\t.\tC\tT\t50\tPASS\tAC=3000000000;AN=4\tGT\t0|1\t1|1',
             '22\t4000\t.\tG\tA\t50\tPASS\tAN=8\tGT\t0/1/1/1\t0/0/0/1',
             '22\t4500\t.\tG\tA,C,T,GA,GC,GT,GG,N,TT\t50\tPASS\tAN=8\tGT\t9/2/1\t8|3',
             '22\t4600\t.\tG\tA\t50\tPASS\tAC=' + '7' * 40 + ';AN=' + '3' * 30 + '\tGT\t0|1\t0|0',
             '22\t5000\t.\tT\tC\t50\tPASS\tAC=1;AN=4\tGT\t0|1\t0|0']
    path = str(tmp_path / 'lim.vcf')
    open(path, 'w').write('\n'.join(lines) + '\n')
    store = Store.build([('lim.vcf', path)], device=0)
    orc = OracleVcf(path)
    base = dict(passthrough={'includeSamples': True}, dataset_id='d', query_id='q', reference_bases='N', end_min=0,
                end_max=10**9, variant_type=None, include_details=True, requested_granularity='record',
                variant_min_length=0, variant_max_length=-1, vcf_location='lim.vcf')
    payloads = []
    for a, b in [(900, 1500), (1500, 2500), (2500, 3500), (3500, 4550), (4450, 5500), (1, 10000), (1, 1999)]:
        for alt in ('N', 'G', 'T', 'GA', None):
            for gran, det in (('record', True), ('boolean', True), ('count', False)):
                payloads.append(dict(base, region=f'22:{a}-{b}', alternate_bases=alt, requested_granularity=gran,
                                     include_details=det, variant_type=None if alt else 'INS'))
        payloads.append(dict(base, region=f'22:{a}-{b}', alternate_bases='N',
                             passthrough={'sampleNames': ['S1'], 'selectedSamplesOnly': True}))
    _vs_oracle(store, orc, payloads)
    big = [r for r in store.query(payloads).responses() if not isinstance(r, Exception) and r.call_count > 2**63]
    assert big  # the 40-digit AC came back exact


@pytest.fixture(scope='module')
def general_store():
    from sbeacon.engine import Store
    return Store.build([('general22.vcf', os.path.join(FIXTURES, 'general22.vcf'))], device=0)


def test_general_goldens(general_goldens, general_store):
    """Reference goldens over general records (tests/golden/
    make_general_goldens.py): > 64 ALTs, AC / AN past int64 (exact Python
    ints, up to 4300 digits), GT fallbacks in CPython set order, ploidy > 3,
    huge GT tokens -- through the device, bit for bit."""
    got = general_store.query([c['payload'] for c in general_goldens]).responses()
    for g, c in zip(got, general_goldens):
        _cmp(g, c)


def test_general_vs_oracle_random(general_store):
    """Random payloads over the general-record fixture (every scan
    specialisation hands its slices to general_slice_kernel) against the C
    oracle."""
    from oracle.oracle import OracleVcf
    path = os.path.join(FIXTURES, 'general22.vcf')
    recs, names = read_records(path)
    rng = random.Random(31)
    payloads = [random_payload(rng, recs, names, 'general22.vcf') for _ in range(1500)]
    _vs_oracle(general_store, OracleVcf(path), payloads)


def test_concurrent_query_batches(fixture_stores, goldens):
    """sb_query_batch from 8 host threads at once on one store (the store
    mutex serialises device batches): every thread's responses equal the
    single-threaded ones."""
    from concurrent.futures import ThreadPoolExecutor
    store = fixture_stores['tiny22']
    cases = [c['payload'] for c in goldens if c['fixture'] == 'tiny22' and c['oracle'] == 'patched-oracle']
    cases += [c['payload'] for c in goldens if c['fixture'] == 'tiny22' and c['error'] is None][:400]
    rng = random.Random(9)
    sets = [rng.sample(cases, 120) for _ in range(32)]

    def run(ps):
        return [r.dump() if not isinstance(r, Exception) else type(r).__name__
                for r in store.query(ps).responses()]

    expected = [run(ps) for ps in sets]
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(run, sets))
    assert got == expected
