"""Device duplicateVariantSearch (sb_dedup_count) vs the C restatement
(oracle/summarise_oracle.c orc_dedup_count): random (VCF set, contig, range)
jobs answered in one batched device sort, forced 64-bit-word collisions
(host recount path), the decimal-concatenation key collisions the reference
has, IUPAC records (reference throws), and size-independent properties on a
larger synthetic store."""
import os
import random

import pytest

from conftest import FIXTURES

pytestmark = pytest.mark.gpu

HEADER = b'##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\tS2\n'


def gen_vcf(seed, pool, share=0.7, n_own=400):
    """Records drawn from a shared pool (70 %) plus private ones, sorted."""
    rng = random.Random(seed)
    recs = [r for r in pool if rng.random() < share]
    bases = 'ACGTN'
    for _ in range(n_own):
        chrom = rng.choice(['22', '22', '22', 'X'])
        pos = rng.randrange(1, 3000)
        ref = ''.join(rng.choice(bases) for _ in range(rng.choice([1, 1, 2, 3, 9])))
        alt = rng.choice(['G', 'T,C', '<DEL>', '*', '.', 'ACGTACGTAC', 'g', 'a,,t'])
        recs.append((chrom, pos, ref, alt))
    recs.sort(key=lambda r: (r[0] != '22', r[1]))
    return HEADER + b''.join(f'{c}\t{p}\t.\t{r}\t{a}\t.\tPASS\tAC=1;AN=4\tGT\t0|1\t1|1\n'.encode()
                             for c, p, r, a in recs)


def make_pool(seed=3):
    rng = random.Random(seed)
    pool = []
    for _ in range(600):
        pos = rng.randrange(1, 3000)
        ref = rng.choice(['A', 'C', 'GA', 'GAC', 'TTTTTTTT'])
        alt = rng.choice(['G', 'T', 'C,G', '<DUP:TANDEM>', 'AC'])
        pool.append(('22', pos, ref, alt))
    # decimal-concatenation collisions: "12"+GAC'_G' == "121"+C'_G'
    for p in (12, 34, 56, 230, 251):
        pool.append(('22', p, 'GAC', 'G'))
        pool.append(('22', p * 10 + 1, 'C', 'G'))
    return pool


@pytest.fixture(scope='module')
def texts():
    pool = make_pool()
    t = {f'dd{i}.vcf.gz': gen_vcf(100 + i, pool) for i in range(4)}
    # a VCF with IUPAC codes at known places
    t['iupac.vcf.gz'] = HEADER + (b'22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n'
                                  b'22\t200\t.\tR\tG\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n'
                                  b'22\t300\t.\tA\tM\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n'
                                  b'22\t400\t.\tA\tC\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n')
    for name in ('tiny22', 'quirk22'):
        t[name + '.vcf.gz'] = open(os.path.join(FIXTURES, name + '.vcf'), 'rb').read()
    return t


@pytest.fixture(scope='module')
def store(texts):
    from sbeacon.engine import Store
    return Store.build(list(texts.items()), device=0)


def oracle(texts, locs, contig, lo, hi):
    from oracle.oracle import dedup_count
    try:
        return dedup_count([texts[l] for l in locs], contig, lo, hi)
    except ValueError:
        return ValueError


def random_jobs(texts, rng, n):
    names = [k for k in texts if k.startswith('dd')]
    jobs = []
    for _ in range(n):
        k = rng.randrange(1, len(names) + 1)
        locs = rng.sample(names, k)
        if rng.random() < 0.2:
            locs = rng.choice([['tiny22.vcf.gz'], ['quirk22.vcf.gz'], ['iupac.vcf.gz'], locs + ['iupac.vcf.gz']])
        contig = rng.choice(['22', '22', '22', 'X', '1'])
        lo = rng.randrange(0, 3000)
        hi = lo + rng.choice([0, 1, 10, 500, 3000, 10**8])
        if rng.random() < 0.1:
            lo, hi = 0, 2**40
        jobs.append((locs, contig, lo, hi))
    if 'tiny22.vcf.gz' in texts:
        jobs.append((['tiny22.vcf.gz', 'quirk22.vcf.gz'], '22', 0, 10**9))
    return jobs


def check(texts, jobs, got):
    for j, g in zip(jobs, got):
        e = oracle(texts, *j)
        if e is ValueError:
            assert isinstance(g, NotImplementedError), j
        else:
            assert g == e, (j, g, e)


@pytest.mark.parametrize('exact', ['window', 'window_small', 'bucket', 'radix', 'overflow'])
def test_dedup_batch_vs_oracle(texts, store, monkeypatch, exact):
    """windows (default: each job's runs cut by effective position, one read
    of every key; window_small: windows of ~3 keys, so displaced keys land in
    other windows than their POS and in the gaps between them), the exact
    stream by hash buckets, by the full radix sort, and by buckets whose hash
    sets 'overflow' (a cap of 4 keys per workgroup): the same answers."""
    if exact == 'radix':
        monkeypatch.setenv('SBEACON_DEDUP_EXACT', 'radix')
    elif exact == 'bucket':
        monkeypatch.setenv('SBEACON_DEDUP_EXACT', 'bucket')
    elif exact == 'overflow':
        monkeypatch.setenv('SBEACON_DEDUP_EXACT', 'bucket')
        monkeypatch.setenv('SBEACON_DEDUP_BUCKET_CAP', '4')
    elif exact == 'window_small':
        monkeypatch.setenv('SBEACON_DEDUP_WIN_TARGET', '3')
    rng = random.Random(11)
    jobs = random_jobs(texts, rng, 300)
    got, st = store.dedup_counts(jobs, with_stats=True)
    check(texts, jobs, got)
    assert st['keys'] > 0
    assert st['path'] == {'radix': 'radix', 'bucket': 'buckets', 'overflow': 'radix'}.get(exact, 'windows')
    if exact == 'window_small':
        assert st['windows'] > st['keys'] // 8
    # a single-job call agrees with the batched call
    for j, g in list(zip(jobs, got))[:20]:
        assert store.dedup_counts([j]) == [g]


def test_window_pileup_takes_the_sorted_path(monkeypatch):
    """One POS holding more keys than a window (3,072) cannot be cut: the
    call is answered by the bucket / radix path, with the same count."""
    from oracle.oracle import dedup_count
    from sbeacon.engine import Store
    rows = []
    for i in range(3200):  # 3,200 distinct multi-base REFs at one POS
        ref = ''.join('ACGT'[(i >> (2 * k)) & 3] for k in range(6))
        rows.append(f'22\t500\t.\t{ref}\tA\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n')
    t = HEADER + ''.join(rows).encode() + b'22\t501\t.\tA\tC\t.\t.\tAC=1;AN=2\tGT\t0|1\t0|0\n'
    st = Store.build([('pile.vcf.gz', t)], device=0)
    got, stats = st.dedup_counts([(['pile.vcf.gz'], '22', 0, 10**9), (['pile.vcf.gz'], '22', 501, 501)],
                                 with_stats=True)
    assert stats['path'] != 'windows'
    assert got == [dedup_count([t], '22', 0, 10**9), 1]


def test_decimal_concat_collisions_are_counted_as_the_reference_does(texts, store):
    from oracle.oracle import dedup_count
    t = HEADER + b'22\t12\t.\tGAC\tG\t.\t.\t.\tGT\t0|1\t0|0\n'
    # on the device: the pool's (12, GAC, G) and (121, C, G) entries are one key
    locs = ['dd0.vcf.gz', 'dd1.vcf.gz', 'dd2.vcf.gz', 'dd3.vcf.gz']
    got = store.dedup_counts([(locs, '22', 12, 121), (locs, '22', 13, 121)])
    assert got == [dedup_count([texts[l] for l in locs], '22', 12, 121),
                   dedup_count([texts[l] for l in locs], '22', 13, 121)]
    assert dedup_count([t + b'22\t121\t.\tC\tG\t.\t.\t.\tGT\t0|1\t0|0\n'], '22', 0, 1000) == 1


def test_forced_word_collisions_take_the_exact_host_recount(texts, store, monkeypatch):
    rng = random.Random(12)
    jobs = random_jobs(texts, rng, 120)
    monkeypatch.setenv('SBEACON_DEDUP_HASH_BITS', '3')
    got, st = store.dedup_counts(jobs, with_stats=True)
    assert st['collisions'] > 0
    check(texts, jobs, got)


def test_empty_and_unknown(texts, store):
    assert store.dedup_counts([]) == []
    assert store.dedup_counts([(['dd0.vcf.gz'], 'nope', 0, 10**9), ([], '22', 0, 10**9),
                               (['dd0.vcf.gz'], '22', 50, 10)]) == [0, 0, 0]


def test_handler_with_region_paths(texts):
    import json

    from sbeacon import dedup, engine
    from sbeacon.engine import Store
    locs = ['s3://bkt/dir/dd0.vcf.gz', 's3://bkt/dir/dd1.vcf.gz']
    st = Store.build([(l, texts[l.rsplit('/', 1)[1]]) for l in locs], device=0)
    engine.registry.register(st)
    try:
        tally = dedup.DuplicateTally()
        tally.expect('22', 'ds', [(0, 1499), (1500, 10**9)])
        paths = [f'vcf-summaries/contig/22/{dedup.bucket_key(l)}/regions/1-2999' for l in locs]
        assert paths[0] == 'vcf-summaries/contig/22/bkt%dir%dd0/regions/1-2999'
        msgs = [{'bucket': 'b', 'rangeStart': a, 'rangeEnd': b, 'contig': '22', 'targetFilepaths': paths,
                 'dataset': 'ds'} for a, b in [(0, 1499), (1500, 10**9)]]
        # these keys name no real region file: the intended-range extension
        r0 = dedup.lambda_handler({'Records': [{'Sns': {'Message': json.dumps(msgs[0])}}]}, tally=tally,
                                  strict=False)
        assert r0['statusCode'] == 200
        r1 = dedup.dedup_batch([msgs[1]], tally=tally, strict=False)
        names = ['dd0.vcf.gz', 'dd1.vcf.gz']
        assert r0['uniqueVariants'] == oracle(texts, names, '22', 0, 1499)
        assert r1[0] == oracle(texts, names, '22', 1500, 10**9)
        assert tally.dataset_counts == {'ds': r0['uniqueVariants'] + r1[0]}
    finally:
        engine.registry.clear()


def test_synthetic_store_properties():
    """200k-record chr22-shape VCF A and a subset B of its lines: the union is
    |A|, A alone matches the oracle, and a range split sums to the whole."""
    from oracle.oracle import dedup_count
    from sbeacon.engine import Store
    from sbeacon.workload import SyntheticVcf
    g = SyntheticVcf(n_records=200000, n_samples=4, seed=4)
    a = b''.join(g.chunks(sites_only=True))
    lines = a.split(b'\n')
    rng = random.Random(5)
    b = b'\n'.join(l for l in lines if l.startswith(b'#') or (l and rng.random() < 0.5)) + b'\n'
    st = Store.build([('A.vcf.gz', a), ('B.vcf.gz', b)], device=0, keep_genotypes=False)
    pos = g.positions()
    mid = int(pos[len(pos) // 2])
    whole, union, left, right = st.dedup_counts([(['A.vcf.gz'], '22', 0, 2**32), (['A.vcf.gz', 'B.vcf.gz'], '22', 0, 2**32),
                                                 (['A.vcf.gz'], '22', 0, mid), (['A.vcf.gz'], '22', mid + 1, 2**32)])
    assert whole == dedup_count([a], '22', 0, 2**32)
    assert union == whole
    assert left + right == whole


def test_many_vcfs_in_one_job_fall_back_to_the_sorted_path():
    """A job over more VCFs than a window holds runs (64) is declined by the
    window planner and answered by the sorted path with the same count; a
    job over fewer takes the windows."""
    from oracle.oracle import dedup_count
    from sbeacon.engine import Store
    pool = make_pool(seed=9)
    texts = {f'm{i}.vcf.gz': gen_vcf(500 + i, pool, share=0.3, n_own=40) for i in range(70)}
    st = Store.build(list(texts.items()), device=0)
    names = list(texts)
    got, stats = st.dedup_counts([(names, '22', 0, 10**9)], with_stats=True)
    assert stats['path'] != 'windows'
    assert got == [dedup_count([texts[n] for n in names], '22', 0, 10**9)]
    got, stats = st.dedup_counts([(names[:40], '22', 0, 10**9)], with_stats=True)
    assert stats['path'] == 'windows'
    assert got == [dedup_count([texts[n] for n in names[:40]], '22', 0, 10**9)]

