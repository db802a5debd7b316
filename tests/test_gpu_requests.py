"""Request batches (sb_requests_prepare / sb_requests_run: the splitQuery
fan-out in the library, rows + dense hit lists in request order) against the
per-slice path: every request's row equals the route-level reduction of its
splitQuery slices' responses and its hit list the concatenation of theirs;
on the config-3 genome shape also against the C oracle."""
import os
import random
import tempfile

import numpy as np
import pytest

from conftest import FIXTURES

pytestmark = pytest.mark.gpu


def _split_payload(rng, recs, names, loc, chrom='22'):
    pos = recs[rng.randrange(len(recs))][1]
    width = rng.choice([0, 1, 50, 5000, 9999, 10000, 25000, 100000, 330000])
    smin = max(1, pos - rng.randrange(0, width + 1))
    smax = smin + width
    u = rng.random()
    ref, alt, vt = 'N', None, rng.choice(['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV', None])
    if u < 0.25:
        alt = 'N'
    elif u < 0.35:
        alt, ref = 'A', rng.choice(['N', 'C', 'G'])
    gran = rng.choice(['record', 'record', 'aggregated', 'count', 'boolean'])
    pt = {}
    r = rng.random()
    if r < 0.1:
        pt = {'includeSamples': True}
    elif r < 0.15 and names:
        pt = {'sampleNames': rng.sample(names, rng.randrange(1, len(names) + 1)), 'selectedSamplesOnly': True}
    emin, emax = (smin, smax + rng.choice([0, 10, 10**6])) if rng.random() < 0.7 else (0, 10**9)
    vmin, vmax = (0, -1) if rng.random() < 0.6 else (rng.choice([0, 1, 2]), rng.choice([-1, 1, 3, 10]))
    return dict(passthrough=pt, dataset_id='d', query_id='q', reference_bases=ref, start_min=smin, start_max=smax,
                end_min=emin, end_max=emax, alternate_bases=alt, variant_type=vt,
                include_datasets=rng.choice(['HIT', 'HIT', 'ALL', 'NONE']), vcf_locations={loc: chrom},
                vcf_groups=[], requested_granularity=gran, variant_min_length=vmin, variant_max_length=vmax)


def _expected(store, split_payloads):
    """Per-slice path: splitQuery's payloads through store.query, reduced per
    request row (route-level sums) + concatenated hit lists."""
    pls, owner = [], []
    for i, sp in enumerate(split_payloads):
        for p in split_payloads_of(sp):
            pls.append(p)
            owner.append(i)
    rs = store.query(pls)
    res = rs.responses()
    # route-level sums per row (sb_request_partial), Python ints wrapped to int64 as the device rows hold them
    acc = [[0, 0, 0, 0, 0] for _ in split_payloads]
    for o, r in zip(owner, res):
        if isinstance(r, Exception):
            acc[o][4] += 1
            continue
        d = r.dump()
        acc[o][0] += 1 if d['exists'] else 0
        acc[o][1] += len(d['variants'])
        acc[o][2] += d['call_count']
        acc[o][3] += d['all_alleles_count']
    # a row whose exact sums leave int64 holds their low 64 bits and is
    # flagged (sb_requests_inexact_rows)
    wrap = lambda x: ((x + 2**63) % 2**64) - 2**63  # noqa: E731
    rows = np.array([[wrap(x) for x in a] for a in acc], dtype=np.int64).reshape(len(split_payloads), 5)
    wide = np.array([any(not -2**63 <= x < 2**63 for x in a[2:4]) for a in acc], dtype=bool)
    hits = [[] for _ in split_payloads]
    for j, o in enumerate(owner):
        if not isinstance(res[j], Exception):
            hits[o].extend(int(r) | (int(a) << 32) for r, a in rs.hits(j))
    return rows, hits, wide


def split_payloads_of(sp):
    from sbeacon.split_query import split_payloads
    return split_payloads(sp)


@pytest.mark.parametrize('fixture', ['tiny22', 'quirk22', 'general22'])
def test_requests_match_slices(fixture):
    from payload_gen import read_records
    from sbeacon.engine import Store
    from sbeacon.requests import RequestBatch, requests_from_split_payloads
    path = os.path.join(FIXTURES, fixture + '.vcf')
    store = Store.build([(fixture + '.vcf', path)], device=0)
    recs, names = read_records(path)
    rng = random.Random(hash(fixture) % 1000)
    sps = [_split_payload(rng, recs, names, fixture + '.vcf') for _ in range(400)]
    sps.append(dict(sps[0], vcf_locations={fixture + '.vcf': 'chrUnknown'}))  # contig the VCF lacks
    sps.append(dict(sps[1], start_min=sps[1]['start_max'] + 1))               # no slices
    arr, keep, owners = requests_from_split_payloads(store, sps)
    b = RequestBatch(store, arr, len(owners))
    rows, hits, ro = b.answer()
    exp_rows, exp_hits, exp_wide = _expected(store, sps)
    np.testing.assert_array_equal(rows, exp_rows)
    np.testing.assert_array_equal(b.inexact_rows(), exp_wide)
    if fixture == 'general22':
        assert exp_wide.any()  # the fixture's AC / AN past int64 reach some rows
    assert np.all(np.diff(ro) == rows[:, 1])
    for w in range(len(sps)):
        assert [int(x) for x in hits[ro[w]:ro[w + 1]]] == exp_hits[w], (w, sps[w])
    st = b.stats()
    assert st['chains'] > 0  # some requests took the chain path
    # the same requests as columns (sb_requests_prepare_columns): identical answers
    cols, keep_c, owners_c = requests_from_split_payloads(store, sps, columns=True)
    assert owners_c == owners
    rows_c, hits_c, ro_c = RequestBatch(store, cols, len(owners)).answer()
    np.testing.assert_array_equal(rows_c, rows)
    np.testing.assert_array_equal(ro_c, ro)
    np.testing.assert_array_equal(hits_c, hits)


@pytest.mark.parametrize('fixture', ['quirk22', 'general22'])
def test_index_staged_hits_match(fixture, monkeypatch):
    """request_eval_kernel stages each hit as its record number (the
    store's records fit 29 bits) or, for larger stores, as its candidate
    index that request_deliver_kernel maps through vc_idx: the index form,
    forced with SBEACON_REQ_INDEX_STAGE (a test hook), gives the same rows
    and hit lists, full-width and compact.  Compact outputs hold every
    answer: rows that do not fit u32 (raising slices, general records) and
    ALT labels past 6 escape (sb_requests_escapes), and the widened outputs
    equal the wide ones -- general22 has hits on ALT indexes past 7."""
    from payload_gen import read_records
    from sbeacon.engine import Store
    from sbeacon.requests import COMPACT_ALL, COMPACT_HITS, RequestBatch, requests_from_split_payloads
    path = os.path.join(FIXTURES, fixture + '.vcf')
    store = Store.build([(fixture + '.vcf', path)], device=0)
    recs, names = read_records(path)
    rng = random.Random(7 + len(fixture))
    sps = [_split_payload(rng, recs, names, fixture + '.vcf') for _ in range(300)]
    arr, keep, owners = requests_from_split_payloads(store, sps)  # keep: the buffers arr points into
    exp_rows, exp_hits, _ = _expected(store, sps)
    # u32 hits hold ALT labels 0..6 directly; 7 and past escape to the batch's side table
    wide_alt = any(h >> 32 > 7 for hl in exp_hits for h in hl)
    assert wide_alt == (fixture == 'general22')
    raising = bool((exp_rows[:, 4] > 0).any())  # rows whose slices raise: no compact row holds them
    for index_stage in ('0', '1'):
        monkeypatch.setenv('SBEACON_REQ_INDEX_STAGE', index_stage)
        for mode in (0, COMPACT_HITS, COMPACT_ALL):
            b = RequestBatch(store, arr, len(owners))
            b.set_compact(mode)
            rows, hits, ro = b.answer()
            er, eh = b.escape_flags()
            assert eh == (mode != 0 and wide_alt), (mode, eh)
            assert (er if mode == COMPACT_ALL and raising else True) and (mode == COMPACT_ALL or not er), (mode, er)
            np.testing.assert_array_equal(rows, exp_rows)
            for w in range(len(sps)):
                assert [int(x) for x in hits[ro[w]:ro[w + 1]]] == exp_hits[w], (index_stage, mode, w)
    assert ro[-1] > 0


def test_genome_requests_match_oracle_and_slices():
    """Config-3 shape (small): shard request batches at world 1 and 2 vs the
    per-slice shard batches (rows + hit lists) and the C oracle (rows; at
    world 1 also every hit list, rendered as (chrom, POS, ALT) against the
    oracle's variant strings in order)."""
    from oracle.oracle import OracleVcf
    from sbeacon.genome import (GenomeShape, config3_requests, prepare_shard_batch, prepare_shard_requests,
                                shard_record_base, shard_requests, shard_slices, slice_payloads)
    from sbeacon.shard import request_rows_from_responses
    import torch
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    reqs = config3_requests(shape, n=2000, seed=1003)
    with tempfile.TemporaryDirectory() as tmp:
        full = os.path.join(tmp, 'full.vcf')
        with open(full, 'wb') as f:
            for c in shape.shard_chunks(1, 0):
                f.write(c)
        orc = OracleVcf(full, load_gt=False)
        whole = shard_slices(shape, reqs, 1, 0)
        res = orc.perform_query_batch(slice_payloads(whole), patched=True)
        exp = request_rows_from_responses(whole.req, res, whole.n_rows)
        exp_v = [[] for _ in range(len(reqs))]
        for o, r in zip(whole.req, res):
            if isinstance(r, dict):
                exp_v[o].extend(tuple(v.split('\t')[i] for i in (0, 1, 3)) for v in r['variants'])
        orc.close()
    alts = {}

    def variant(g, k):  # global record g, ALT k -> (chrom, POS, ALT) from the generator
        ci = int(np.searchsorted(shape.offsets, g, side='right') - 1)
        i = g - int(shape.offsets[ci])
        if (ci, i) not in alts:
            line = shape.gen(ci).records(i, i + 1, sites_only=True).decode().split('\t')
            alts[(ci, i)] = (line[0], line[1], line[4].split(','))
        c, pos, a = alts[(ci, i)]
        return c, pos, a[k]
    for world in (1, 2):
        total = np.zeros((len(reqs), 5), dtype=np.int64)
        for rank in range(world):
            store = shape.build_shard_store(world, rank, device=0)
            sr = shard_requests(shape, reqs, world, rank)
            sl = shard_slices(shape, reqs, world, rank)
            assert (sr.row_lo, sr.n_rows) == (sl.row_lo, sl.n_rows)
            base = shard_record_base(shape, world, rank)
            b = prepare_shard_requests(store, sr)
            rows, hits, ro = b.answer(rec_base=base)
            # the per-slice shard batch (rows + hit lists by sb_batch_deliver)
            sb = prepare_shard_batch(store, sl)
            part = torch.zeros((sl.n_rows, 5), dtype=torch.int64, device='cuda:0')
            h2 = torch.zeros(max(sb.stats()['hits'], 1), dtype=torch.int64, device='cuda:0')
            ro2 = torch.zeros(sl.n_rows + 1, dtype=torch.int64, device='cuda:0')
            sb.set_stream(torch.cuda.current_stream().cuda_stream)
            sb.run()
            sb.deliver(part.data_ptr(), h2.data_ptr(), ro2.data_ptr(), base)
            sb.sync()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(rows, part.cpu().numpy())
            ro2 = ro2.cpu().numpy()
            h2 = h2.cpu().numpy().view(np.uint64)
            for w in range(sr.n_rows):
                assert sorted(hits[ro[w]:ro[w + 1]].tolist()) == sorted(h2[ro2[w]:ro2[w + 1]].tolist()), w
            total[sr.row_lo:sr.row_lo + sr.n_rows] += rows
            if world == 1:
                hv = hits.view(np.uint64)
                checked = 0
                for w in range(sr.n_rows):
                    got = [variant(x & 0xffffffff, x >> 32) for x in hv[ro[w]:ro[w + 1]].tolist()]
                    assert got == exp_v[sr.row_lo + w], w
                    checked += len(got)
                assert checked == int(exp[:, 1].sum()) > 0  # every variant the oracle emits
        np.testing.assert_array_equal(total, exp)


def test_large_batch_scans_multiple_rounds(monkeypatch):
    """A batch past one round of the pass's scans (> 4,096 eval workgroups =
    > 1,048,576 requests for the tile scan; > 16 staging tiles): its rows
    and hit lists equal those of the same requests answered as two batches
    (each within one round), in the compact-hit form the bench step uses."""
    from sbeacon.genome import GenomeShape, Requests, config3_requests, prepare_shard_requests, shard_requests
    from sbeacon.requests import COMPACT_HITS
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    reqs = config3_requests(shape, n=1_150_000, seed=1009)
    store = shape.build_shard_store(1, 0, device=0)

    def answer(r):
        b = prepare_shard_requests(store, shard_requests(shape, r, 1, 0))
        b.set_compact(COMPACT_HITS)
        out = b.answer()
        b.free()
        return out

    rows, hits, ro = answer(reqs)
    assert len(rows) == len(reqs) and (len(reqs) + 63) // 64 > 4 * 4096
    # (past 4,096 eval workgroups the delivery's group sums take a second
    # round of loads; the tile scan gives the same offsets)
    monkeypatch.setenv('SBEACON_REQ_TILE_SCAN', '1')
    rows_t, hits_t, ro_t = answer(reqs)
    monkeypatch.delenv('SBEACON_REQ_TILE_SCAN')
    np.testing.assert_array_equal(rows_t, rows)
    np.testing.assert_array_equal(ro_t, ro)
    np.testing.assert_array_equal(hits_t, hits)
    k = 600_000
    part = [answer(Requests(*(getattr(reqs, f)[sl] for f in ('ci', 'start', 'width', 'vt', 'vmin', 'vmax'))))
            for sl in (slice(0, k), slice(k, None))]
    np.testing.assert_array_equal(rows, np.concatenate([part[0][0], part[1][0]]))
    np.testing.assert_array_equal(ro, np.concatenate([part[0][2][:-1], part[1][2] + part[0][2][-1]]))
    np.testing.assert_array_equal(hits, np.concatenate([part[0][1], part[1][1]]))
    assert ro[-1] > 0


def test_request_batch_is_repeatable():
    """Back-to-back passes (ticket / status re-zeroed per pass) give the same
    rows and hits; the spill path (more hits per run than the LDS buffer)
    is exercised by a dense fixture."""
    from payload_gen import read_records
    from sbeacon.engine import Store
    from sbeacon.requests import RequestBatch, requests_from_split_payloads
    path = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('tiny22.vcf', path)], device=0)
    recs, names = read_records(path)
    lo, hi = recs[0][1], recs[-1][1]
    sps = []
    for k in range(64):  # wide variantType requests over the whole fixture: many hits per run
        sps.append(dict(passthrough={}, dataset_id='d', query_id='q', reference_bases='N', start_min=lo + k,
                        start_max=min(hi, lo + k + 300000), end_min=0, end_max=10**9, alternate_bases=None,
                        variant_type=['DEL', 'INS', 'CNV', 'DUP'][k % 4], include_datasets='HIT',
                        vcf_locations={'tiny22.vcf': '22'}, vcf_groups=[], requested_granularity='record',
                        variant_min_length=0, variant_max_length=-1))
    arr, keep, owners = requests_from_split_payloads(store, sps)
    b = RequestBatch(store, arr, len(owners))
    first = b.answer()
    for _ in range(3):
        again = b.answer()
        for x, y in zip(first, again):
            np.testing.assert_array_equal(x, y)
    exp_rows, exp_hits, _ = _expected(store, sps)
    rows, hits, ro = first
    np.testing.assert_array_equal(rows, exp_rows)
    for w in range(len(sps)):
        assert [int(x) for x in hits[ro[w]:ro[w + 1]]] == exp_hits[w], w
    assert ro[-1] > 320  # more than one LDS buffer of hits in some run


def test_pass_invariants_fail_the_batch(monkeypatch):
    """The request pass checks its per-chain sums against the wave's own
    totals (query_kernels.hip request_eval_kernel): with one chain's
    exists-slice count (SBEACON_REQ_INJECT=1), call-count pull (=2) or AN
    pull (=3) perturbed on the device (a test hook) the batch fails at sync
    with SB_EINTERNAL instead of returning its rows; the SAME batch then
    answers normally once the hook is off (the error word is cleared at the
    sync that reports it)."""
    from payload_gen import read_records
    from sbeacon._lib import SB_EINTERNAL, SbError
    from sbeacon.engine import Store
    from sbeacon.requests import COMPACT_ALL, RequestBatch, requests_from_split_payloads
    path = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('tiny22.vcf', path)], device=0)
    recs, _ = read_records(path)
    lo, hi = recs[0][1], recs[-1][1]
    sps = [dict(passthrough={}, dataset_id='d', query_id='q', reference_bases='N', start_min=lo + k,
                start_max=min(hi, lo + k + 300000), end_min=0, end_max=10**9, alternate_bases=None,
                variant_type=['DEL', 'INS', 'CNV', 'DUP'][k % 4], include_datasets='HIT',
                vcf_locations={'tiny22.vcf': '22'}, vcf_groups=[], requested_granularity='record',
                variant_min_length=0, variant_max_length=-1) for k in range(16)]
    arr, _, owners = requests_from_split_payloads(store, sps)
    exp_rows, _, _ = _expected(store, sps)
    for mode in ('1', '2', '3'):
        for compact in (0, COMPACT_ALL):
            b = RequestBatch(store, arr, len(owners))
            b.set_compact(compact)
            monkeypatch.setenv('SBEACON_REQ_INJECT', mode)
            with pytest.raises(SbError) as e:
                b.answer()
            assert e.value.code == SB_EINTERNAL, (mode, compact)
            monkeypatch.delenv('SBEACON_REQ_INJECT')
            rows, _, _ = b.answer()
            np.testing.assert_array_equal(rows, exp_rows)
            b.free()


def test_shard_plan_stores_on_device():
    """sbeacon.sharding over real fixture VCFs on the device: three shard
    stores (sb_builder_set_record_range: core + halo), every golden payload
    routed to its rank and answered there equals the reference golden; the
    request-level fan-out (split_requests) summed over the ranks equals the
    unsharded store's request rows, hit lists concatenated in rank order."""
    import json
    from conftest import GOLDEN, normalise
    from sbeacon.engine import Store
    from sbeacon.requests import RequestBatch
    from sbeacon.sharding import ShardPlan
    names = ('tiny22', 'quirk22', 'general22')
    sources = [(n + '.vcf', os.path.join(FIXTURES, n + '.vcf')) for n in names]
    world = 3
    plan = ShardPlan.from_sources(sources, world)
    stores = [plan.build_store(r, device=0) for r in range(world)]
    cases = json.load(open(os.path.join(GOLDEN, 'perform_query_golden.json')))['cases']
    cases += json.load(open(os.path.join(GOLDEN, 'general_golden.json')))['cases']
    for c in cases:
        c['payload']['vcf_location'] = c['fixture'] + '.vcf'
    route = plan.route_payloads([c['payload'] for c in cases])
    for r in range(world):
        for oracle in ('reference', 'patched-oracle'):
            idx = [j for j in np.flatnonzero(route == r).tolist() if cases[j]['oracle'] == oracle]
            got = stores[r].query([cases[j]['payload'] for j in idx],
                                  strict_variant_type=oracle == 'reference').responses()
            for j, g in zip(idx, got):
                c = cases[j]
                if c['error']:
                    assert isinstance(g, Exception) and type(g).__name__ == c['error'], (r, c['payload'])
                else:
                    assert not isinstance(g, Exception), (r, c['payload'], g)
                    assert normalise(g.dump()) == normalise(c['response']), (r, c['payload'])
    # request level
    from payload_gen import read_records
    rng = random.Random(77)
    sps = []
    for n in names:
        recs, smp = read_records(os.path.join(FIXTURES, n + '.vcf'))
        sps += [_split_payload(rng, recs, smp, n + '.vcf') for _ in range(120)]
    full = Store.build(sources, device=0)
    from sbeacon.requests import requests_from_split_payloads
    arr, keep, owners = requests_from_split_payloads(full, sps)
    exp_rows, exp_hits, exp_ro = RequestBatch(full, arr, len(owners)).answer()
    tot = np.zeros_like(exp_rows)
    hits_by_row = [[] for _ in owners]
    for r in range(world):
        arr, keep, ow = plan.split_requests(sps, r)
        assert ow == owners
        rows, hits, ro = RequestBatch(stores[r], arr, len(ow)).answer()
        tot += rows
        for w in range(len(ow)):
            hits_by_row[w].extend(hits[ro[w]:ro[w + 1]].tolist())
    np.testing.assert_array_equal(tot, exp_rows)
    # record ids differ between the shard stores and the full store: compare
    # (POS, ALT index) through each store's records
    assert sum(len(h) for h in hits_by_row) == int(exp_ro[-1])


def test_request_batches_concurrent_streams():
    """Request batches take no store lock (sb_requests_prepare / _run): four
    host threads, each preparing its own batch and running it on its own
    stream, give the answers the batches give one at a time."""
    import threading
    import torch
    from payload_gen import read_records
    from sbeacon.engine import Store
    from sbeacon.requests import RequestBatch, requests_from_split_payloads
    path = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('tiny22.vcf', path)], device=0)
    recs, names = read_records(path)
    sets = []
    for t in range(4):
        rng = random.Random(100 + t)
        sets.append([_split_payload(rng, recs, names, 'tiny22.vcf') for _ in range(300)])
    expect = []
    for sps in sets:
        arr, keep, owners = requests_from_split_payloads(store, sps, columns=True)
        expect.append(RequestBatch(store, arr, len(owners)).answer())
    got = [None] * 4
    errors = []

    def work(t):
        try:
            with torch.cuda.stream(torch.cuda.Stream(device=0)):
                arr, keep, owners = requests_from_split_payloads(store, sets[t], columns=True)
                b = RequestBatch(store, arr, len(owners))
                for _ in range(3):
                    got[t] = b.answer()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(4):
        for x, y in zip(got[t], expect[t]):
            np.testing.assert_array_equal(x, y)


def test_device_planned_requests_match_host_planned(monkeypatch):
    """sb_requests_prepare_columns with batch-wide scalar filters plans on the
    device (request_plan_kernel: runs of 64 rows, candidate ranges from the
    coarse index); the same requests as an sb_request array plan on the host.
    Wide requests (up to 5 Mb, hundreds of slices) put more than 4 k
    candidates into some runs (chain starts found past the start bitmap).
    Both must give identical rows, offsets and hit lists."""
    from sbeacon.genome import (CONTIGS, LOCATION, VARIANT_TYPES, GenomeShape, Requests, config3_requests,
                                prepare_shard_requests, shard_requests)
    from sbeacon.requests import RequestBatch, requests_array
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    base = config3_requests(shape, n=3000, seed=77)
    rng = np.random.default_rng(5)
    width = base.width.copy()
    wide = rng.random(len(width)) < 0.1  # 1 - 250 Mb: up to ~25 k slices
    width[wide] = rng.integers(1_000_000, 250_000_000, int(wide.sum()))
    # 192 requests over the whole of contig 1, first in (contig, start)
    # order: three runs of 64 whole-contig chains, each well past the
    # chain-start bitmap's 4 k candidate positions
    k = 192
    ci = np.concatenate([np.zeros(k, dtype=base.ci.dtype), base.ci])
    start = np.concatenate([np.arange(k, dtype=base.start.dtype), base.start])
    width = np.concatenate([np.full(k, 248_000_000, dtype=width.dtype), width])
    vt = np.concatenate([rng.integers(0, len(VARIANT_TYPES), k).astype(base.vt.dtype), base.vt])
    vmin = np.concatenate([np.zeros(k, dtype=base.vmin.dtype), base.vmin])
    vmax = np.concatenate([np.full(k, -1, dtype=base.vmax.dtype), base.vmax])
    order = np.lexsort((start, ci))
    reqs = Requests(ci[order], start[order], width[order], vt[order], vmin[order], vmax[order])
    store = shape.build_shard_store(1, 0, device=0)
    sr = shard_requests(shape, reqs, 1, 0)
    dev_b = prepare_shard_requests(store, sr)  # scalar filters: planned on the device
    names = store.contigs(LOCATION)
    at = {c: i for i, c in enumerate(names)}
    cmap = np.array([at.get(c, 0xffffffff) for c in CONTIGS], dtype=np.uint32)
    arr, keep = requests_array(
        sr.n_rows, vcf_id=store.vcf_id(LOCATION), contig=cmap[sr.ci], start_min=sr.start_min,
        start_max=sr.start_max, end_min=sr.end_min, end_max=sr.end_max, reference=('N',), alternate=(None,),
        variant_type=VARIANT_TYPES, variant_type_code=sr.vt, variant_min_length=sr.vmin,
        variant_max_length=sr.vmax, granularity='record', include_details=1)
    host_b = RequestBatch(store, arr, sr.n_rows)
    sd, sh = dev_b.stats(), host_b.stats()
    assert sd['chains'] == sh['chains'] > 0
    assert sd['hits'] == sh['hits']  # the same staging capacity, however the runs are cut
    rows_d, hits_d, ro_d = dev_b.answer()
    rows_h, hits_h, ro_h = host_b.answer()
    np.testing.assert_array_equal(rows_d, rows_h)
    np.testing.assert_array_equal(ro_d, ro_h)
    np.testing.assert_array_equal(hits_d, hits_h)
    # the first runs of 64 rows (device plan) stage more than 4 k hits, so
    # their candidates run past the chain-start bitmap's 4 k positions
    runs = np.add.reduceat(rows_d[:, 1], np.arange(0, len(rows_d), 64))
    assert runs[:3].min() > 4096, runs[:3]
    # every pass re-planned on the device (the bench step): the same answers
    # pass after pass
    from sbeacon import _lib
    # (fixed-stride staging: each eval wave plans its own run; with
    # SBEACON_REQ_PLAN_APART request_plan_kernel runs first, as before)
    dev_b.set_replan(True)
    # (the delivery sums the eval workgroup totals itself; with
    # SBEACON_REQ_TILE_SCAN request_tile_scan_kernel runs before it)
    for apart, tile in (('0', '0'), ('1', '0'), ('0', '1'), ('0', '0')):
        monkeypatch.setenv('SBEACON_REQ_PLAN_APART', apart)
        monkeypatch.setenv('SBEACON_REQ_TILE_SCAN', tile)
        rows_r, hits_r, ro_r = dev_b.answer()
        assert dev_b.plan_fused() == (apart == '0')  # (this batch stages at a fixed stride)
        np.testing.assert_array_equal(rows_r, rows_h)
        np.testing.assert_array_equal(ro_r, ro_h)
        np.testing.assert_array_equal(hits_r, hits_h)
    with pytest.raises(_lib.SbError):
        host_b.set_replan(True)  # planned on the host: nothing to re-plan from
    # the compact output form (u32 rows, offsets and hits), widened on the host: the same answers,
    # with hits staged as records and (SBEACON_REQ_INDEX_STAGE) as candidate indices
    from sbeacon.requests import COMPACT_HITS
    for b, index_stage in ((dev_b, '0'), (host_b, '0'), (dev_b, '1')):
        monkeypatch.setenv('SBEACON_REQ_INDEX_STAGE', index_stage)
        # u32 hits with wide rows: any batch (per-slice rows included)
        b.set_compact(COMPACT_HITS)
        rows_c, hits_c, ro_c = b.answer()
        np.testing.assert_array_equal(rows_c, rows_h)
        np.testing.assert_array_equal(ro_c, ro_h)
        np.testing.assert_array_equal(hits_c, hits_h)
        b.set_compact(False)
        b.set_compact(True)  # (rows answered per slice narrow too, or escape)
        rows_c, hits_c, ro_c = b.answer()
        np.testing.assert_array_equal(rows_c, rows_h)
        np.testing.assert_array_equal(ro_c, ro_h)
        np.testing.assert_array_equal(hits_c, hits_h)
        b.set_compact(False)
    del keep, dev_b, host_b


def _genome_oracle(shape, reqs, path, patched=True):
    """(request rows, per-request [(chrom, POS, ALT)] in hit order) of the
    C oracle over every splitQuery slice of reqs on the VCF at path."""
    from oracle.oracle import OracleVcf
    from sbeacon.genome import shard_slices, slice_payloads
    from sbeacon.shard import request_rows_from_responses
    orc = OracleVcf(path, load_gt=False)
    whole = shard_slices(shape, reqs, 1, 0)
    res = orc.perform_query_batch(slice_payloads(whole), patched=patched)
    exp = request_rows_from_responses(whole.req, res, whole.n_rows)
    exp_v = [[] for _ in range(len(reqs))]
    for o, r in zip(whole.req, res):
        if isinstance(r, dict):
            exp_v[o].extend(tuple(v.split('\t')[i] for i in (0, 1, 3)) for v in r['variants'])
    orc.close()
    return exp, exp_v


def _vcf_records(path):
    """(chrom, POS, ALTs) of every record in file order (= the store's record ids for one VCF)."""
    out = []
    with open(path) as f:
        for line in f:
            if line[0] == '#':
                continue
            c = line.split('\t', 5)
            out.append((c[0], c[1], c[4].split(',')))
    return out


@pytest.mark.parametrize('n_streams', [1, 2])
def test_timed_step_variant_matches_oracle(n_streams):
    """The exact form the bench step times (bench_genome.py main_genome): 4
    request batches prepared once, each re-planned on the device inside
    every pass (sb_requests_set_replan; the planning fused into
    request_eval_kernel: plan_fused), compact outputs (SB_COMPACT_ALL), run
    in rotation into their own buffers -- on one stream, or (the bench's
    default, --streams 2) batch k on CU-masked stream k mod 2 with two
    batches in flight -- every batch's rows and every hit list against the
    C oracle (patched variantType semantics), not against another device
    path."""
    import torch
    from bench_genome import step_streams
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_requests, shard_requests
    from sbeacon.requests import COMPACT_ALL, widen_compact
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    store = shape.build_shard_store(1, 0, device=0)
    dev = torch.device('cuda', 0)
    ss, ss_destroy = step_streams(torch, dev, n_streams) if n_streams > 1 else \
        ([torch.cuda.current_stream(dev)], lambda: None)
    B = []
    for k in range(4):
        reqs = config3_requests(shape, n=4000, seed=1003 + k)
        sr = shard_requests(shape, reqs, 1, 0)
        b = prepare_shard_requests(store, sr)
        b.set_stream(ss[k % n_streams].cuda_stream)
        b.set_replan(True)
        b.set_compact(COMPACT_ALL)
        cap = max(int(b.stats()['hits']), 1)
        B.append(dict(reqs=reqs, sr=sr, b=b, rows=torch.zeros((sr.n_rows, 4), dtype=torch.int32, device=dev),
                      hits=torch.zeros(cap, dtype=torch.int32, device=dev),
                      ro=torch.zeros(sr.n_rows + 1, dtype=torch.int32, device=dev)))
    for i in range(10):  # the rotation (the bench's warmup + steps)
        x = B[i % 4]
        x['b'].run(x['rows'].data_ptr(), x['hits'].data_ptr(), x['ro'].data_ptr(), 0)
    for x in B:
        x['b'].sync()
        assert x['b'].plan_fused()  # the timed variant: planning inside the eval kernel
        assert x['b'].escape_flags() == (False, False)
        x['b'].set_stream(None)  # (off the step streams before they are destroyed)
    torch.cuda.synchronize()
    ss_destroy()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'full.vcf')
        with open(path, 'wb') as f:
            for c in shape.shard_chunks(1, 0):
                f.write(c)
        recs = _vcf_records(path)
        checked = 0
        for x in B:
            ro32 = x['ro'].cpu().numpy().view(np.uint32)
            rows, hits, ro = widen_compact(x['rows'].cpu().numpy(), x['hits'][:int(ro32[-1])].cpu().numpy(), ro32)
            exp, exp_v = _genome_oracle(shape, x['reqs'], path)
            np.testing.assert_array_equal(rows, exp[x['sr'].row_lo:x['sr'].row_lo + x['sr'].n_rows])
            for w in range(x['sr'].n_rows):
                got = [(recs[h & 0xffffffff][0], recs[h & 0xffffffff][1], recs[h & 0xffffffff][2][h >> 32])
                       for h in hits[ro[w]:ro[w + 1]].tolist()]
                assert got == exp_v[x['sr'].row_lo + w], w
                checked += len(got)
        assert checked > 200


def test_compact_escapes_in_genome_batch():
    """A config-3-shape batch whose windows reach a record with 10 ALTs and
    one with an AC past 2^32 (general record): those requests are answered
    per slice inside the batch, and SB_COMPACT_ALL still answers the whole
    batch -- the ALT labels past 6 and the rows past u32 escape to the
    batch's side tables (sb_requests_escapes), and the widened rows and hit
    lists equal the C oracle's."""
    from sbeacon.engine import Store
    from sbeacon.genome import (CONTIGS, LOCATION, GenomeShape, Requests, config3_requests, prepare_shard_requests,
                                shard_requests)
    from sbeacon.requests import COMPACT_ALL
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    ci_y = len(CONTIGS) - 1
    _, last = shape.span(ci_y)
    p1, p2 = last + 100, last + 300
    ref = 'ACGTACGTACG'
    alts = [ref[:k] for k in range(1, 11)]  # ten deletions: ALT indexes 0..9
    extra = (f'{CONTIGS[ci_y]}\t{p1}\t.\t{ref}\t{",".join(alts)}\t.\tPASS\tAC={",".join(str(k + 1) for k in range(10))};'
             f'AN=5008;VT=INDEL\n'
             f'{CONTIGS[ci_y]}\t{p2}\t.\tACGT\tA\t.\tPASS\tAC=5000000000;AN=5000000000;VT=INDEL\n')
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'esc.vcf')
        with open(path, 'wb') as f:
            for c in shape.shard_chunks(1, 0):
                f.write(c)
            f.write(extra.encode())
        store = Store.build([(LOCATION, path)], device=0)
        base = config3_requests(shape, n=3000, seed=21)
        k = 200  # DEL requests whose windows hold the two records
        rng = np.random.default_rng(8)
        start = (p1 - 1 - rng.integers(0, 5000, k)).astype(base.start.dtype)
        reqs_ci = np.concatenate([base.ci, np.full(k, ci_y, dtype=base.ci.dtype)])
        reqs_start = np.concatenate([base.start, start])
        width = np.concatenate([base.width, rng.integers(5400, 30000, k).astype(base.width.dtype)])
        vt = np.concatenate([base.vt, np.zeros(k, dtype=base.vt.dtype)])  # DEL
        vmin = np.concatenate([base.vmin, np.zeros(k, dtype=base.vmin.dtype)])
        vmax = np.concatenate([base.vmax, np.full(k, -1, dtype=base.vmax.dtype)])
        order = np.lexsort((reqs_start, reqs_ci))
        reqs = Requests(reqs_ci[order], reqs_start[order], width[order], vt[order], vmin[order], vmax[order])
        sr = shard_requests(shape, reqs, 1, 0)
        b = prepare_shard_requests(store, sr)
        assert b.stats()['n_queries'] > 0  # some requests went per slice
        b.set_compact(COMPACT_ALL)
        rows, hits, ro = b.answer()
        assert b.escape_flags() == (True, True)
        exp, exp_v = _genome_oracle(shape, reqs, path)
        recs = _vcf_records(path)
        np.testing.assert_array_equal(rows, exp[sr.row_lo:sr.row_lo + sr.n_rows])
        big = 0
        for w in range(sr.n_rows):
            got = [(recs[h & 0xffffffff][0], recs[h & 0xffffffff][1], recs[h & 0xffffffff][2][h >> 32])
                   for h in hits[ro[w]:ro[w + 1]].tolist()]
            assert got == exp_v[sr.row_lo + w], w
            big += sum(1 for h in hits[ro[w]:ro[w + 1]].tolist() if h >> 32 >= 7)
        assert big > 0 and (rows[:, 2] > 2**32).any()
