"""Batched g_variants route (sbeacon.route_batch: one request pass for many
events, bodies folded by sb_route_bodies) against the REFERENCE route's
responses (tests/golden/route_golden.json, made by
tests/golden/make_route_goldens.py from the reference route -> splitQuery ->
performQuery chain).

* CPU: a host-only store (SB_HOST_ONLY) supplies the request planning and
  the text columns sb_route_bodies reads; the request rows and hit lists come
  from the C oracle per splitQuery slice (test-only injection of
  route_batch._answer: the product path is the device pass).
* ``-m gpu``: the device pass (wide and compact outputs), the same goldens;
  config-3-shape requests against the per-slice route on the same store.

Bodies are compared with ``results`` sorted by variantInternalId (the
reference lists them in thread-completion order)."""
import json
import os

import numpy as np
import pytest

from conftest import FIXTURES, GOLDEN

HOST_ONLY = -1
SOURCES = [('tiny22.vcf', os.path.join(FIXTURES, 'tiny22.vcf')), ('quirk22.vcf', os.path.join(FIXTURES, 'quirk22.vcf'))]


@pytest.fixture(scope='module')
def route_golden():
    with open(os.path.join(GOLDEN, 'route_golden.json')) as f:
        return json.load(f)


def _catalog(g):
    from sbeacon.catalog import Catalog, Dataset
    cat = Catalog()
    for d in g['datasets']:
        cat.add(Dataset(**d))
    return cat


def _norm_body(body: str):
    b = json.loads(body)
    for rs in b.get('response', {}).get('resultSets', []):
        rs['results'] = sorted(rs['results'], key=lambda r: r['variantInternalId'])
    return b


def _records(path):
    """(POS, REF, ALTs, VT) of every record in file order."""
    out = []
    with open(path) as f:
        for line in f:
            if line.startswith('#'):
                continue
            c = line.rstrip('\n').split('\t')
            vt = 'N/A'
            for kv in c[7].split(';'):
                if kv.startswith('VT='):
                    vt = kv[3:]
            out.append((int(c[1]), c[3], c[4].split(','), vt))
    return out


def oracle_answerer(sources, patched=False):
    """route_batch._answer from the C oracle: per request row, its splitQuery
    slices through the oracle; each variant string mapped back to (record,
    ALT) of the store (records numbered in file order, VCFs in build order)."""
    from oracle.oracle import OracleVcf
    from sbeacon.split_query import split_payloads
    orcs, index = {}, {}
    base = 0
    for loc, path in sources:
        orcs[loc] = OracleVcf(path)
        recs = _records(path)
        ix = {}
        for r, (pos, ref, alts, vt) in enumerate(recs):
            for k, a in enumerate(alts):
                ix.setdefault((pos, ref, a, vt), base + r | k << 32)
        index[loc] = ix
        base += len(recs)

    def answer(store, payloads, owners, cols, n_rows):
        rows = np.zeros((n_rows, 5), np.int64)
        hits, row_off = [], [0]
        for w, (pi, loc) in enumerate(owners):
            sp = dict(payloads[pi])
            sp['vcf_locations'] = {loc: sp['vcf_locations'][loc]}
            for q in split_payloads(sp):
                try:
                    r = orcs[loc].perform_query(q, patched=patched)
                except Exception:  # noqa: BLE001 (the reference raises on this slice)
                    r = None
                if not isinstance(r, dict):
                    rows[w, 4] += 1
                    continue
                rows[w, 0] += int(r['exists'])
                rows[w, 1] += len(r['variants'])
                for v in r['variants']:
                    _, pos, ref, alt, vt = v.split('\t')
                    hits.append(index[loc][(int(pos), ref, alt, vt)])
            row_off.append(len(hits))
        return rows, np.array(hits, dtype=np.uint64), np.array(row_off, dtype=np.int64)
    return answer


def _check(g, out):
    n_ok = 0
    for c, got in zip(g['cases'], out):
        ev = c['event']
        if c['error']:
            assert isinstance(got, Exception), (ev, got)
            continue
        assert not isinstance(got, Exception), (ev, got)
        exp = c['response']
        assert got['statusCode'] == exp['statusCode'] and got['headers'] == exp['headers'], ev
        assert _norm_body(got['body']) == _norm_body(exp['body']), ev
        n_ok += 1
    return n_ok


def test_route_batch_goldens_host_with_oracle(route_golden, monkeypatch):
    """Every golden event through route_batch on CPU; the /g_variants events
    take the batched form (request batch planned in the library, bodies by
    sb_route_bodies), the others route() with the oracle behind it."""
    from oracle.oracle import OracleVcf
    from sbeacon import engine, route_batch as rb
    import sbeacon.variant_search as vs
    from sbeacon.engine import Store
    from sbeacon.payloads import PerformQueryResponse
    store = Store.build(SOURCES, device=HOST_ONLY)
    engine.registry.register(store)
    orcs = {loc: OracleVcf(p) for loc, p in SOURCES}

    def oracle_batch(payloads, **kw):
        out = []
        for p in payloads:
            try:
                r = orcs[p['vcf_location']].perform_query(p, patched=False)
            except Exception as e:  # noqa: BLE001
                out.append(e)
                continue
            out.append(r('reference error') if isinstance(r, type) else PerformQueryResponse(**r))
        return out

    monkeypatch.setattr(vs, 'perform_query_batch', oracle_batch)
    monkeypatch.setattr(rb, '_answer', oracle_answerer(SOURCES))
    try:
        cases = route_golden['cases']
        out = rb.route_batch([c['event'] for c in cases], [c['query_id'] for c in cases],
                             catalog=_catalog(route_golden))
        n = _check(route_golden, out)
        assert n >= 150
        assert rb.last_stats['batched'] >= 165, rb.last_stats
    finally:
        engine.registry.clear()


def test_route_bodies_dedup_and_envelopes():
    """sb_route_bodies on hand-made rows: equal strings from two VCFs count
    once; equal (pos, ref, alt) with another VT count twice but give one
    entry; boolean / count / record / other granularities; an errored row
    and an escaped compact label go back to route() (status 1)."""
    import base64
    from sbeacon.engine import Store
    from sbeacon.route_batch import route_bodies
    from sbeacon import responses
    tiny = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('a.vcf', tiny), ('b.vcf', tiny)], device=HOST_ONLY)
    recs = _records(tiny)
    n = len(recs)
    # a record with an extra ALT, two records: row 0 (VCF a), row 1 (VCF b) hit the same lines
    multi = next(i for i, r in enumerate(recs) if len(r[2]) > 1)
    picks = [(multi, 0), (multi, 1), (0, 0)]
    h0 = [r | k << 32 for r, k in picks]
    h1 = [n + r | k << 32 for r, k in picks]
    # events 0-2 and 5: rows (a, b) hitting the same lines; 3: one empty row; 4: a raising slice
    pair_rows = [0, 2, 4, 8]
    rows = np.zeros((10, 5), np.int64)
    hit_parts, off = [], [0]
    for r in range(10):
        if r in pair_rows or r - 1 in pair_rows:
            rows[r, 0] = 1
            hit_parts += h0 if r in pair_rows else h1
        off.append(len(hit_parts))
    rows[7, 4] = 1
    hits = np.array(hit_parts, dtype=np.uint64)
    row_off = np.array(off, dtype=np.int64)
    vcf = np.array([0, 1] * 5, np.uint32)
    b = route_bodies(store, rows=rows, hits=hits, row_off=row_off, compact=False,
                     row_lo=[0, 2, 4, 6, 7, 8], row_hi=[2, 4, 6, 7, 8, 10],
                     granularity=[3, 1, 0, 3, 3, 255], check_all=[1, 1, 1, 1, 1, 1],
                     row_vcf=vcf, row_contig=0)
    assert list(b.status) == [0, 0, 0, 0, 1, 2]
    rec = json.loads(b.text(0))
    exp_ids = []
    for r, k in picks:
        pos, ref, alts, vt = recs[r]
        iid = f'GRCh38\t22\t{pos}\t{ref}\t{alts[k]}'
        exp_ids.append(base64.b64encode(iid.encode()).decode())
    assert [e['variantInternalId'] for e in rec['response']['resultSets'][0]['results']] == exp_ids
    assert rec['responseSummary'] == {'exists': True, 'numTotalResults': 3}
    e0 = rec['response']['resultSets'][0]['results'][0]
    pos, ref, alts, vt = recs[multi]
    assert e0 == responses.get_variant_entry(exp_ids[0], 'GRCh38', ref, alts[0], pos, pos + len(alts[0]), vt)
    body = responses.get_result_sets_response(setType='genomicVariant', exists=True, total=3,
                                              results=rec['response']['resultSets'][0]['results'],
                                              reqPagination=responses.get_pagination_object(0, 100))
    assert b.text(0) == json.dumps(body)
    assert b.text(1) == json.dumps(responses.get_counts_response(exists=True, count=3))
    assert b.text(2) == json.dumps(responses.get_boolean_response(exists=True))
    assert b.text(3) == json.dumps(responses.get_result_sets_response(
        setType='genomicVariant', exists=False, total=0, results=[],
        reqPagination=responses.get_pagination_object(0, 100)))
    b.free()
    # compact rows and hits: label 7 is an escape -> route(); others as wide
    rows32 = np.zeros((2, 4), np.uint32)
    rows32[:, 0] = 1
    hits32 = np.array([r | k << 29 for r, k in picks] + [(n + multi) | 7 << 29], dtype=np.uint32)
    off32 = np.array([0, 3, 4], dtype=np.uint32)
    b = route_bodies(store, rows=rows32, hits=hits32, row_off=off32, compact=True, row_lo=[0, 1], row_hi=[1, 2],
                     granularity=[1, 1], check_all=[1, 1], row_vcf=np.array([0, 1], np.uint32), row_contig=0)
    assert list(b.status) == [0, 1]
    assert json.loads(b.text(0))['responseSummary']['numTotalResults'] == 3
    b.free()


def test_route_bodies_same_line_other_vt():
    """Two records with the same POS/REF/ALT and different VT: two variant
    strings (count 2) and one entry (the first seen), as the route's set and
    its `found` set give (route_g_variants.py:157-171)."""
    import tempfile
    from sbeacon.engine import Store
    from sbeacon.route_batch import route_bodies
    hdr = '##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n'
    body = ('22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2;VT=SNP\n'
            '22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2;VT=X\n'
            '22\t100\t.\tA\tG\t.\t.\tAC=1;AN=2;VT=SNP\n')
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, 'v.vcf')
        with open(p, 'w') as f:
            f.write(hdr + body)
        store = Store.build([('v.vcf', p)], device=HOST_ONLY)
        rows = np.zeros((1, 5), np.int64)
        rows[0, 0] = 1
        b = route_bodies(store, rows=rows, hits=np.array([0, 1, 2], np.uint64), row_off=np.array([0, 3], np.int64),
                         compact=False, row_lo=[0], row_hi=[1], granularity=[3], check_all=[1])
        out = json.loads(b.text(0))
        assert out['responseSummary']['numTotalResults'] == 2
        res = out['response']['resultSets'][0]['results']
        assert len(res) == 1 and res[0]['variation']['variantType'] == 'SNP'
        b.free()


@pytest.mark.gpu
@pytest.mark.parametrize('compact', [False, True])
def test_route_batch_goldens_device(route_golden, monkeypatch, compact):
    """The product path: every golden event through route_batch on device 0
    (one request pass per call), wide and compact outputs."""
    from sbeacon import engine, perform_query, route_batch as rb
    from sbeacon.engine import Store
    monkeypatch.setattr(perform_query, 'STRICT_VARIANT_TYPE', True)  # the reference crashes on variantType
    monkeypatch.setattr(rb, 'COMPACT', compact)
    store = Store.build(SOURCES, device=0)
    engine.registry.register(store)
    try:
        cases = route_golden['cases']
        out = rb.route_batch([c['event'] for c in cases], [c['query_id'] for c in cases],
                             catalog=_catalog(route_golden))
        n = _check(route_golden, out)
        assert n >= 150
        assert rb.last_stats['batched'] >= 165, rb.last_stats
    finally:
        engine.registry.clear()


@pytest.mark.gpu
def test_route_batch_genome_matches_route():
    """Config-3-shape events (POST /g_variants, variantType + length bounds,
    every granularity and includeResultsetResponses) on a 240 k-record
    genome store: route_batch (one request pass, compact outputs, bodies by
    sb_route_bodies) equals route() per event (the per-slice device path the
    reference goldens pin), body for body."""
    import random
    from sbeacon import engine, route_batch as rb
    from sbeacon.catalog import Catalog, Dataset
    from sbeacon.genome import CONTIGS, LOCATION, VARIANT_TYPES, GenomeShape, config3_requests
    from sbeacon.route_g_variants import route
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    store = shape.build_shard_store(1, 0, device=0)
    engine.registry.register(store)
    cat = Catalog()
    cat.add(Dataset(id='wgs', assemblyId='GRCh38', vcfLocations=[LOCATION],
                    vcfChromosomeMap=[{'vcf': LOCATION, 'chromosomes': store.contigs(LOCATION)}]))
    reqs = config3_requests(shape, n=600, seed=11)
    rng = random.Random(3)
    events = []
    for i in range(len(reqs)):
        s = int(reqs.start[i])
        w = int(reqs.width[i]) * (rng.choice([1, 6, 30]))  # (up to 3 Mb: some rows past 64 slices go per slice)
        rp = {'start': [s], 'end': [s + w], 'assemblyId': 'GRCh38',
              'referenceName': CONTIGS[int(reqs.ci[i])], 'referenceBases': 'N',
              'variantType': VARIANT_TYPES[int(reqs.vt[i])], 'variantMinLength': int(reqs.vmin[i]),
              'variantMaxLength': int(reqs.vmax[i])}
        q = {'requestParameters': rp, 'requestedGranularity': rng.choice(['record', 'record', 'count', 'boolean',
                                                                          'aggregated']),
             'includeResultsetResponses': rng.choice(['HIT', 'ALL', 'NONE'])}
        if rng.random() < 0.2:
            q['pagination'] = {'skip': rng.randrange(5), 'limit': rng.randrange(1, 50)}
        events.append({'resource': '/g_variants', 'httpMethod': 'POST', 'body': json.dumps({'query': q})})
    try:
        got = rb.route_batch(events, [f'q{i}' for i in range(len(events))], catalog=cat)
        assert rb.last_stats['batched'] == len(events), rb.last_stats
        n_res = 0
        for i, ev in enumerate(events):
            exp = route(ev, f'q{i}', catalog=cat)
            assert not isinstance(got[i], Exception), got[i]
            assert got[i]['statusCode'] == exp['statusCode'] and got[i]['headers'] == exp['headers']
            assert _norm_body(got[i]['body']) == _norm_body(exp['body']), ev
            n_res += len(json.loads(exp['body']).get('response', {}).get('resultSets', [{}])[0].get('results', []))
        assert n_res > 50
    finally:
        engine.registry.clear()
