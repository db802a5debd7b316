"""g_variants route parity against responses the
REFERENCE route produced (tests/golden/make_route_goldens.py: the whole
route -> splitQuery -> performQuery chain run unmodified in this container).

* ``-m gpu``: the product path — sbeacon.route_g_variants over the HBM store
  (one device batch per request).
* CPU: the same host logic (parameter parsing, fan-out, aggregation,
  envelopes) with the per-slice answers supplied by the C oracle; this pins
  the route layer without a GPU.

The reference iterates performQuery responses in thread-completion order, so
``results`` is compared as a list sorted by variantInternalId; everything else
in the body must be identical.  Reference error cases (performQuery crashes
surfacing as a failed Lambda payload, a missing ``end``) must raise here too.
"""
import json
import os

import pytest

from conftest import FIXTURES, GOLDEN


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


def _run_cases(g, catalog):
    from sbeacon import responses
    from sbeacon.route_g_variants import route, route_id
    assert responses.BEACON_API_VERSION == g['env']['BEACON_API_VERSION']
    assert responses.BEACON_ID == g['env']['BEACON_ID']
    n_ok = 0
    for c in g['cases']:
        ev = c['event']
        fn = route if ev['resource'] == '/g_variants' else route_id
        try:
            got = fn(ev, c['query_id'], catalog=catalog)
            err = None
        except Exception as e:  # noqa: BLE001
            got, err = None, e
        if c['error']:
            assert err is not None, (ev, got)
            continue
        assert err is None, (ev, err)
        exp = c['response']
        assert got['statusCode'] == exp['statusCode'] and got['headers'] == exp['headers'], ev
        assert _norm_body(got['body']) == _norm_body(exp['body']), ev
        n_ok += 1
    return n_ok


def test_request_hash_matches_reference(route_golden):
    from sbeacon.request_hash import hash_query
    for c in route_golden['cases']:
        assert hash_query(c['event']) == c['query_id']


def test_route_goldens_host_logic_with_oracle(route_golden, monkeypatch):
    """Route layer on CPU: the per-slice answers come from the C oracle
    (test-only injection; the product path is the device batch)."""
    from oracle.oracle import OracleVcf
    import sbeacon.variant_search as vs
    orcs = {n: OracleVcf(os.path.join(FIXTURES, n)) for n in ('tiny22.vcf', 'quirk22.vcf')}

    def oracle_batch(payloads, **kw):
        out = []
        for p in payloads:
            r = orcs[p['vcf_location']].perform_query(p, patched=False)
            if isinstance(r, type):
                out.append(r('reference error'))
            else:
                from sbeacon.payloads import PerformQueryResponse
                out.append(PerformQueryResponse(**r))
        return out

    monkeypatch.setattr(vs, 'perform_query_batch', oracle_batch)
    n = _run_cases(route_golden, _catalog(route_golden))
    assert n >= 150


@pytest.mark.gpu
def test_route_goldens_device(route_golden, monkeypatch):
    from sbeacon import engine, perform_query
    from sbeacon.engine import Store
    monkeypatch.setattr(perform_query, 'STRICT_VARIANT_TYPE', True)  # the reference crashes on variantType
    store = Store.build([(n, os.path.join(FIXTURES, n)) for n in ('tiny22.vcf', 'quirk22.vcf')], device=0)
    engine.registry.register(store)
    try:
        n = _run_cases(route_golden, _catalog(route_golden))
    finally:
        engine.registry.clear()
    assert n >= 150


@pytest.mark.gpu
def test_library_aggregation_matches_python():
    """aggregate() over device responses deduplicates the variant strings in
    the library (sb_result_distinct_variants); the same responses without
    their result-set link take the Python set path.  Wide requests, two
    datasets sharing a VCF and a second VCF with the same lines (equal
    strings from different records): identical exists / variants / results."""
    import random
    from sbeacon import engine
    from sbeacon.engine import Store
    from sbeacon.route_g_variants import aggregate
    from sbeacon.catalog import Dataset
    from sbeacon.variant_search import perform_variant_search_sync
    tiny = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('tiny22.vcf', tiny), ('copy22.vcf', tiny)], device=0)  # same lines in two VCFs
    engine.registry.register(store)
    try:
        ds = [Dataset(id='a', assemblyId='G', vcfLocations=['tiny22.vcf'],
                      vcfChromosomeMap=[{'vcf': 'tiny22.vcf', 'chromosomes': ['22']}]),
              Dataset(id='b', assemblyId='G', vcfLocations=['tiny22.vcf', 'copy22.vcf'],
                      vcfChromosomeMap=[{'vcf': v, 'chromosomes': ['22']} for v in ('tiny22.vcf', 'copy22.vcf')])]
        rng = random.Random(4)
        for _ in range(40):
            a = rng.randrange(16050000, 16100000)
            rs = perform_variant_search_sync(
                datasets=ds, referenceName='22', referenceBases='N', alternateBases=rng.choice(['N', 'A', 'T']),
                start=[a], end=[a + rng.choice([100, 5000, 60000])], variantType=None, variantMinLength=0,
                variantMaxLength=-1, requestedGranularity='record', includeResultsetResponses='ALL')
            lib_side = aggregate(rs, granularity='record', check_all=True, assembly_id='G')
            for r in rs:
                r._src = None
            py_side = aggregate(rs, granularity='record', check_all=True, assembly_id='G')
            assert lib_side[0] == py_side[0] and lib_side[1] == py_side[1]
            key = lambda e: e['variantInternalId']  # noqa: E731
            assert sorted(lib_side[2], key=key) == sorted(py_side[2], key=key)
    finally:
        engine.registry.clear()
