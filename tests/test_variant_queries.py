"""The async variant-search fan-in (sbeacon.variant_queries):
search_variants.py:27-155 (perform_variant_search: record, publish, fan-out,
poll, yield in response-number order), performQuery's async tail
(search_variants.py:273-317) and the VariantQuery / VariantResponse records
(variant_queries.py:29-59).

CPU: the fan-in bookkeeping with the device batch replaced by a stub (the
coordinates, fan-out sizes, response numbering, the poll's completion and
timeout, the 300 KB checkS3 mark, the handler's SNS path recording).  GPU:
the same search on a real store yields, slice for slice, what the C oracle
(oracle/sbeacon_oracle.c, pinned to the reference goldens) answers for the
payloads the fan-out published, and what perform_variant_search_sync
returns."""
import json
import os
import sys

import pytest

from conftest import FIXTURES, PKG, REPO  # noqa: F401

sys.path.insert(0, os.path.dirname(__file__))
from test_host_logic import _DS  # noqa: E402

KW = dict(referenceName='22', referenceBases='N', alternateBases='N', variantType=None, variantMinLength=0,
          variantMaxLength=-1, requestedGranularity='record', includeResultsetResponses='HIT')


def _stub(seen, big=False):
    from sbeacon import payloads as P

    def batch(payloads, **kw):
        seen.extend(payloads)
        return [P.PerformQueryResponse(exists=True, vcf_location=p['vcf_location'], dataset_id=p['dataset_id'],
                                       all_alleles_count=k, variants=['x' * (400_000 if big and k == 0 else 3)],
                                       call_count=k) for k, p in enumerate(payloads)]
    return batch


def test_fan_in_counts_numbers_and_yields_every_slice(monkeypatch):
    from sbeacon import perform_query, variant_queries as vq
    seen = []
    monkeypatch.setattr(perform_query, 'perform_query_batch', _stub(seen, big=True))
    out = list(vq.perform_variant_search(datasets=[_DS('d1', ['a.vcf', 'b.vcf']), _DS('d2', ['c.vcf'])],
                                         start=[99], end=[25000], query_id='q-fan', timeout=30, **KW))
    # 3 slices (search_variants.py:179-199 coordinates) x 3 VCFs
    assert vq.get_split_query_fan_out(100, 25001) == 3
    assert len(seen) == 9 and len(out) == 9
    assert seen[0]['region'] == 'chr22:100-10099' and seen[0]['query_id'] == 'q-fan'
    assert sorted(r.call_count for r in out) == list(range(9))
    q = vq.VariantQuery('q-fan')
    q.refresh()
    assert (q.fanOut, q.responses, q.responsesCounter, q.complete) == (0, 9, 9, True)
    rows = vq.VariantResponse.batch_get([('q-fan', k) for k in range(1, 10)])
    assert [r.responseNumber for r in rows] == list(range(1, 10))
    assert sum(r.checkS3 for r in rows) == 1  # the one body past 300 KB (performQuery :283)
    assert json.loads(rows[0].result)['dataset_id'] in ('d1', 'd2')


def test_fan_in_times_out_when_a_slice_never_finishes(monkeypatch):
    from sbeacon import perform_query, variant_queries as vq
    from sbeacon import payloads as P

    def failing(payloads, **kw):  # the first slice's Lambda fails: it never marks itself finished
        return [RuntimeError('boom') if k == 0 else
                P.PerformQueryResponse(exists=False, vcf_location=p['vcf_location'], dataset_id=p['dataset_id'],
                                       all_alleles_count=0, variants=[], call_count=0)
                for k, p in enumerate(payloads)]
    monkeypatch.setattr(perform_query, 'perform_query_batch', failing)
    out = list(vq.perform_variant_search(datasets=[_DS('d1', ['a.vcf'])], start=[99], end=[25000],
                                         query_id='q-timeout', timeout=0.5, **KW))
    assert out == []  # the reference's poll loop leaves with no results
    q = vq.VariantQuery('q-timeout')
    q.refresh()
    assert q.fanOut == 1 and q.responses == 2


def test_bad_coordinates_yield_nothing():
    from sbeacon import variant_queries as vq
    assert list(vq.perform_variant_search(datasets=[_DS('d1', ['a.vcf'])], start=[1], end=[], query_id='q-bad',
                                          **KW)) == []


def test_sns_handler_records_its_response(monkeypatch):
    """lambda_function.py:33-39: an SNS-wrapped event is the async path; its
    response is numbered and marked finished under the payload's query id."""
    from sbeacon import perform_query, variant_queries as vq
    from sbeacon import payloads as P
    monkeypatch.setattr(perform_query, 'query_payloads', lambda ps, **kw: [
        P.PerformQueryResponse(exists=True, vcf_location=p['vcf_location'], dataset_id=p['dataset_id'],
                               all_alleles_count=2, variants=['22\t5\tA\tT\tSNP'], call_count=1) for p in ps])
    payload = dict(passthrough={}, dataset_id='d', query_id='q-sns', region='22:1-100', reference_bases='N',
                   end_min=1, end_max=100, alternate_bases='N', variant_type=None, include_details=True,
                   requested_granularity='record', variant_min_length=0, variant_max_length=-1,
                   vcf_location='a.vcf')
    vq.VariantQuery('q-sns').save()
    vq.VariantQuery('q-sns').add_fan_out(1)
    perform_query.lambda_handler({'Records': [{'Sns': {'Message': json.dumps(payload)}}]}, None)
    perform_query.lambda_handler(payload, None)  # a sync invoke records nothing
    q = vq.VariantQuery('q-sns')
    q.refresh()
    assert (q.fanOut, q.responses) == (0, 1)
    (row,) = vq.VariantResponse.batch_get([('q-sns', 1)])
    assert json.loads(row.result)['call_count'] == 1


@pytest.mark.gpu
@pytest.mark.parametrize('kw', [dict(referenceBases='N', alternateBases='N'),
                                dict(referenceBases='N', alternateBases=None, variantType='DEL'),
                                dict(referenceBases='N', alternateBases=None, variantType='INS', variantMaxLength=20),
                                dict(requestedGranularity='boolean', includeResultsetResponses='NONE')])
def test_async_search_matches_oracle_on_device(kw):
    """The async fan-in (search_variants.py:27-155 + performQuery's SNS tail
    :273-317) on the device: every slice response it yields equals the C
    oracle's answer to the payload it published (variantType payloads: the
    patched-oracle intent, as the goldens), and the multiset equals the
    sync search's."""
    sys.path.insert(0, REPO)
    from oracle.oracle import OracleVcf
    from sbeacon import engine, perform_query
    from sbeacon.engine import Store
    from sbeacon.variant_queries import perform_variant_search
    from sbeacon.variant_search import perform_variant_search_sync
    fx = os.path.join(FIXTURES, 'tiny22.vcf')
    store = Store.build([('tiny22.vcf', fx)], device=0)
    engine.registry.register(store)
    published = []
    real = perform_query.perform_query_batch

    def spy(payloads, **k):
        published.extend(payloads)
        return real(payloads, **k)
    orc = OracleVcf(fx)
    try:
        ds = [_DS('d1', ['tiny22.vcf'])]
        ds[0]._vcfChromosomeMap = [{'vcf': 'tiny22.vcf', 'chromosomes': ['22']}]
        args = dict(KW, start=[16050000], end=[16110000])
        args.update(kw)
        sync = perform_variant_search_sync(datasets=ds, **args)
        perform_query.perform_query_batch = spy
        got = list(perform_variant_search(datasets=ds, query_id=f'q-dev-{len(published)}-{id(kw)}', timeout=60,
                                          **args))
        key = lambda d: json.dumps(d, sort_keys=True)  # noqa: E731
        assert len(published) == len(got) > 1
        exp = []
        for p in published:
            e = orc.perform_query(p, patched=p.get('variant_type') is not None)
            e['sample_indices'] = sorted(e['sample_indices'])
            exp.append(key(e))
        dumps = []
        for r in got:
            d = r.dump()
            d['sample_indices'] = sorted(d['sample_indices'])
            dumps.append(key(d))
        assert sorted(dumps) == sorted(exp)
        assert sorted(dumps) == sorted(key(dict(r.dump(), sample_indices=sorted(r.dump()['sample_indices'])))
                                       for r in sync)
    finally:
        perform_query.perform_query_batch = real
        orc.close()
        engine.registry.clear()
