"""Host logic that surrounds the device path: splitQuery slicing,
coordinate conversion, chromosome matching, payload round trips."""
import pytest

from sbeacon import payloads as P
from sbeacon import split_query, variant_search
from sbeacon.chrom_matching import get_matching_chromosome, match_chromosome_name


def _split(start_min, start_max, vcfs, include='HIT'):
    return P.SplitQueryPayload(passthrough={'x': 1}, dataset_id='d', query_id='q', reference_bases='N',
                               start_min=start_min, start_max=start_max, end_min=start_min, end_max=start_max,
                               alternate_bases='N', variant_type=None, include_datasets=include,
                               vcf_locations=vcfs, vcf_groups=[], requested_granularity='record',
                               variant_min_length=0, variant_max_length=-1)


def test_split_slices_follow_reference():
    # lambda/splitQuery/lambda_function.py:82-106
    ps = split_query.split_payloads(_split(1, 25000, {'a.vcf': '22', 'b.vcf': 'chr22'}))
    assert [p['region'] for p in ps] == ['22:1-10000', 'chr22:1-10000', '22:10001-20000', 'chr22:10001-20000',
                                         '22:20001-25000', 'chr22:20001-25000']
    assert all(p['include_details'] is True for p in ps)
    assert ps[0]['passthrough'] == {'x': 1}
    assert ps[1]['vcf_location'] == 'b.vcf'
    assert split_query.split_payloads(_split(5, 4, {'a.vcf': '22'})) == []
    one = split_query.split_payloads(_split(7, 7, {'a.vcf': '22'}, include='NONE'))
    assert [p['region'] for p in one] == ['22:7-7'] and one[0]['include_details'] is False


def test_payload_round_trip():
    p = P.PerformQueryPayload(region='22:1-2', end_min=1, end_max=2)
    d = p.dump()
    assert P.PerformQueryPayload.load(d).dump() == d
    assert d['query_id'] == 'test' and d['passthrough'] == {}
    r = P.PerformQueryResponse(exists=True, vcf_location='v', dataset_id='d', all_alleles_count=3,
                               variants=['x'], call_count=1)
    assert list(r.dump()) == ['exists', 'vcf_location', 'dataset_id', 'all_alleles_count', 'variants',
                              'call_count', 'sample_indices', 'sample_names']


@pytest.mark.parametrize('name,canon', [('chr1', '1'), ('1', '1'), ('chrX', 'X'), ('chrM', 'MT'), ('Chr22', '22'),
                                        ('x', 'X'), ('GL000.1', '1'), ('HLA-A', None), ('chr12', '12')])
def test_match_chromosome_name(name, canon):
    # shared_resources/utils/chrom_matching.py:71-79: first matching suffix wins, so
    # 'chr12' -> '12' and (reference quirk) 'GL000.1' -> '1'
    assert match_chromosome_name(name) == canon


def test_get_matching_chromosome():
    assert get_matching_chromosome(['chr1', 'chr22'], '22') == 'chr22'
    assert get_matching_chromosome(['chr1'], 'chr1') is None


class _DS:
    def __init__(self, i, vcfs):
        self.id = i
        self._vcfLocations = vcfs
        self._vcfChromosomeMap = [{'vcf': v, 'chromosomes': ['chr22', 'chr1']} for v in vcfs]


def test_variant_search_coordinates(monkeypatch):
    seen = []

    def fake_batch(payloads, **kw):
        seen.extend(payloads)
        return [P.PerformQueryResponse(exists=False, vcf_location=p['vcf_location'], dataset_id=p['dataset_id'],
                                       all_alleles_count=0, variants=[], call_count=0) for p in payloads]

    monkeypatch.setattr(variant_search, 'perform_query_batch', fake_batch)
    kw = dict(referenceName='22', referenceBases='N', alternateBases='N', variantType=None, variantMinLength=0,
              variantMaxLength=-1, requestedGranularity='count', includeResultsetResponses='HIT')
    out = variant_search.perform_variant_search_sync(datasets=[_DS('d1', ['a.vcf']), _DS('d2', ['b.vcf'])],
                                                     start=[99], end=[25000], **kw)
    # shared_resources/variantutils/search_variants.py:179-199: +1, start_max = end_max
    assert len(out) == 6
    assert seen[0]['region'] == 'chr22:100-10099' and seen[0]['end_min'] == 100 and seen[0]['end_max'] == 25001
    assert seen[-1]['region'] == 'chr22:20100-25001'
    seen.clear()
    variant_search.perform_variant_search_sync(datasets=[_DS('d1', ['a.vcf'])], start=[10, 20], end=[30, 40],
                                               dataset_samples=[['S1']], **kw)
    assert seen[0]['region'] == 'chr22:11-21' and (seen[0]['end_min'], seen[0]['end_max']) == (31, 41)
    assert seen[0]['passthrough'] == {'sampleNames': ['S1'], 'selectedSamplesOnly': True}
    # missing end -> (False, []) exactly like the reference's except branch
    assert variant_search.perform_variant_search_sync(datasets=[_DS('d1', ['a.vcf'])], start=[1], end=[],
                                                      **kw) == (False, [])
