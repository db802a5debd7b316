"""initDuplicateVariantSearch range planning against
outputs of the REFERENCE functions (tests/golden/make_range_goldens.py ran
getFileNameInfo + sort + calcRangeSplits from
lambda/summariseDataset/initDuplicateVariantSearch.py on 300 key lists)."""
import json
import os

import pytest

from conftest import GOLDEN


@pytest.fixture(scope='module')
def golden():
    with open(os.path.join(GOLDEN, 'range_golden.json')) as f:
        return json.load(f)


def test_calc_range_splits_matches_reference(golden):
    from sbeacon.dedup import calc_range_splits, get_file_name_info
    n_ok = 0
    for c in golden['cases']:
        region = sorted((get_file_name_info(k) for k in c['keys']), key=lambda x: x.startRange)
        if c['error'] == 'timeout':
            with pytest.raises(RuntimeError):
                calc_range_splits(region, golden['abs_max_data_split'], max_iterations=200_000)
            continue
        if c['error']:
            with pytest.raises(Exception) as ei:
                calc_range_splits(region, golden['abs_max_data_split'])
            assert type(ei.value).__name__ == c['error']
            continue
        got = calc_range_splits(region, golden['abs_max_data_split'])
        assert [{'start': s.start, 'end': s.end, 'filePaths': s.filePaths} for s in got] == c['splits']
        n_ok += 1
    assert n_ok >= 250


def test_init_duplicate_variant_search_messages_and_tally():
    from sbeacon.dedup import DuplicateTally, init_duplicate_variant_search
    keys = ['vcf-summaries/contig/22/b%ds%a/regions/100-5000-300',
            'vcf-summaries/contig/22/b%ds%a/regions/9000-12000-500',
            'vcf-summaries/contig/22/b%other/regions/100-5000-300',
            'vcf-summaries/contig/X/b%ds%a/regions/7-70-10']
    tally = DuplicateTally()
    msgs = init_duplicate_variant_search('ds', ['s3://b/ds/a.vcf.gz'], keys, tally=tally, abs_max=1000)
    assert {m['contig'] for m in msgs} == {'22', 'X'}
    m22 = [m for m in msgs if m['contig'] == '22']
    assert all('other' not in p for m in m22 for p in m['targetFilepaths'])
    assert tally.items[('22', 'ds')]['toUpdate'] == {(m['rangeStart'], m['rangeEnd']) for m in m22}
