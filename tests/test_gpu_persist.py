"""Persisted stores on the device: a store saved (sb_store_save) and re-opened
(sb_store_open: the device image streamed back, no VCF re-read) answers
every reference golden, the general-record goldens, summariseSlice, dedup
and config-3-shape request batches exactly as the store it was saved from."""
import os
import random
import tempfile

import numpy as np
import pytest

from conftest import FIXTURES, normalise

pytestmark = pytest.mark.gpu


def _same(a, b):
    if isinstance(a, Exception):
        assert type(a) is type(b), (a, b)
    else:
        assert normalise(a.dump()) == normalise(b.dump())


@pytest.mark.parametrize('fixture', ['tiny22', 'quirk22', 'general22'])
def test_reopened_store_answers_like_the_original(goldens, general_goldens, fixture):
    from sbeacon.engine import Store
    path = os.path.join(FIXTURES, fixture + '.vcf')
    st = Store.build([(fixture + '.vcf', path)], device=0)
    with tempfile.TemporaryDirectory() as tmp:
        st.save(tmp)
        again = Store.open(tmp, device=0)
    assert again.info()['n_records'] == st.info()['n_records']
    cases = [c for c in goldens + general_goldens if c['fixture'] == fixture]
    assert cases
    pay = [c['payload'] for c in cases]
    for strict in (False, True):
        a = st.query(pay, strict_variant_type=strict).responses()
        b = again.query(pay, strict_variant_type=strict).responses()
        for x, y in zip(a, b):
            _same(x, y)
    if fixture == 'tiny22':
        jobs = [([fixture + '.vcf'], '22', lo, lo + span) for lo, span in ((0, 10**9), (16050000, 200000), (5, 5))]
        assert again.dedup_counts(jobs) == st.dedup_counts(jobs)


def test_reopened_genome_store_request_batches():
    """Config-3 shape (240 k records): request rows and hit lists from the
    re-opened store equal the original's."""
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_requests, shard_requests
    from sbeacon.engine import Store
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    reqs = config3_requests(shape, n=4000, seed=21)
    st = shape.build_shard_store(1, 0, device=0)
    with tempfile.TemporaryDirectory() as tmp:
        st.save(tmp)
        again = Store.open(tmp, device=0)
    sr = shard_requests(shape, reqs, 1, 0)
    a = prepare_shard_requests(st, sr).answer()
    b = prepare_shard_requests(again, sr).answer()
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert a[2][-1] > 0
