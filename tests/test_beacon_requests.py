"""sb_requests_prepare_beacon: the route's query parameters (int64 columns)
turned into SplitQueryPayloads and cut to a shard's core inside the library
(search_variants.py:179-197, lambda/splitQuery/lambda_function.py:74-110,
ShardPlan.slice_runs) plan the same batch as shard_requests +
prepare_shard_requests (numpy routing + sb_requests_prepare_columns).

CPU: host-only stores (the host planner) -- the plan statistics (chains,
chained slices, staging capacity) agree for every rank of worlds 1-3 and
with requests straddling the cuts.  GPU: rows and hit lists equal."""
import os
import sys

import numpy as np
import pytest

from conftest import PKG, REPO  # noqa: F401

sys.path.insert(0, os.path.dirname(__file__))
from test_shard_gloo import _requests_straddling, _shape  # noqa: E402

HOST_ONLY = -1


def _straddling(shape, world):
    """The gloo tests' requests as int64 columns (the Beacon request dtype)."""
    from sbeacon.genome import Requests
    r = _requests_straddling(shape, world)
    return Requests(*(np.asarray(x, dtype=np.int64) for x in (r.ci, r.start, r.width, r.vt, r.vmin, r.vmax)))


def _same_rows(shape, reqs, world, rank):
    from sbeacon.genome import shard_requests, shard_rows
    sr = shard_requests(shape, reqs, world, rank)
    lo, hi = shard_rows(shape, reqs, world, rank)
    assert (lo, hi - lo) == (sr.row_lo, sr.n_rows)
    return sr


@pytest.mark.parametrize('world', [1, 2, 3])
def test_beacon_batch_plans_like_the_sharded_columns(world):
    from sbeacon.genome import prepare_beacon_shard, prepare_shard_requests
    shape = _shape()
    reqs = _straddling(shape, world)
    for rank in range(world):
        # the rank's own shard store: it holds only the contigs of its
        # records (store contig indexes differ from the plan's contig codes)
        store = shape.build_shard_store(world, rank, device=HOST_ONLY)
        try:
            sr = _same_rows(shape, reqs, world, rank)
            a = prepare_shard_requests(store, sr)
            lo, n, b = prepare_beacon_shard(store, shape, reqs, world, rank)
            sa, sb = a.stats(), b.stats()
            for k in ('n_queries', 'hits', 'chained_slices', 'chains'):
                assert sa[k] == sb[k], (world, rank, k, sa, sb)
            assert sa['chained_slices'] > 0
            a.free()
            b.free()
        finally:
            store.close()


def test_beacon_columns_two_element_ranges_and_errors():
    """start / end of two elements (search_variants.py:179-190), codes out of
    range and absent contigs."""
    from sbeacon import _lib
    from sbeacon.genome import LOCATION, VARIANT_TYPES, config3_requests
    from sbeacon.requests import RequestBatch, beacon_requests, request_columns
    shape = _shape()
    reqs = config3_requests(shape, n=600, seed=8)
    store = shape.build_shard_store(1, 0, device=HOST_ONLY)
    try:
        n = len(reqs)
        vid = store.vcf_id(LOCATION)
        s2 = reqs.start + reqs.width // 3
        e1 = reqs.start + reqs.width // 2
        e2 = reqs.start + reqs.width
        q, keep = beacon_requests(n, vcf_id=vid, contig=reqs.ci, start=reqs.start, start2=s2, end=e1, end2=e2,
                                  variant_type=VARIANT_TYPES, variant_type_code=reqs.vt,
                                  variant_min_length=reqs.vmin, variant_max_length=reqs.vmax)
        b = RequestBatch(store, q, n)
        c, keep2 = request_columns(n, vcf_id=vid, contig=reqs.ci.astype(np.uint32), start_min=reqs.start + 1,
                                   start_max=s2 + 1, end_min=e1 + 1, end_max=e2 + 1, variant_type=VARIANT_TYPES,
                                   variant_type_code=reqs.vt, variant_min_length=reqs.vmin,
                                   variant_max_length=reqs.vmax, include_details=1)
        a = RequestBatch(store, c, n)
        sa, sb = a.stats(), b.stats()
        for k in ('n_queries', 'hits', 'chained_slices', 'chains'):
            assert sa[k] == sb[k], (k, sa, sb)
        a.free()
        b.free()
        bad = reqs.vt.copy()
        bad[7] = len(VARIANT_TYPES)
        q, keep = beacon_requests(n, vcf_id=vid, contig=reqs.ci, start=reqs.start, end=e2,
                                  variant_type=VARIANT_TYPES, variant_type_code=bad)
        with pytest.raises(_lib.SbError, match='request 7'):
            RequestBatch(store, q, n)
        # a contig code past the map: no slices for that row
        cm = np.arange(5, dtype=np.uint32)
        q, keep = beacon_requests(n, vcf_id=vid, contig=reqs.ci, contig_map=cm, start=reqs.start, end=e2)
        b = RequestBatch(store, q, n)
        assert b.stats()['chains'] == int((reqs.ci < 5).sum())
        b.free()
    finally:
        store.close()


@pytest.mark.gpu
@pytest.mark.parametrize('world', [1, 2])
def test_beacon_batch_answers_like_the_sharded_columns(world):
    from sbeacon.genome import prepare_beacon_shard, prepare_shard_requests
    shape = _shape()
    reqs = _straddling(shape, world)
    for rank in range(world):
        store = shape.build_shard_store(world, rank, device=0)
        sr = _same_rows(shape, reqs, world, rank)
        ra, ha, oa = prepare_shard_requests(store, sr).answer()
        lo, n, b = prepare_beacon_shard(store, shape, reqs, world, rank)
        rb, hb, ob = b.answer()
        np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(oa, ob)
        np.testing.assert_array_equal(ha, hb)
        assert oa[-1] > 0
        store.close()
