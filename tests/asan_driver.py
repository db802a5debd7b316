"""Host-code workload for the sanitizer build (tests/test_host_sanitizers.py).

Runs in a child process with the clang AddressSanitizer runtime preloaded and
SBEACON_LIB pointing at build/asan/libsbeacon_hip_asan.so (host code under
ASan + UBSan, request-plan invariant checks on).  No GPU: every store is
host-only (SB_HOST_ONLY).  Covers: VCF ingest (text, BGZF files, the
general-record side table), CSI / TBI writing, request planning (host path:
classification, runs of up to 64 chains, descriptors, staging capacities --
the planner behind the round-3 64-slot fault) on the fixtures and on a
240 k-record genome shape with whole-contig requests, and the performQuery
wire parser (events parsed, then the device call refused).
"""
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (HERE, REPO, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

from sbeacon import _lib  # noqa: E402
from sbeacon.engine import Store  # noqa: E402

FIX = os.path.join(HERE, 'golden', 'fixtures')
HOST_ONLY = -1


def split_payload(rng, recs, loc):
    pos = recs[rng.randrange(len(recs))][1]
    width = rng.choice([0, 1, 50, 5000, 9999, 10000, 25000, 100000, 330000, 3_000_000])
    smin = max(1, pos - rng.randrange(0, width + 1))
    u = rng.random()
    ref, alt = 'N', None
    if u < 0.25:
        alt = 'N'
    elif u < 0.35:
        alt, ref = 'A', rng.choice(['N', 'C', 'G'])
    vt = rng.choice(['DEL', 'INS', 'DUP', 'DUP:TANDEM', 'CNV', 'INV', None])
    emin, emax = (smin, smin + width + rng.choice([0, 10, 10**6])) if rng.random() < 0.7 else (0, 10**9)
    return dict(passthrough={}, dataset_id='d', query_id='q', reference_bases=ref, start_min=smin,
                start_max=smin + width, end_min=emin, end_max=emax, alternate_bases=alt, variant_type=vt,
                include_datasets=rng.choice(['HIT', 'ALL', 'NONE']), vcf_locations={loc: '22'}, vcf_groups=[],
                requested_granularity=rng.choice(['record', 'aggregated', 'count', 'boolean']),
                variant_min_length=rng.choice([0, 1]), variant_max_length=rng.choice([-1, 3, 10]))


def plan_requests(store, payloads):
    from sbeacon.requests import RequestBatch, requests_from_split_payloads
    for columns in (False, True):
        arr, keep, owners = requests_from_split_payloads(store, payloads, columns=columns)
        b = RequestBatch(store, arr, len(owners))  # planning only: a host-only store has no pass
        st = b.stats()
        b.free()
        del keep
    return st


def main():
    from payload_gen import random_payload, read_records
    rng = random.Random(3)
    # 1. fixtures: ingest, request planning, wire parsing
    for fx in ('tiny22', 'quirk22', 'general22'):
        path = os.path.join(FIX, fx + '.vcf')
        store = Store.build([(fx + '.vcf', path)], device=HOST_ONLY)
        recs, names = read_records(path)
        st = plan_requests(store, [split_payload(rng, recs, fx + '.vcf') for _ in range(500)])
        assert st['chains'] > 0, st
        from sbeacon import engine
        from sbeacon.wire import pack_events, perform_query_events_packed
        import json
        engine.registry.register(store)
        try:
            evs = [json.dumps(random_payload(rng, recs, names, fx + '.vcf')) for _ in range(300)]
            evs += ['{"Records": [{"Sns": {"Message": ' + json.dumps(evs[0]) + '}}]}', '{', '[1, 2]', '\xff']
            buf, off = pack_events(evs)
            try:
                perform_query_events_packed(buf, off)
                raise AssertionError('a host-only store answered a device batch')
            except _lib.SbError as e:
                assert e.code == -3, e  # SB_EHIP after the events were parsed and planned
        finally:
            engine.registry.clear()
        store.close()
    # 2. CSI / TBI of BGZF fixtures (index.cpp)
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    from index_fixtures import FIXTURES, write_fixture
    from sbeacon.summarise_vcf import write_index
    with tempfile.TemporaryDirectory() as tmp:
        for name, spec in FIXTURES.items():
            p = write_fixture(name, tmp)
            for fmt in spec[3]:
                assert len(write_index(p, fmt)) > 28
            store = Store.build([(name, p)], device=HOST_ONLY)  # BGZF ingest
            store.close()
    # 3. config-3 shape: runs of 64 whole-contig chains, both request sources
    from sbeacon.genome import (GenomeShape, Requests, VARIANT_TYPES, config3_requests, prepare_shard_requests,
                                shard_requests)
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    base = config3_requests(shape, n=4000, seed=5)
    k = 256
    ci = np.concatenate([np.zeros(k, dtype=base.ci.dtype), base.ci])
    start = np.concatenate([np.arange(k, dtype=base.start.dtype), base.start])
    width = np.concatenate([np.full(k, 248_000_000, dtype=base.width.dtype), base.width])
    vt = np.concatenate([np.arange(k, dtype=base.vt.dtype) % len(VARIANT_TYPES), base.vt])
    vmin = np.concatenate([np.zeros(k, dtype=base.vmin.dtype), base.vmin])
    vmax = np.concatenate([np.full(k, -1, dtype=base.vmax.dtype), base.vmax])
    order = np.lexsort((start, ci))
    reqs = Requests(ci[order], start[order], width[order], vt[order], vmin[order], vmax[order])
    store = shape.build_shard_store(1, 0, device=HOST_ONLY)
    b = prepare_shard_requests(store, shard_requests(shape, reqs, 1, 0))
    st = b.stats()
    assert st['chains'] == len(reqs), st
    b.free()
    store.close()
    print('asan driver ok', flush=True)


if __name__ == '__main__':
    main()
