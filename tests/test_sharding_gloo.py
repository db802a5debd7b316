"""ShardPlan over real VCF files (sbeacon/sharding.py) on CPU: gloo ranks
(world 2 and 3) each take their record range of three fixture VCFs (core +
10 kb halo), answer the payloads routed to them with the C oracle over that
shard's text only, and rank 0 gathers the answers.  They must equal the
REFERENCE goldens (and so the unsharded answers) for every payload; the
request-level routing (split_requests) must hand every splitQuery slice to
exactly one rank."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import FIXTURES, GOLDEN, PKG, REPO, normalise  # noqa: F401

NAMES = ('tiny22', 'quirk22', 'general22')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cases():
    cases = json.load(open(os.path.join(GOLDEN, 'perform_query_golden.json')))['cases']
    cases += json.load(open(os.path.join(GOLDEN, 'general_golden.json')))['cases']
    for c in cases:
        c['payload']['vcf_location'] = c['fixture'] + '.vcf'
    return cases


def _plan(world):
    from sbeacon.sharding import ShardPlan
    return ShardPlan.from_sources([(n + '.vcf', os.path.join(FIXTURES, n + '.vcf')) for n in NAMES], world)


def _worker(rank, world, port, tmp, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from oracle.oracle import OracleVcf
        plan = _plan(world)
        cases = _cases()
        route = plan.route_payloads([c['payload'] for c in cases])
        assert (route >= 0).all()
        oracles = {}
        for v, lay in enumerate(plan.layouts):
            path = os.path.join(tmp, f'w{world}_r{rank}_{v}.vcf')
            with open(path, 'wb') as f:
                f.write(plan.shard_text(rank, v))
            oracles[lay.location] = OracleVcf(path)
        mine = []
        for j in np.flatnonzero(route == rank).tolist():
            c = cases[j]
            try:
                got = oracles[c['payload']['vcf_location']].perform_query(
                    c['payload'], patched=c['oracle'] == 'patched-oracle')
                got = normalise(got)
            except Exception as e:  # noqa: BLE001 - the exception class is the contract
                got = type(e).__name__
            mine.append((j, got))
        out = [None] * world if rank == 0 else None
        dist.gather_object(mine, out, dst=0)
        if rank == 0:
            q.put(('answers', [x for part in out for x in part]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_answers_equal_reference_goldens(world):
    cases = _cases()
    plan = _plan(world)
    sizes = [sum(hi - lo for lo, hi in (plan.record_range(r, v) for v in range(len(NAMES)))) for r in range(world)]
    assert all(s > 0 for s in sizes) and sum(sizes) >= sum(l.n for l in plan.layouts)
    with tempfile.TemporaryDirectory() as tmp:
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, tmp, q)) for r in range(world)]
        for p in procs:
            p.start()
        kind, answers = q.get(timeout=300)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    assert sorted(j for j, _ in answers) == list(range(len(cases)))  # every payload answered once
    bad = []
    for j, got in answers:
        c = cases[j]
        if c['error']:
            ok = got == c['error']
        else:
            ok = isinstance(got, dict) and got == normalise(c['response'])
        if not ok:
            bad.append((j, c['fixture'], c['payload']['region']))
    assert not bad, bad[:5]


def test_cuts_respect_pos_runs_and_halo():
    """No cut splits records of one POS; every rank's range holds each of
    its slices' records (the halo)."""
    plan = _plan(3)
    for r in range(1, 3):
        g = plan.cuts[r]
        v, i, k = plan._locate(g)
        lay = plan.layouts[v]
        if i > lay.contigs[k][1]:
            assert lay.pos[i] != lay.pos[i - 1]
    rng = np.random.default_rng(4)
    for v, lay in enumerate(plan.layouts):
        for _ in range(300):
            a = int(rng.integers(int(lay.pos[0]) - 100, int(lay.pos[-1]) + 100))
            r = int(plan.route(v, 0, a))
            lo, hi = plan.record_range(r, v)
            want = np.flatnonzero((lay.pos >= a) & (lay.pos <= a + 9999))
            assert all(lo <= x < hi for x in want.tolist()), (v, a, r)


def test_split_requests_cover_every_slice_once():
    from sbeacon.requests import request_dtype
    import ctypes as C
    plan = _plan(3)
    rng = np.random.default_rng(9)
    sps = []
    for k in range(200):
        lay = plan.layouts[k % 3]
        smin = int(rng.integers(int(lay.pos[0]) - 20000, int(lay.pos[-1])))
        sps.append(dict(passthrough={}, dataset_id='d', query_id='q', reference_bases='N', start_min=smin,
                        start_max=smin + int(rng.integers(0, 120000)), end_min=0, end_max=10**9,
                        alternate_bases='N', variant_type=None, include_datasets='HIT',
                        vcf_locations={lay.location: '22'}, vcf_groups=[], requested_granularity='record',
                        variant_min_length=0, variant_max_length=-1))
    seen = [[] for _ in sps]
    for r in range(3):
        arr, keep, owners = plan.split_requests(sps, r)
        v = np.frombuffer((C.c_char * (C.sizeof(arr) )).from_address(C.addressof(arr)), dtype=request_dtype())
        for w, (i, loc) in enumerate(owners):
            a, b = int(v['start_min'][w]), int(v['start_max'][w])
            s = a
            while s <= b:
                seen[i].append((s, min(s + 9999, b), r))
                s += 10000
    for i, sp in enumerate(sps):
        exp, s = [], sp['start_min']
        while s <= sp['start_max']:
            exp.append((s, min(s + 9999, sp['start_max'])))
            s += 10000
        got = sorted(seen[i])
        assert [x[:2] for x in got] == exp, i
        vloc = plan.vcf_index[next(iter(sp['vcf_locations']))]
        for a, b, r in got:
            assert int(plan.route(vloc, 0, a)) == r
