"""The config-3 bench step itself (bench_genome.shard_setup + make_step) on
CPU, world 2 over gloo: each rank routes the requests through the product
sharder (ShardPlan via GenomeShape.plan), answers its sub-requests with the C
oracle over its shard's text in place of the device pass, and runs the
bench's step (answer, then ResultExchange).  Every request's row and hit
list reaches exactly one rank and equals the UNSHARDED oracle's."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO  # noqa: F401

sys.path.insert(0, os.path.dirname(__file__))
from test_shard_gloo import _hit_map, _requests_straddling, _rows_and_hits, _shape, _write  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step_requests(shape, world, scaling):
    """The bench's step requests (bench_genome.step_requests: 300 per GPU
    under weak scaling, 300 in total under strong) plus requests straddling
    every shard cut (their rows travel to the first slice's rank)."""
    import argparse
    from bench_genome import step_requests
    from sbeacon.genome import Requests
    a = step_requests(shape, argparse.Namespace(genome_requests=300, scaling=scaling), world, 0)
    b = _requests_straddling(shape, world)
    r = Requests(*(np.concatenate([getattr(a, f), getattr(b, f)]) for f in ('ci', 'start', 'width', 'vt', 'vmin',
                                                                          'vmax')))
    o = np.lexsort((r.start, r.ci))
    return Requests(r.ci[o], r.start[o], r.width[o], r.vt[o], r.vmin[o], r.vmax[o])


def _worker(rank, world, port, tmp, mode, compact, scaling, q):
    for p in (REPO, PKG, os.path.dirname(__file__)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from bench_genome import make_step, shard_setup
        from oracle.oracle import OracleVcf
        from sbeacon.genome import shard_slices, slice_payloads
        from sbeacon.shard import ResultExchange
        shape = _shape()
        reqs = _step_requests(shape, world, scaling)
        sr, owners, base = shard_setup(shape, reqs, world, rank, mode)
        path = _write(os.path.join(tmp, f'b{world}_{rank}.vcf'), shape.shard_chunks(world, rank))
        sl = shard_slices(shape, reqs, world, rank)
        assert (sl.row_lo, sl.n_rows) == (sr.row_lo, sr.n_rows)
        res = OracleVcf(path, load_gt=False).perform_query_batch(slice_payloads(sl), patched=True)
        rows, hits, row_off = _rows_and_hits(sl, res, _hit_map(os.path.join(tmp, 'full.vcf')))
        # the store's first record is global record `base`: the shard text starts there
        with open(path) as f:
            first = next(line for line in f if not line.startswith('#')).split('\t')[:2]
        assert _hit_map(os.path.join(tmp, 'full.vcf'))[(first[0], int(first[1]))][0] == base

        from sbeacon.requests import widen_hits, widen_rows
        dt = torch.int64
        if compact:  # the bench step's narrow outputs: u32 rows, offsets and hits (record | ALT << 29)
            rows = rows[:, :4].astype(np.uint32).view(np.int32)
            h = hits.view(np.uint64)
            hits = ((h & np.uint64(0xffffffff)) | ((h >> np.uint64(32)) << np.uint64(29))).astype(np.uint32).view(np.int32)
            row_off = row_off.astype(np.int32)
            dt = torch.int32

        def run(p, h, o):  # the oracle in place of the device pass
            p.copy_(torch.from_numpy(rows))
            h[:len(hits)].copy_(torch.from_numpy(hits))
            o.copy_(torch.from_numpy(row_off))

        part = torch.zeros((max(sr.n_rows, 1), 4 if compact else 5), dtype=dt)
        # 'first': room for the received hits, so the merge writes in place;
        # 'rank0': none, so it writes new buffers (both merge paths run)
        hbuf = torch.zeros(len(hits) + (4096 if mode == 'first' else 8), dtype=dt)
        obuf = torch.zeros(sr.n_rows + 1, dtype=dt)
        ex = ResultExchange(dist, rank, world, sr.row_lo, sr.n_rows, owners, 'cpu', row_fields=4 if compact else 5,
                            row_dtype=dt)
        step = make_step(run, ex, part, hbuf, obuf)
        for _ in range(3):  # later steps re-issue the cached P2P op list and the cached merge plan
            got = step()
        mh, mo = ex.merge()
        if ex.recv_hits_n and any(ex.recv_hits_n.values()):
            assert (mh.data_ptr() == hbuf.data_ptr()) == (mode == 'first'), (mode, rank)
        assert not ex.row_overflow()
        if compact:
            mh, mo = widen_hits(mh.numpy()), mo.numpy().astype(np.int64)
            rows_got = widen_rows(got.numpy()[:ex.n_own])
            hl = {k: [int(h) for h in widen_hits(np.array(v, dtype=np.uint64).astype(np.uint32))]
                  for k, v in ex.hit_lists().items()}
        else:
            mh, mo = mh.numpy().view(np.uint64), mo.numpy()
            rows_got = got.numpy()[:ex.n_own].copy()
            hl = {k: [int(h) for h in v] for k, v in ex.hit_lists().items()}
        merged = {ex.own_lo + i: [int(h) for h in mh[mo[i]:mo[i + 1]]] for i in range(ex.n_own)}
        q.put((rank, ex.own_lo, ex.n_own, rows_got, hl, merged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('compact,scaling', [(False, 'weak'), (True, 'weak'), (True, 'strong')])
@pytest.mark.parametrize('mode', ['first', 'rank0'])
def test_bench_step_world2_matches_unsharded_oracle(mode, compact, scaling):
    from oracle.oracle import OracleVcf
    from sbeacon.genome import shard_slices, slice_payloads
    world = 2
    shape = _shape()
    reqs = _step_requests(shape, world, scaling)
    assert len(reqs) == 300 * (world if scaling == 'weak' else 1) + len(_requests_straddling(shape, world))
    with tempfile.TemporaryDirectory() as tmp:
        full = _write(os.path.join(tmp, 'full.vcf'), shape.shard_chunks(1, 0))
        whole = shard_slices(shape, reqs, 1, 0)
        res = OracleVcf(full, load_gt=False).perform_query_batch(slice_payloads(whole), patched=True)
        exp_rows, exp_hits, exp_off = _rows_and_hits(whole, res, _hit_map(full))
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, tmp, mode, compact, scaling, q))
                 for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    owned = np.zeros(len(reqs), dtype=np.int64)
    for rank, lo, n, rows, hl, merged in got:
        if mode == 'rank0' and rank:
            assert n == 0
        owned[lo:lo + n] += 1
        np.testing.assert_array_equal(rows, exp_rows[lo:lo + n])
        for r in range(lo, lo + n):
            e = [int(h) for h in exp_hits.view(np.uint64)[exp_off[r]:exp_off[r + 1]]]
            assert hl.get(r, []) == e, (rank, r)
            assert merged[r] == e, (rank, r, 'merged')
    assert (owned == 1).all()
    assert exp_off[-1] > 20
