"""Contig sharding + the request-row gather on CPU (gloo, world 2 and 3).

Each rank writes its shard of a small whole-genome store (core + 10 kb halo,
sbeacon/genome.py) as VCF text and answers its slices with the C oracle;
the per-request rows go through sbeacon.shard.RequestGather (torch.distributed
gather) exactly as the GPU path does with RCCL.  Rank 0 checks the combined
table against the oracle over the UNSHARDED genome, and every rank checks
that each of its slices sees exactly the records the whole genome has there
(the halo makes slices shard-local).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shape():
    from sbeacon.genome import GenomeShape
    return GenomeShape(n_total=240_000, seed=3, n_samples=0)


def _requests(shape):
    from sbeacon.genome import config3_requests
    return config3_requests(shape, n=1500, seed=1003)


def _write(path, chunks):
    with open(path, 'wb') as f:
        for c in chunks:
            f.write(c)
    return path


def _answer(orc, sl):
    from sbeacon.genome import slice_payloads
    from sbeacon.shard import request_rows_from_responses
    res = orc.perform_query_batch(slice_payloads(sl), patched=True)
    return request_rows_from_responses(sl.req, res, sl.n_rows)


def _worker(rank, world, port, tmp, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from oracle.oracle import OracleVcf
        from sbeacon.genome import CONTIGS, shard_slices
        from sbeacon.shard import RequestGather
        shape = _shape()
        reqs = _requests(shape)
        path = _write(os.path.join(tmp, f'shard{world}_{rank}.vcf'), shape.shard_chunks(world, rank))
        orc = OracleVcf(path, load_gt=False)
        sl = shard_slices(shape, reqs, world, rank)
        full = OracleVcf(os.path.join(tmp, 'full.vcf'), load_gt=False)
        for j in range(0, len(sl), 7):  # halo: the shard holds every record of each of its slices
            region = f'{CONTIGS[sl.ci[j]]}:{sl.a[j]}-{sl.b[j]}'
            assert orc.records_in_region(region) == full.records_in_region(region), region
        rows = _answer(orc, sl)
        g = RequestGather(dist, rank, world, sl.row_lo, sl.n_rows, len(reqs), 'cpu')
        g.part[:sl.n_rows] = torch.from_numpy(rows)
        tot = g.exchange()
        if rank == 0:
            q.put(('total', tot.numpy().copy(), len(sl)))
        else:
            q.put(('n', None, len(sl)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_gather_matches_unsharded_oracle(world):
    from oracle.oracle import OracleVcf
    from sbeacon.genome import request_slices, shard_slices
    shape = _shape()
    reqs = _requests(shape)
    with tempfile.TemporaryDirectory() as tmp:
        _write(os.path.join(tmp, 'full.vcf'), shape.shard_chunks(1, 0))
        # expected: every slice of every request against the whole genome
        whole = shard_slices(shape, reqs, 1, 0)
        assert len(whole) == len(request_slices(reqs)[0])
        exp = _answer(OracleVcf(os.path.join(tmp, 'full.vcf'), load_gt=False), whole)
        assert exp[:, 1].sum() > 0 and exp[:, 0].sum() > 0  # the workload has hits
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, tmp, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    total = next(t for k, t, _ in got if k == 'total')
    assert sum(n for _, _, n in got) == len(whole)  # every slice answered exactly once
    np.testing.assert_array_equal(total, exp)


def test_cuts_partition_records():
    shape = _shape()
    for world in (1, 2, 5, 8):
        cores = []
        cuts = shape.cuts(world)
        assert cuts[0] == (0, 0) and len(cuts) == world + 1
        assert all(cuts[i] <= cuts[i + 1] for i in range(world))
        tot = 0
        for r in range(world):
            n = shape.shard_records(world, r)
            cores.append(n)
            tot += n
        assert tot >= shape.n_total  # halos only add records
        assert max(cores) - min(cores) <= 0.05 * shape.n_total / world + 200


def test_vectorised_queries_match_payload_path():
    """genome.shard_query_array == engine.queries_from_payloads(slice_payloads)."""
    import ctypes as C
    from sbeacon.engine import queries_from_payloads
    from sbeacon.genome import shard_query_array, shard_slices, slice_payloads
    shape = _shape()
    sl = shard_slices(shape, _requests(shape), 2, 1)
    a, _k1 = shard_query_array(sl, 7)
    b, _k2 = queries_from_payloads(slice_payloads(sl), lambda loc: 7)
    strs = [('region', 'region_len'), ('reference_bases', 'reference_len'), ('alternate_bases', 'alternate_len'),
            ('variant_type', 'variant_type_len'), ('sample_names', 'sample_names_len')]
    scal = ['vcf_id', 'end_min', 'end_max', 'variant_min_length', 'variant_max_length', 'granularity',
            'include_details', 'include_samples', 'selected_samples_only', 'strict_variant_type']
    assert len(sl) > 100
    for i in range(len(sl)):
        for f in scal:
            assert getattr(a[i], f) == getattr(b[i], f), (i, f)
        for pf, lf in strs:
            va, vb = getattr(a[i], pf), getattr(b[i], pf)
            assert (va is None) == (vb is None), (i, pf)
            la, lb = getattr(a[i], lf), getattr(b[i], lf)
            assert la == lb, (i, lf)
            if va is not None:
                assert va[:la] == vb[:lb], (i, pf)


def _hit_map(path):
    """(chrom, pos) -> (global record index, ALT list) of a whole-genome VCF
    written in (contig, POS) order: the record numbering shard stores use
    (genome.shard_record_base + shard record index)."""
    m = {}
    gid = 0
    with open(path) as f:
        for line in f:
            if line.startswith('#'):
                continue
            c = line.split('\t', 5)
            m[(c[0], int(c[1]))] = (gid, c[4].split(','))
            gid += 1
    return m


def _rows_and_hits(sl, responses, hmap):
    """Per-request rows + dense hit lists (sb_batch_compact_hits layout) from
    per-slice oracle responses: hit = global record | ALT index << 32."""
    from sbeacon.shard import request_rows_from_responses
    rows = request_rows_from_responses(sl.req, responses, sl.n_rows)
    per_row = [[] for _ in range(sl.n_rows)]
    for o, r in zip(sl.req, responses):
        if isinstance(r, dict):
            for v in r['variants']:
                chrom, pos, ref, alt, _ = v.split('\t')
                gid, alts = hmap[(chrom, int(pos))]
                per_row[o].append(gid | (alts.index(alt) << 32))
    row_off = np.zeros(sl.n_rows + 1, dtype=np.int64)
    row_off[1:] = np.cumsum([len(x) for x in per_row])
    hits = np.array([h for x in per_row for h in x] or [0], dtype=np.uint64).view(np.int64)
    return rows, hits, row_off


def _requests_straddling(shape, world):
    """The test requests plus, at every shard cut, requests whose slices fall
    on both sides (their rows must travel to the first slice's rank)."""
    from sbeacon.genome import Requests
    base = _requests(shape)
    ci, st, wd, vt = [], [], [], []
    for c, p in shape.cuts(world)[1:-1]:
        for k in range(5):
            ci.append(c)
            st.append(p - 25000 + 3000 * k)
            wd.append(60000 + 9000 * k)
            vt.append(k % 5)
    n = len(ci)
    r = Requests(np.concatenate([base.ci, ci]), np.concatenate([base.start, st]),
                 np.concatenate([base.width, wd]), np.concatenate([base.vt, vt]),
                 np.concatenate([base.vmin, np.zeros(n, dtype=base.vmin.dtype)]),
                 np.concatenate([base.vmax, -np.ones(n, dtype=base.vmax.dtype)]))
    o = np.lexsort((r.start, r.ci))
    return Requests(r.ci[o], r.start[o], r.width[o], r.vt[o], r.vmin[o], r.vmax[o])


def _exchange_worker(rank, world, port, tmp, mode, q):
    import sys
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from oracle.oracle import OracleVcf
        from sbeacon.genome import first_rank_of_rows, shard_slices, slice_payloads
        from sbeacon.shard import ResultExchange, owner_ranks
        shape = _shape()
        reqs = _requests_straddling(shape, world)
        path = _write(os.path.join(tmp, f'x{world}_{rank}.vcf'), shape.shard_chunks(world, rank))
        sl = shard_slices(shape, reqs, world, rank)
        res = OracleVcf(path, load_gt=False).perform_query_batch(slice_payloads(sl), patched=True)
        rows, hits, row_off = _rows_and_hits(sl, res, _hit_map(os.path.join(tmp, 'full.vcf')))
        owners = owner_ranks(first_rank_of_rows(shape, reqs, world, sl), mode, rank)
        ex = ResultExchange(dist, rank, world, sl.row_lo, sl.n_rows, owners, 'cpu')
        for _ in range(2):  # repeated steps reuse the receive buffers (part is rewritten every step)
            got = ex.exchange(torch.from_numpy(rows.copy()), torch.from_numpy(hits), torch.from_numpy(row_off))
        q.put((rank, ex.own_lo, ex.n_own, len(ex.recvs), got.numpy()[:ex.n_own].copy(),
               {k: [int(h) for h in v] for k, v in ex.hit_lists().items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,mode', [(2, 'first'), (3, 'first'), (2, 'rank0'), (3, 'rank0')])
def test_result_exchange_rows_and_hit_lists(world, mode):
    """Every request's combined row and hit list reach exactly one rank (its
    host-facing rank) and equal the unsharded oracle's; 'rank0' = all at 0."""
    from oracle.oracle import OracleVcf
    from sbeacon.genome import shard_slices, slice_payloads
    shape = _shape()
    reqs = _requests_straddling(shape, world)
    with tempfile.TemporaryDirectory() as tmp:
        full = _write(os.path.join(tmp, 'full.vcf'), shape.shard_chunks(1, 0))
        whole = shard_slices(shape, reqs, 1, 0)
        res = OracleVcf(full, load_gt=False).perform_query_batch(slice_payloads(whole), patched=True)
        exp_rows, exp_hits, exp_off = _rows_and_hits(whole, res, _hit_map(full))
        assert exp_off[-1] > 20 and (exp_rows[:, 1] > 0).sum() > 10
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, tmp, mode, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    owned = np.zeros(len(reqs), dtype=np.int64)
    assert sum(k for _, _, _, k, _, _ in got) >= (world - 1 if mode == 'first' else world - 1)
    for rank, lo, n, _, rows, hl in got:
        if mode == 'rank0' and rank:
            assert n == 0
        owned[lo:lo + n] += 1
        np.testing.assert_array_equal(rows, exp_rows[lo:lo + n])
        for r in range(lo, lo + n):
            e = [int(h) for h in exp_hits.view(np.uint64)[exp_off[r]:exp_off[r + 1]]]
            assert hl.get(r, []) == e, (rank, r)
    assert (owned == 1).all()
