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
