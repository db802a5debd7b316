"""Whole-genome sharding on the device (config 3 shape, small): two shard
stores + the unsharded store on one MI355X.  Per-slice answers of each
shard's vectorised batch (genome.prepare_shard_batch) are checked against the
C oracle, the device per-request rows (sb_batch_reduce_requests) against the
host statement of the same reduction, and the summed shard rows against the
unsharded store's rows."""
import os
import tempfile

import numpy as np
import pytest

from conftest import normalise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def genome():
    from sbeacon.genome import GenomeShape, config3_requests
    shape = GenomeShape(n_total=240_000, seed=3, n_samples=0)
    return shape, config3_requests(shape, n=1500, seed=1003)


def _rows(batch, n_rows):
    import torch
    out = torch.zeros((max(n_rows, 1), 5), dtype=torch.int64, device='cuda:0')
    batch.run()
    batch.reduce_requests(out.data_ptr())
    batch.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy()[:n_rows]


@pytest.mark.parametrize('spw', ['0', '8'])
def test_shards_match_oracle_and_unsharded(genome, monkeypatch, spw):
    """spw '8': slice runs (8 slices per wave, candidate positions mapped in
    the run prologue) on a batch small enough to default to one per wave."""
    if spw != '0':
        monkeypatch.setenv('SBEACON_SLICES_PER_WAVE', spw)
    from oracle.oracle import OracleVcf
    from sbeacon.genome import prepare_shard_batch, shard_slices, slice_payloads
    from sbeacon.shard import combine_host, request_rows_from_responses
    shape, reqs = genome
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        full_path = os.path.join(tmp, 'full.vcf')
        with open(full_path, 'wb') as f:
            for c in shape.shard_chunks(1, 0):
                f.write(c)
        orc = OracleVcf(full_path, load_gt=False)
        whole = shard_slices(shape, reqs, 1, 0)
        exp = request_rows_from_responses(whole.req, orc.perform_query_batch(slice_payloads(whole), patched=True),
                                          whole.n_rows)
        full_store = shape.build_shard_store(1, 0, device=0)
        got_full = _rows(prepare_shard_batch(full_store, whole), whole.n_rows)
        np.testing.assert_array_equal(got_full, exp)
        windows, parts = [], []
        for r in range(world):
            store = shape.build_shard_store(world, r, device=0)
            sl = shard_slices(shape, reqs, world, r)
            b = prepare_shard_batch(store, sl)
            rows = _rows(b, sl.n_rows)
            pl = slice_payloads(sl)
            ores = orc.perform_query_batch(pl, patched=True)
            np.testing.assert_array_equal(rows, request_rows_from_responses(sl.req, ores, sl.n_rows))
            b.payloads = pl
            rs = b.fetch()
            for j in range(0, len(sl), 5):  # per-slice answers, bit-exact
                e = ores[j]
                g = rs.response(j)
                assert normalise(g.dump()) == normalise(e), pl[j]
            windows.append((sl.row_lo, sl.n_rows))
            parts.append(rows)
        np.testing.assert_array_equal(combine_host(windows, parts, len(reqs)), exp)


@pytest.mark.parametrize('chains', ['1', '0'])
def test_compact_hits_match_fetch(genome, monkeypatch, chains):
    """sb_batch_compact_hits (device scan + gather, chain-dense regions) and
    the fused sb_batch_deliver give each request row the concatenation of its
    slices' fetched hits, with the shard's global record base added, on the
    caller's torch stream."""
    import torch
    if chains == '0':
        monkeypatch.setenv('SBEACON_NO_CHAINS', '1')
    from sbeacon.genome import prepare_shard_batch, shard_record_base, shard_slices, slice_payloads
    shape, reqs = genome
    world, rank = 2, 1
    store = shape.build_shard_store(world, rank, device=0)
    sl = shard_slices(shape, reqs, world, rank)
    b = prepare_shard_batch(store, sl)
    b.set_stream(torch.cuda.current_stream().cuda_stream)
    cap = b.stats()['hits']
    hits = torch.full((max(cap, 1),), -1, dtype=torch.int64, device='cuda:0')
    row_off = torch.zeros(sl.n_rows + 1, dtype=torch.int64, device='cuda:0')
    part = torch.zeros((sl.n_rows, 5), dtype=torch.int64, device='cuda:0')
    base = shard_record_base(shape, world, rank)
    for k in range(3):  # without / with the reduced rows handed over, then the fused deliver
        b.run()
        if k < 2:
            b.reduce_requests(part.data_ptr())
            b.compact_hits(hits.data_ptr(), row_off.data_ptr(), base, rows_ptr=part.data_ptr() if k else 0)
        else:
            hits.fill_(-1)
            row_off.zero_()
            part.zero_()
            b.deliver(part.data_ptr(), hits.data_ptr(), row_off.data_ptr(), base)
    b.sync()
    torch.cuda.synchronize()
    ro = row_off.cpu().numpy()
    h = hits.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(np.diff(ro), part.cpu().numpy()[:, 1])
    b.payloads = slice_payloads(sl)
    rs = b.fetch()
    per_row = [[] for _ in range(sl.n_rows)]
    for j, o in enumerate(sl.req):
        per_row[o].extend((base + r) | (a << 32) for r, a in rs.hits(j))
    assert ro[-1] == sum(len(x) for x in per_row) > 0
    for w in range(sl.n_rows):
        assert [int(x) for x in h[ro[w]:ro[w + 1]]] == per_row[w], w


def test_genotype_bitmatrix_shard_answers_like_gt_text():
    """The config-3 store with its carrier bit-matrix attached
    (build_shard_store(genotypes=True): sites-only text + the planes the GT
    columns would give, sb_builder_attach_carriers), on the second shard of
    two (carrier rows aligned to the shard's record range): sample-collecting
    payloads answer exactly as the oracle over the same records' GT text."""
    import random
    from oracle.oracle import OracleVcf
    from sbeacon.genome import CONTIGS, LOCATION, GenomeShape
    shape = GenomeShape(n_total=120_000, seed=3, n_samples=96)
    world, rank = 2, 1
    pieces = shape.shard_pieces(world, rank)
    store = shape.build_shard_store(world, rank, device=0, genotypes=True)
    assert store.info()['device_bytes'] > 0
    rng = random.Random(17)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'shard_gt.vcf')
        with open(path, 'wb') as f:
            f.write(shape.gen(pieces[0][0]).header(sites_only=False))
            for ci, a, b in pieces:
                f.write(shape.gen(ci).records(a, b, sites_only=False))
        orc = OracleVcf(path)
        payloads = []
        for _ in range(60):
            ci, a, b = pieces[rng.randrange(len(pieces))]
            pos = shape.gen(ci).positions()[a:b]
            x = int(pos[rng.randrange(len(pos))])
            pt = {'includeSamples': True}
            if len(payloads) % 2:  # a sample subset (the selected-samples path)
                pt = {'includeSamples': True, 'selectedSamplesOnly': True,
                      'sampleNames': rng.sample(shape.gen(0).sample_names(), 20)}
            payloads.append(dict(passthrough=pt, dataset_id='d', query_id='g',
                                 region=f'{CONTIGS[ci]}:{x}-{x + rng.randrange(1, 9999)}', reference_bases='N',
                                 end_min=0, end_max=10**9, alternate_bases='N', variant_type=None,
                                 include_details=True, requested_granularity='record', variant_min_length=0,
                                 variant_max_length=-1, vcf_location=LOCATION))
        rs = store.query(payloads)
        hits = 0
        for i, p in enumerate(payloads):
            got = rs.response(i).dump()
            exp = orc.perform_query(p)
            assert normalise(got) == normalise(exp), p
            hits += len(got['sample_names'])
        assert hits > 0
    store.close()
