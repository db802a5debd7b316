#!/usr/bin/env python3
"""Config 3 bench (``python bench.py --workload genome``): whole-genome
1000G-shape store sharded by contig across the GPUs (sbeacon/genome.py), 1 M
variantType Beacon requests (strong scaling: the same requests whatever N).

One step = every rank answers the slices in its core (one device pass), reduces
them into per-request rows on the device (sb_batch_reduce_requests), and the
rows are gathered to rank 0 (torch.distributed gather = RCCL over xGMI) and
summed into the request table.  Barrier + torch.cuda.synchronize() bracket the
K timed steps; the time is the max over ranks.  Prints one JSON line on rank 0.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, 'terraform-aws-serverless-beacon_amd')
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main_genome(args):
    import numpy as np
    import torch
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_batch, shard_slices, union_rows
    from sbeacon.shard import RequestGather

    t0 = time.perf_counter()
    shape = GenomeShape(n_total=args.genome_records, seed=3)
    n_shard = shape.shard_records(world, rank)
    last = [0.0]

    def progress(contig, done):
        if time.perf_counter() - last[0] > 20:
            last[0] = time.perf_counter()
            log(f'[rank {rank}] ingest: {done}/{n_shard} records (contig {contig}), {last[0] - t0:.0f} s')

    store = shape.build_shard_store(world, rank, device=local, threads=args.threads, progress=progress)
    info = store.info()
    t_ingest = time.perf_counter() - t0
    log(f'[rank {rank}] shard: {info["n_records"]} records, {info["device_bytes"] / 2**20:.0f} MiB HBM, '
        f'ingest {t_ingest:.1f} s')
    t0 = time.perf_counter()
    reqs = config3_requests(shape, n=args.genome_requests, seed=1003)
    sl = shard_slices(shape, reqs, world, rank)
    batch = prepare_shard_batch(store, sl)
    g = RequestGather(dist, rank, world, sl.row_lo, sl.n_rows, len(reqs), torch.device('cuda', local))
    log(f'[rank {rank}] {len(reqs)} requests, {len(sl)} slices on this rank (rows {sl.row_lo}+{sl.n_rows}), '
        f'prepare {time.perf_counter() - t0:.1f} s')

    def step():
        batch.run()
        batch.reduce_requests(g.part_ptr)
        batch.sync()
        g.exchange()

    for _ in range(args.warmup):
        step()
    batch.timing()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t1
    if dist:
        dist.barrier()
    timing = batch.timing()  # HIP events around the query kernels, averaged over the timed steps
    rs = batch.fetch()
    st = rs.stats()
    scanned, hits = st['records_scanned'], st['hits']
    # Overlapping slices re-scan the same records (~16x here); those re-reads
    # are served from L2 / MALL, so the HBM roofline is priced on the unique
    # rows of the step (the union of the slice windows) at 32 B/row, + 8 B/hit.
    uniq = union_rows(shape, sl)
    scan_bytes = 32.0 * uniq + 8.0 * hits
    achieved = scan_bytes / (timing['scan_ms'] * 1e-3) / 1e9 if timing['scan_ms'] > 0 else 0.0
    traffic = None  # HBM bytes per step from the PMC passes (tools/gpu_pmc_genome_traffic.sh)
    tf = os.path.join(REPO, 'profiles', 'traffic_genome.json')
    if world == 1 and os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get('records') == shape.n_total and tj.get('requests') == len(reqs):
                traffic = tj.get('scan_kernel_hbm_bytes_per_launch')
        except Exception:
            traffic = None
    vals = [elapsed, timing['scan_ms'], float(len(sl)), float(scanned), float(hits), achieved, float(uniq)]
    if dist:
        t = torch.tensor(vals, dtype=torch.float64, device='cuda')
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        allv = [x.tolist() for x in allv]
    else:
        allv = [vals]
    elapsed = max(v[0] for v in allv)
    tot_slices = sum(v[2] for v in allv)
    tot_scanned = sum(v[3] for v in allv)
    tot_hits = sum(v[4] for v in allv)
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline_and_parity(args, shape, reqs, g.total.cpu().numpy())
    out = {
        'metric': 'region queries/sec (Beacon g_variants variantType requests, whole-genome store sharded by contig)',
        'value': round(len(reqs) * args.steps / elapsed, 1),
        'unit': 'requests/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'int64',
        'data': 'synthetic (seeded whole-genome 1000G-shape VCF text per contig shard, generated + ingested in-process)',
        'config': {'workload': 'config3-wgs-1000g-shape', 'records': shape.n_total, 'requests': len(reqs),
                   'slice_queries': int(tot_slices),
                   'parallelism': f'contig shards x{world} (+10 kb halo), per-request rows gathered to rank 0'},
        'records_scanned_per_s': round(tot_scanned * args.steps / elapsed, 1),
        'hits_per_step': int(tot_hits),
        'device_ms_per_step': {'query_kernels_rank0': round(timing['scan_ms'], 4),
                               'query_kernels_max': round(max(v[1] for v in allv), 4)},
        'roofline': {'bound': 'hbm', 'achieved': round(allv[0][5], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(allv[0][5] / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': 'rank 0 query step: vt_kernel (the batch is one variantType group) + request_reduce_kernel; HIP events spanning the step',
                     'algorithmic_bytes_per_launch': 32.0 * allv[0][6] + 8.0 * allv[0][4],
                     'unique_rows_per_launch': int(allv[0][6]),
                     'rows_scanned_per_launch': int(allv[0][3]),
                     'note': '32 B x unique rows (union of slice windows) + 8 B/hit; counting every '
                             're-scan of overlapping slices would give '
                             f'{(32.0 * allv[0][3] + 8.0 * allv[0][4]) / (allv[0][1] * 1e-3) / 1e9:.0f} GB/s'},
        'cpu_baseline': cpu,
        'parity_sample': parity,
        'ingest_s': round(t_ingest, 2),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_and_parity(args, shape, reqs, total, n_sample=20000, seed=7):
    """C oracle (OpenMP) over a random sample of the requests, on a VCF that
    holds exactly the records those requests can reach; also checks the
    device's request rows for the sample."""
    import numpy as np
    from oracle.oracle import OracleVcf
    from sbeacon.genome import CONTIGS, Requests, request_slices, shard_slices, slice_payloads
    from sbeacon.shard import request_rows_from_responses
    rng = np.random.default_rng(seed)
    pick = np.sort(rng.choice(len(reqs), size=min(n_sample, len(reqs)), replace=False))
    sub = Requests(reqs.ci[pick], reqs.start[pick], reqs.width[pick], reqs.vt[pick], reqs.vmin[pick],
                   reqs.vmax[pick])
    tmp = tempfile.mkdtemp(prefix='sbeacon-genome-')
    path = os.path.join(tmp, 'sample.vcf')
    with open(path, 'wb') as f:
        first = True
        for ci in range(len(CONTIGS)):
            m = sub.ci == ci
            if not m.any():
                continue
            gen = shape.gen(ci)
            pos = gen.positions()
            los = np.searchsorted(pos, sub.start[m] + 1, side='left')
            his = np.searchsorted(pos, sub.start[m] + sub.width[m] + 1 + 10000, side='right')
            if first:
                f.write(gen.header(sites_only=True))
                first = False
            cur = 0
            for lo, hi in sorted(zip(los.tolist(), his.tolist())):
                lo = max(lo, cur)
                if hi > lo:
                    f.write(gen.records(lo, hi, sites_only=True, threads=args.threads))
                    cur = hi
    orc = OracleVcf(path, load_gt=False)
    whole = shard_slices(shape, sub, 1, 0)
    pl = slice_payloads(whole)
    dt, passes = orc.time_batch(pl, patched=True, threads=args.threads, min_seconds=args.cpu_seconds)
    res = orc.perform_query_batch(pl, patched=True, threads=args.threads)
    exp = request_rows_from_responses(whole.req, res, whole.n_rows)
    got = total[pick]
    bad = int((got != exp).any(axis=1).sum())
    cpu = {'value': round(passes * len(pick) / dt, 1), 'unit': 'requests/s', 'cores': args.threads, 'kind': 'port',
           'sample': f'{len(pick)} random requests ({len(pl)} slice payloads) x {passes} passes through oracle/sbeacon_oracle.c '
                     f'(CPU restatement of search_variants.py, patched variantType branch), OpenMP x{args.threads}, '
                     f'on a sites-only VCF holding the records those requests reach',
           'seconds': round(dt, 2), 'host_cpus': os.cpu_count()}
    parity = {'requests': len(pick), 'slice_queries': len(pl), 'mismatched_requests': bad,
              'variants_checked': int(exp[:, 1].sum())}
    orc.close()
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    return cpu, parity
