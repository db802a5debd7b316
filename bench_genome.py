#!/usr/bin/env python3
"""Config 3 bench (the default of ``python bench.py``): whole-genome
1000G-shape store sharded by contig across the GPUs (sbeacon/genome.py) and
variantType Beacon requests -- 1 M per GPU (weak scaling, the default: N M
genome-wide requests routed to the shards by position) or 1 M in total
(``--scaling strong``).

One step = every rank answers the slices in its core (chain_kernel: one wave
per request's slices), reduces them into per-request rows
(sb_batch_reduce_requests), writes the rows' dense hit lists with global
record ids (sb_batch_compact_hits), and delivers rows + hits to each
request's host-facing rank (sbeacon.shard.ResultExchange: all_gather of
counts, then RCCL send/recv over xGMI of the straddling requests' rows and
hits; ``--deliver rank0`` sends everything to rank 0).  Barrier +
torch.cuda.synchronize() bracket the K timed steps; the time is the max over
ranks.  Prints one JSON line on rank 0.
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
    dev = torch.device('cuda', local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=dev)
    from sbeacon.genome import (GenomeShape, config3_requests, first_rank_of_rows, prepare_shard_batch,
                                shard_record_base, shard_slices, union_rows)
    from sbeacon.shard import ResultExchange, owner_ranks

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
    # weak scaling (default): genome-wide requests, args.genome_requests per GPU, routed
    # to the shards by position; strong: args.genome_requests in total
    n_req = args.genome_requests * (world if args.scaling == 'weak' else 1)
    reqs = config3_requests(shape, n=n_req, seed=1003)
    sl = shard_slices(shape, reqs, world, rank)
    batch = prepare_shard_batch(store, sl)
    batch.set_stream(torch.cuda.current_stream().cuda_stream)  # one stream: kernels, torch ops, RCCL
    # the step delivers request rows + hit lists: chained slices skip their
    # per-slice QRes rows (turned back on below for the per-slice fetch)
    batch.set_slice_results(False)
    pst = batch.stats()
    part = torch.zeros((max(sl.n_rows, 1), 5), dtype=torch.int64, device=dev)
    hits = torch.zeros(max(int(pst['hits']), 1), dtype=torch.int64, device=dev)
    row_off = torch.zeros(sl.n_rows + 1, dtype=torch.int64, device=dev)
    base = shard_record_base(shape, world, rank)
    owners = owner_ranks(first_rank_of_rows(shape, reqs, world, sl), args.deliver, rank)
    ex = ResultExchange(dist, rank, world, sl.row_lo, sl.n_rows, owners, dev)
    log(f'[rank {rank}] {n_req} requests, {len(sl)} slices on this rank (rows {sl.row_lo}+{sl.n_rows}, '
        f'{pst["chains"]} chains), delivery {args.deliver}: owns {ex.n_own} rows, receives {len(ex.recvs)} '
        f'range(s), prepare {time.perf_counter() - t0:.1f} s')

    def step():  # answer + deliver: chain kernel, request rows, dense hit lists, exchange
        batch.run()
        batch.deliver(part.data_ptr(), hits.data_ptr(), row_off.data_ptr(), base)  # request rows + hit lists
        ex.exchange(part, hits, row_off)

    for _ in range(args.warmup):
        step()
    batch.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    batch.sync()  # records the closing event on the stream
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t1
    if dist:
        dist.barrier()
    step_dev_ms = batch.timing()['scan_ms']  # HIP events on the stream: first run -> sync, / steps
    # the dominant kernel alone (chain_kernel): K back-to-back runs between two events
    for _ in range(args.steps):
        batch.run()
    batch.sync()
    kern_ms = batch.timing()['scan_ms']
    batch.set_slice_results(True)
    batch.run()
    batch.sync()
    rs = batch.fetch()
    st = rs.stats()
    scanned, nhits = st['records_scanned'], st['hits']
    # Roofline of chain_pack_kernel, priced on the bytes one launch must move
    # at least once: chain descriptors (80 B), their two
    # coarse-index entries (8 B), the request-row partial (40 B), the
    # candidate words in the union of the chain windows (POS 4 + VtHot 16 +
    # record 4 = 24 B, each candidate once however many overlapping requests
    # read it) and hits (8 B).  Beside it the SURVEY §8d contract figure:
    # 32 B x unique records in the slice windows + 8 B / hit.
    chains, cslices = st['chains'], st['chained_slices']
    comp = 80.0 * chains + 8.0 * chains + 40.0 * chains + 24.0 * st['cand_unique'] + 8.0 * nhits
    achieved = comp / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    uniq = union_rows(shape, sl)
    contract = 32.0 * uniq + 8.0 * nhits
    traffic = None  # HBM bytes per launch from the PMC passes (tools/gpu_pmc_genome_traffic.sh)
    tf = os.path.join(REPO, 'profiles', 'traffic_genome.json')
    if world == 1 and os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get('records') == shape.n_total and tj.get('requests') == len(reqs) and tj.get('kernel') == 'chain_pack_kernel<false>':
                traffic = tj.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None
    vals = [elapsed, kern_ms, float(len(sl)), float(scanned), float(nhits), achieved, float(uniq), comp, contract,
            step_dev_ms]
    if dist:
        t = torch.tensor(vals, dtype=torch.float64, device=dev)
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
        cpu, parity = cpu_baseline_and_parity(args, shape, reqs, ex.exchange(part, hits, row_off).cpu().numpy(),
                                              hits.cpu().numpy(), row_off.cpu().numpy())
    r0 = allv[0]
    out = {
        'metric': 'region queries/sec (Beacon g_variants variantType requests, whole-genome store sharded by contig)',
        'value': round(n_req * args.steps / elapsed, 1),
        'unit': 'requests/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': args.scaling,
        'vs_baseline': None,
        'dtype': 'int64',
        'data': 'synthetic (seeded whole-genome 1000G-shape VCF text per contig shard, generated + ingested in-process)',
        'config': {'workload': 'config3-wgs-1000g-shape', 'records': shape.n_total, 'requests': n_req,
                   'requests_per_gpu': args.genome_requests if args.scaling == 'weak' else None,
                   'slice_queries': int(tot_slices),
                   'parallelism': f'contig shards x{world} (+10 kb halo); request rows + hit lists delivered to '
                                  f'the {"first slice" if args.deliver == "first" else "rank 0"} rank over '
                                  f'{"RCCL" if world > 1 else "(no peer)"}'},
        'step': 'chain_pack_kernel (request-row partials + dense chain hits; per-slice rows off) + request rows '
                '+ dense hit lists (scan, gather) + exchange (all_gather of counts, send/recv of straddling rows and '
                'hits)',
        'records_scanned_per_s': round(tot_scanned * args.steps / elapsed, 1),
        'hits_per_step': int(tot_hits),
        'device_ms_per_step': {'step_rank0': round(r0[9], 4), 'chain_kernel_rank0': round(r0[1], 4),
                               'chain_kernel_max': round(max(v[1] for v in allv), 4)},
        'roofline': {'bound': 'hbm', 'achieved': round(r0[5], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(r0[5] / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': 'chain_kernel (rank 0), HIP events around K back-to-back launches on its stream',
                     'algorithmic_bytes_per_launch': r0[7],
                     'pricing': 'bytes one launch must move at least once: 128 B/chain (80 B descriptor + 2 '
                                'index entries + 40 B request-row partial) + 24 B per candidate in the union of the '
                                'chain windows + 8 B/hit (the step keeps request rows, not per-slice rows)',
                     'candidates': {'unique': int(st['cand_unique']), 'in_windows': int(st['cand_window']),
                                    'loaded': int(st['cand_loaded'])},
                     'contract_bytes_per_launch': r0[8],
                     'contract_frac': round(r0[8] / (r0[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if r0[1] > 0 else None,
                     'contract_note': 'SURVEY 8d: 32 B x unique records in the slice windows (a full scan of them) '
                                      '+ 8 B/hit; the candidate index reads a few % of those records'},
        'cpu_baseline': cpu,
        'parity_sample': parity,
        'ingest_s': round(t_ingest, 2),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_and_parity(args, shape, reqs, total, hits, row_off, n_sample=20000, seed=7):
    """C oracle (OpenMP) over a random sample of the requests, on a VCF that
    holds exactly the records those requests can reach; also checks the
    device's request rows and hit lists for the sample."""
    import numpy as np
    from oracle.oracle import OracleVcf
    from sbeacon.genome import CONTIGS, Requests, shard_slices, slice_payloads
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
    # hit lists: the device's (global record, ALT index) pairs of each sampled
    # request, rendered as (chrom, POS, ALT) through the generator, against the
    # oracle's variant strings in order
    exp_v = [[] for _ in range(len(pick))]
    for o, r in zip(whole.req, res):
        if isinstance(r, dict):
            exp_v[o].extend(tuple(v.split('\t')[i] for i in (0, 1, 3)) for v in r['variants'])
    h = hits.view(np.uint64)
    bad_hits = 0
    alts_cache = {}
    for j, r in enumerate(pick.tolist()):
        dv = []
        for x in h[row_off[r]:row_off[r + 1]].tolist():
            g, k = x & 0xffffffff, x >> 32
            ci = int(np.searchsorted(shape.offsets, g, side='right') - 1)
            i = g - int(shape.offsets[ci])
            if (ci, i) not in alts_cache:
                line = shape.gen(ci).records(i, i + 1, sites_only=True).decode().split('\t')
                alts_cache[(ci, i)] = (line[0], line[1], line[4].split(','))
            c, p, alts = alts_cache[(ci, i)]
            dv.append((c, p, alts[k]))
        bad_hits += int(dv != exp_v[j])
    cpu = {'value': round(passes * len(pick) / dt, 1), 'unit': 'requests/s', 'cores': args.threads, 'kind': 'port',
           'sample': f'{len(pick)} random requests ({len(pl)} slice payloads) x {passes} passes through oracle/sbeacon_oracle.c '
                     f'(CPU restatement of search_variants.py, patched variantType branch), OpenMP x{args.threads}, '
                     f'on a sites-only VCF holding the records those requests reach',
           'seconds': round(dt, 2), 'host_cpus': os.cpu_count()}
    parity = {'requests': len(pick), 'slice_queries': len(pl), 'mismatched_requests': bad,
              'mismatched_hit_lists': bad_hits, 'variants_checked': int(exp[:, 1].sum())}
    orc.close()
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    return cpu, parity
