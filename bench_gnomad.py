#!/usr/bin/env python3
"""Config 5 bench (``python bench.py --workload gnomad``): gnomAD-shape sites
(750 M records, AN = 152,312) with a 2,504-sample carrier bit-matrix, sharded
into 8 record-balanced shards, shard r resident on GPU r (~94 M sites +
~30 GB of carrier planes each; sbeacon/gnomad.py).

One step = every rank answers its shard's slices in one device pass (half AC/AN
aggregation ranges, half sample-subset queries that OR carrier rows and AND the
subset mask).  Weak scaling: per-GPU work is fixed, no data-path collective.
Barrier + torch.cuda.synchronize() bracket the K timed steps; the time is the
max over ranks.  Prints one JSON line on rank 0.
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


def main_gnomad(args):
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
    from sbeacon.gnomad import SHARDS, GnomadShape, config5_slices, sample_subsets, slice_payloads
    if world > SHARDS:
        raise SystemExit(f'config 5 has {SHARDS} shards; run at most {SHARDS} ranks')

    t0 = time.perf_counter()
    shape = GnomadShape(n_total=args.gnomad_records)
    n_shard = shape.shard_records(SHARDS, rank)
    last = [0.0]

    def progress(contig, done):
        if time.perf_counter() - last[0] > 20:
            last[0] = time.perf_counter()
            log(f'[rank {rank}] ingest: {done}/{n_shard} records ({contig}), {last[0] - t0:.0f} s')

    log(f'[rank {rank}] shard {rank}/{SHARDS}: {n_shard} records; generating carrier planes')
    store = shape.build_gnomad_store(rank, device=local, threads=args.threads, progress=progress)
    info = store.info()
    t_ingest = time.perf_counter() - t0
    log(f'[rank {rank}] store: {info["n_records"]} records, {info["n_alt_rows"]} alt rows, '
        f'{info["device_bytes"] / 2**30:.1f} GiB HBM, ingest {t_ingest:.1f} s')
    t0 = time.perf_counter()
    subsets = sample_subsets(shape.n_samples, shape.sample_names())
    sl = config5_slices(shape, rank, args.gnomad_requests)
    payloads = slice_payloads(sl, subsets)
    batch = store.prepare(payloads)
    log(f'[rank {rank}] {sl.n_requests} requests -> {len(sl)} slices '
        f'({int(sl.kind.sum())} sample-subset), prepare {time.perf_counter() - t0:.1f} s')

    # --streams N: N copies of the batch in flight on CU-masked streams (one
    # hardware queue each: bench_genome.step_streams), step i runs copy
    # i mod N; the kernels' own time (the roofline's) from one copy run
    # one pass at a time afterwards
    n_streams = max(1, getattr(args, 'streams', 1))
    batches, ss_destroy = [batch], (lambda: None)
    if n_streams > 1:
        from bench_genome import step_streams
        ss, ss_destroy = step_streams(torch, torch.device('cuda', local), n_streams)
        batches += [store.prepare(payloads) for _ in range(n_streams - 1)]
        for b, s_ in zip(batches, ss):
            b.set_stream(s_.cuda_stream)
    for i in range(max(args.warmup, n_streams)):
        batches[i % n_streams].run()
    for b in batches:
        b.sync()
    batch.timing()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(args.steps):
        batches[i % n_streams].run()
    for b in batches:
        b.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t1
    if dist:
        dist.barrier()
    if n_streams > 1:
        for b in batches[1:]:
            b.free()
        batch.set_stream(None)
        ss_destroy()
        for _ in range(args.steps):
            batch.run()
        batch.sync()
    timing = batch.timing()
    rs = batch.fetch()
    st = rs.stats()
    scanned, hits = st['records_scanned'], st['hits']
    samp_idx = np.flatnonzero(sl.kind == 1)
    samp_hits = int(sum(rs.view(int(j)).n_variants for j in samp_idx))
    words = (shape.n_samples + 63) // 64
    # rows inside the slices, per kind (host count over the generator's POS)
    rows_kind = [0, 0]
    for ci in np.unique(sl.ci).tolist():
        pos = shape.gen(int(ci)).positions()
        m = sl.ci == ci
        n_in = np.searchsorted(pos, sl.b[m], side='right') - np.searchsorted(pos, sl.a[m], side='left')
        for k in (0, 1):
            rows_kind[k] += int(n_in[sl.kind[m] == k].sum())
    # algorithmic bytes = what the kernels must read at least once: the 8 B
    # RangeHot8 word per aggregation row, the 16 B RecHot word per sample-path
    # row, one carrier row (words x 8 B) per hit ALT of a sample-subset query,
    # 8 B per hit written.  SURVEY §8d's 32 B/row contract is reported beside it.
    alg = 8.0 * rows_kind[0] + 16.0 * rows_kind[1] + 8.0 * words * samp_hits + 8.0 * hits
    contract = 32.0 * scanned + 8.0 * hits + 8.0 * words * samp_hits
    achieved = alg / (timing['scan_ms'] * 1e-3) / 1e9 if timing['scan_ms'] > 0 else 0.0
    traffic = None  # HBM bytes per step from the PMC passes (tools/gpu_pmc_gnomad.sh)
    tf = os.path.join(REPO, 'profiles', 'traffic_gnomad.json')
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get('records') == shape.n_total and tj.get('requests') == args.gnomad_requests:
                traffic = tj.get('scan_kernel_hbm_bytes_per_launch')
        except Exception:
            traffic = None
    vals = [elapsed, timing['scan_ms'], float(sl.n_requests), float(len(sl)), float(scanned), float(hits),
            achieved, alg, float(samp_hits), contract]
    if dist:
        t = torch.tensor(vals, dtype=torch.float64, device='cuda')
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        allv = [x.tolist() for x in allv]
    else:
        allv = [vals]
    elapsed = max(v[0] for v in allv)
    tot_req = sum(v[2] for v in allv)
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline_and_parity(args, shape, sl, subsets, rs)
    out = {
        'metric': 'region queries/sec (Beacon g_variants requests: AC/AN aggregation + sample-subset genotype masks, '
                  'gnomAD-shape sites shard per GPU)',
        'value': round(tot_req * args.steps / elapsed, 1),
        'unit': 'requests/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'streams': n_streams,
        'dtype': 'int64',
        'data': 'synthetic (seeded gnomAD-shape sites VCF text per shard + 2504-sample carrier bit-matrix, '
                'generated + ingested in-process)',
        'config': {'workload': 'config5-gnomad-shape', 'records': shape.n_total, 'shards': SHARDS,
                   'records_per_gpu': int(info['n_records']), 'samples': shape.n_samples,
                   'requests_per_gpu': int(allv[0][2]), 'slice_queries_per_gpu': int(allv[0][3]),
                   'parallelism': f'shard r of {SHARDS} on rank r (x{world}), no data-path collective'},
        'slice_queries_per_s': round(sum(v[3] for v in allv) * args.steps / elapsed, 1),
        'records_scanned_per_s': round(sum(v[4] for v in allv) * args.steps / elapsed, 1),
        'hits_per_step': int(sum(v[5] for v in allv)),
        'sample_path_hits_per_step': int(sum(v[8] for v in allv)),
        'device_ms_per_step': {'query_kernels_rank0': round(timing['scan_ms'], 4),
                               'query_kernels_max': round(max(v[1] for v in allv), 4)},
        'roofline': {'bound': 'hbm', 'achieved': round(allv[0][6], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(allv[0][6] / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': 'rank 0 query step (range_n + sample-path scan launches); HIP events spanning the step (not a rocprof average)',
                     'algorithmic_bytes_per_launch': allv[0][7],
                     'pricing': f'8 B/aggregation row (RangeHot8) + 16 B/sample-path row (RecHot) + {8 * words} B '
                                f'carrier row per sample-path hit ALT + 8 B/hit written',
                     'rows_in_slices': {'aggregation': rows_kind[0], 'sample_subset': rows_kind[1]},
                     'contract_bytes_per_launch': allv[0][9],
                     'contract_note': 'SURVEY 8d prices 32 B per row scanned; the packed words are 8-16 B, so that '
                                      'figure is rows covered, not bytes moved'},
        'cpu_baseline': cpu,
        'parity_sample': parity,
        'ingest_s': round(t_ingest, 2),
        'device_gib': round(info['device_bytes'] / 2**30, 2),
    }
    del batch, rs
    store.close()
    torch.cuda.empty_cache()
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


def _write_vcf(path, shape, sl, idx, sites_only, threads):
    """VCF holding the records slices `idx` can reach (their [a, b])."""
    import numpy as np
    from sbeacon.genome import CONTIGS
    with open(path, 'wb') as f:
        first = True
        for ci in range(len(CONTIGS)):
            m = idx[sl.ci[idx] == ci]
            if not len(m):
                continue
            gen = shape.gen(ci)
            pos = gen.positions()
            los = np.searchsorted(pos, sl.a[m], side='left')
            his = np.searchsorted(pos, sl.b[m], side='right')
            if first:
                f.write(gen.header(sites_only=sites_only))
                first = False
            cur = 0
            for lo, hi in sorted(zip(los.tolist(), his.tolist())):
                lo = max(lo, cur)
                if hi > lo:
                    f.write(gen.records(lo, hi, sites_only=sites_only, threads=threads))
                    cur = hi


def cpu_baseline_and_parity(args, shape, sl, subsets, rs, n_agg=2000, n_samp=1000, seed=9):
    """C oracle (OpenMP) on samples of both request kinds: aggregation slices
    over a sites-only VCF, sample-subset slices over a VCF with the 2,504 GT
    columns (the oracle's regex-equivalent token match per sample, :233-236).
    Also checks the device's full responses for those slices."""
    import numpy as np
    from oracle.oracle import OracleVcf
    from sbeacon.gnomad import slice_payloads
    rng = np.random.default_rng(seed)
    agg = np.flatnonzero(sl.kind == 0)
    samp = np.flatnonzero(sl.kind == 1)
    agg = np.sort(rng.choice(agg, size=min(n_agg, len(agg)), replace=False))
    samp = np.sort(rng.choice(samp, size=min(n_samp, len(samp)), replace=False))
    tmp = tempfile.mkdtemp(prefix='sbeacon-gnomad-')
    out = {}
    bad = checked = variants = 0
    for name, idx, sites in (('agg', agg, True), ('samp', samp, False)):
        path = os.path.join(tmp, f'{name}.vcf')
        _write_vcf(path, shape, sl, idx, sites, args.threads)
        orc = OracleVcf(path, load_gt=not sites)
        pl = slice_payloads(sl, subsets, idx)
        dt, passes = orc.time_batch(pl, threads=args.threads, min_seconds=args.cpu_seconds / 2)
        res = orc.perform_query_batch(pl, threads=args.threads)
        for j, exp in zip(idx.tolist(), res):
            got = rs.response(j).dump()
            if isinstance(exp, dict) and 'errorType' not in exp:
                got['sample_indices'] = sorted(got['sample_indices'])
                exp = dict(exp)
                exp['sample_indices'] = sorted(exp['sample_indices'])
                bad += got != exp
                variants += len(exp['variants'])
            else:
                bad += 1
            checked += 1
        # per-request CPU time: this kind's slices per request x time per slice
        per_slice = dt / (passes * len(pl))
        out[name] = per_slice * len(sl.req[sl.kind == (0 if sites else 1)]) / max(
            1, len(np.unique(sl.req[sl.kind == (0 if sites else 1)])))
        out[name + '_passes'] = passes
        out[name + '_s'] = dt
        orc.close()
        os.remove(path)
    os.rmdir(tmp)
    # the workload's request mix (half of each kind)
    n0 = len(np.unique(sl.req[sl.kind == 0]))
    n1 = len(np.unique(sl.req[sl.kind == 1]))
    t_req = (n0 * out['agg'] + n1 * out['samp']) / (n0 + n1)
    cpu = {'value': round(1.0 / t_req, 1), 'unit': 'requests/s', 'cores': args.threads, 'kind': 'port',
           'sample': f'{len(agg)} aggregation slices x {out["agg_passes"]} passes (sites-only VCF) + {len(samp)} '
                     f'sample-subset slices x {out["samp_passes"]} passes (VCF with 2504 GT columns) through '
                     f'oracle/sbeacon_oracle.c (CPU restatement of search_variants.py / '
                     f'search_variants_in_samples.py), OpenMP x{args.threads}; per-request times weighted by '
                     f'this shard\'s request mix',
           'seconds': round(out['agg_s'] + out['samp_s'], 2), 'host_cpus': os.cpu_count()}
    parity = {'slice_queries': checked, 'mismatches': int(bad), 'variants_checked': int(variants),
              'sample_subset_slices': len(samp)}
    return cpu, parity
