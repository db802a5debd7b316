#!/usr/bin/env python3
"""Benchmark: batched Beacon g_variants requests on an HBM-resident store.

Default workload (BASELINE.json configs[2], SURVEY.md §8d config 3,
``bench_genome.py``): the whole-genome 1000G-shape store (85 M records)
sharded by contig across the GPUs, 1 M variantType requests per GPU; a step
answers every request's 10 kb slices (chain_kernel), reduces them into
request rows, compacts the hit lists and delivers rows + hits to each
request's host-facing rank over RCCL.  ``--workload chr22`` is config 2
(1000G chr22 shape, 10 k range / point requests, replicas), ``--workload
gnomad`` config 5 (gnomAD-shape sites + carrier bit-matrix).

``--gpus N`` without torch.distributed's environment starts
``torch.distributed.run`` with N ranks (one per GPU) as a child process
before anything touches a GPU, and exits with its code.  Every rank prints
its log to stderr; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, 'terraform-aws-serverless-beacon_amd')
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--records', type=int, default=1103547)
    ap.add_argument('--samples', type=int, default=2504)
    ap.add_argument('--range-requests', type=int, default=5000)
    ap.add_argument('--point-requests', type=int, default=5000)
    ap.add_argument('--threads', type=int, default=None,
                    help='host ingest / CPU-baseline threads (default: every CPU the process may use, host_cores())')
    ap.add_argument('--batches', type=int, default=4,
                    help='config 3: request batches the step rotates over (each answered every --batches steps)')
    ap.add_argument('--streams', type=int, default=2,
                    help='configs 3 and 2: HIP streams the step\'s batches alternate over (batch k on stream k mod N: N '
                         'independent batches in flight, as a serving loop keeps them; 1 = every step behind the last)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0, help='target CPU-baseline sample duration')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--parity-requests', type=int, default=2000,
                    help='requests re-checked against the C oracle after timing (rank 0)')
    ap.add_argument('--workload', choices=['chr22', 'genome', 'gnomad'], default='genome',
                    help='genome: config 3 (default; whole-genome store sharded by contig across the GPUs, '
                         'request rows + hit lists delivered over RCCL). chr22: config 2 (replicas across GPUs). '
                         'gnomad: config 5 (gnomAD-shape sites + carrier bit-matrix, shard r of 8 per GPU)')
    ap.add_argument('--genome-records', type=int, default=85_000_000)
    ap.add_argument('--genome-requests', type=int, default=1_000_000,
                    help='config-3 requests per GPU (weak scaling) or in total (strong)')
    ap.add_argument('--scaling', choices=['weak', 'strong'], default='weak')
    ap.add_argument('--deliver', choices=['first', 'rank0'], default='first',
                    help="config 3: each request's rows + hits go to the rank of its first slice, or all to rank 0")
    ap.add_argument('--no-config4', action='store_true',
                    help='config 3 only: skip the config-4 sub-object (summariseSlice + duplicateVariantSearch on the '
                         '50-dataset cohort, bench_paths.py) the default N=1 run appends')
    ap.add_argument('--config4-datasets', type=int, default=50)
    ap.add_argument('--no-config5', action='store_true',
                    help='config 3 only: skip the config-5 sub-object (gnomAD-shape shard, bench_gnomad.py)')
    ap.add_argument('--no-config2', action='store_true',
                    help='config 3 only: skip the config-2 sub-object (chr22-shape requests + the wire figure)')
    ap.add_argument('--gnomad-records', type=int, default=750_000_000)
    ap.add_argument('--gnomad-requests', type=int, default=50_000, help='config-5 requests per GPU')
    args = ap.parse_args()
    if args.threads is None:
        args.threads = host_cores()['cores']
    return args


def config4_lines(args) -> dict:
    """BASELINE configs[3] beside the headline (N=1): bench_paths.run over the
    50-dataset cohort after the config-3 store is freed -- summariseSlice over
    every slice of the 100 VCFs in one call, the per-dataset
    duplicateVariantSearch jobs in one call, the reference-exact mode over
    the first 10 datasets' messages, each with its C-oracle parity sample and
    CPU baseline.  Times measured inside bench_paths as in its own lines."""
    import bench_paths
    a = bench_paths.parse(['--datasets', str(args.config4_datasets), '--threads', str(args.threads)] +
                          (['--no-cpu-baseline'] if args.no_cpu_baseline else []))
    t0 = time.perf_counter()
    lines = bench_paths.run(a)
    keep = ('metric', 'value', 'unit', 'ms_per_step', 'device_ms_per_step', 'config', 'roofline', 'cpu_baseline',
            'parity_sample', 'strict_mode', 'union', 'path', 'windows', 'ingest_s')
    out = {x['config']['workload']: {k: x[k] for k in keep if k in x} for x in lines}
    out['seconds'] = round(time.perf_counter() - t0, 1)
    return out


def host_cores() -> dict:
    """The CPUs this process may run on: its affinity mask, capped by the
    cgroup's CPU quota when one is set (a 16-CPU quota on a 256-CPU affinity
    mask gives 16 CPUs' worth of time: more threads only time-slice), with the
    CPU model (lscpu's "Model name", from /proc/cpuinfo)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return {'cores': cores, 'affinity': aff, 'cgroup_cpu_quota': quota, 'model': model}


def unique_rows(gen, payloads) -> int:
    """Records inside the union of the payloads' POS windows."""
    import numpy as np
    iv = []
    for p in payloads:
        a, b = p['region'].split(':')[1].split('-')
        iv.append((int(a), int(b)))
    iv.sort()
    merged = []
    for a, b in iv:
        if merged and a <= merged[-1][1] + 1:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    pos = np.asarray(gen.positions())
    return int(sum(np.searchsorted(pos, b, side='right') - np.searchsorted(pos, a, side='left') for a, b in merged))


def spawn_ranks(args) -> int:
    """`--gpus N` outside torch.distributed: run N ranks under
    torch.distributed.run as a child (nothing here has touched a GPU)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(('127.0.0.1', 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log('launching: ' + ' '.join(cmd))
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(args))
    if args.workload == 'genome':
        from bench_genome import main_genome
        out = main_genome(args)
        if out is not None:  # rank 0
            if int(os.environ.get('WORLD_SIZE', 1)) == 1:
                # the other BASELINE configs beside the headline, each after
                # the previous store is released (N=1 only; each carries its
                # own timing, roofline, CPU baseline and oracle parity sample)
                # a sub-line that raises (a parity mismatch included) is
                # recorded as its error; the headline line is still printed
                def sub(key, fn):
                    t0 = time.perf_counter()
                    try:
                        out[key] = fn()
                    except Exception as e:  # noqa: BLE001 -- reported in the line, not swallowed
                        import traceback
                        log(traceback.format_exc())
                        out[key] = {'error': f'{type(e).__name__}: {e}'}
                        import torch
                        torch.cuda.empty_cache()
                    out[key]['seconds'] = round(time.perf_counter() - t0, 1)

                if not args.no_config4:
                    sub('config4', lambda: config4_lines(args))
                if not args.no_config5:
                    from bench_gnomad import main_gnomad
                    sub('config5', lambda: sub_line(main_gnomad(args)))
                if not args.no_config2:
                    sub('config2', lambda: sub_line(main_chr22(args)))
            print(json.dumps(out), flush=True)
        return
    if args.workload == 'gnomad':
        from bench_gnomad import main_gnomad
        out = main_gnomad(args)
    else:
        out = main_chr22(args)
    if out is not None:  # rank 0
        print(json.dumps(out), flush=True)


def sub_line(out: dict) -> dict:
    """A workload's line as a sub-object of the headline line."""
    keep = ('metric', 'value', 'unit', 'ms_per_step', 'streams', 'dtype', 'device_ms_per_step', 'config', 'roofline',
            'delivered', 'cpu_baseline', 'parity_sample', 'ingest_s', 'device_gib')
    return {k: out[k] for k in keep if k in out}


def main_chr22(args):
    """Config 2 (BASELINE configs[1]): 10 k range / point requests on the
    chr22-shape store, replicas across ranks.  Returns rank 0's line (None
    on the other ranks); the store is released before returning."""
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(local)

    from sbeacon.workload import SyntheticVcf, config2_requests, requests_to_payloads

    t0 = time.perf_counter()
    gen = SyntheticVcf(seed=22, n_records=args.records, n_samples=args.samples)
    loc = 'synthetic/chr22-1000g-shape.vcf.gz'
    store = gen.build_store(loc, device=local, keep_genotypes=True, threads=args.threads)
    info = store.info()
    t_ingest = time.perf_counter() - t0
    log(f'[rank {rank}] store: {info["n_records"]} records, {info["n_alt_rows"]} alt rows, '
        f'{info["device_bytes"] / 2**20:.0f} MiB HBM, ingest {t_ingest:.1f} s')
    reqs = config2_requests(gen, n_range=args.range_requests, n_point=args.point_requests, seed=1022 + rank)
    payloads, owner = requests_to_payloads(reqs, vcf_location=loc, chrom='22')
    batch = store.prepare(payloads)
    log(f'[rank {rank}] {len(reqs)} requests -> {len(payloads)} slice queries')

    # --streams N: N copies of the batch (the same payloads, each its own
    # buffers) alternate over N CU-masked streams, one hardware queue each,
    # as config 3's step does (bench_genome.step_streams): step i runs copy
    # i mod N, so one pass's ramp and drain overlap the next pass
    n_streams = max(1, args.streams)
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
    if n_streams > 1:  # the kernels' own time (the roofline's): one copy, one pass at a time, on the store's stream
        for b in batches[1:]:
            b.free()
        batches = [batch]
        batch.set_stream(None)
        ss_destroy()
        for _ in range(args.steps):
            batch.run()
        batch.sync()
    timing = batch.timing()  # HIP events spanning K back-to-back launches of one batch, / K (set at its last sync)
    rs = batch.fetch()
    st = rs.stats()
    n_req, n_slice = len(reqs), len(payloads)
    scanned, hits = st['records_scanned'], st['hits']
    if dist:
        t = torch.tensor([elapsed, timing['scan_ms'], timing['total_ms']], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, scan_ms_max, total_ms_max = t.tolist()
        tot = torch.tensor([n_req, n_slice, scanned, hits], dtype=torch.float64, device='cuda')
        dist.all_reduce(tot)
        tot_req, tot_slice, tot_scanned, tot_hits = tot.tolist()
    else:
        tot_req, tot_slice, tot_scanned, tot_hits = n_req, n_slice, scanned, hits

    ms_per_step = elapsed / args.steps * 1e3
    value = tot_req * args.steps / elapsed
    # roofline of the dominant kernel (the range scan), algorithmic bytes per
    # launch: 32 B per scanned record + 8 B per emitted hit
    scan_bytes = 32.0 * scanned + 8.0 * hits
    achieved = scan_bytes / (timing['scan_ms'] * 1e-3) / 1e9 if timing['scan_ms'] > 0 else 0.0
    # beside it (SURVEY §8d cache caveat): the same price over UNIQUE records
    # -- the union of the slice windows, each record counted once however
    # many slices scan it (the chr22 scan columns sit in L2 / MALL, so the
    # re-scans are cache hits; HBM-bound claims rest on configs 3 and 5)
    uniq = unique_rows(gen, payloads)
    uniq_bytes = 32.0 * uniq + 8.0 * hits
    uniq_gbs = uniq_bytes / (timing['scan_ms'] * 1e-3) / 1e9 if timing['scan_ms'] > 0 else 0.0
    traffic = None
    tf = os.path.join(REPO, 'profiles', 'traffic.json')
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get('records') == args.records and tj.get('requests') == n_req:
                traffic = tj.get('scan_kernel_hbm_bytes_per_launch')
        except Exception:
            traffic = None

    # what a drop-in handler sees (weak item of round 1): PerformQueryPayload
    # dicts in, PerformQueryResponse objects out through the registry --
    # prepare (host planning + upload), device pass, fetch (D2H) and response
    # building (variant strings formatted lazily, on first access)
    delivered = None
    if rank == 0 and world == 1:
        from sbeacon import engine
        from sbeacon.perform_query import perform_query_batch
        engine.registry.register(store)
        try:
            perform_query_batch(payloads[:64], lazy_variants=True)
            reps = 3
            t2 = time.perf_counter()
            for _ in range(reps):
                resp = perform_query_batch(payloads, lazy_variants=True)
            dt = (time.perf_counter() - t2) / reps
            delivered = {'requests_per_s': round(n_req / dt, 1), 'slice_payloads_per_s': round(n_slice / dt, 1),
                         'ms_per_batch': round(dt * 1e3, 2), 'responses': len(resp),
                         'note': 'one batch of all requests\' payload dicts -> PerformQueryResponse objects '
                                 '(prepare + device pass + fetch + responses; host-bound, not the timed step)'}
            # at the wire: the performQuery events as the Lambda runtime receives
            # them (JSON text) -> the JSON text it would send back, for the whole
            # batch in one library call (sbeacon/wire.py, csrc/wire.cpp)
            from sbeacon.wire import pack_events, perform_query_events_packed
            ebuf, eoff = pack_events([json.dumps(p) for p in payloads])
            wout = perform_query_events_packed(ebuf, eoff)  # warm: the output / event buffers sized once
            tw = []
            for _ in range(5):  # steady state: the previous output released outside the timed call
                wout = None
                t2 = time.perf_counter()
                wout = perform_query_events_packed(ebuf, eoff)
                tw.append(time.perf_counter() - t2)
            dtw = sorted(tw)[len(tw) // 2]  # median call
            delivered['wire'] = {'requests_per_s': round(n_req / dtw, 1), 'slice_payloads_per_s': round(n_slice / dtw, 1),
                                 'ms_per_batch': round(dtw * 1e3, 2), 'event_bytes': len(ebuf),
                                 'response_bytes': len(wout.buf), 'python_fallbacks': int(wout.fallback.sum()),
                                 'call_ms': [round(t * 1e3, 2) for t in tw],
                                 'note': 'event JSON texts in -> response JSON texts out (json.dumps(response.dump()) '
                                         'byte for byte): C++ parse + one device batch + C++ formatting; median of 5 '
                                         'calls after a warm-up call'}
        finally:
            engine.registry.clear()

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline_and_parity(args, gen, reqs, payloads, owner, rs)

    out = {
        'metric': 'region queries/sec (Beacon g_variants requests, 10 kb-sliced performQuery payloads)',
        'value': round(value, 1),
        'unit': 'requests/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'streams': n_streams,
        'dtype': 'int64',
        'data': 'synthetic (seeded 1000G chr22-shape VCF, generated + ingested in-process)',
        'config': {'workload': 'config2-chr22-shape', 'records': args.records, 'samples': args.samples,
                   'requests_per_gpu': n_req, 'slice_queries_per_gpu': n_slice,
                   'parallelism': f'replicas x{world} (independent slices, no data-path collective)'},
        'slice_queries_per_s': round(tot_slice * args.steps / elapsed, 1),
        'records_scanned_per_s': round(tot_scanned * args.steps / elapsed, 1),
        'hits_per_step': int(tot_hits),
        'device_ms_per_step': {'scan_kernel': round(timing['scan_ms'], 4)},
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': 'query step: fused_kernel (range_n + exact groups in one launch); HIP events spanning the K timed launches / K',
                     'algorithmic_bytes_per_launch': scan_bytes,
                     'pricing': '32 B per scanned record per slice (re-scans of overlapping slices counted) + 8 B/hit',
                     'unique_records': int(uniq), 'unique_bytes_per_launch': uniq_bytes,
                     'unique_achieved': round(uniq_gbs, 1), 'unique_frac': round(uniq_gbs / HBM_PEAK_GBS, 4)},
        'delivered': delivered,
        'cpu_baseline': cpu,
        'parity_sample': parity,
        'ingest_s': round(t_ingest, 2),
    }
    del batch, rs
    store.close()
    torch.cuda.empty_cache()
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


def cpu_baseline_and_parity(args, gen, reqs, payloads, owner, rs):
    """C oracle (the CPU restatement of the reference loop, OpenMP over the
    host cores) on a bounded sample of the same requests; also re-checks the
    device answers for a sample of requests against it."""
    from oracle.oracle import OracleVcf
    tmp = tempfile.mkdtemp(prefix='sbeacon-bench-')
    path = os.path.join(tmp, 'sites.vcf')
    gen.write(path, sites_only=True, threads=args.threads)  # config 2 queries read no GT
    orc = OracleVcf(path, load_gt=False)
    threads = args.threads
    by_req = {}
    for j, r in enumerate(owner):
        by_req.setdefault(r, []).append(j)
    # interleave request kinds so the sample is representative of the mix
    order = []
    nr = args.range_requests
    for k in range(max(nr, len(reqs) - nr)):
        if k < nr:
            order.append(k)
        if nr + k < len(reqs):
            order.append(nr + k)
    # the whole request set, payloads converted once; C time only, repeated
    # passes until ~cpu_seconds (the oracle takes no Python per query)
    pl = [payloads[j] for r in order for j in by_req[r]]
    dt, passes = orc.time_batch(pl, patched=True, threads=threads, min_seconds=args.cpu_seconds)
    done = passes * len(order)
    sample = f'all {len(reqs)} requests ({len(pl)} slice payloads) x {passes} passes'
    cpu = {'value': round(done / dt, 1), 'unit': 'requests/s', 'cores': threads, 'kind': 'port', 'host': host_cores(),
           'sample': sample + f' through oracle/sbeacon_oracle.c (CPU restatement of search_variants.py), '
                              f'OpenMP x{threads}, sites-only VCF text (config-2 queries read no GT)',
           'seconds': round(dt, 2), 'host_cpus': os.cpu_count()}
    # parity: device answers vs oracle for a sample of requests
    chk = order[:args.parity_requests]
    idx = [j for r in chk for j in by_req[r]]
    exp = orc.perform_query_batch([payloads[j] for j in idx], patched=True, threads=threads)
    bad = 0
    for j, e in zip(idx, exp):
        try:
            g = rs.response(j).dump()
        except Exception as ex:  # noqa: BLE001
            g = type(ex)
        if isinstance(e, type) or isinstance(g, type):
            bad += int(e is not g)
        else:
            g['sample_indices'] = sorted(g['sample_indices'])
            e['sample_indices'] = sorted(e['sample_indices'])
            bad += int(g != e)
    parity = {'requests': len(chk), 'slice_queries': len(idx), 'mismatches': bad,
              'variants_checked': int(sum(len(e['variants']) for e in exp if isinstance(e, dict)))}
    orc.close()
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    return cpu, parity


if __name__ == '__main__':
    main()
