#!/usr/bin/env python3
"""Config 3 bench (the default of ``python bench.py``): whole-genome
1000G-shape store sharded across the GPUs by the product sharder
(sbeacon.sharding.ShardPlan over the generated genome VCF: record-balanced
(contig, POS) cores + 10 kb halo) and variantType Beacon requests -- 1 M per
GPU (weak scaling, the default: N M genome-wide requests routed to the shards
by ShardPlan.route / slice_runs) or 1 M in total (``--scaling strong``).

One step = every rank runs its request batch (request_eval_kernel: each
request's slices on this rank as one chain; request_tile_scan_kernel +
request_deliver_kernel: request rows, row offsets and dense hit lists with
global record ids), then delivers rows + hits to each request's host-facing
rank (sbeacon.shard.ResultExchange: sizes gathered once per batch, then one
RCCL send/recv group over xGMI per step for the straddling requests;
``--deliver rank0`` sends everything to rank 0).  Barrier +
torch.cuda.synchronize() bracket the K timed steps; the time is the max over
ranks.  Prints one JSON line on rank 0.  tests/test_bench_step_gloo.py runs
this step (shard_setup + make_step) at world 2 over gloo against the
unsharded oracle.
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


def step_streams(torch, dev, n):
    """n streams for the bench step, each on a hardware queue of its own.
    HIP hands a process's streams its few hardware queues (GPU_MAX_HW_QUEUES,
    4) and two plain streams shared one (measured: the steps never
    overlapped, 0.085 ms/step as on one stream); a stream created with a CU
    mask gets a queue of its own, and a mask over every CU restricts nothing
    (0.0675 ms/step; the first stream at high priority instead: 0.0724).
    SBEACON_BENCH_STREAMS (measurement): 'cumask' (default), 'prio', 'plain'."""
    import ctypes
    mode = os.environ.get('SBEACON_BENCH_STREAMS', 'cumask')
    if mode == 'cumask':
        # torch's own HIP runtime (the one process-wide copy the library binds to as well)
        p = os.path.join(os.path.dirname(torch.__file__), 'lib', 'libamdhip64.so')
        hip = ctypes.CDLL(p if os.path.exists(p) else 'libamdhip64.so')
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        words = (n_cu + 31) // 32
        mask = (ctypes.c_uint32 * words)(*([0xffffffff] * words))
        out, raw = [], []
        for _ in range(n):
            h = ctypes.c_void_p()
            if hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask) != 0:
                raise RuntimeError('hipExtStreamCreateWithCUMask failed')
            raw.append(h)
            out.append(torch.cuda.ExternalStream(h.value, device=dev))

        def destroy():  # (ours, not torch's: destroyed once the steps are done, not left to process exit)
            torch.cuda.synchronize()
            for h in raw:
                hip.hipStreamDestroy(h)
        return out, destroy
    if mode == 'prio':
        lo, hi = torch.cuda.Stream.priority_range()
        return [torch.cuda.Stream(device=dev, priority=hi if k == 0 else lo) for k in range(n)], lambda: None
    return [torch.cuda.Stream(device=dev) for _ in range(n)], lambda: None


def main_genome(args):
    import numpy as np
    import torch
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    # the step's streams (--streams, below), created before the store and
    # the library's own streams: HIP hands a process's streams its few
    # hardware queues (GPU_MAX_HW_QUEUES) as they are created, and two step
    # streams created later shared one queue (measured: no overlap at all)
    n_streams = max(1, args.streams)
    ss, ss_destroy = step_streams(torch, dev, n_streams) if n_streams > 1 else (None, lambda: None)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=dev)
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_requests, union_rows, shard_slices
    from sbeacon.requests import COMPACT_ALL, widen_compact, widen_hits, widen_rows
    from sbeacon.shard import ResultExchange

    t0 = time.perf_counter()
    shape = GenomeShape(n_total=args.genome_records, seed=3)
    n_shard = shape.shard_records(world, rank)
    last = [0.0]

    def progress(contig, done):
        if time.perf_counter() - last[0] > 20:
            last[0] = time.perf_counter()
            log(f'[rank {rank}] ingest: {done}/{n_shard} records (contig {contig}), {last[0] - t0:.0f} s')

    # the store north_star describes: sites + the 2,504-sample carrier
    # bit-matrix (~320 B per ALT row; the requests never read it)
    store = shape.build_shard_store(world, rank, device=local, threads=args.threads, progress=progress,
                                    genotypes=True)
    info = store.info()
    t_ingest = time.perf_counter() - t0
    log(f'[rank {rank}] shard: {info["n_records"]} records, {info["device_bytes"] / 2**20:.0f} MiB HBM, '
        f'ingest {t_ingest:.1f} s')
    # weak scaling (default): genome-wide requests, args.genome_requests per GPU, routed
    # to the shards by position; strong: args.genome_requests in total.  The
    # step rotates over args.batches independently drawn request sets (seeds
    # 1003, 1004, ...), each prepared once: a step answers a batch the device
    # did not answer in the previous step (its ~220 MB working set is out of
    # the 256 MB MALL by the time it comes round again), starting from the
    # packed requests resident in HBM -- the planning kernels run inside the
    # step (sb_requests_set_replan)
    n_req = step_request_count(args, world)
    stream = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    B = []
    for k in range(args.batches):
        reqs_k = step_requests(shape, args, world, k)
        sr, owners, base = shard_setup(shape, reqs_k, world, rank, args.deliver)  # ShardPlan routing
        batch = prepare_shard_requests(store, sr)      # request batch: packing + upload + planning (C++)
        batch.set_stream(stream)  # torch's stream: kernels, torch ops and RCCL in one order
        batch.set_replan(True)
        # the narrow outputs (sb_requests_set_compact): rows as four u32 sums
        # (16 B instead of 40), u32 row offsets, hits as u32 (record + base) |
        # ALT << 29 -- the genome's 85 M records fit 29 bits and a request's
        # sums 32; the library refuses a batch or fails a pass (SB_EINTERNAL)
        # that would not fit, and the exchange flags a cross-rank row sum
        # past 32 bits (row_overflow)
        batch.set_compact(COMPACT_ALL)
        pst = batch.stats()
        B.append(dict(reqs=reqs_k, sr=sr, batch=batch, pst=pst,
                      part=torch.zeros((max(sr.n_rows, 1), 4), dtype=torch.int32, device=dev),
                      hits=torch.zeros(max(int(pst['hits']), 1), dtype=torch.int32, device=dev),
                      row_off=torch.zeros(sr.n_rows + 1, dtype=torch.int32, device=dev),
                      ex=ResultExchange(dist, rank, world, sr.row_lo, sr.n_rows, owners, dev, row_fields=4,
                                        row_dtype=torch.int32)))
    t_prepare = (time.perf_counter() - t0) / args.batches
    reqs, sr, batch, pst = B[0]['reqs'], B[0]['sr'], B[0]['batch'], B[0]['pst']
    part, hits, row_off, ex = B[0]['part'], B[0]['hits'], B[0]['row_off'], B[0]['ex']
    log(f'[rank {rank}] {args.batches} batches of {n_req} requests; batch 0: rows {sr.row_lo}+{sr.n_rows}, '
        f'{pst["chains"]} chains, delivery {args.deliver}: owns {ex.n_own} rows, receives {len(ex.recvs)} '
        f'range(s), prepare {t_prepare:.2f} s per batch')

    # answer + deliver: request rows + dense hit lists (one pass), exchange.
    # Consecutive steps' batches alternate over args.streams HIP streams
    # (batch k on stream k mod N, its exchange too): independent batches in
    # flight, as a serving loop keeps them -- one batch's delivery and its
    # eval's ramp and drain overlap the next batch's eval.  Every step's work
    # is inside the bracket (torch.cuda.synchronize() waits for every stream)
    if ss is None:
        ss = [torch.cuda.current_stream()]
    for k, b in enumerate(B):
        b['stream'] = ss[k % n_streams]
        b['batch'].set_stream(b['stream'].cuda_stream)

    def on_stream(f, s):
        def g():
            with torch.cuda.stream(s):
                return f()
        return g

    steps = [on_stream(make_step(lambda p, h, o, b=b: b['batch'].run(p.data_ptr(), h.data_ptr(), o.data_ptr(), base),
                                 b['ex'], b['part'], b['hits'], b['row_off']), b['stream']) for b in B]

    for i in range(max(args.warmup, args.batches)):
        steps[i % len(steps)]()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ea = [torch.cuda.Event(enable_timing=True) for _ in ss]
    ez = [torch.cuda.Event(enable_timing=True) for _ in ss]
    t1 = time.perf_counter()
    for e, s_ in zip(ea, ss):
        e.record(s_)
    for i in range(args.steps):
        steps[i % len(steps)]()
    for e, s_ in zip(ez, ss):
        e.record(s_)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t1
    if dist:
        dist.barrier()
    # events on every step stream around the K steps: first start to last end
    step_dev_ms = max(ea[0].elapsed_time(e) for e in ez) / args.steps
    # the measurements below time one batch at a time on torch's stream (the
    # eval kernel alone, the serial pass): each batch's runs synced first (the
    # invariant word of every timed pass is checked here: SB_EINTERNAL raises)
    for b in B:
        b['batch'].sync()
        b['batch'].set_stream(stream)
    ss_destroy()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if any(b['ex'].row_overflow() for b in B):  # (u32 rows: a cross-rank sum left 32 bits)
        raise RuntimeError('a request row sum left 32 bits in the exchange: compact rows cannot hold it')
    # the dominant kernel (request_eval_kernel) alone: events around its launch
    # in each pass on its stream (sb_requests_time_eval), the same rotation
    for b in B:
        b['batch'].time_eval(True)
    for i in range(args.steps):
        b = B[i % len(B)]
        b['batch'].run(b['part'].data_ptr(), b['hits'].data_ptr(), b['row_off'].data_ptr(), base)
    n_pass = [len(range(k, args.steps, len(B))) for k in range(len(B))]
    eval_ms = []
    for b, n in zip(B, n_pass):
        b['batch'].sync()
        if n:
            eval_ms.append((b['batch'].timing()['scan_ms'], n))
        b['batch'].time_eval(False)
    kern_ms = sum(t * n for t, n in eval_ms) / max(sum(n for _, n in eval_ms), 1)
    # the memory level: the same rotation with L2 and the 256 MiB Infinity
    # Cache evicted before every pass (a 1 GiB device buffer written between
    # passes, outside the eval kernel's events), against the store's
    # candidate columns (the VcQ words + record ids the eval reads)
    n_cand, cand_bytes = store.candidates()
    flush = torch.empty(1 << 28, dtype=torch.int32, device=dev)
    for b in B:
        b['batch'].time_eval(True)
    for i in range(args.steps):
        flush.fill_(i)
        b = B[i % len(B)]
        b['batch'].run(b['part'].data_ptr(), b['hits'].data_ptr(), b['row_off'].data_ptr(), base)
    cold = []
    for b, n in zip(B, n_pass):
        b['batch'].sync()
        if n:
            cold.append((b['batch'].timing()['scan_ms'], n))
        b['batch'].time_eval(False)
    cold_ms = sum(t * n for t, n in cold) / max(sum(n for _, n in cold), 1)
    del flush
    # the pass without the exchange (re-plan + eval + tile scan + deliver), same rotation
    torch.cuda.synchronize()
    e0.record()
    for i in range(args.steps):
        b = B[i % len(B)]
        b['batch'].run(b['part'].data_ptr(), b['hits'].data_ptr(), b['row_off'].data_ptr(), base)
    e1.record()
    torch.cuda.synchronize()
    pass_ms = e0.elapsed_time(e1) / args.steps
    nhits = int(row_off[-1].item())
    # candidate statistics of each batch's chains (the slice view of the same
    # requests), averaged over the rotation as the timing is
    from sbeacon.genome import prepare_shard_batch
    agg = dict(chains=0.0, cand_unique=0.0, cand_window=0.0, cand_loaded=0.0, hits=0.0, slices=0.0, uniq=0.0,
               rows=0.0)
    for b, n in zip(B, n_pass):
        sl = shard_slices(shape, b['reqs'], world, rank)  # slice view (statistics / roofline pricing only)
        sbat = prepare_shard_batch(store, sl)
        st = sbat.stats()
        sbat.free()
        w = n / max(args.steps, 1)
        agg['chains'] += w * float(b['pst']['chains'])
        agg['cand_unique'] += w * st['cand_unique']
        agg['cand_window'] += w * st['cand_window']
        agg['cand_loaded'] += w * st['cand_loaded']
        agg['hits'] += w * float(b['row_off'][-1].item())
        agg['slices'] += w * len(sl)
        agg['uniq'] += w * union_rows(shape, sl)
        agg['rows'] += w * b['sr'].n_rows
    st = {'cand_unique': agg['cand_unique'], 'cand_window': agg['cand_window'], 'cand_loaded': agg['cand_loaded']}
    # Roofline of the request pass, priced on the bytes it must move at least
    # once.  request_eval_kernel: per request its 32 B chain
    # descriptor (ReqChain), 16 B row and 4 B row count (the compact outputs
    # the step writes); 16 B per candidate in
    # the union of the chain windows (the VcQ word: POS, END, VtHot word, AC;
    # each once however many overlapping requests read it; runs under a
    # common AN read nothing else); 4 B per hit staged.  Beside it the round-4
    # basis (24 B per candidate, 8 B per hit: what the round-4 kernel read and
    # wrote) and the SURVEY §8d contract: 32 B x unique records in the slice
    # windows + 8 B / hit.
    chains, hits_avg = agg['chains'], agg['hits']
    comp = (32.0 + 16.0 + 4.0) * chains + 16.0 * st['cand_unique'] + 4.0 * hits_avg
    achieved = comp / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    comp_r04 = (32.0 + 40.0 + 8.0) * chains + 24.0 * st['cand_unique'] + 8.0 * hits_avg
    # the whole pass: the planning kernels (32 B packed request read, 32 B
    # descriptor written per request), eval, tile scan, delivery (+ 4 B row
    # count read and 4 B row offset written per request; per hit its staged word read (4 B), its record id
    # read (4 B), the 4 B hit written: u32 hits, sb_requests_set_compact).  The record id is priced once
    # per hit although the eval now loads it beside each candidate's VcQ word (coalesced, instead of the
    # delivery's per-hit gather): the pricing counts what the answer needs, not what the kernel reads.
    # -- when the eval kernel plans its runs itself (sb_requests_plan_fused: a
    # fixed-stride re-planning pass) the descriptors never reach HBM and the
    # eval's 32 B per request is the packed request (ReqIn) instead: no
    # planning bytes of their own
    fused = all(b['batch'].plan_fused() for b in B)
    comp_pass = comp + (0.0 if fused else 64.0) * agg['rows'] + 8.0 * chains + 12.0 * hits_avg
    achieved_pass = comp_pass / (pass_ms * 1e-3) / 1e9 if pass_ms > 0 else 0.0
    uniq = agg['uniq']
    contract = 32.0 * uniq + 8.0 * hits_avg
    traffic = None  # HBM bytes per launch from the PMC passes (tools/gpu_r03_pmc.sh)
    tf = os.path.join(REPO, 'profiles', 'traffic_genome.json')
    if world == 1 and os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get('records') == shape.n_total and tj.get('requests') == len(reqs) and \
                    tj.get('kernel') == 'request_eval_kernel' and tj.get('batches') == args.batches:
                traffic = tj.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None
    # delivered: requests in host memory -> rows + hit lists in host memory,
    # everything inside the timed region (routing to the rank, planning,
    # upload, the pass, D2H); rank-local (no exchange)
    delivered = None
    if world == 1:
        serial = delivered_passes(args, store, shape, reqs, world, rank, base, dev)
        chunked = delivered_pipelined(args, store, shape, reqs, world, rank, base, dev)
        streaming = delivered_streaming(args, store, shape, reqs, world, rank, base, dev)
        if chunked['hits_returned'] != serial['hits_returned']:
            raise RuntimeError(f'pipelined delivery returned {chunked["hits_returned"]} hits, serial '
                               f'{serial["hits_returned"]}')
        # full-size property: the step's rows + hit lists (one batch, resident),
        # the serial delivered pass, the pipelined chunks and the streamed
        # batches are bit-identical
        step_digest = digest(widen_rows(part[:sr.n_rows].cpu().numpy()), [widen_hits(hits[:nhits].cpu().numpy())])
        if not (step_digest == serial['digest'] == chunked['digest'] == streaming['digest']) or \
                not streaming['hits_equal_every_batch']:
            raise RuntimeError(f'delivery digests differ: step {step_digest}, serial {serial["digest"]}, '
                               f'pipelined {chunked["digest"]}, streaming {streaming["digest"]}')
        # the headline delivered figure is the serving loop's steady state
        # (round 6); one batch's makespan, serial and chunk-pipelined, beside it
        delivered = {'requests_per_s': streaming['requests_per_s'], 'ms_per_batch': streaming['ms_per_batch'],
                     'form': 'streaming: back-to-back 1 M-request batches, the next prepared on a host thread '
                             'while the current runs and copies back',
                     'digests_equal_step': True, 'streaming': streaming, 'serial': serial,
                     'pipelined_chunks': chunked}
        delivered['cold_launch'] = cold_launch_probe(store, shape, reqs, world, rank, base, dev)
        delivered['cold_launch']['note'] = (
            'request_eval_kernel of a freshly prepared batch, HIP events: first and second launch after a 50 ms idle '
            'gap, and after ~8 fp32 GEMMs (a busy device); round 3 traced 0.76-0.81 ms launches in its serial '
            'delivered passes')
        route_out, route_bodies_last = route_bodies_passes(args, store, shape, reqs, world, rank, base, dev)
        if route_out['hits_returned'] != serial['hits_returned']:
            raise RuntimeError(f'route bodies pass returned {route_out["hits_returned"]} hits, serial '
                               f'{serial["hits_returned"]}')
    # per-rank load (the first multi-GPU run shows its imbalance): rows
    # answered, rows owned (host-facing), straddling rows sent / received
    # by the exchange, hits staged
    sent = sum(b - a for _, a, b in ex.sends)
    recv = sum(n for _, _, n in ex.recvs)
    vals = [elapsed, kern_ms, agg['slices'], float(st['cand_loaded']), hits_avg, achieved, float(uniq), comp,
            contract, step_dev_ms, pass_ms, achieved_pass, comp_pass, comp_r04, float(agg['rows']), float(ex.n_own),
            float(sent), float(recv)]
    if dist:
        t = torch.tensor(vals, dtype=torch.float64, device=dev)
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        allv = [x.tolist() for x in allv]
    else:
        allv = [vals]
    elapsed = max(v[0] for v in allv)
    tot_slices = sum(v[2] for v in allv)
    tot_cand = sum(v[3] for v in allv)
    tot_hits = sum(v[4] for v in allv)
    cpu = parity = None
    if world != 1:
        route_out = route_bodies_last = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline_and_parity(args, shape, reqs, widen_rows(ex.exchange(part, hits, row_off).cpu().numpy()),
                                              widen_hits(hits.cpu().numpy()),
                                              row_off.cpu().numpy().view(np.uint32).astype(np.int64),
                                              bodies=route_bodies_last)
        if route_out is not None:
            route_out['parity'] = parity.pop('bodies')
        if route_bodies_last is not None:
            route_bodies_last.free()
        # the other batches of the rotation: a smaller sample each, parity only
        parity['other_batches'] = []
        for k, b in enumerate(B[1:], start=1):
            _, pk = cpu_baseline_and_parity(args, shape, b['reqs'],
                                            widen_rows(b['ex'].exchange(b['part'], b['hits'], b['row_off']).cpu().numpy()),
                                            widen_hits(b['hits'].cpu().numpy()),
                                            b['row_off'].cpu().numpy().view(np.uint32).astype(np.int64), n_sample=4000,
                                            seed=7 + k, timed=False)
            pk['batch'] = k
            parity['other_batches'].append(pk)
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
        'dtype': 'u32',  # compact outputs: rows as checked u32 sums, u32 offsets and hits
        'data': 'synthetic (seeded whole-genome 1000G-shape VCF text per contig shard + its 2504-sample carrier '
                'bit-matrix, generated + ingested in-process)',
        'config': {'workload': 'config3-wgs-1000g-shape', 'records': shape.n_total, 'requests': n_req,
                   'requests_per_gpu': args.genome_requests if args.scaling == 'weak' else None,
                   'slice_queries': int(tot_slices),
                   'parallelism': f'contig shards x{world} (+10 kb halo); request rows + hit lists delivered to '
                                  f'the {"first slice" if args.deliver == "first" else "rank 0"} rank over '
                                  f'{"RCCL" if world > 1 else "(no peer)"}'},
        'step': f'one request batch of a rotation over {args.batches} independently drawn 1 M-request batches '
                f'(step i answers batch i mod {args.batches}; packed requests resident in HBM): '
                + ('request_eval_kernel planning each run in the wave (each request\'s candidate range by a batched '
                   'lower / upper bound of its splitQuery window in the (segment, kind) index; fixed-stride staging; '
                   'sb_requests_plan_fused) and evaluating it ' if fused else
                   'planning (request_plan_kernel: each request\'s candidate range by a batched lower / upper bound '
                   'of its splitQuery window in the (segment, kind) index + its staging capacity), '
                   'request_eval_kernel ')
                + '(every request = one chain of its 10 kb slices, rows + hits staged per run), '
                'request_deliver_kernel (each workgroup\'s output base summed from the eval workgroup totals -- '
                'request_tile_scan_kernel\'s tile offsets with SBEACON_REQ_TILE_SCAN=1 --, row offsets, dense hit lists '
                'in request order; compact outputs: rows as four u32 sums, u32 offsets and hits), '
                'then the exchange (send/recv of straddling rows and hits)'
                + (f'; consecutive steps on {n_streams} HIP streams (batch k on stream k mod {n_streams}: '
                   f'{n_streams} independent batches in flight, one batch\'s delivery and its eval\'s ramp and drain '
                   'overlapping the next batch\'s eval; every step inside the synchronize bracket)'
                   if n_streams > 1 else ''),
        'streams': n_streams,
        'slice_queries_per_s': round(tot_slices * args.steps / elapsed, 1),
        'candidates_loaded_per_s': round(tot_cand * args.steps / elapsed, 1),
        'hits_per_step': int(tot_hits),
        'device_ms_per_step': {'step_rank0': round(r0[9], 4), 'pass_rank0': round(r0[10], 4),
                               'eval_kernel_rank0': round(r0[1], 4),
                               'eval_kernel_max': round(max(v[1] for v in allv), 4)},
        'per_rank': [{'rank': r, 'step_ms': round(v[0] / args.steps * 1e3, 4), 'eval_kernel_ms': round(v[1], 4),
                      'pass_ms': round(v[10], 4), 'rows': int(v[14]), 'owned_rows': int(v[15]),
                      'straddling_rows_sent': int(v[16]), 'straddling_rows_received': int(v[17]),
                      'hits_per_step': int(v[4]), 'slice_queries': int(v[2])} for r, v in enumerate(allv)],
        'roofline': {'bound': 'hbm', 'achieved': round(r0[5], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(r0[5] / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'kernel': 'request_eval_kernel (rank 0, the dominant kernel of the pass): HIP events around '
                               'its launch in each of K rotating passes on one stream, one pass at a time (not beside '
                               'another batch as the timed steps run), averaged; rocprof: the launches of that serial '
                               'phase (the timed steps\' launches share the device with the other stream\'s), '
                               'profiles/',
                     'algorithmic_bytes_per_launch': r0[7],
                     'pricing': 'bytes the launch must move at least once: 52 B/request (32 B '
                                + ('packed request, planned in the wave' if fused else 'chain descriptor')
                                + ' + 16 B row + 4 B row count: the compact outputs) + 16 B per candidate in the '
                                'union of the chain windows (POS, END, VtHot word, AC) + 4 B/hit staged',
                     'planning_fused': fused,
                     'limiter': 'VALU issue, not memory: SQ_INSTS_VALU 1,869 per wave x 15.6 k waves is ~47 us of '
                                'issue at 4 cycles per wave64 op on 1,024 SIMDs; without the candidate loop the '
                                'kernel runs 18.9 us; HBM-cold it is 1.2x slower, not the ~2x of a bandwidth-bound '
                                'kernel (profiles/r06_eval/sq_tables.txt, ab.log; DESIGN.md 3.1)',
                     'memory_level': {
                         'candidate_columns_bytes': int(cand_bytes), 'candidates': int(n_cand),
                         'infinity_cache_bytes': 256 << 20,
                         'eval_ms_warm': round(kern_ms, 4), 'eval_ms_cold': round(cold_ms, 4),
                         'frac_cold': round(comp / (cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if cold_ms > 0 else None,
                         'note': 'warm: the rotation as timed above; cold: the same passes with a 1 GiB device buffer '
                                 'written before each (L2 and the MALL evicted; HIP events around the eval kernel '
                                 'only).  candidate_columns_bytes: the whole store\'s VcQ words + record ids; a '
                                 'batch reads those of its windows\' unique candidates (candidates.unique x 20 B)'},
                     'r04_basis': {'bytes': r0[13], 'frac': round(r0[13] / (r0[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                   if r0[1] > 0 else None,
                                   'note': 'the round-4 pricing (80 B per request, 24 B per candidate, 8 B per hit '
                                           'staged: what the round-4 kernel read and wrote) over this kernel time, '
                                           'for comparison'},
                     'pass': {'ms': round(r0[10], 4), 'achieved': round(r0[11], 1),
                              'frac': round(r0[11] / HBM_PEAK_GBS, 4), 'bytes': r0[12],
                              'note': ('eval with its planning (no descriptors in HBM)' if fused else
                                       'planning (+64 B/request: packed request read, descriptor written) + eval')
                                      + ' + delivery (+8 B/request: row count read, offset written; '
                                      '+12 B/hit: staged word and record id read, 4 B hit written)'},
                     'candidates': {'unique': int(st['cand_unique']), 'in_windows': int(st['cand_window']),
                                    'loaded': int(st['cand_loaded'])},
                     'contract_bytes_per_launch': r0[8],
                     'contract_frac': round(r0[8] / (r0[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if r0[1] > 0 else None,
                     'contract_note': 'SURVEY 8d prices a full scan of every record in the slice windows (32 B x '
                                      'unique records + 8 B/hit); the candidate index never reads most of them, so '
                                      'this is records covered per second, not bytes moved'},
        'delivered': delivered,
        'route_bodies': route_out,
        'cpu_baseline': cpu,
        'parity_sample': parity,
        'ingest_s': round(t_ingest, 2),
        'prepare_s': round(t_prepare, 3),
        'batches': args.batches,
    }
    # the store and the batches' buffers go before the caller's next workload
    for b in B:
        b['batch'].free()
    del B, steps, part, hits, row_off, ex
    store.close()
    torch.cuda.empty_cache()
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


def step_request_count(args, world) -> int:
    """Requests per step in total: args.genome_requests per GPU (weak
    scaling: the per-GPU work is fixed as the world grows) or in total
    (strong: the world splits a fixed batch)."""
    return args.genome_requests * (world if args.scaling == 'weak' else 1)


def step_requests(shape, args, world, k):
    """Batch k of the step's rotation: genome-wide config-3 requests (seed
    1003 + k), step_request_count of them, ordered by (contig, start); every
    rank draws the same set and routes its part (shard_setup)."""
    from sbeacon.genome import config3_requests
    return config3_requests(shape, n=step_request_count(args, world), seed=1003 + k)


def shard_setup(shape, reqs, world, rank, deliver):
    """One rank's routing, all through the product sharder
    (sbeacon.sharding.ShardPlan over the genome's layout, GenomeShape.plan):
    its sub-requests (ShardPlan.slice_runs: the splitQuery slices whose first
    base its core holds), the host-facing rank of each of its rows
    (ShardPlan.route of the request's first slice, or rank 0) and the first
    record of its store (ShardPlan.record_range)."""
    import numpy as np
    from sbeacon.genome import rank_of_slices, shard_record_base, shard_requests
    from sbeacon.shard import owner_ranks
    sr = shard_requests(shape, reqs, world, rank)
    rows = sr.row_lo + np.arange(sr.n_rows)
    first = rank_of_slices(shape, world, reqs.ci[rows], reqs.start[rows] + 1)
    return sr, owner_ranks(first, deliver, rank), shard_record_base(shape, world, rank)


def digest(rows, hit_parts) -> str:
    """blake2b over the request rows (int64 [n, 5]) and the hit lists in
    request order (uint64 arrays, concatenated): the delivery paths' outputs
    compared at full size without keeping copies."""
    import hashlib
    import numpy as np
    h = hashlib.blake2b(digest_size=16)
    h.update(np.ascontiguousarray(rows, dtype=np.int64).tobytes())
    for x in hit_parts:
        h.update(np.ascontiguousarray(x).view(np.uint64).tobytes())
    return h.hexdigest()


def make_step(run, ex, part, hits, row_off):
    """The bench step: ``run(part, hits, row_off)`` answers the rank's
    sub-requests into its rows / dense hit lists, then ResultExchange
    delivers them to their host-facing ranks and merges each owned request's
    received hits into the owner's dense lists (ResultExchange.merge).
    Returns the owned rows."""
    def step():
        run(part, hits, row_off)
        rows = ex.exchange(part, hits, row_off)
        if ex.world > 1:
            ex.merge()
        return rows
    return step


def delivered_passes(args, store, shape, reqs, world, rank, base, dev, passes=5):
    """End to end on one GPU: requests (numpy, host) -> the rank's row range
    (shard_rows) -> request batch planning + upload
    (sb_requests_prepare_beacon: conversion, the core cut and packing in C++,
    then the planning kernels) -> one pass in the compact output form
    (sb_requests_set_compact: 16 B rows, u32 row offsets, u32 hits) -> rows,
    row offsets and the hit lists copied back into pinned host memory.  Every
    part inside the timed region; a fresh batch each pass."""
    import numpy as np
    import torch
    from sbeacon.genome import prepare_beacon_shard, shard_rows
    from sbeacon.requests import widen_compact
    t_route = t_prep = t_dev = 0.0
    best = None
    rows_h = hits_h = ro_h = None
    for k in range(passes + 1):  # pass 0 warms the allocator / pinned buffers (untimed)
        torch.cuda.synchronize()
        a = time.perf_counter()
        rr = shard_rows(shape, reqs, world, rank)
        b0 = time.perf_counter()
        _, n_rows, batch = prepare_beacon_shard(store, shape, reqs, world, rank, rows=rr)
        batch.set_stream(torch.cuda.current_stream().cuda_stream)
        batch.set_compact(True)
        cap = int(batch.stats()['hits'])
        c0 = time.perf_counter()
        if rows_h is None or rows_h.shape[0] < n_rows or hits_h.shape[0] < cap:
            rows_d = torch.empty((max(n_rows, 1), 4), dtype=torch.int32, device=dev)
            ro_d = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
            hits_d = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
            rows_h = torch.empty(rows_d.shape, dtype=torch.int32, pin_memory=True)
            ro_h = torch.empty(ro_d.shape, dtype=torch.int32, pin_memory=True)
            hits_h = torch.empty(hits_d.shape, dtype=torch.int32, pin_memory=True)
        batch.run(rows_d.data_ptr(), hits_d.data_ptr(), ro_d.data_ptr(), base)
        rows_h[:n_rows].copy_(rows_d[:n_rows], non_blocking=True)
        ro_h.copy_(ro_d, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        total = int(ro_h[-1].numpy().view(np.uint32))
        hits_h[:total].copy_(hits_d[:total], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        d0 = time.perf_counter()
        batch.sync()  # (the pass's invariant word; outside the timed region)
        batch.free()
        if k == 0:
            continue
        t_route += b0 - a
        t_prep += c0 - b0
        t_dev += d0 - c0
        best = (d0 - a) if best is None else min(best, d0 - a)
    dt = (t_route + t_prep + t_dev) / passes
    n = len(reqs)
    total = int(ro_h[-1].numpy().view(np.uint32))
    rows_w, hits_w, _ = widen_compact(rows_h[:n_rows].numpy(), hits_h[:total].numpy(), ro_h.numpy())
    return {'requests_per_s': round(n / dt, 1), 'ms_per_pass': round(dt * 1e3, 2),
            'best_ms': round(best * 1e3, 2), 'passes': passes,
            'split_ms': {'route_rows': round(t_route / passes * 1e3, 2),
                         'prepare_upload': round(t_prep / passes * 1e3, 2),
                         'device_pass_and_d2h': round(t_dev / passes * 1e3, 2)},
            'hits_returned': total,
            'd2h_bytes': int(16 * n_rows + 4 * (n_rows + 1) + 4 * total),
            'digest': digest(rows_w, [hits_w]),
            'note': 'requests as numpy columns in host memory -> compact rows (16 B) + u32 row offsets + u32 hit '
                    'lists in pinned host memory; routing, planning, upload, the pass and both D2H copies inside '
                    'the timed region (digest over the widened outputs)'}


def delivered_streaming(args, store, shape, reqs, world, rank, base, dev, batches=8, blocking=True):
    """A serving loop's steady state: consecutive 1 M-request batches, batch
    i + 1 routed and prepared on a host thread (sb_requests_prepare_beacon on
    every core the library's pool holds) while batch i runs and copies its
    rows, offsets and hits back into pinned host memory on the stream.  Each
    batch is the full delivered path of `delivered_passes` (a fresh batch:
    routing, packing, upload, planning, the pass, both D2H copies); the
    figure is requests over the wall time of the whole sequence, the first
    batch's preparation included (nothing is prepared before the clock
    starts).  What `delivered_passes` and the chunked form measure is one
    batch's makespan; this is the throughput of back-to-back batches."""
    import numpy as np
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from sbeacon.genome import prepare_beacon_shard, shard_rows
    from sbeacon.requests import widen_compact
    stream = torch.cuda.current_stream()

    def prep():
        rr = shard_rows(shape, reqs, world, rank)
        _, m, bt = prepare_beacon_shard(store, shape, reqs, world, rank, rows=rr)
        return m, bt, int(bt.stats()['hits'])

    # buffers sized by one untimed batch
    m, bt, cap = prep()
    bt.free()
    rows_d = torch.empty((max(m, 1), 4), dtype=torch.int32, device=dev)
    ro_d = torch.empty(m + 1, dtype=torch.int32, device=dev)
    hits_d = torch.empty(max(cap, 1) + (cap >> 4), dtype=torch.int32, device=dev)
    rows_h = torch.empty(rows_d.shape, dtype=torch.int32, pin_memory=True)
    ro_h = torch.empty(ro_d.shape, dtype=torch.int32, pin_memory=True)
    hits_h = torch.empty(hits_d.shape, dtype=torch.int32, pin_memory=True)
    totals = []

    # the main thread waits for its copies with a blocking-sync event (it
    # sleeps instead of spinning on a core the preparing thread's pack needs)
    def wait():
        if not blocking:
            stream.synchronize()
            return
        e = torch.cuda.Event(blocking=True)
        e.record(stream)
        e.synchronize()

    import gc
    gc.collect()
    gc.disable()
    with ThreadPoolExecutor(1) as ex:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fut = ex.submit(prep)
        for i in range(batches):
            m, bt, cap = fut.result()
            if i + 1 < batches:
                fut = ex.submit(prep)  # the next batch's host work, beside this batch's device work
            if cap > hits_d.shape[0]:
                raise RuntimeError('streaming: a batch outgrew the hit buffers sized on the first')
            bt.set_stream(stream.cuda_stream)
            bt.set_compact(True)
            bt.run(rows_d.data_ptr(), hits_d.data_ptr(), ro_d.data_ptr(), base)
            rows_h[:m].copy_(rows_d[:m], non_blocking=True)
            ro_h.copy_(ro_d, non_blocking=True)
            wait()
            total = int(ro_h[m].numpy().view(np.uint32))
            hits_h[:total].copy_(hits_d[:total], non_blocking=True)
            wait()
            bt.sync()  # the pass's invariant word (a serving loop checks it too)
            bt.free()  # its buffers back to the store's pool for batch i + 2
            totals.append(total)
            last = (m, total)
        dt = time.perf_counter() - t0
    gc.enable()
    m, total = last
    rows_w, hits_w, _ = widen_compact(rows_h[:m].numpy(), hits_h[:total].numpy(), ro_h[:m + 1].numpy())
    n = len(reqs)
    return {'requests_per_s': round(n * batches / dt, 1), 'ms_per_batch': round(dt / batches * 1e3, 2),
            'batches': batches, 'hits_returned': total, 'hits_equal_every_batch': len(set(totals)) == 1,
            'digest': digest(rows_w, [hits_w]),
            'blocking_waits': blocking,
            'note': 'steady state of back-to-back 1 M-request batches: batch i+1 routed + prepared on one host '
                    'thread while batch i runs and copies back (compact rows, u32 offsets and hits into pinned '
                    'host memory; the main thread waits on blocking-sync events); requests over the wall time of '
                    'all batches, the first preparation included'}


def cold_launch_probe(store, shape, reqs, world, rank, base, dev):
    """The eval launch of a freshly prepared batch, timed alone (HIP events
    around request_eval_kernel): its first launch, a second launch of the
    same batch right after, and the first launch of another fresh batch
    issued right behind ~2 ms of unrelated GPU work (a busy device: no clock
    ramp)."""
    import torch
    from sbeacon.genome import prepare_shard_requests, shard_requests
    sr = shard_requests(shape, reqs, world, rank)
    out = {}
    for label in ('fresh', 'after_busy'):
        torch.cuda.synchronize()
        time.sleep(0.05)  # an idle device, as after host planning
        bt = prepare_shard_requests(store, sr)
        bt.set_stream(torch.cuda.current_stream().cuda_stream)
        cap = int(bt.stats()['hits'])
        rows = torch.empty((max(sr.n_rows, 1), 5), dtype=torch.int64, device=dev)
        hits = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        ro = torch.empty(sr.n_rows + 1, dtype=torch.int64, device=dev)
        if label == 'after_busy':
            a = torch.randn(4096, 4096, device=dev)
            for _ in range(8):
                a = a @ a
                a = a / a.norm()
        bt.time_eval(True)
        ms = []
        for _ in range(2):
            bt.run(rows.data_ptr(), hits.data_ptr(), ro.data_ptr(), base)
            bt.sync()
            ms.append(round(bt.timing()['scan_ms'], 4))
        bt.time_eval(False)
        bt.free()
        out[label] = {'first_ms': ms[0], 'second_ms': ms[1]}
    return out


def delivered_pipelined(args, store, shape, reqs, world, rank, base, dev, passes=7, chunks=8, workers=2):
    """The delivered path in chunks of consecutive request rows, pipelined:
    two host threads route and prepare chunks ahead (the chunk's row range,
    then sb_requests_prepare_beacon: the Beacon columns converted, cut to the
    rank's core and packed in one pass, uploaded, and the planning kernels on
    the thread's planning stream) while the main thread enqueues each
    prepared chunk's pass (compact outputs) and its row / row-offset D2H on
    the torch stream, and a chunk's hit list D2H once its row offsets are
    back.  Requests in host memory -> compact rows (16 B), u32 row offsets
    (per chunk) and u32 hit lists in pinned host memory, all inside the timed
    region."""
    import numpy as np
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from sbeacon.genome import prepare_beacon_shard
    from sbeacon.requests import widen_compact
    n = len(reqs)
    # chunk sizes tapered at both ends (a quarter, then 0.6, of the others):
    # the pipeline fills and drains sooner (`profiles/r04_y/` sweep)
    w = np.ones(chunks)
    if chunks > 3:
        w[0] = w[-1] = 0.25
        w[1] = w[-2] = 0.6
    cuts = np.round(np.concatenate([[0], np.cumsum(w)]) / w.sum() * n).astype(np.int64)
    stream = torch.cuda.current_stream()

    def prep(k):
        a, b = int(cuts[k]), int(cuts[k + 1])
        lo, m, bt = prepare_beacon_shard(store, shape, reqs.rows(a, b), world, rank)
        return a + lo, m, bt, int(bt.stats()['hits'])

    rows_h = torch.empty((n, 4), dtype=torch.int32, pin_memory=True)
    ro_h = torch.empty(n + chunks, dtype=torch.int32, pin_memory=True)
    rows_d = torch.empty((n, 4), dtype=torch.int32, device=dev)
    ro_d = torch.empty(n + chunks, dtype=torch.int32, device=dev)
    hits_d, hits_h = [None] * chunks, [None] * chunks
    hit_n = [0] * chunks
    times, total_hits = [], 0
    import gc
    gc.collect()
    gc.disable()  # as timeit does: a collector pause inside a ~2 ms pass is noise, not the path
    with ThreadPoolExecutor(workers) as ex:
        for p in range(passes + 1):  # pass 0 sizes the hit buffers (untimed)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            futs = [ex.submit(prep, k) for k in range(chunks)]
            live, pend = [], []
            total_hits = 0
            for k in range(chunks):
                a, m, bt, cap = futs[k].result()
                if hits_d[k] is None or hits_d[k].numel() < max(cap, 1):
                    hits_d[k] = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
                    hits_h[k] = torch.empty(max(cap, 1), dtype=torch.int32, pin_memory=True)
                bt.set_stream(stream.cuda_stream)
                bt.set_compact(True)
                ro = ro_d[a + k:a + k + m + 1]
                bt.run(rows_d[a:a + m].data_ptr(), hits_d[k].data_ptr(), ro.data_ptr(), base)
                rows_h[a:a + m].copy_(rows_d[a:a + m], non_blocking=True)
                ro_h[a + k:a + k + m + 1].copy_(ro, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                pend.append((k, ev, a + k + m))
                live.append(bt)
                while len(pend) > 1:  # the previous chunk's hits, once its offsets are back
                    kk, e, last = pend.pop(0)
                    e.synchronize()
                    nh = hit_n[kk] = int(ro_h[last].numpy().view(np.uint32))
                    total_hits += nh
                    hits_h[kk][:nh].copy_(hits_d[kk][:nh], non_blocking=True)
            for kk, e, last in pend:
                e.synchronize()
                nh = hit_n[kk] = int(ro_h[last].numpy().view(np.uint32))
                total_hits += nh
                hits_h[kk][:nh].copy_(hits_d[kk][:nh], non_blocking=True)
            stream.synchronize()
            dt = time.perf_counter() - t0
            for bt in live:
                bt.sync()  # (the passes' invariant words; outside the timed region)
                bt.free()
            if p:
                times.append(dt)
    gc.enable()
    dt = sorted(times)[len(times) // 2]  # the median pass (host threads make single passes noisy)
    rows_w, _, _ = widen_compact(rows_h.numpy(), np.zeros(0, np.uint32), np.zeros(1, np.uint32))
    hit_parts = [widen_compact(np.zeros((0, 4), np.uint32), hits_h[k][:hit_n[k]].numpy(), np.zeros(1, np.uint32))[1]
                 for k in range(chunks)]
    return {'requests_per_s': round(n / dt, 1), 'ms_per_pass': round(dt * 1e3, 2),
            'mean_ms': round(sum(times) / len(times) * 1e3, 2), 'best_ms': round(min(times) * 1e3, 2),
            'pass_ms': [round(t * 1e3, 2) for t in times], 'passes': passes, 'chunks': chunks, 'workers': workers,
            'hits_returned': total_hits,
            'd2h_bytes': int(16 * n + 4 * (n + chunks) + 4 * total_hits),
            'digest': digest(rows_w, hit_parts),
            'note': f'pipelined: the requests cut into chunks of consecutive rows; {workers} host threads route + '
                    'prepare chunks ahead (sb_requests_prepare_beacon: Beacon int64 columns -> SplitQueryPayloads '
                    'cut to the core and packed in the library) while each prepared chunk runs and copies back '
                    '(compact rows, per-chunk u32 row offsets, u32 hits into pinned host memory); everything inside '
                    'the timed region (digest over the widened outputs)'}


def route_bodies_passes(args, store, shape, reqs, world, rank, base, dev, passes=3):
    """The drop-in at the route: Beacon /g_variants requests (the route's
    parameters as int64 columns in host memory, one event per request) ->
    the route's response bodies (JSON text in host memory).  Inside the timed
    region: the rank's row range, sb_requests_prepare_beacon (SplitQueryPayload
    per request, packing, device planning), one pass with compact outputs,
    the D2H copies, and sb_route_bodies (route_g_variants.py:153-198 per
    event: exists OR, distinct variant strings, one get_variant_entry per
    distinct internal id, the result-set envelope as json.dumps writes it).
    Returns (summary, the last pass's Bodies) -- the parity sample compares
    those bodies with the reference fold over the oracle's responses."""
    import numpy as np
    import torch
    from sbeacon.genome import LOCATION, prepare_beacon_shard, shard_rows
    from sbeacon.route_batch import GRAN_CODE, route_bodies
    vid = store.vcf_id(LOCATION)
    times, split = [], np.zeros(3)
    last = None
    rows_h = hits_h = ro_h = None
    for k in range(passes + 1):  # pass 0 warms the pinned buffers and the body buffer (untimed)
        if last is not None:
            last.free()
            last = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lo, hi = shard_rows(shape, reqs, world, rank)
        lo, n, batch = prepare_beacon_shard(store, shape, reqs, world, rank, rows=(lo, hi))
        batch.set_stream(torch.cuda.current_stream().cuda_stream)
        batch.set_compact(True)
        cap = int(batch.stats()['hits'])
        if rows_h is None or rows_h.shape[0] < n or hits_h.shape[0] < cap:
            rows_d = torch.empty((max(n, 1), 4), dtype=torch.int32, device=dev)
            ro_d = torch.empty(n + 1, dtype=torch.int32, device=dev)
            hits_d = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
            rows_h = torch.empty(rows_d.shape, dtype=torch.int32, pin_memory=True)
            ro_h = torch.empty(ro_d.shape, dtype=torch.int32, pin_memory=True)
            hits_h = torch.empty(hits_d.shape, dtype=torch.int32, pin_memory=True)
        t1 = time.perf_counter()
        batch.run(rows_d.data_ptr(), hits_d.data_ptr(), ro_d.data_ptr(), base)
        rows_h[:n].copy_(rows_d[:n], non_blocking=True)
        ro_h[:n + 1].copy_(ro_d[:n + 1], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        total = int(ro_h[n].numpy().view(np.uint32))
        hits_h[:total].copy_(hits_d[:total], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        t2 = time.perf_counter()
        cmap = store.__dict__['_genome_cmap'][LOCATION]
        ev = np.arange(n + 1, dtype=np.uint32)
        last = route_bodies(store, rows=rows_h[:n].numpy(), hits=hits_h[:total].numpy(), row_off=ro_h[:n + 1].numpy(),
                            compact=True, rec_base=base, row_lo=ev[:n], row_hi=ev[1:], granularity=GRAN_CODE['record'],
                            check_all=1, assembly=('GRCh38',), row_vcf=vid, row_contig=cmap[reqs.ci[lo:lo + n]])
        t3 = time.perf_counter()
        batch.sync()  # (the pass's invariant word; outside the timed region)
        batch.free()
        if k:
            times.append(t3 - t0)
            split += (t1 - t0, t2 - t1, t3 - t2)
    dt = sorted(times)[len(times) // 2]
    st = np.bincount(last.status, minlength=3)
    out = {'requests_per_s': round(len(reqs) / dt, 1), 'ms_per_pass': round(dt * 1e3, 2),
           'best_ms': round(min(times) * 1e3, 2), 'passes': passes,
           'split_ms': {'prepare_upload': round(split[0] / passes * 1e3, 2),
                        'device_pass_and_d2h': round(split[1] / passes * 1e3, 2),
                        'route_bodies': round(split[2] / passes * 1e3, 2)},
           'hits_returned': total, 'body_bytes': int(last.n_bytes),
           'body_gb_per_s': round(last.n_bytes / (split[2] / passes) / 1e9, 2),
           'events': int(n), 'status': {'body': int(st[0]), 'route_fallback': int(st[1]), 'none': int(st[2])},
           'note': 'one GET/POST /g_variants event per request (granularity record, includeResultsetResponses HIT): '
                   'Beacon int64 request columns in host memory -> the route\'s response bodies (json.dumps text of '
                   'get_result_sets_response with one get_variant_entry per distinct internal id) in host memory; '
                   'planning, the device pass (compact outputs), both D2H copies and sb_route_bodies inside the timed '
                   'region (median pass)'}
    return out, last


def cpu_baseline_and_parity(args, shape, reqs, total, hits, row_off, n_sample=20000, seed=7, timed=True, bodies=None):
    from bench import host_cores
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
    if timed:
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
    cpu = None if not timed else {
           'value': round(passes * len(pick) / dt, 1), 'unit': 'requests/s', 'cores': args.threads, 'kind': 'port',
           'host': host_cores(),
           'sample': f'{len(pick)} random requests ({len(pl)} slice payloads) x {passes} passes through oracle/sbeacon_oracle.c '
                     f'(CPU restatement of search_variants.py, patched variantType branch), OpenMP x{args.threads}, '
                     f'on a sites-only VCF holding the records those requests reach',
           'seconds': round(dt, 2), 'host_cpus': os.cpu_count()}
    parity = {'requests': len(pick), 'slice_queries': len(pl), 'mismatched_requests': bad,
              'mismatched_hit_lists': bad_hits, 'variants_checked': int(exp[:, 1].sum())}
    if bodies is not None:
        # the route's own fold (route_g_variants.aggregate + the result-set
        # envelope) over the oracle's per-slice responses of each sampled
        # request, against the body sb_route_bodies wrote for it
        import json as _json
        from sbeacon import responses as R
        from sbeacon.payloads import PerformQueryResponse
        from sbeacon.route_g_variants import _finish, aggregate
        per = [[] for _ in range(len(pick))]
        for o, r in zip(whole.req, res):
            per[o].append(PerformQueryResponse(**r) if isinstance(r, dict) else r)
        bad_b, n_entries = 0, 0
        for j, r in enumerate(pick.tolist()):
            if any(not isinstance(x, PerformQueryResponse) for x in per[j]):
                bad_b += 1
                continue
            ex, vs, rs = aggregate(per[j], granularity='record', check_all=True, assembly_id='GRCh38')
            want = _json.loads(_finish('record', ex, vs, rs, 'q', R.get_pagination_object(0, 100))['body'])
            got = _json.loads(bodies.text(r)) if int(bodies.status[r]) == 0 else None
            for b in (want, got):
                if b is not None:
                    for s_ in b['response']['resultSets']:
                        s_['results'].sort(key=lambda e: e['variantInternalId'])
            bad_b += int(got != want)
            n_entries += len(want['response']['resultSets'][0]['results'])
        parity['bodies'] = {'requests': len(pick), 'mismatched_bodies': bad_b, 'entries_checked': n_entries,
                            'note': 'each sampled request\'s body from sb_route_bodies vs the reference route fold '
                                    '(route_g_variants.aggregate + get_result_sets_response) over the C oracle\'s '
                                    'per-slice responses; results compared as sets'}
    orc.close()
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    return cpu, parity
