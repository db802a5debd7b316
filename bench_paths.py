#!/usr/bin/env python3
"""Benchmark of the ingest-side hot paths on config 4:
summariseSlice over index-style slices, then per-dataset
duplicateVariantSearch, plus the cross-dataset union count (extension).

Workload: D datasets (default 10; config 4 names 50) over one chr22-shape
site pool (1,103,547 records, seed 4); each dataset = two VCFs with the same
sites (a vcfGroup split by samples), 70 % of records shared with the pool.
The VCFs are written as BGZF (sites-only text to bound generation time —
neither path reads genotypes except through summariseSlice's skip-heuristic
delimiter count, which the sites-only records still exercise) and ingested
from the files, so virtual offsets are real.

Prints one JSON line per workload (rank 0, one GPU):
  summarise: every slice of every VCF (summariseVcf's partition) in one
             sb_summarise_slices call; unit records/s.
  dedup:     one sb_dedup_count call holding the D per-dataset jobs (whole
             contig each); unit region keys/s.  The union job is reported in
             the same line.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--datasets', type=int, default=10)
    ap.add_argument('--records', type=int, default=1103547)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--threads', type=int, default=None,
                    help='host threads (ingest, CPU baselines); default: every CPU the process may use')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--only', choices=['summarise', 'dedup'], default=None)
    ap.add_argument('--strict-datasets', type=int, default=10,
                    help='datasets whose messages also run in the reference-exact dedup mode (0: skip)')
    args = ap.parse_args(argv)
    from bench import host_cores
    if args.threads is None:
        args.threads = host_cores()['cores']
    return args


def main():
    for line in run(parse()):
        print(json.dumps(line), flush=True)


def run(args) -> list:
    """The config-4 lines (summarise, dedup) as dicts."""
    import torch
    torch.cuda.set_device(0)
    from sbeacon.engine import Store
    from sbeacon.summarise_vcf import plan_slices
    from sbeacon.workload import config4_cohort, write_bgzf

    tmp = tempfile.mkdtemp(prefix='sbeacon-paths-')
    try:
        t0 = time.perf_counter()
        pool, datasets = config4_cohort(n_datasets=args.datasets, n_records=args.records)
        files = []
        for ds, parts in datasets:
            for loc, gen in parts:
                p = os.path.join(tmp, loc.replace('/', '_').replace(':', ''))
                if parts.index((loc, gen)) == 0:
                    write_bgzf(p, gen.chunks(sites_only=True, threads=args.threads), level=1, threads=args.threads)
                    first = p
                else:
                    shutil.copyfile(first, p)  # same sites: the vcfGroup's other sample half
                files.append((loc, p))
        t_gen = time.perf_counter() - t0
        t0 = time.perf_counter()
        store = Store.build(files, device=0, keep_genotypes=False, n_threads=args.threads)
        t_ingest = time.perf_counter() - t0
        info = store.info()
        log(f'{len(files)} VCFs, {info["n_records"]} records, {info["device_bytes"] / 2**20:.0f} MiB HBM; '
            f'generate {t_gen:.1f} s, ingest {t_ingest:.1f} s')
        out = []
        if args.only != 'dedup':
            out.append(summarise_line(args, store, files, plan_slices))
        if args.only != 'summarise':
            out.append(dedup_line(args, store, datasets, files))
        for x in out:
            x['ingest_s'] = round(t_ingest, 2)
        store.close()
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def pmc_traffic(records, kernels):
    """HBM bytes per launch of the named kernels from the committed PMC passes
    (tools/gpu_pmc_r02.sh -> profiles/traffic_paths.json), when they were
    measured on this workload; else None."""
    tf = os.path.join(REPO, 'profiles', 'traffic_paths.json')
    try:
        tj = json.load(open(tf))
    except (OSError, ValueError):
        return None
    if tj.get('records') != records:
        return None
    ks = tj.get('kernels', {})
    if not all(k in ks for k in kernels):
        return None
    return sum(ks[k]['hbm_bytes_per_launch'] for k in kernels)


def summarise_line(args, store, files, plan_slices):
    # summariseVcf's plan per VCF from its CSI index (written by the ingest
    # side, sb_index_vcf; one host thread per VCF)
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(args.threads) as ex:
        plans = list(ex.map(lambda f: plan_slices(store, f[0]), files))
    log(f'summariseVcf plans (CSI written + read) for {len(files)} VCFs: {time.perf_counter() - t0:.1f} s')
    slices = []
    for (loc, _), pl in zip(files, plans):
        slices += [(loc, a, b) for a, b in pl]
    for _ in range(args.warmup):
        store.summarise_slices(slices)
    dev = []
    t = time.perf_counter()
    for _ in range(args.steps):
        res, ms = store.summarise_slices(slices, with_timing=True)
        dev.append(ms)
    wall = (time.perf_counter() - t) / args.steps
    recs = sum(r['records'] for r in res if isinstance(r, dict))
    n_records = store.info()['n_records']
    dev_ms = sum(dev) / len(dev)
    # algorithmic bytes: 8 B per record; the chunk kernel reads
    # one packed 8-byte word per record (the wide SumHot, cursor and delimiter
    # count only for escapes and overshooting records)
    alg = 8.0 * n_records
    achieved = alg / (dev_ms * 1e-3) / 1e9
    cpu = parity = None
    if not args.no_cpu_baseline:
        k = max(1, min(args.threads, len(files)))  # one VCF per host thread
        cpu, parity = summarise_cpu(files[:k], [[s for s in slices if s[0] == f[0]] for f in files[:k]],
                                    [[r for s, r in zip(slices, res) if s[0] == f[0]] for f in files[:k]],
                                    args.threads)
    return ({
        'metric': 'summariseSlice records/s (all slices of every VCF in one call)',
        'value': round(n_records / (wall * 1e-0), 1) if wall > 0 else None,
        'unit': 'records/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(wall * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'uint64', 'data': 'synthetic config-4 cohort, sites-only BGZF',
        'config': {'workload': f'config4-summarise-{args.datasets}ds', 'vcfs': len(files), 'records': n_records,
                   'slices': len(slices), 'records_visited': recs},
        'device_ms_per_step': round(dev_ms, 4),
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'traffic': pmc_traffic(n_records, ['summarise_chunk_kernel', 'summarise_finish_kernel']),
                     'kernel': 'summarise_chunk_kernel + summarise_finish_kernel',
                     'algorithmic_bytes_per_launch': alg},
        'cpu_baseline': cpu, 'parity_sample': parity})


def summarise_cpu(files, slices, got, threads):
    """oracle/summarise_oracle.c over every slice of the first VCFs (one per
    host thread), the slices spread over a pool of `threads` host threads
    (ctypes drops the GIL in the C call); each VCF inflated in memory first
    (inflate time excluded)."""
    from concurrent.futures import ThreadPoolExecutor

    from bench import host_cores
    from oracle.oracle import OracleBgzf
    orcs = [OracleBgzf(f[1]) for f in files]
    work = [(o, a, b) for o, sl in zip(orcs, slices) for _, a, b in sl]
    with ThreadPoolExecutor(threads) as ex:
        t = time.perf_counter()
        exp = list(ex.map(lambda w: w[0].summarise_slice(w[1], w[2]), work))
        dt = time.perf_counter() - t
    recs = sum(e['records'] for e in exp)
    flat = [g for gs in got for g in gs]
    bad = sum(int(g != e) for g, e in zip(flat, exp))
    for o in orcs:
        o.close()
    cpu = {'value': round(recs / dt, 1), 'unit': 'records/s', 'cores': threads, 'kind': 'port', 'host': host_cores(),
           'sample': f'every slice of {len(files)} VCFs ({len(work)} slices, {recs} records) through '
                     f'oracle/summarise_oracle.c on {threads} host threads (inflated streams in memory; inflate '
                     'time excluded)',
           'seconds': round(dt, 3)}
    return cpu, {'slices': len(work), 'mismatches': bad}


def dedup_line(args, store, datasets, files):
    jobs = [([loc for loc, _ in parts], '22', 0, 2**32 - 1) for _, parts in datasets]
    union = [([loc for loc, _ in files], '22', 0, 2**32 - 1)]
    log(f'dedup: {len(jobs)} jobs, warmup')
    for _ in range(args.warmup):
        store.dedup_counts(jobs)
    dev, keys = [], 0
    t = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        res, st = store.dedup_counts(jobs, with_stats=True)
        if os.environ.get('SBEACON_DEDUP_DEBUG'):
            log(f'dedup call {1e3 * (time.perf_counter() - t1):.3f} ms')
        dev.append(st['device_ms'])
        keys = st['keys']
    wall = (time.perf_counter() - t) / args.steps
    dev_ms = sum(dev) / len(dev)
    log(f'dedup: {wall * 1e3:.3f} ms per call, device {dev_ms:.3f} ms')
    ures, ust = store.dedup_counts(union, with_stats=True)
    ures, ust = store.dedup_counts(union, with_stats=True)
    alg = 8.0 * keys  # compulsory: one read of the 64-bit key stream
    if st['path'] == 'windows':
        # implementation bytes: one 8 B class word per key + the 8 B hash of
        # keys outside the exact class (~5 %) + 16 B per window descriptor;
        # bodies of colliding hashed keys and deferred displaced keys are noise
        impl = 8.0 * keys + 8.0 * 0.05 * keys + 16.0 * st['windows']
        kern = ('window_dedupe_kernel (one workgroup per POS window: one read of every key, LDS hash set) + '
                'deferred_dedupe_kernel (displaced keys with a possible copy at a larger POS)')
    else:
        # exact stream, ~97 % of keys, bucket path: gather (20 B/key) + two
        # radix passes on the word's mix (24 B/key each) + the bucket hash-set
        # pass (8 B/key); the hashed stream's 8 passes of 28 B/key on top
        impl = 20.0 * keys + 2 * 24.0 * keys + 8.0 * keys + 0.03 * 8 * 28.0 * keys
        kern = 'gather + 2 mix-digit radix passes + bucket hash sets (exact stream); radix sort + unique (hashed stream)'
    achieved = alg / (dev_ms * 1e-3) / 1e9
    cpu = parity = None
    if not args.no_cpu_baseline:
        from concurrent.futures import ThreadPoolExecutor

        from bench import host_cores
        from oracle.oracle import dedup_count
        k = max(1, min(args.threads, len(datasets)))  # one dataset job per host thread
        texts = [b''.join(parts[0][1].chunks(sites_only=True, threads=args.threads)) for _, parts in datasets[:k]]
        with ThreadPoolExecutor(args.threads) as ex:
            t = time.perf_counter()
            exp = list(ex.map(lambda x: dedup_count([x, x], '22', 0, 2**32 - 1), texts))
            dt = time.perf_counter() - t
        cpu = {'value': round(k * 2 * args.records / dt, 1), 'unit': 'keys/s', 'cores': args.threads, 'kind': 'port',
               'host': host_cores(),
               'sample': f'the first {k} datasets\' jobs (2 VCFs each, {2 * args.records} records per job) through '
                         f'orc_dedup_count (string keys, qsort + unique; text parse included), one job per host '
                         f'thread on {args.threads} threads', 'seconds': round(dt, 3)}
        parity = {'jobs': k, 'mismatches': int(sum(r != e for r, e in zip(res[:k], exp))), 'unique_first': exp[0]}
    strict = strict_sample(args, store, datasets) if args.strict_datasets else None
    return ({
        'metric': 'duplicateVariantSearch region keys/s (per-dataset unique counts, one batched call)',
        'value': round(keys / wall, 1) if wall > 0 else None,
        'unit': 'keys/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(wall * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'uint64', 'data': 'synthetic config-4 cohort, sites-only BGZF',
        'config': {'workload': f'config4-dedup-{args.datasets}ds', 'jobs': len(jobs), 'keys': keys,
                   'unique_per_dataset_mean': sum(r for r in res if isinstance(r, int)) / max(len(res), 1)},
        'device_ms_per_step': round(dev_ms, 4), 'path': st['path'], 'windows': st['windows'],
        'union': {'vcfs': len(files), 'keys': ust['keys'], 'unique': ures[0], 'device_ms': round(ust['device_ms'], 4)},
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'traffic': (pmc_traffic(store.info()['n_records'], ['window_dedupe_kernel', 'deferred_dedupe_kernel'])
                                 if st['path'] == 'windows' else None),
                     'kernel': kern, 'algorithmic_bytes_per_launch': alg,
                     'implementation_bytes_per_launch_upper_bound': impl,
                     'implementation_GBs': round(impl / (dev_ms * 1e-3) / 1e9, 1)},
        'cpu_baseline': cpu, 'parity_sample': parity, 'strict_mode': strict})


def strict_sample(args, store, datasets):
    """The reference-exact duplicateVariantSearch (the default mode:
    every region file a message names read as ReadVcfData::getVcfData reads
    it, sb_dedup_count_files) beside the intended-range device path, over the
    same initDuplicateVariantSearch messages of the first datasets: the
    summariseVcf / summariseSlice / region-file steps run once, untimed; the
    timed part is one dedup_batch call of all those messages per mode."""
    from sbeacon.dedup import DuplicateTally, dedup_batch, init_duplicate_variant_search
    from sbeacon.summarise import _single_store_registry, region_file_keys
    from sbeacon.summarise_vcf import summarise_vcf
    reg = _single_store_registry(store)
    msgs, refs = [], {}
    for ds, parts in datasets[:args.strict_datasets]:
        keys = []
        for loc, _ in parts:
            slices, _, _ = summarise_vcf(store, loc)
            keys += region_file_keys(store, loc, slices, refs)
        msgs += init_duplicate_variant_search(ds, [loc for loc, _ in parts], keys, tally=DuplicateTally())
        log(f'strict: dataset {ds} planned ({len(msgs)} messages, {len(refs)} region files)')
    out = {'datasets': min(args.strict_datasets, len(datasets)), 'messages': len(msgs),
           'region_files': len(refs)}
    for mode, strict in (('strict', True), ('intended', False)):
        t = time.perf_counter()
        dedup_batch(msgs, registry=reg, file_refs=refs, strict=strict)
        first = time.perf_counter() - t  # strict: writes (gzip level 9) and caches the slices' region files
        log(f'strict: {mode} first call {first * 1e3:.2f} ms')
        reps = 3
        t = time.perf_counter()
        for _ in range(reps):
            res = dedup_batch(msgs, registry=reg, file_refs=refs, strict=strict)
        dt = (time.perf_counter() - t) / reps
        log(f'strict: {mode} {dt * 1e3:.2f} ms per call')
        out[mode] = {'ms_per_call': round(dt * 1e3, 2), 'first_call_ms': round(first * 1e3, 2),
                     'unique_sum': int(sum(r for r in res if isinstance(r, int))),
                     'raised': int(sum(isinstance(r, Exception) for r in res))}
    out['note'] = ('one dedup_batch call of every message of these datasets per mode; strict = the reference\'s '
                   'reader over the region files (host walk + device keys), intended = the device window path; '
                   'first_call_ms includes writing the region files (gzip level 9, once per slice: summariseSlice\'s '
                   'output in the reference, cached per store here), ms_per_call reads them')
    return out


if __name__ == '__main__':
    main()
