#!/usr/bin/env python3
"""Config-3 query step timing over kernel knobs on ONE ingested store (the
ingest dominates a bench run): chain run length (SBEACON_CHAIN_RUN) and the
per-slice path (SBEACON_NO_CHAINS=1).  Prints one JSON line per setting."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)


def main():
    import torch
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_batch, shard_slices
    records = int(os.environ.get('RECORDS', 85_000_000))
    nreq = int(os.environ.get('REQUESTS', 1_000_000))
    steps = int(os.environ.get('STEPS', 10))
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    shape = GenomeShape(n_total=records, seed=3)
    store = shape.build_shard_store(1, 0, device=0, threads=16)
    print(f'ingest {time.perf_counter() - t0:.1f} s', file=sys.stderr, flush=True)
    reqs = config3_requests(shape, n=nreq, seed=1003)
    sl = shard_slices(shape, reqs, 1, 0)
    out = torch.zeros((max(sl.n_rows, 1), 5), dtype=torch.int64, device='cuda')
    base = None
    for setting in os.environ.get('SETTINGS', 'seq8,pack').split(','):
        env = {}
        if setting == 'pack':  # packed kernel (host-built runs of up to pack_run_max() chains)
            pass
        elif setting.startswith('pack'):  # packed kernel, runs of at most N chains
            env['SBEACON_PACK_RUN'] = setting[4:]
        elif setting.startswith('seq'):  # chain-sequential kernel
            env['SBEACON_CHAIN_RUN'] = setting[3:]
            env['SBEACON_CHAIN_KERNEL'] = 'seq'
        elif setting.startswith('dbg'):  # packed kernel timing ablation (results invalid)
            env['SBEACON_PACK_DBG'] = setting[3:]
        elif setting == 'nochain':
            env['SBEACON_NO_CHAINS'] = '1'
        for k in ('SBEACON_CHAIN_RUN', 'SBEACON_NO_CHAINS', 'SBEACON_CHAIN_KERNEL', 'SBEACON_PACK_DBG', 'SBEACON_PACK_RUN'):
            os.environ.pop(k, None)
        os.environ.update(env)
        t1 = time.perf_counter()
        batch = prepare_shard_batch(store, sl)
        if os.environ.get('ROWS_ONLY', '1') == '1':
            batch.set_slice_results(False)
        tp = time.perf_counter() - t1
        batch.run()
        batch.sync()
        for _ in range(steps):
            batch.run()
        batch.sync()
        run_ms = batch.timing()['scan_ms']
        for _ in range(steps):
            batch.run()
            batch.reduce_requests(out.data_ptr())
        batch.sync()
        step_ms = batch.timing()['scan_ms']
        rows = out.cpu().numpy().copy()
        same = None
        if base is None:
            base = rows
        else:
            same = bool((rows == base).all())
        batch.set_slice_results(True)
        batch.run()
        batch.sync()
        st = batch.fetch().stats()
        print(json.dumps({'setting': setting, 'run_ms': round(run_ms, 4), 'run_plus_reduce_ms': round(step_ms, 4),
                          'prepare_s': round(tp, 2), 'chained_slices': st['chained_slices'], 'hits': st['hits'],
                          'rows_equal_first_setting': same}), flush=True)
        batch.free()


if __name__ == '__main__':
    main()
