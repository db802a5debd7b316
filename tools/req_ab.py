#!/usr/bin/env python3
"""Config-3 A/B on one store: the request batch (request_rows_kernel) on the
requests in their drawn order and sorted by (contig, start), and the round-2
slice batch (chain kernel + sb_batch_deliver).  Prints one JSON line of
per-step device times (HIP events, K back-to-back passes)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    from sbeacon.genome import (GenomeShape, Requests, config3_requests, prepare_shard_batch, prepare_shard_requests,
                                shard_requests, shard_slices)
    K = int(os.environ.get('AB_STEPS', '20'))
    shape = GenomeShape(n_total=int(os.environ.get('AB_RECORDS', '85000000')), seed=3)
    store = shape.build_shard_store(1, 0, device=0, threads=16)
    reqs = config3_requests(shape, n=1_000_000, seed=1003)
    o = np.lexsort((reqs.start, reqs.ci))
    sreqs = Requests(reqs.ci[o], reqs.start[o], reqs.width[o], reqs.vt[o], reqs.vmin[o], reqs.vmax[o])
    out = {}
    for name, rq in (('request_order', reqs), ('sorted', sreqs)):
        sr = shard_requests(shape, rq, 1, 0)
        b = prepare_shard_requests(store, sr)
        b.set_stream(torch.cuda.current_stream().cuda_stream)
        part = torch.zeros((sr.n_rows, 5), dtype=torch.int64, device=dev)
        hits = torch.zeros(int(b.stats()['hits']) + 1, dtype=torch.int64, device=dev)
        ro = torch.zeros(sr.n_rows + 1, dtype=torch.int64, device=dev)
        for _ in range(3):
            b.run(part.data_ptr(), hits.data_ptr(), ro.data_ptr(), 0)
        b.sync()
        b.timing()
        for _ in range(K):
            b.run(part.data_ptr(), hits.data_ptr(), ro.data_ptr(), 0)
        b.sync()
        out[name] = {'kernel_ms': round(b.timing()['scan_ms'], 4), 'runs_stats': b.stats()}
        b.free()
        print(name, out[name], file=sys.stderr, flush=True)
    # round-2 path: slice batch, chain kernel + deliver
    sl = shard_slices(shape, reqs, 1, 0)
    b = prepare_shard_batch(store, sl)
    b.set_stream(torch.cuda.current_stream().cuda_stream)
    b.set_slice_results(False)
    part = torch.zeros((sl.n_rows, 5), dtype=torch.int64, device=dev)
    hits = torch.zeros(int(b.stats()['hits']) + 1, dtype=torch.int64, device=dev)
    ro = torch.zeros(sl.n_rows + 1, dtype=torch.int64, device=dev)
    for _ in range(3):
        b.run()
        b.deliver(part.data_ptr(), hits.data_ptr(), ro.data_ptr(), 0)
    b.sync()
    b.timing()
    for _ in range(K):
        b.run()
    b.sync()
    kern = b.timing()['scan_ms']
    for _ in range(K):
        b.run()
        b.deliver(part.data_ptr(), hits.data_ptr(), ro.data_ptr(), 0)
    b.sync()
    out['r02_chain_path'] = {'chain_kernel_ms': round(kern, 4), 'step_ms': round(b.timing()['scan_ms'], 4)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
