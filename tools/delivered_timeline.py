"""Config-3 delivered path diagnostics (compact outputs, as the bench's delivered path): the device planner's phase times
(SBEACON_PREP_TRACE, one serial prepare of 1 M requests) and a per-chunk
timeline of the pipelined path (worker prepare start/end, main-thread
enqueue, offsets back, hits back) for a few chunk / worker settings.  Builds
the 85 M record store once (as bench.py does)."""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))


def chunk_cuts(n, chunks, taper):
    import numpy as np
    if not taper:
        return np.linspace(0, n, chunks + 1).astype(np.int64)
    # small first and last chunks: the pipeline fills and drains sooner
    w = np.ones(chunks)
    w[0] = w[-1] = 0.25
    if chunks > 3:
        w[1] = w[-2] = 0.6
    c = np.concatenate([[0], np.cumsum(w)]) / w.sum() * n
    return np.round(c).astype(np.int64)


def timeline(store, shape, reqs, base, dev, chunks, workers, passes=5, taper=False):
    import numpy as np
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from sbeacon.genome import prepare_beacon_shard
    n = len(reqs)
    cuts = chunk_cuts(n, chunks, taper)
    stream = torch.cuda.current_stream()
    rows_h = torch.empty((n, 4), dtype=torch.int32, pin_memory=True)
    ro_h = torch.empty(n + chunks, dtype=torch.int32, pin_memory=True)
    rows_d = torch.empty((n, 4), dtype=torch.int32, device=dev)
    ro_d = torch.empty(n + chunks, dtype=torch.int32, device=dev)
    hits_d, hits_h = [None] * chunks, [None] * chunks
    out = []
    with ThreadPoolExecutor(workers) as ex:
        for p in range(passes + 1):
            ev = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()

            def prep(k):
                a0 = time.perf_counter()
                a, b = int(cuts[k]), int(cuts[k + 1])
                lo, m, bt = prepare_beacon_shard(store, shape, reqs.rows(a, b), 1, 0)
                cap = int(bt.stats()['hits'])
                ev[k] = {'thr': threading.get_ident() % 1000, 'prep0': a0 - t0, 'prep1': time.perf_counter() - t0}
                return a + lo, m, bt, cap

            futs = [ex.submit(prep, k) for k in range(chunks)]
            live, pend = [], []
            for k in range(chunks):
                a, m, bt, cap = futs[k].result()
                ev[k]['got'] = time.perf_counter() - t0
                if hits_d[k] is None or hits_d[k].numel() < max(cap, 1):
                    hits_d[k] = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
                    hits_h[k] = torch.empty(max(cap, 1), dtype=torch.int32, pin_memory=True)
                bt.set_stream(stream.cuda_stream)
                bt.set_compact(True)
                ro = ro_d[a + k:a + k + m + 1]
                bt.run(rows_d[a:a + m].data_ptr(), hits_d[k].data_ptr(), ro.data_ptr(), base)
                rows_h[a:a + m].copy_(rows_d[a:a + m], non_blocking=True)
                ro_h[a + k:a + k + m + 1].copy_(ro, non_blocking=True)
                e = torch.cuda.Event()
                e.record(stream)
                ev[k]['enq'] = time.perf_counter() - t0
                pend.append((k, e, a + k + m))
                live.append(bt)
                while len(pend) > 1:
                    kk, e2, last = pend.pop(0)
                    e2.synchronize()
                    ev[kk]['off'] = time.perf_counter() - t0
                    nh = int(ro_h[last].numpy().view(np.uint32))
                    hits_h[kk][:nh].copy_(hits_d[kk][:nh], non_blocking=True)
            for kk, e2, last in pend:
                e2.synchronize()
                ev[kk]['off'] = time.perf_counter() - t0
                nh = int(ro_h[last].numpy().view(np.uint32))
                hits_h[kk][:nh].copy_(hits_d[kk][:nh], non_blocking=True)
            stream.synchronize()
            dt = time.perf_counter() - t0
            for bt in live:
                bt.sync()
                bt.free()
            if p:
                out.append({'ms': round(dt * 1e3, 2),
                            'chunks': [{k2: (round(v * 1e3, 2) if isinstance(v, float) else v) for k2, v in ev[k].items()}
                                       for k in range(chunks)]})
    return out


def main():
    import torch
    from sbeacon.genome import GenomeShape, config3_requests, prepare_beacon_shard, shard_record_base
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    shape = GenomeShape(n_total=85_000_000, seed=3)
    store = shape.build_shard_store(1, 0, device=0, threads=16)
    reqs = config3_requests(shape, n=1_000_000, seed=1003)
    base = shard_record_base(shape, 1, 0)
    for _ in range(2):
        b = prepare_beacon_shard(store, shape, reqs, 1, 0)[2]
        b.free()
    os.environ['SBEACON_PREP_TRACE'] = '1'
    for _ in range(2):
        t = time.perf_counter()
        b = prepare_beacon_shard(store, shape, reqs, 1, 0)[2]
        print(json.dumps({'serial_prepare_ms': round((time.perf_counter() - t) * 1e3, 2)}), flush=True)
        b.free()
    del os.environ['SBEACON_PREP_TRACE']
    for chunks, workers, taper in ((8, 2, True), (4, 1, True), (8, 1, True), (4, 2, True), (6, 1, True)):
        tl = timeline(store, shape, reqs, base, dev, chunks, workers, passes=7, taper=taper)
        ms = sorted(x['ms'] for x in tl)
        print(json.dumps({'chunks': chunks, 'workers': workers, 'taper': taper, 'median_ms': ms[len(ms) // 2],
                          'ms': [x['ms'] for x in tl]}), flush=True)
        print(json.dumps(tl[-1]['chunks']), flush=True)


if __name__ == '__main__':
    main()
