#!/usr/bin/env python3
"""Config-3 request-pass A/B harness (kernel tuning, not the bench): the
whole-genome store (sites only unless --genotypes; --save DIR writes it with
sb_store_save, --open DIR re-opens it in ~0.5 s so library variants
(SBEACON_LIB) can be compared on one box without re-ingesting), 4 rotating
1 M-request batches re-planned every pass as bench.py's step does.  Prints
one JSON line: per-kernel medians from HIP events (eval alone; the pass)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--records', type=int, default=85_000_000)
    ap.add_argument('--requests', type=int, default=1_000_000)
    ap.add_argument('--batches', type=int, default=4)
    ap.add_argument('--rounds', type=int, default=15)
    ap.add_argument('--save', default=None)
    ap.add_argument('--open', default=None)
    ap.add_argument('--genotypes', action='store_true')
    ap.add_argument('--streams', type=int, default=1,
                    help='also time the rotation with batch k on stream k %% N (N > 1: independent batches overlap)')
    ap.add_argument('--digest', action='store_true', help='blake2b of every batch\'s rows + hits (A/B parity)')
    ap.add_argument('--wide', action='store_true', help='wide outputs (int64 rows, offsets, hits) instead of the '
                                                         'compact ones the bench step writes')
    args = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    from sbeacon.engine import Store
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_requests, shard_requests
    shape = GenomeShape(n_total=args.records, seed=3)
    t0 = time.perf_counter()
    if args.open:
        store = Store.open(args.open, device=0)
    else:
        store = shape.build_shard_store(1, 0, device=0, genotypes=args.genotypes)
        if args.save:
            store.save(args.save)
    t_store = time.perf_counter() - t0
    stream = torch.cuda.current_stream().cuda_stream
    B = []
    for k in range(args.batches):
        sr = shard_requests(shape, config3_requests(shape, n=args.requests, seed=1003 + k), 1, 0)
        b = prepare_shard_requests(store, sr)
        b.set_stream(stream)
        b.set_replan(True)
        n = sr.n_rows
        if args.wide:
            B.append((b, torch.zeros((max(n, 1), 5), dtype=torch.int64, device=dev),
                      torch.zeros(int(b.stats()['hits']) + 1, dtype=torch.int64, device=dev),
                      torch.zeros(n + 1, dtype=torch.int64, device=dev)))
        else:  # the bench step's form (sb_requests_set_compact)
            b.set_compact(True)
            B.append((b, torch.zeros((max(n, 1), 4), dtype=torch.int32, device=dev),
                      torch.zeros(int(b.stats()['hits']) + 1, dtype=torch.int32, device=dev),
                      torch.zeros(n + 1, dtype=torch.int32, device=dev)))

    def run(b, p, h, o):
        b.run(p.data_ptr(), h.data_ptr(), o.data_ptr(), 0)

    for _ in range(2):
        for x in B:
            run(*x)
    torch.cuda.synchronize()
    ev, pas = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for x in B:
            x[0].time_eval(True)
        for x in B:
            run(*x)
        for x in B:
            x[0].sync()
            ev.append(x[0].timing()['scan_ms'])
            x[0].time_eval(False)
        e0.record()
        for x in B:
            run(*x)
        e1.record()
        torch.cuda.synchronize()
        pas.append(e0.elapsed_time(e1) / len(B))
    ev.sort()
    pas.sort()
    pas_ms = []
    if args.streams > 1:  # batch k on stream k % N (no cross-stream waits: events on each stream)
        ss = [torch.cuda.Stream() for _ in range(args.streams)]
        for k, x in enumerate(B):
            x[0].sync()  # (the runs above: a batch changes stream only between a run's sync and the next run)
            x[0].set_stream(ss[k % len(ss)].cuda_stream)
        for _ in range(args.rounds):
            torch.cuda.synchronize()
            a = [torch.cuda.Event(enable_timing=True) for _ in ss]
            z = [torch.cuda.Event(enable_timing=True) for _ in ss]
            for e, s_ in zip(a, ss):
                e.record(s_)
            for _ in range(4):
                for x in B:
                    run(*x)
            for e, s_ in zip(z, ss):
                e.record(s_)
            torch.cuda.synchronize()
            pas_ms.append(max(a[0].elapsed_time(e) for e in z) / (4 * len(B)))
        for x in B:
            x[0].sync()
        pas_ms.sort()
    out = {'lib': os.environ.get('SBEACON_LIB', 'in-tree'), 'records': args.records, 'store_s': round(t_store, 2),
           'eval_ms_median': round(ev[len(ev) // 2], 4), 'eval_ms_min': round(ev[0], 4),
           'pass_ms_median': round(pas[len(pas) // 2], 4), 'pass_ms_min': round(pas[0], 4)}
    if pas_ms:
        out.update({'streams': args.streams, 'pass_ms_streams_median': round(pas_ms[len(pas_ms) // 2], 4),
                    'pass_ms_streams_min': round(pas_ms[0], 4)})
    if args.digest:  # over the wide form (compact outputs widened): one digest for both forms
        import hashlib
        from sbeacon.requests import widen_compact
        h = hashlib.blake2b(digest_size=16)
        for b, p, hh, o in B:
            if args.wide:
                ro = o.cpu().numpy()
                rows, hits = p[:len(ro) - 1].cpu().numpy(), hh[:int(ro[-1])].cpu().numpy()
            else:
                ro32 = o.cpu().numpy().view(np.uint32)
                rows, hits, ro = widen_compact(p[:len(ro32) - 1].cpu().numpy(), hh[:int(ro32[-1])].cpu().numpy(), ro32)
                hits = hits.view(np.int64)
            h.update(rows.tobytes())
            h.update(hits.tobytes())
            h.update(ro.tobytes())
        out['digest'] = h.hexdigest()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
