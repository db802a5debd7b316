#!/usr/bin/env python3
"""Config-3 delivered-path A/B (host preparation and, with --routes, the
route-body fold; not the bench): re-opens a
store saved by tools/req_tune.py --save (library variants via SBEACON_LIB on
one box), then times sb_requests_prepare_beacon of 1 M requests alone
(median of --rounds) and the bench's serial and streaming delivered forms
(bench_genome.delivered_passes / delivered_streaming).  One JSON line."""
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
    ap.add_argument('--open', required=True)
    ap.add_argument('--records', type=int, default=85_000_000)
    ap.add_argument('--rounds', type=int, default=15)
    ap.add_argument('--routes', action='store_true', help='also time requests -> route bodies (route_bodies_passes)')
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    import bench_genome
    from sbeacon.engine import Store
    from sbeacon.genome import GenomeShape, config3_requests, prepare_beacon_shard, shard_record_base
    shape = GenomeShape(n_total=args.records, seed=3)
    store = Store.open(args.open, device=0)
    reqs = config3_requests(shape, n=1_000_000, seed=1003)
    base = shard_record_base(shape, 1, 0)
    t = []
    for k in range(args.rounds + 1):
        a = time.perf_counter()
        b = prepare_beacon_shard(store, shape, reqs, 1, 0)[2]
        dt = time.perf_counter() - a
        b.free()
        if k:
            t.append(dt)
    t.sort()
    serial = bench_genome.delivered_passes(None, store, shape, reqs, 1, 0, base, dev)
    stream = [bench_genome.delivered_streaming(None, store, shape, reqs, 1, 0, base, dev) for _ in range(3)]
    stream.sort(key=lambda x: x['ms_per_batch'])
    spin = [bench_genome.delivered_streaming(None, store, shape, reqs, 1, 0, base, dev, blocking=False) for _ in range(3)]
    spin.sort(key=lambda x: x['ms_per_batch'])
    routes = None
    if args.routes:
        r, _ = bench_genome.route_bodies_passes(None, store, shape, reqs, 1, 0, base, dev)
        routes = {'ms_per_pass': r['ms_per_pass'], 'best_ms': r['best_ms'], 'split_ms': r['split_ms'],
                  'body_bytes': r['body_bytes']}
    print(json.dumps({'routes': routes, 'lib': os.environ.get('SBEACON_LIB', 'in-tree'),
                      'prepare_ms_median': round(t[len(t) // 2] * 1e3, 3), 'prepare_ms_min': round(t[0] * 1e3, 3),
                      'serial_ms': serial['ms_per_pass'], 'serial_split': serial['split_ms'],
                      'streaming_ms': [x['ms_per_batch'] for x in stream],
                      'streaming_spin_ms': [x['ms_per_batch'] for x in spin],
                      'digest': serial['digest'], 'streaming_digest': stream[0]['digest']}), flush=True)


if __name__ == '__main__':
    main()
