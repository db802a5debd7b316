#!/usr/bin/env python3
"""Where a request batch's host preparation goes (the delivered path's
host side): prepare_beacon_shard over 1 M config-3 requests (and over 1/8 of
them, a pipelined chunk), wall time per call with the library's phase ticks
(SBEACON_PREP_TRACE=1 prints them to stderr)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)


def main():
    import torch
    torch.cuda.set_device(0)
    from sbeacon.genome import GenomeShape, config3_requests, prepare_beacon_shard, shard_rows
    shape = GenomeShape(n_total=int(os.environ.get('PT_RECORDS', '20000000')), seed=3)
    store = shape.build_shard_store(1, 0, device=0)
    reqs = config3_requests(shape, n=1_000_000, seed=1003)
    for label, r in (('1M', reqs), ('125k', reqs.rows(0, 125_000))):
        for k in range(4):
            t = time.perf_counter()
            rr = shard_rows(shape, r, 1, 0)
            t1 = time.perf_counter()
            _, n, b = prepare_beacon_shard(store, shape, r, 1, 0, rows=rr)
            t2 = time.perf_counter()
            b.free()
            print(f'{label} call {k}: rows {1e3 * (t1 - t):.2f} ms, prepare {1e3 * (t2 - t1):.2f} ms', file=sys.stderr,
                  flush=True)


if __name__ == '__main__':
    main()
