#!/usr/bin/env python3
"""Config-2 wire path split: event packing, the library call
(sb_perform_query_events: parse / query / format / concat with
SBEACON_WIRE_TRACE=1), and the Python-side copy.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))
sys.path.insert(0, REPO)


def main():
    import torch
    torch.cuda.set_device(0)
    from sbeacon import engine
    from sbeacon.wire import pack_events, perform_query_events_packed
    from sbeacon.workload import SyntheticVcf, config2_requests, requests_to_payloads
    gen = SyntheticVcf(seed=22, n_records=1103547, n_samples=2504)
    loc = 'synthetic/chr22-1000g-shape.vcf.gz'
    store = gen.build_store(loc, device=0, keep_genotypes=True, threads=16)
    engine.registry.register(store)
    reqs = config2_requests(gen, seed=1022)
    payloads, _ = requests_to_payloads(reqs, vcf_location=loc, chrom='22')
    t0 = time.perf_counter()
    buf, off = pack_events([json.dumps(p) for p in payloads])
    t_pack = time.perf_counter() - t0
    out = {}
    r = None
    for rep in range(4):
        print(f'--- rep {rep}', file=sys.stderr, flush=True)
        t1 = time.perf_counter()
        r = None  # the previous result freed outside the timed call
        t_free = time.perf_counter() - t1
        t0 = time.perf_counter()
        r = perform_query_events_packed(buf, off)
        out = {'call_ms': round((time.perf_counter() - t0) * 1e3, 2), 'free_ms': round(t_free * 1e3, 2),
               'pack_ms': round(t_pack * 1e3, 2),
               'events': len(payloads), 'requests': len(reqs), 'response_bytes': len(r.buf),
               'fallbacks': int(r.fallback.sum())}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
