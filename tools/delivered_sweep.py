"""Config-3 delivered path: pipelined chunk / worker counts side by side,
and the cold-launch probe (bench_genome.cold_launch_probe).  Builds the 85 M
record store once (as bench.py does)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))


def main():
    import torch
    import bench_genome as bg
    from sbeacon.genome import GenomeShape, config3_requests, shard_record_base
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    shape = GenomeShape(n_total=85_000_000, seed=3)
    store = shape.build_shard_store(1, 0, device=0, threads=16)
    reqs = config3_requests(shape, n=1_000_000, seed=1003)
    base = shard_record_base(shape, 1, 0)

    class A:
        pass
    print(json.dumps({'cold': bg.cold_launch_probe(store, shape, reqs, 1, 0, base, dev)}), flush=True)
    for chunks, workers in ((8, 2), (8, 3), (16, 3), (16, 4), (4, 2)):
        d = bg.delivered_pipelined(A(), store, shape, reqs, 1, 0, base, dev, chunks=chunks, workers=workers)
        print(json.dumps({'chunks': chunks, 'workers': workers, 'requests_per_s': d['requests_per_s'],
                          'ms': d['ms_per_pass'], 'best_ms': d['best_ms']}), flush=True)


if __name__ == '__main__':
    main()
