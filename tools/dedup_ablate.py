"""Config-4 dedup (50 datasets) timed with the window kernel's ablation
switches (SBEACON_DEDUP_WIN_DBG: 4 = key loads only, 1 = no exact inserts,
2 = no hashed inserts, 3 = neither): which part of window_dedupe_kernel
costs what.  Ingests once (--save DIR keeps the store, --open DIR re-opens
it, so library variants -- SBEACON_LIB -- are compared on one store); prints
one line per mode with a digest of the counts."""
import argparse
import hashlib
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--save', default=None)
    ap.add_argument('--open', default=None)
    ap.add_argument('--modes', default='0,4,3,1,2,0')
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from sbeacon.engine import Store
    from sbeacon.workload import config4_cohort, write_bgzf
    # the sources stay beside a saved store (re-opening checks them)
    tmp = args.save + '.src' if args.save else tempfile.mkdtemp(prefix='sbeacon-abl-')
    os.makedirs(tmp, exist_ok=True)
    try:
        pool, datasets = config4_cohort(n_datasets=50, n_records=1103547)
        jobs = [([loc for loc, _ in parts], '22', 0, 2**32 - 1) for _, parts in datasets]
        if args.open:
            store = Store.open(args.open, device=0)
        else:
            files = []
            for ds, parts in datasets:
                for loc, gen in parts:
                    p = os.path.join(tmp, loc.replace('/', '_').replace(':', ''))
                    if parts.index((loc, gen)) == 0:
                        write_bgzf(p, gen.chunks(sites_only=True, threads=16), level=1, threads=16)
                        first = p
                    else:
                        shutil.copyfile(first, p)
                    files.append((loc, p))
            store = Store.build(files, device=0, keep_genotypes=False, n_threads=16)
            if args.save:
                store.save(args.save)
        base = None
        for mode in args.modes.split(','):
            os.environ['SBEACON_DEDUP_WIN_DBG'] = mode
            for _ in range(2):
                store.dedup_counts(jobs)
            dev = []
            for _ in range(10):
                res, st = store.dedup_counts(jobs, with_stats=True)
                dev.append(st['device_ms'])
            if mode == '0':
                base = res
            dig = hashlib.blake2b(repr(list(res)).encode(), digest_size=8).hexdigest()
            print(f'mode {mode}: device {sum(dev) / len(dev):.3f} ms (min {min(dev):.3f}), windows {st["windows"]}, '
                  f'path {st["path"]}, same answer {res == base}, digest {dig}', flush=True)
    finally:
        if not args.save:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
