"""Config-4 dedup (50 datasets) timed with the window kernel's ablation
switches (SBEACON_DEDUP_WIN_DBG: 4 = key loads only, 1 = no exact inserts,
2 = no hashed inserts, 3 = neither): which part of window_dedupe_kernel
costs what.  Ingests once; prints one line per mode."""
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))


def main():
    import torch
    torch.cuda.set_device(0)
    from sbeacon.engine import Store
    from sbeacon.workload import config4_cohort, write_bgzf
    tmp = tempfile.mkdtemp(prefix='sbeacon-abl-')
    try:
        pool, datasets = config4_cohort(n_datasets=50, n_records=1103547)
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
        jobs = [([loc for loc, _ in parts], '22', 0, 2**32 - 1) for _, parts in datasets]
        base = None
        for mode in ('0', '4', '3', '1', '2', '0'):
            os.environ['SBEACON_DEDUP_WIN_DBG'] = mode
            for _ in range(2):
                store.dedup_counts(jobs)
            dev = []
            for _ in range(10):
                res, st = store.dedup_counts(jobs, with_stats=True)
                dev.append(st['device_ms'])
            if mode == '0':
                base = res
            print(f'mode {mode}: device {sum(dev) / len(dev):.3f} ms (min {min(dev):.3f}), windows {st["windows"]}, '
                  f'path {st["path"]}, same answer {res == base}', flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
