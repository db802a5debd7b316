"""Config 3 persisted: ingest the 85 M-record whole-genome shape (as bench.py
does), save it (sb_store_save), re-open it (sb_store_open) and answer the
same 1 M requests from both stores; prints one JSON line (ingest, save, open
seconds, bytes on disk, answers equal).  The re-open reads device.bin back
through the page cache the save just filled (a warm restart; a cold disk
adds its read time)."""
import argparse
import hashlib
import json
import os
import shutil
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'terraform-aws-serverless-beacon_amd'))


def digest(batch, dev):
    import torch
    b = batch
    n = b.n
    rows = torch.zeros((max(n, 1), 5), dtype=torch.int64, device=dev)
    hits = torch.zeros(max(int(b.stats()['hits']), 1), dtype=torch.int64, device=dev)
    ro = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    b.set_stream(torch.cuda.current_stream().cuda_stream)
    b.run(rows.data_ptr(), hits.data_ptr(), ro.data_ptr(), 0)
    b.sync()
    h = hashlib.sha256()
    for t in (rows[:n], ro, hits[:int(ro[-1].item())]):
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--records', type=int, default=85_000_000)
    ap.add_argument('--requests', type=int, default=1_000_000)
    ap.add_argument('--dir', default='/tmp/sbeacon_config3_store')
    ap.add_argument('--threads', type=int, default=16)
    args = ap.parse_args()
    import torch
    from sbeacon.engine import Store
    from sbeacon.genome import GenomeShape, config3_requests, prepare_shard_requests, shard_requests
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    shape = GenomeShape(n_total=args.records, seed=3)
    st = shape.build_shard_store(1, 0, device=0, threads=args.threads)
    t_ingest = time.perf_counter() - t0
    print(f'ingest {t_ingest:.1f} s', file=sys.stderr, flush=True)
    shutil.rmtree(args.dir, ignore_errors=True)
    t0 = time.perf_counter()
    st.save(args.dir)
    t_save = time.perf_counter() - t0
    size = sum(os.path.getsize(os.path.join(args.dir, f)) for f in os.listdir(args.dir))
    print(f'save {t_save:.1f} s, {size / 2**30:.1f} GiB', file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    again = Store.open(args.dir, device=0)
    t_open = time.perf_counter() - t0
    print(f'open {t_open:.2f} s', file=sys.stderr, flush=True)
    reqs = config3_requests(shape, n=args.requests, seed=1003)
    sr = shard_requests(shape, reqs, 1, 0)
    d0 = digest(prepare_shard_requests(st, sr), dev)
    d1 = digest(prepare_shard_requests(again, sr), dev)
    info = again.info()
    print(json.dumps({'workload': 'config3-wgs-1000g-shape', 'records': info['n_records'],
                      'device_bytes': info['device_bytes'], 'ingest_s': round(t_ingest, 2),
                      'save_s': round(t_save, 2), 'open_s': round(t_open, 3), 'bytes_on_disk': size,
                      'open_GBs': round(size / t_open / 1e9, 2), 'answers_equal': d0 == d1, 'digest': d0[:16],
                      'note': 'open = host.bin + device.bin read back through the page cache the save filled '
                              '(warm restart), device buffers re-allocated and streamed up, pointers remapped'}),
          flush=True)
    again.close()
    st.close()
    shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == '__main__':
    main()
