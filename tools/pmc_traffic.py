#!/usr/bin/env python3
"""Fold two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of a short
bench.py run into profiles/traffic.json: HBM-side bytes per step of the
timed query phase (the fused query launch: range_n + exact groups).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are
reported in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read, so it is doubled.  Both counters include
Infinity-Cache hits (they are L2 memory-side request counters).

usage: pmc_traffic.py FETCH_DIR WRITE_DIR [--out profiles/traffic.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sys

PHASE = re.compile(r'(request_\w+_kernel|fused_kernel|range_n8?_kernel|vt_kernel|scan_kernel|request_reduce_kernel|chain_\w*kernel|upsweep_kernel|downsweep_kernel|gather_kernel|bucket_dedupe_kernel|unique_kernel|scan_reduce_kernel|scan_top_kernel|scan_down_kernel|summarise_\w+_kernel|row_reduce_kernel|row_gather_kernel|field_tile_\w+_kernel|tile_scan_kernel|hit_\w+_kernel|compact_kernel|dedup\w*|radix\w*|summ\w*)')


def load(d, counter):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        sys.exit(f'no counter_collection.csv under {d}')
    per = {}  # kernel name -> list of values in dispatch order
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row['Counter_Name'] != counter:
                    continue
                name = row['Kernel_Name']
                if not PHASE.search(name):
                    continue
                per.setdefault(name, []).append((int(row['Dispatch_Id']), float(row['Counter_Value']),
                                                 int(row.get('Grid_Size') or 0)))
    # a bench run launches a kernel at several sizes (the timed batches, the
    # delivered path's chunks, probes): only the full-batch launches -- grids
    # within 20 % of the largest (the rotating batches differ a little) -- are
    # priced
    out = {}
    for k, x in per.items():
        g = max(v[2] for v in x)
        out[k] = [v for _, v, gs in sorted(x) if gs >= 0.8 * g]
    return out


def short(name):
    m = re.search(r'(\w+_kernel<[^>]*>|\w+_kernel)', name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('--out', default='profiles/traffic.json')
    ap.add_argument('--records', type=int, default=1103547)
    ap.add_argument('--requests', type=int, default=10000)
    ap.add_argument('--kernel', default=None, help='the dominant kernel the bench line prices (top-level entry)')
    ap.add_argument('--batches', type=int, default=None, help='rotating batches of the measured run (config 3)')
    a = ap.parse_args()
    fetch = load(a.fetch_dir, 'FETCH_SIZE')
    write = load(a.write_dir, 'WRITE_SIZE')
    kernels = {}
    step_bytes = 0.0
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fb = 2.0 * 1024.0 * sum(f) / max(1, len(f))   # gfx950 streaming-read correction, KiB -> B
        wb = 1024.0 * sum(w) / max(1, len(w))
        # profiles/r02_fetch_calib: x2 for coalesced streams (any lane width), x1
        # for scattered 64 B lines; x2 is the upper bound, x1 the lower
        kernels[short(name)] = {'dispatches': [len(f), len(w)], 'fetch_bytes_per_launch': fb,
                                'fetch_bytes_per_launch_x1': fb / 2.0,
                                'write_bytes_per_launch': wb, 'hbm_bytes_per_launch': fb + wb,
                                'hbm_bytes_per_launch_x1': fb / 2.0 + wb}
        step_bytes += fb + wb
    out = {
        'records': a.records,
        'requests': a.requests,
        'batches': a.batches,
        'phase': 'query step = one launch of each kernel below (fused_kernel: range_n8 + exact groups)',
        'kernels': kernels,
        'scan_kernel_hbm_bytes_per_launch': step_bytes,
        'method': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, kernel trace only), '
                  'FETCH_SIZE x2 (gfx950 streaming correction, calibrated at 4/8/16 B per lane in '
                  'profiles/r02_fetch_calib; scattered 64 B lines need x1: *_x1 is that lower bound), KiB->B; '
                  'includes Infinity-Cache hits',
    }
    if a.kernel:
        hit = [k for k in kernels if k.startswith(a.kernel)]
        if hit:
            out['kernel'] = a.kernel
            out['hbm_bytes_per_launch'] = kernels[hit[0]]['hbm_bytes_per_launch']
            out['fetch_bytes_per_launch'] = kernels[hit[0]]['fetch_bytes_per_launch']
            out['write_bytes_per_launch'] = kernels[hit[0]]['write_bytes_per_launch']
            out['hbm_bytes_per_launch_x1'] = kernels[hit[0]]['hbm_bytes_per_launch_x1']
    with open(a.out, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
