#!/usr/bin/env python3
"""Per-kernel duration table (median / min / max per kernel and grid) from a
rocprofv3 kernel-trace CSV: python tools/kernel_table.py trace.csv [top]."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    by = collections.defaultdict(list)
    for r in rows:
        by[(r['Kernel_Name'][:60], r['Grid_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]:
        v.sort()
        print(f'{k[0]:60s} grid={k[1]:>8s} n={len(v):4d} med={v[len(v) // 2]:8.1f} min={v[0]:8.1f} max={v[-1]:8.1f} us')


if __name__ == '__main__':
    main()
