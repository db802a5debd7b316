#!/usr/bin/env python3
"""Per-kernel duration table (median / min / max per kernel and grid) from a
rocprofv3 kernel-trace CSV: python tools/kernel_table.py trace.csv [top].
Each (kernel, grid) row is also split into launches that ran alone and
launches whose interval overlapped another kernel's (two streams in flight,
the bench's timed steps): a launch sharing the device takes longer than one
timed alone."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), i) for i, r in enumerate(rows))
    over = [False] * len(rows)
    end_max, end_arg = -1, -1  # sweep: a launch overlaps one that started earlier and ends after it starts
    for s, e, i in iv:
        if end_max > s:
            over[i] = True
            over[end_arg] = True
        if e > end_max:
            end_max, end_arg = e, i
    by = collections.defaultdict(list)
    for i, r in enumerate(rows):
        by[(r['Kernel_Name'][:60], r['Grid_Size_X'])].append(
            ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, over[i]))
    med = lambda v: v[len(v) // 2] if v else float('nan')
    for k, v in sorted(by.items(), key=lambda kv: -sum(d for d, _ in kv[1]))[:top]:
        a = sorted(d for d, _ in v)
        al = sorted(d for d, o in v if not o)
        ov = sorted(d for d, o in v if o)
        print(f'{k[0]:60s} grid={k[1]:>8s} n={len(a):4d} med={med(a):8.1f} min={a[0]:8.1f} max={a[-1]:8.1f} us | '
              f'alone n={len(al)} med={med(al):.1f} | overlapped n={len(ov)} med={med(ov):.1f}')


if __name__ == '__main__':
    main()
