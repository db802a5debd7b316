"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (sums over
dispatches, divided by the dispatch count)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f'{d}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][-48:]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    print(d)
    for k, v in agg.items():
        n = len(disp[k])
        wc = v.get('SQ_WAVE_CYCLES', 0) or 1
        print(f'  {k} x{n}: ' + ', '.join(f'{c}={x / n:.3g}' for c, x in sorted(v.items())) +
              f' | wait {v.get("SQ_WAIT_ANY", 0) / wc:.2f} active {v.get("SQ_ACTIVE_INST_ANY", 0) / wc:.2f}'
              f' valu/wave {v.get("SQ_INSTS_VALU", 0) / max(v.get("SQ_WAVES", 1), 1):.0f}'
              f' salu/wave {v.get("SQ_INSTS_SALU", 0) / max(v.get("SQ_WAVES", 1), 1):.0f}')
