"""Per-kernel SQ counter means (per launch and per wave) from rocprofv3
--pmc CSV directories: python3 tools/sq_table.py DIR [DIR ...]."""
import collections
import csv
import glob
import os
import re
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        m = re.search(r'(\w+_kernel)(<[^>]*>)?', r['Kernel_Name'])
        agg[m.group(0) if m else r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
    print(d)
    for k, v in agg.items():
        if 'request' not in k:
            continue
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = max(m.get('SQ_WAVES', 1), 1)
        print(f'  {k}: waves {w:.0f}; per wave ' + ', '.join(
            f'{c[8:] if c.startswith("SQ_INSTS") else c[3:]} {m[c] / w:.0f}' for c in sorted(m) if c != 'SQ_WAVES'))
