"""Summarise rocprofv3 CSV outputs of a profiling tag (kernel stats + PMC)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else 'lt_'
for f in sorted(glob.glob(os.path.join(root, '*', 'run_kernel_stats.csv'))):
    print('==', f)
    print(open(f).read())
for f in sorted(glob.glob(os.path.join(root, '*', 'run_counter_collection.csv'))):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    disp = set()
    for r in rows:
        if kern in r.get('Kernel_Name', ''):
            agg[(int(r['Dispatch_Id']), r['Counter_Name'])] += float(r['Counter_Value'])
            disp.add(int(r['Dispatch_Id']))
    if not disp:
        continue
    last = max(disp)
    print('==', os.path.basename(os.path.dirname(f)), 'dispatch', last,
          {c: '%.4g' % v for (d, c), v in sorted(agg.items()) if d == last})
