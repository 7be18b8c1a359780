"""Per-kernel mean of every PMC counter found under <root>/*/run_counter_collection.csv."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else 'lt_'
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, '**', 'run_counter_collection.csv'), recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            per[(r['Kernel_Name'].split('(')[0][:48], int(r['Dispatch_Id']), r['Counter_Name'])] += float(r['Counter_Value'])
    for (k, d, c), v in per.items():
        vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print('%-48s %-28s n=%d mean=%.6g' % (k, c, len(v), sum(v) / len(v)))
