"""Per-kernel mean of every PMC counter found under <root>/*/run_counter_collection.csv.

Kernels are keyed by name.  rocprofv3 reports the decode kernels by their bare
name, so the op-counting launch of tools/prof_decode.py (COUNT = true, the
first dispatch of the kernel) is dropped when the kernel has later dispatches.
"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else 'lt_'
per_dispatch = len(sys.argv) > 3 and sys.argv[3] == 'dispatch'   # one row per dispatch
NAME = re.compile(r'(\w+)(<[^()]*>)?\s*\(')
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, '**', 'run_counter_collection.csv'), recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        kn = r['Kernel_Name']
        if kern not in kn:
            continue
        m = [x for x in NAME.finditer(kn) if kern in x.group(1)]
        name = (m[0].group(1) + (m[0].group(2) or '')) if m else kn[:64]
        per[(name, int(r['Dispatch_Id']), r['Counter_Name'])] += float(r['Counter_Value'])
    first = {}
    for (k, d, c) in per:
        first[k] = min(first.get(k, d), d)
    multi = {k for (k, d, c) in per if d != first[k]}
    for (k, d, c), v in per.items():
        if not per_dispatch and k in multi and d == first[k]:
            continue
        vals[(k, d, c) if per_dispatch else (k, c)].append(v)
for key, v in sorted(vals.items()):
    print('%-44s ' % key[0] + ' '.join('%-28s' % x for x in key[1:]) + ' n=%d mean=%.6g' % (len(v), sum(v) / len(v)))
