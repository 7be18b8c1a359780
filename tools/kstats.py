"""Per-kernel duration statistics of a rocprofv3 kernel trace, warm-up
launches dropped: the first SKIP dispatches of every distinct kernel name
(template instance) are left out, so the mean covers the steady-state
launches the bench's timed region measures (round-3 verdict: the stats must
not mix cold launches into the figure they back).

    python tools/kstats.py TRACE_DIR SKIP OUT_CSV

TRACE_DIR: a rocprofv3 -d directory (searched for *kernel_trace.csv).  Prints
and writes one row per kernel name: calls kept, mean / median / min / max ns.
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    root, skip, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            rows[r['Kernel_Name']].append((int(r['Dispatch_Id']), int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
    if not rows:
        raise SystemExit('no kernel trace under %s' % root)
    table = []
    for name, v in rows.items():
        v.sort()
        d = [x for _, x in v[skip:]] or [x for _, x in v]
        table.append({'kernel': name, 'calls_total': len(v), 'calls_kept': len(d), 'skipped': len(v) - len(d),
                      'mean_ns': statistics.fmean(d), 'median_ns': statistics.median(d),
                      'min_ns': min(d), 'max_ns': max(d)})
    table.sort(key=lambda t: -t['mean_ns'] * t['calls_kept'])
    with open(out, 'w', newline='') as fh:
        w = csv.DictWriter(fh, fieldnames=list(table[0]))
        w.writeheader()
        w.writerows(table)
    for t in table:
        print('%-60s kept %4d/%-4d mean %12.0f ns  median %12.0f  min %12.0f  max %12.0f'
              % (t['kernel'][:60], t['calls_kept'], t['calls_total'], t['mean_ns'], t['median_ns'],
                 t['min_ns'], t['max_ns']))


if __name__ == '__main__':
    main()
