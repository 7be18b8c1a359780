"""HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes of bench.py (MI355X_MICROARCH.md, HBM section: FETCH_SIZE counts half
the bytes of 16 B/lane reads on gfx950 -> doubled; WRITE_SIZE as is; both in
KiB).  Appends one entry per configuration to the JSON list in OUT.

    python tools/traffic_summary.py OUT FETCH_DIR WRITE_DIR KERNEL K SENTENCES FEATURES SEED [LAYOUT]

LAYOUT (default: bench.LAYOUT) tags the entry with the batch layout it was
measured on; bench.py only reads entries of its own layout.  The figures are
fabric bytes: FETCH_SIZE counts Infinity-Cache hits as well as HBM reads.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(root, counter, kern):
    vals = collections.defaultdict(float)
    for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter and r['Kernel_Name'].startswith(kern):
                vals[int(r['Dispatch_Id'])] += float(r['Counter_Value'])
    return [vals[d] for d in sorted(vals)]


def main():
    out, fdir, wdir, kern, k, sents, feats, seed = sys.argv[1:9]
    if len(sys.argv) > 9:
        layout = sys.argv[9]
    else:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
        from bench import LAYOUT as layout
    f = per_dispatch(fdir, 'FETCH_SIZE', kern)
    w = per_dispatch(wdir, 'WRITE_SIZE', kern)
    if not f or not w:
        raise SystemExit('no %s dispatches with FETCH_SIZE/WRITE_SIZE' % kern)
    # the first dispatch is the counting launch (lt_count_ops); use the timed-shape ones
    fk = sum(f[1:]) / len(f[1:]) if len(f) > 1 else f[0]
    wk = sum(w[1:]) / len(w[1:]) if len(w) > 1 else w[0]
    entry = {'kernel': kern, 'k': int(k), 'sentences': int(sents), 'features': int(feats),
             'seed': int(seed), 'layout': layout, 'fetch_size_kib_raw': fk, 'write_size_kib': wk,
             'dispatches': [len(f), len(w)],
             'traffic_bytes_per_launch': int(round((2.0 * fk + wk) * 1024.0))}
    data = json.load(open(out)) if os.path.exists(out) else []
    key = lambda e: (e['kernel'], e['k'], e['sentences'], e['features'], e['seed'], e.get('layout'))  # noqa: E731
    data = [e for e in data if key(e) != key(entry)]
    data.append(entry)
    json.dump(data, open(out, 'w'), indent=1)
    print(json.dumps(entry))


if __name__ == '__main__':
    main()
