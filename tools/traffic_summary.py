"""HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes of bench.py (MI355X_MICROARCH.md, HBM section: FETCH_SIZE counts half
the bytes of 16 B/lane reads on gfx950 -> doubled; WRITE_SIZE as is; both in
KiB).  Appends one entry per configuration to the JSON list in OUT.

    python tools/traffic_summary.py OUT FETCH_DIR WRITE_DIR KERNEL K SENTENCES FEATURES SEED
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
    f = per_dispatch(fdir, 'FETCH_SIZE', kern)
    w = per_dispatch(wdir, 'WRITE_SIZE', kern)
    if not f or not w:
        raise SystemExit('no %s dispatches with FETCH_SIZE/WRITE_SIZE' % kern)
    # the first dispatch is the counting launch (lt_count_ops); use the timed-shape ones
    fk = sum(f[1:]) / len(f[1:]) if len(f) > 1 else f[0]
    wk = sum(w[1:]) / len(w[1:]) if len(w) > 1 else w[0]
    entry = {'kernel': kern, 'k': int(k), 'sentences': int(sents), 'features': int(feats),
             'seed': int(seed), 'fetch_size_kib_raw': fk, 'write_size_kib': wk,
             'dispatches': [len(f), len(w)],
             'traffic_bytes_per_launch': int(round((2.0 * fk + wk) * 1024.0))}
    data = json.load(open(out)) if os.path.exists(out) else []
    data = [e for e in data if (e['kernel'], e['k'], e['sentences'], e['features'], e['seed']) !=
            (entry['kernel'], entry['k'], entry['sentences'], entry['features'], entry['seed'])]
    data.append(entry)
    json.dump(data, open(out, 'w'), indent=1)
    print(json.dumps(entry))


if __name__ == '__main__':
    main()
