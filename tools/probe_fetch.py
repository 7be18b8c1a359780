"""Where does the PCIe-inclusive step time go?  Times, on the 64K config-3
batch: decode alone, result fetch alone, and decode + fetch, each synced.

    python tools/probe_fetch.py [--sentences 65536] [--k 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lattice_based_tagger_amd import _capi  # noqa: E402
import bench  # noqa: E402


def timeit(fn, reps):
    best, tot = 1e30, 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        best = min(best, dt)
        tot += dt
    return {'best_ms': best * 1e3, 'avg_ms': tot / reps * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=65536)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    _capi.load()
    raw, lay, sm, packed, keys, coefs = bench.make_workload(a.sentences, 0, 1_000_000)
    ctx = _capi.Context(0)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, packed, max_k=a.k)
    k = a.k

    def dec():
        db.launch(dm, k)
        ctx.sync()

    def fetch():
        db.fetch()
        ctx.sync()

    def both():
        db.launch(dm, k)
        db.fetch()
        ctx.sync()
    dec()
    fetch()
    out = {'decode': timeit(dec, a.reps), 'fetch': timeit(fetch, a.reps), 'decode_fetch': timeit(both, a.reps)}
    for name in ('fetch_results',):
        fn = getattr(db, name, None)
        if fn:
            out[name] = timeit(fn, a.reps)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
