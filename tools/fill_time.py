"""Time of the k=1 lane-schedule fill (lt_k1_sched) alone: lt_batch_create of
a beam-1 batch runs it behind the uploads; lt_batch_prep_ms reads its events.
No decode is launched.  LT_LIBRARY selects the library (timing builds of the
fill: -DLT_K1_FILL_STAGES=1 / 2).

    python tools/fill_time.py [--sentences 65536] [--reps 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from lattice_based_tagger_amd import _capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=65536)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    import bench
    packed = bench.make_workload(a.sentences, 0, 1_000_000)[3]     # the bench batch
    ctx = _capi.Context(0)
    ms = []
    for _ in range(a.reps):
        db = _capi.DeviceBatch(ctx, packed, max_k=1)
        ms.append(db.prep_ms())
        db.close()
    print(json.dumps({'library': os.environ.get('LT_LIBRARY', 'liblt.so'), 'sentences': a.sentences,
                      'fill_ms': ms}))


if __name__ == '__main__':
    main()
