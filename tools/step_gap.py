"""Where the time between back-to-back k=1 decodes goes: the bench batch
(bench.make_workload, seed 0) decoded K times in a row
  launch_only   the decode alone (no result D2H)
  launch_fetch  decode + result D2H on the copy stream (the bench step)
per-step wall time against the kernel's HIP-event time.  One JSON line.

    python tools/step_gap.py [--steps 40] [--k 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lattice_based_tagger_amd import _capi  # noqa: E402

_capi.load()
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--sentences', type=int, default=65536)
    a = ap.parse_args()
    base_n = min(a.sentences, bench.BASE_SENTENCES)
    raw, lay, sm, packed, keys, coefs = bench.make_workload(base_n, 0, 1_000_000)
    order = bench.batch_order(a.sentences, base_n, 0)
    piece = packed if order is None else packed.take(order)
    ctx = _capi.Context(0)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, piece, max_k=a.k)
    out = {'k': a.k, 'sentences': a.sentences, 'steps': a.steps}

    def run(name, step):
        for _ in range(3):
            step()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        ctx.sync()
        el = (time.perf_counter() - t0) / a.steps * 1e3
        kern = ctx.kernel_ms_recent(a.steps)
        km = sum(kern) / len(kern)
        out[name] = {'step_ms': el, 'kernel_ms': km, 'gap_ms': el - km}

    run('launch_only', lambda: db.launch(dm, a.k))

    def with_fetch():
        db.launch(dm, a.k)
        db.fetch()
    run('launch_fetch', with_fetch)
    run('launch_only_again', lambda: db.launch(dm, a.k))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
