"""Decode launches of the bench workload for counter passes (rocprofv3 --pmc):
the 64K config-3 batch (bench.make_workload), then one counting launch
(lt_count_ops), --warmup and --steps decodes with the result copy, as
bench.py's step.  Prints one JSON line with the kernel
name and the dispatch count, so a counter table can be read per dispatch.

    python tools/prof_decode.py --k 1 [--steps 3] [--cache /tmp/ltw]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lattice_based_tagger_amd import _capi  # noqa: E402


def workload(sentences, seed):
    """The bench batch (bench.make_workload), generated in this process (a
    cache of selected PackedBatch fields went stale when the batch gained
    implicit-Unknown records)."""
    import bench
    _, _, _, packed, keys, coefs = bench.make_workload(sentences, seed, 1_000_000)
    return packed, keys, coefs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--sentences', type=int, default=65536)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--cache', default=None, help='(ignored; kept for the scripts that pass it)')
    a = ap.parse_args()
    lib = _capi.load()
    packed, keys, coefs = workload(a.sentences, a.seed)
    ctx = _capi.Context(0)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, packed, max_k=a.k)
    ops = db.count_ops(dm, a.k)
    for _ in range(a.warmup):
        db.launch(dm, a.k)
        db.fetch()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        db.launch(dm, a.k)
        db.fetch()
    ctx.sync()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({'kernel': lib.lt_kernel_name(a.k).decode(), 'k': a.k, 'sentences': a.sentences,
                      'dispatches': 1 + a.warmup + a.steps, 'count_dispatch': 0, 'ms_per_step': dt * 1e3,
                      'kernel_ms': ctx.kernel_ms_recent(a.steps), 'ops': ops, 'pieces': db.pieces}))
    db.close()
    dm.close()
    ctx.close()


if __name__ == '__main__':
    main()
