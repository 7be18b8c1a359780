#!/usr/bin/env python3
"""CPU-only timing of Tagger.tag_batch's host stages on unique synthetic text
(tools/bench_tagger.unique_text): lookup, pack, and the re-materialisation of
the best paths (beam._materialise_bulk) fed with the C oracle's decode of the
same batch in the compact result layout -- no GPU needed.  Test/diagnostic
tool: the oracle only stands in for the device's results here.

    python tools/prof_materialise.py [--sentences 16384] [--k 1] [--threads 8] [--profile]
"""
import argparse
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

from bench_tagger import unique_text  # noqa: E402
from golden_io import load  # noqa: E402
from test_lookup import _fixture, fixture_lexicon  # noqa: E402
from lattice_based_tagger_amd.beam import _materialise_bulk, lowered_model  # noqa: E402
from lattice_based_tagger_amd.native_packer import packer_for  # noqa: E402
from oracle import lt_oracle  # noqa: E402


def compact(count, length, score, codes, sent_n, k):
    """The oracle's padded results in PackedResults' compact layout."""
    S = len(sent_n)
    n = np.asarray(sent_n, dtype=np.int64)
    cum = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(n, out=cum[1:])
    L = length.ravel().astype(np.int64)
    e = np.repeat(np.arange(L.size, dtype=np.int64), L)
    off = np.zeros(S * k + 1, dtype=np.int64)
    np.cumsum(L, out=off[1:])
    s, t = e // k, e % k
    j = np.arange(int(L.sum()), dtype=np.int64) - off[e]
    return SimpleNamespace(k=k, count=count, length=length, score=score,
                           codes=codes[k * cum[s] + t * n[s] + j], off=off)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=16384)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--profile', action='store_true')
    a = ap.parse_args()
    entry = _fixture()['base']
    lex = fixture_lexicon(entry)
    model = lowered_model(load('base')[0].funcs)
    npk = packer_for(model)
    sents = unique_text(entry['sentences'], a.sentences, 7)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        lat = lex.lookup(sents, n_threads=a.threads)
        t1 = time.perf_counter()
        packed, views = npk.pack_lattices(lat, max_len=8)
        t2 = time.perf_counter()
        print('lookup %.3f s  pack %.3f s' % (t1 - t0, t2 - t1), flush=True)
    count, length, score, codes, _, _ = lt_oracle.decode(packed, model.keys, model.coefs, a.k, nthreads=a.threads)
    res = compact(count, length, score, codes, packed.sent_n, a.k)
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = _materialise_bulk(packed, views, lat.chars, 1, res, model)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        del out
    print('materialise best of %d: %.3f s (%d sentences, %d path words)' % (a.reps, best, len(sents),
                                                                        int(res.length[:, 0].sum())))
    # the two halves Tagger.tag_batch runs on different threads (round 6)
    from lattice_based_tagger_amd.beam import materialise_prepared, prepare_bulk
    bp = bm = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        prep = prepare_bulk(packed, views, lat.chars, 1, res, model)
        t1 = time.perf_counter()
        out = materialise_prepared(prep)
        t2 = time.perf_counter()
        bp = t1 - t0 if bp is None else min(bp, t1 - t0)
        bm = t2 - t1 if bm is None else min(bm, t2 - t1)
        del out, prep
    print('  prepare (decode-stage worker) %.3f s, build (caller, GIL) %.3f s' % (bp, bm))
    if a.profile:
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        _materialise_bulk(packed, views, lat.chars, 1, res, model)
        prof.disable()
        pstats.Stats(prof).sort_stats('tottime').print_stats(15)


if __name__ == '__main__':
    main()
