#!/usr/bin/env python3
"""Host stages of Tagger.tag_batch on the CPU (no GPU): native lookup, native
pack, and the caller's best-path materialisation (beam._materialise_bulk)
fed with results from the C restatement (oracle/lt_oracle.c; test
infrastructure used here as a stand-in for the device results, which it
equals byte for byte).  Times each stage over --reps; --profile adds a
cProfile of one materialisation.

    python tools/host_stages.py [--sentences 16384] [--threads 8] [--reps 3] [--profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

from bench_tagger import unique_text  # noqa: E402
from golden_io import load  # noqa: E402
from test_lookup import _fixture, fixture_lexicon  # noqa: E402
from lattice_based_tagger_amd import beam as BM  # noqa: E402
from lattice_based_tagger_amd.beam import lowered_model  # noqa: E402
from lattice_based_tagger_amd.native_packer import packer_for  # noqa: E402
from oracle import lt_oracle  # noqa: E402


class _Res:
    """The compact result layout (_capi.PackedResults) from padded codes."""

    def __init__(self, count, length, score, codes, sent_n, k):
        S = len(count)
        self.k = k
        self.count = count
        self.length = length.reshape(S, k)
        self.score = score.reshape(S, k)
        cum = np.zeros(S + 1, dtype=np.int64)
        np.cumsum(np.asarray(sent_n, dtype=np.int64), out=cum[1:])
        parts = []
        for s in range(S):
            for t in range(min(int(count[s]), k)):
                a = k * cum[s] + t * int(sent_n[s])
                parts.append(codes[a:a + int(self.length[s, t])])
        self.codes = np.concatenate(parts) if parts else np.zeros(0, np.int32)
        self.off = np.zeros(S * k + 1, dtype=np.int64)
        np.cumsum(self.length.ravel(), out=self.off[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=16384)
    ap.add_argument('--threads', type=int, default=os.cpu_count())
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--profile', action='store_true')
    a = ap.parse_args()
    entry = _fixture()['base']
    funcs = load('base')[0].funcs
    sents = unique_text(entry['sentences'], a.sentences, 7)
    lex = fixture_lexicon(entry)
    model = lowered_model(funcs)
    npk = packer_for(model)
    lat = lex.lookup(sents, n_threads=a.threads)
    packed, views = npk.pack_lattices(lat, max_len=8)
    keys, coefs = model.keys, model.coefs
    count, length, score, codes, _, _ = lt_oracle.decode(packed, keys, coefs, a.k, nthreads=a.threads)
    res = _Res(count, length, score, codes, packed.sent_n, a.k)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        lat2 = lex.lookup(sents, n_threads=a.threads)
        t1 = time.perf_counter()
        p2, v2 = npk.pack_lattices(lat2, max_len=8)
        t2 = time.perf_counter()
        out = BM._materialise_bulk(packed, views, lat.chars, 1, res, model)
        t3 = time.perf_counter()
        print('lookup %.3f s  pack %.3f s  materialise %.3f s  (%d sentences, %d nodes)'
              % (t1 - t0, t2 - t1, t3 - t2, len(sents), p2.n_nodes))
        del lat2, p2, v2, out
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        BM._materialise_bulk(packed, views, lat.chars, 1, res, model)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats('cumulative').print_stats(18)


if __name__ == '__main__':
    main()
