#!/usr/bin/env python3
"""beam_search_batch throughput from reference-style lattices (lists of Word
per begin slot, as ``sentence_lookup_as_begin_index`` returns them): native
pack of the Word lists + HIP decode + the matures re-materialised with the
caller's Word objects.  One JSON line.

    python tools/bench_beam_api.py [--sentences 4096] [--k 1 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lattice_based_tagger_amd import _capi, synth, score_funcs as SF, feature as FE  # noqa: E402

_capi.load()
from lattice_based_tagger_amd.beam import beam_search_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=4096)
    ap.add_argument('--k', type=int, nargs='+', default=[1, 5])
    a = ap.parse_args()
    raw = synth.make_lattices(a.sentences, seed=3)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=3, n_features=200_000)
    dic, coef = synth.render_model(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    sents = synth.render_sentences(raw, range(raw.S))
    beam_search_batch(sents[:64], funcs, beam_size=1)           # warm: lowering, device model
    out = {}
    for k in a.k:
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            res = beam_search_batch(sents, funcs, beam_size=k)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        assert len(res) == len(sents)
        out[str(k)] = len(sents) / best
    print(json.dumps({'metric': 'beam_search_batch sentences/s (Word-list lattices -> matures)',
                      'sentences': len(sents), 'sentences_per_s': out}))


if __name__ == '__main__':
    main()
