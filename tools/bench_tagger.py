#!/usr/bin/env python3
"""End-to-end Tagger throughput: text -> native lattices -> native packer ->
HIP decode -> best Sequence objects, per phase.

Text (--text): 'unique' (default) -- every sentence a fresh seeded draw of
10-20 eojeols from the 2,087 distinct eojeols of tests/golden/lookup.json.gz's
base-dictionary sentences (the restricted reference dictionary stored there
answers their lookups exactly, and a sentence's lattice is the concatenation
of its eojeols' lattices, `lookup.py:344-369`); 'golden' -- the golden 'base'
sentences of >= 10 eojeols replicated to --sentences (rounds 1-2).  The model
is the golden 'base' set's (RegularizationScore + SimpleTrigramFeatureScore).
One JSON line.

    python tools/bench_tagger.py [--sentences 65536] [--k 1] [--text unique] [--threads 0] [--reps 3]
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from lattice_based_tagger_amd import _capi  # noqa: E402

_capi.load()
from golden_io import load  # noqa: E402
from test_lookup import _fixture, fixture_dictionary, fixture_lexicon  # noqa: E402
from lattice_based_tagger_amd import Tagger  # noqa: E402
from lattice_based_tagger_amd.beam import Decoder, decode_batch, lowered_model  # noqa: E402
from lattice_based_tagger_amd.native_packer import packer_for  # noqa: E402


def unique_text(golden, n, seed):
    """n distinct sentences of 10-20 eojeols drawn from the golden eojeols."""
    import numpy as np
    pool = sorted({w for s in golden for w in s.split()})
    rng = np.random.default_rng(seed)
    lens = rng.integers(10, 21, size=n)
    picks = rng.integers(0, len(pool), size=int(lens.sum()))
    out, at = [], 0
    for m in lens:
        out.append(' '.join(pool[i] for i in picks[at:at + m]))
        at += m
    assert len(set(out)) == n
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=65536)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--threads', type=int, default=0)
    ap.add_argument('--text', choices=('unique', 'golden'), default='unique')
    ap.add_argument('--seed', type=int, default=7)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--chunk', type=int, default=0, help='Tagger.tag_batch pipeline chunk (0: default)')
    ap.add_argument('--profile', action='store_true', help='cProfile the tag_batch call (stderr)')
    ap.add_argument('--api-reps', type=int, default=3, help='timed tag_batch calls (best reported)')
    ap.add_argument('--api-first', action='store_true',
                    help='time the tag_batch calls before the per-phase breakdown (whose 64K-sentence '
                         'batches otherwise precede them)')
    a = ap.parse_args()
    entry = _fixture()['base']
    funcs = load('base')[0].funcs
    if a.text == 'golden':
        base = [s for s in entry['sentences'] if len(s.split()) >= 10]
        sents = (base * (a.sentences // len(base) + 1))[:a.sentences]
    else:
        sents = unique_text(entry['sentences'], a.sentences, a.seed)
    lex = fixture_lexicon(entry)
    tagger = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=lex, score_funcs=funcs)
    if a.chunk:
        Tagger.CHUNK = a.chunk
    # warm-up, as a service does once at start: model lowering, device model,
    # and the pipeline's batch arenas at chunk size (up to four chunks in
    # flight since round 6's decode stage; the context recycles them for every
    # later call)
    tagger.tag_batch(sents[:5 * Tagger.CHUNK], beam_size=a.k)

    call_stats = []

    def api_calls():
        times = []
        out = None
        for _ in range(a.api_reps):
            out = None                            # the previous call's results are freed untimed
            gc.collect()
            t0 = time.perf_counter()
            out = tagger.tag_batch(sents, beam_size=a.k)
            times.append(time.perf_counter() - t0)
            t1 = time.perf_counter()
            gc.collect()                          # (untimed: what the call left for the collector)
            gc_s = time.perf_counter() - t1
            st = dict(tagger.last_stats or {})
            st['call_s'] = times[-1]
            st['gc_after_s'] = gc_s
            call_stats.append({key: round(v, 4) if isinstance(v, float) else v for key, v in st.items()})
        return times, out
    if a.api_first:
        api_times, out = api_calls()
    model = lowered_model(funcs)
    npk = packer_for(model)
    best = {}
    for _ in range(a.reps):
        t = {}
        t0 = time.perf_counter()
        lat = lex.lookup(sents, n_threads=a.threads)
        t['lookup'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        packed, views = npk.pack_lattices(lat, max_len=8)        # (as Tagger.tag_batch packs)
        t['pack'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        # (a context of its own, so that this 64K-sentence batch's arena
        # stays out of the pool of the context the tag_batch calls use)
        dec = Decoder.get(0, 1)
        dm = dec.device_model(model)
        dbs = [_capi.DeviceBatch(dec.ctx, packed, max_k=a.k)]
        t['batch_create_h2d'] = time.perf_counter() - t0
        t0 = time.perf_counter()
        kern = 0.0
        for db in dbs:
            db.launch(dm, a.k)
            dec.ctx.sync()
            kern += dec.ctx.kernel_ms() / 1e3
            db.fetch()
            dec.ctx.sync()
            db.close()
        t['decode_d2h'] = time.perf_counter() - t0
        t['kernel_only'] = kern
        t0 = time.perf_counter()
        matures = decode_batch(packed, views, lat.chars, model, a.k, 0, best_only=True, decoder=dec)
        t['decode_and_materialise_best'] = time.perf_counter() - t0
        t['total'] = t['lookup'] + t['pack'] + t['decode_and_materialise_best']
        if not best or t['total'] < best['total']:
            best = t
            n_words = lat.n_words
    if not a.api_first:
        api_times, out = api_calls()
    api = min(api_times)
    if a.profile:
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        tagger.tag_batch(sents, beam_size=a.k)
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats('tottime').print_stats(25)
    assert len(out) == len(sents) and all(o.score == m[0].score for o, m in zip(out, matures))
    line = {'metric': 'end-to-end Tagger.tag_batch sentences/s (text -> best Sequence)',
            'sentences': len(sents), 'k': a.k, 'text': a.text, 'distinct_sentences': len(set(sents)), 'lattice_nodes': n_words,
            'packed_nodes': int(packed.n_nodes),
            'chars_per_sentence': float(packed.sent_n.mean()),
            'phase_s': best, 'sentences_per_s': {p: len(sents) / v for p, v in best.items()},
            'tag_batch_api_sentences_per_s': len(sents) / api,
            'tag_batch_api_runs_sentences_per_s': [len(sents) / t for t in api_times],
            'tag_batch_api_call_stats': call_stats,
            'lookup_threads': a.threads or os.cpu_count(), 'nproc': os.cpu_count(), 'api_first': a.api_first}
    print(json.dumps(line))


if __name__ == '__main__':
    main()
