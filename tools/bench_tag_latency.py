#!/usr/bin/env python3
"""Tagger.tag(sentence) latency, one sentence per call (the reference's
primary API), on the golden base set's sentences.  One JSON line."""
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


def main():
    entry = _fixture()['base']
    funcs = load('base')[0].funcs
    sents = [s for s in entry['sentences'] if len(s.split()) >= 10]
    tagger = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=fixture_lexicon(entry),
                    score_funcs=funcs)
    out = {}
    for k in (1, 5):
        for s in sents[:10]:
            tagger.tag(s, beam_size=k)                    # warm
        ts = []
        for s in sents * 2:
            t0 = time.perf_counter()
            tagger.tag(s, beam_size=k)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out[str(k)] = {'median_ms': 1e3 * ts[len(ts) // 2], 'p90_ms': 1e3 * ts[int(len(ts) * 0.9)],
                       'calls': len(ts)}
    # per-phase breakdown of one call (k=1): where the latency goes
    from lattice_based_tagger_amd.beam import Decoder, decode_batch, lowered_model
    from lattice_based_tagger_amd.native_packer import packer_for
    model = lowered_model(funcs)
    npk = packer_for(model)
    dec = Decoder.get(0)
    dm = dec.device_model(model)
    lex = tagger.native_lexicon()
    ph = {'lookup': [], 'pack': [], 'batch_create': [], 'decode': [], 'batch_destroy': [], 'decode_batch_whole': []}
    for s in sents:
        t0 = time.perf_counter()
        lat = lex.lookup([s])
        t1 = time.perf_counter()
        packed, views = npk.pack_desc(lat.desc, lat, lat.chars, max_len=8)
        t2 = time.perf_counter()
        db = _capi.DeviceBatch(dec.ctx, packed, max_k=1)
        t3 = time.perf_counter()
        db.decode(dm, 1)
        t4 = time.perf_counter()
        db.close()
        t5 = time.perf_counter()
        decode_batch(packed, views, lat.chars, model, 1, 0, best_only=True)
        t6 = time.perf_counter()
        for key, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            ph[key].append(v)
    med = {key: 1e3 * sorted(v)[len(v) // 2] for key, v in ph.items()}
    print(json.dumps({'metric': 'Tagger.tag latency (one sentence per call)', 'latency': out,
                      'phase_median_ms_k1': med}))


if __name__ == '__main__':
    main()
