"""Golden vectors of ``beam_search(..., debug=True)``: the REFERENCE's printed
per-position dump (`lattice_tagger/beam/beam.py:53-57`) for a selection of the
committed golden cases.

Run in the survey container only (the reference is not on the GPU box):

    PYTHONHASHSEED=0 PYTHONPATH=/root/reference python tests/golden/make_debug_golden.py

Inputs are the committed fixtures (tests/golden/<set>.json.gz, data only);
each case's lattice and scorer specs are rebuilt as the REFERENCE's own
objects (``lattice_tagger.dictionary.Word``, the reference scorers), the
reference decoder runs with ``debug=True`` and its stdout is captured.  Harness
shim as in make_golden.py: ``numpy.int = int``.

Output ``debug.json.gz``: a list of {set, index, beam, stdout, error}.
"""

import contextlib
import gzip
import io
import json
import os

import numpy as np

np.int = int                       # harness shim (make_golden.py)

from lattice_tagger.beam import beam_search as ref_beam_search   # noqa: E402
from lattice_tagger.beam import (BeamScoreFunctions, RegularizationScore,  # noqa: E402
                                 MorphemePreferenceScore, WordPreferenceScore,
                                 SimpleTrigramFeatureScore)
from lattice_tagger.features import SimpleTrigramEncoder        # noqa: E402
from lattice_tagger.dictionary import Word                      # noqa: E402
from lattice_tagger.beam.score_funcs import BeamScoreFunction   # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
import sys                                                      # noqa: E402
sys.path.insert(0, os.path.join(HERE, '..'))
from plugin_defs import edge_from_spec, make_edge_table_class   # noqa: E402

EdgeTableScore = make_edge_table_class(BeamScoreFunction)       # the user plugin, inside the reference

# (set, max chars, how many cases, beams): short sentences keep the dump small
PICK = [('demo', 14, 4, (1, 3)), ('edge', 12, 14, (1, 2)), ('scorers', 30, 3, (1, 4)),
        ('synth', 40, 2, (1, 5)), ('dense', 30, 2, (2,)),
        # the general kernel's configurations: beams above 256, max_len > 8 and < 1
        ('wide', 20, 11, (1, 300)), ('wide', 33, 3, (2,)),
        # user plugins of (wj, wk) (tests/plugin_defs.py)
        ('plugins', 24, 4, (1, 3))]


def ref_funcs(specs):
    funcs = []
    for sp in specs:
        t = sp['type']
        if t == 'RegularizationScore':
            funcs.append(RegularizationScore(sp['unknown_penalty'], sp['known_preference'],
                                             sp['syllable_penalty']))
        elif t == 'MorphemePreferenceScore':
            funcs.append(MorphemePreferenceScore(sp['table']))
        elif t == 'WordPreferenceScore':
            funcs.append(WordPreferenceScore(sp['table']))
        elif t == 'SimpleTrigramFeatureScore':
            dic = {tuple(f): i for i, f in enumerate(sp['features'])}
            coef = np.array([float.fromhex(c) for c in sp['coef']], dtype=np.float64)
            funcs.append(SimpleTrigramFeatureScore(SimpleTrigramEncoder(dic), coef))
        elif t == 'EdgeTableScore':
            funcs.append(edge_from_spec(EdgeTableScore, sp))
        else:
            raise ValueError(t)
    return BeamScoreFunctions(*funcs)


def main():
    out = []
    for name, max_chars, count, beams in PICK:
        with gzip.open(os.path.join(HERE, name + '.json.gz'), 'rt', encoding='utf-8') as f:
            data = json.load(f)
        models = {k: ref_funcs(v) for k, v in data['models'].items()}
        taken = 0
        for idx, c in enumerate(data['cases']):
            if taken >= count or len(c['chars']) > max_chars:
                continue
            taken += 1
            bindex = [[Word(*w) for w in ws] for ws in c['bindex']]
            for k in beams:
                buf = io.StringIO()
                err = None
                with contextlib.redirect_stdout(buf):
                    try:
                        ref_beam_search(bindex, c['chars'], models[c['model']], beam_size=k,
                                        max_len=c['max_len'], debug=True)
                    except Exception as exc:          # the reference's own behaviour
                        err = type(exc).__name__
                out.append({'set': name, 'index': idx, 'beam': k, 'stdout': buf.getvalue(), 'error': err})
    path = os.path.join(HERE, 'debug.json.gz')
    with gzip.open(path, 'wt', encoding='utf-8') as f:
        json.dump(out, f, ensure_ascii=False, separators=(',', ':'))
    print('wrote', path, len(out), 'dumps', os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
