"""Loader of the golden vectors in tests/golden/*.json.gz (data only; produced
by tests/golden/make_golden.py from the reference itself)."""

import gzip
import json
import os

import numpy as np

from lattice_based_tagger_amd import (BeamScoreFunctions, RegularizationScore,
                                      MorphemePreferenceScore, WordPreferenceScore,
                                      SimpleTrigramFeatureScore, SimpleTrigramEncoder, Word)
from lattice_based_tagger_amd.score_funcs import BeamScoreFunction
from plugin_defs import edge_from_spec, make_edge_table_class

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
SETS = ('base', 'demo', 'synth', 'scorers', 'edge', 'dense', 'wide')
# sets whose composites hold user plugins (tests/plugin_defs.py), which the C
# restatement (oracle/lt_oracle.c) does not evaluate
PLUGIN_SETS = ('plugins',)
# composites with several SimpleTrigramFeatureScores (round 6): the general
# kernel; the C restatement (one trigram term) does not take them
MULTI_SETS = ('multitri',)
EdgeTableScore = make_edge_table_class(BeamScoreFunction)


def _tup(x):
    return tuple(x)


def build_funcs(specs):
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
            dic = {_tup(f): i for i, f in enumerate(sp['features'])}
            coef = np.array([float.fromhex(c) for c in sp['coef']], dtype=np.float64)
            funcs.append(SimpleTrigramFeatureScore(SimpleTrigramEncoder(dic), coef))
        elif t == 'EdgeTableScore':
            funcs.append(edge_from_spec(EdgeTableScore, sp))
        else:
            raise ValueError(t)
    return BeamScoreFunctions(*funcs)


class Case:
    def __init__(self, d, funcs):
        self.chars = d['chars']
        self.bindex = [[Word(*w) for w in ws] for ws in d['bindex']]
        self.max_len = d['max_len']
        self.model = d['model']
        self.tag = d['tag']
        self.funcs = funcs
        self.expected = d['expected']

    def node(self, code):
        if code[0] == 'U':
            return None
        return self.bindex[code[0]][code[1]]


def load(name, packable=False):
    """The cases of set ``name``; ``packable``: only those a packed batch can
    hold (max_len >= 1 -- below that beam_search decodes nothing and packs
    nothing, beam.py:29-31)."""
    with gzip.open(os.path.join(GOLDEN, name + '.json.gz'), 'rt', encoding='utf-8') as f:
        data = json.load(f)
    models = {k: build_funcs(v) for k, v in data['models'].items()}
    cases = [Case(c, models[c['model']]) for c in data['cases']]
    return [c for c in cases if c.max_len >= 1] if packable else cases


def beams_of(cases):
    """Beam sizes the reference was run with in any of ``cases``."""
    return sorted({int(k) for c in cases for k in c.expected})


def path_matches(case, codes, path_words):
    """path_words: the decoded path without BOS/EOS.  Dictionary nodes must be
    the very objects of bindex (identity); Unknown nodes must have the
    synthesised fields."""
    if len(codes) != len(path_words):
        return False
    for code, w in zip(codes, path_words):
        if code[0] == 'U':
            b, e = code[1], code[2]
            sub = case.chars[b:e]
            if tuple(w) != (sub, sub, None, 'Unknown', None, e - b, b, e, False):
                return False
        elif w is not case.node(code):
            return False
    return True
