"""Score types of the drop-in (no GPU): the reference's mature score is a
Python sum whose type follows its increments -- int 0 at BOS (beam.py:21),
float from float-valued scorers, numpy.float64 once a trigram feature set is
non-empty (score_funcs.py:141-144).  ``path_score_type`` replays that on the
host for the decoded path; the golden vectors record the reference's type of
every mature."""

import numpy as np
import pytest

from golden_io import MULTI_SETS, SETS, load
from lattice_based_tagger_amd import Word
from lattice_based_tagger_amd.beam import lowered_model, path_score_type, typed_score
from lattice_based_tagger_amd.word import bos_word


def _path(case, codes):
    out = [bos_word()]
    for code in codes:
        w = case.node(code)
        if w is None:
            b, e = code[1], code[2]
            sub = case.chars[b:e]
            w = Word(sub, sub, None, 'Unknown', None, e - b, b, e, False)
        out.append(w)
    return out


@pytest.mark.parametrize('name', SETS + MULTI_SETS)
def test_path_score_type_matches_reference(name):
    seen = set()
    for case in load(name):
        model = lowered_model(case.funcs)
        for k, exp in case.expected.items():
            for codes, shex, kind in exp.get('matures', []):
                if not case.chars:
                    continue                 # [BOS, EOS]: int 0, set by the decoder itself
                t = path_score_type(model, _path(case, codes))
                assert t.__name__ == kind, (case.tag, k, t, kind)
                v = typed_score(t, float.fromhex(shex))
                assert type(v).__name__ == kind and float(v).hex() == shex
                seen.add(kind)
    assert seen


def test_all_three_types_occur():
    kinds = set()
    for name in ('scorers', 'edge'):
        for case in load(name):
            for exp in case.expected.values():
                kinds |= {m[2] for m in exp.get('matures', [])}
    assert kinds == {'int', 'float', 'float64'}
    assert typed_score(int, 3.0) == 3 and type(typed_score(int, 3.0)) is int
    assert type(typed_score(np.float64, 0.5)) is np.float64
