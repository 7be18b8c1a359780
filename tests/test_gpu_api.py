"""Drop-in API behaviours beyond the golden vectors (`lattice_tagger/beam/
score_funcs.py:7-15,35-39`: any BeamScoreFunction subclass plugs in):

* a user plugin that declares ``node_local = True`` is lowered per node and
  decodes exactly as the reference loop calling it per expansion (checked
  against oracle/ref_beam.py, the restatement pinned to the reference's own
  vectors) -- before and after the trigram term;
* a user plugin without that declaration is refused loudly;
* infinite coefficients of one sign decode exactly; NaN, or +inf with -inf
  (whose NaN sums Python's sort orders unreproducibly), are refused.
"""
import numpy as np
import pytest

from golden_io import load
from lattice_based_tagger_amd import (beam_search_batch, BeamScoreFunction, BeamScoreFunctions,
                                      SimpleTrigramFeatureScore, SimpleTrigramEncoder, _capi)
from oracle import ref_beam

pytestmark = pytest.mark.gpu


class NounLength(BeamScoreFunction):
    node_local = True

    def score(self, seq, w):
        return 0.25 * w.len if w.tag0 == 'Noun' else -0.125


class UnknownPenalty(BeamScoreFunction):
    node_local = True

    def __init__(self, v):
        self.v = v

    def score(self, seq, w):
        return self.v if w.tag0 == 'Unknown' else 0


class PathDependent(BeamScoreFunction):
    def score(self, seq, w):
        return len(seq.sequences)


def _cases():
    return [c for c in load('demo') if not any('error' in e for e in c.expected.values())][:40]


def _compare(cases, funcs, k):
    got = beam_search_batch([(c.bindex, c.chars) for c in cases], funcs, beam_size=k,
                            max_len=cases[0].max_len)
    for c, matures in zip(cases, got):
        exp = ref_beam.beam_search(c.bindex, c.chars, funcs, k, c.max_len)
        assert len(matures) == len(exp)
        for m, (path, score) in zip(matures, exp):
            assert float(m.score).hex() == float(score).hex()
            assert [tuple(w) for w in m.sequences] == [tuple(w) for w in path]


def _parts(case):
    funcs = case.funcs.funcs
    tri = [f for f in funcs if type(f).__name__ == 'SimpleTrigramFeatureScore'][0]
    other = [f for f in funcs if f is not tri]
    return tri, other


@pytest.mark.parametrize('k', [1, 5])
def test_node_local_user_plugins(gpu_decoder, k):
    cases = _cases()
    tri, other = _parts(cases[0])
    funcs = BeamScoreFunctions(NounLength(), *other, tri, UnknownPenalty(-0.75))
    _compare(cases, funcs, k)


def test_plugin_without_node_local_is_refused(gpu_decoder):
    c = _cases()[0]
    tri, other = _parts(c)
    with pytest.raises(NotImplementedError):
        beam_search_batch([(c.bindex, c.chars)], BeamScoreFunctions(*other, tri, PathDependent()), 1)


def _with_coefs(tri, fn):
    coef = tri.coefficients.copy()
    fn(coef)
    return SimpleTrigramFeatureScore(SimpleTrigramEncoder(tri.encoder.feature_dic), coef)


@pytest.mark.parametrize('sign', [1.0, -1.0])
@pytest.mark.parametrize('k', [1, 4])
def test_infinite_coefficients_of_one_sign(gpu_decoder, sign, k):
    cases = _cases()
    tri, other = _parts(cases[0])
    rng = np.random.default_rng(3)

    def poke(c):
        c[rng.choice(c.size, max(1, c.size // 50), replace=False)] = sign * np.inf
    funcs = BeamScoreFunctions(*other, _with_coefs(tri, poke))
    _compare(cases, funcs, k)


def test_nan_or_mixed_infinities_are_refused(gpu_decoder):
    c = _cases()[0]
    tri, other = _parts(c)

    def nan(x):
        x[0] = np.nan

    def mixed(x):
        x[0], x[1] = np.inf, -np.inf
    for fn in (nan, mixed):
        with pytest.raises(NotImplementedError):
            beam_search_batch([(c.bindex, c.chars)], BeamScoreFunctions(*other, _with_coefs(tri, fn)), 1)
    # +inf coefficients with a -inf node term: refused by the library at decode
    plus = _with_coefs(tri, lambda x: x.__setitem__(slice(0, 5), np.inf))
    with pytest.raises(_capi.LTError):
        beam_search_batch([(cc.bindex, cc.chars) for cc in _cases()],
                          BeamScoreFunctions(*other, plus, UnknownPenalty(-np.inf)), 1)
