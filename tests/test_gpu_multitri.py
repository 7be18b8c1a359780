"""Composites with several SimpleTrigramFeatureScores (round 6;
`lattice_tagger/beam/score_funcs.py:50-54` sums any scorers in constructor
order): the reference's own vectors are in tests/golden/multitri.json.gz
(test_gpu_parity / test_evaluate); here synthetic batches against the
pure-Python restatement (oracle/ref_beam.py, itself pinned to those vectors
by test_oracle_golden), the lowering's layout and the debug dump."""

import io

import numpy as np
import pytest

from lattice_based_tagger_amd import beam_search, beam_search_batch, synth
from lattice_based_tagger_amd.beam import debug_dump, lowered_model
from lattice_based_tagger_amd.feature import SimpleTrigramEncoder
from lattice_based_tagger_amd.lowering import XTRI_CLASS_STRIDE
from lattice_based_tagger_amd.packer import pack
from lattice_based_tagger_amd.score_funcs import (BeamScoreFunctions, MorphemePreferenceScore,
                                                  RegularizationScore, SimpleTrigramFeatureScore)
from lattice_based_tagger_amd.word import Word
from oracle import ref_beam


def _lattices_and_scorers(n_sent=48, seed=31):
    raw = synth.make_lattices(n_sent, seed=seed, eojeols=5)
    lats, dic_a, coef_a = synth.to_words(raw, synth.make_model(raw, seed=seed, n_features=3000), word_cls=Word)
    _, dic_b, coef_b = synth.to_words(raw, synth.make_model(raw, seed=seed + 1, n_features=2000), word_cls=Word)
    tri_a = SimpleTrigramFeatureScore(SimpleTrigramEncoder(dic_a), coef_a)
    tri_b = SimpleTrigramFeatureScore(SimpleTrigramEncoder(dic_b), coef_b)
    return lats, tri_a, tri_b


def test_lowering_keys_of_each_scorer():
    """Scorer t's keys carry class + 16 t; one vocabulary, masks per scorer."""
    lats, tri_a, tri_b = _lattices_and_scorers(8)
    m = lowered_model(BeamScoreFunctions(RegularizationScore(), tri_a, tri_b))
    assert len(m.trigrams) == 2 and m.n_xtri == 1 and len(m.vmasks) == 2
    cls = m.keys[:, 3]
    assert set(np.unique(cls // XTRI_CLASS_STRIDE).tolist()) == {0, 1}
    assert set(np.unique(cls % XTRI_CLASS_STRIDE).tolist()) <= {0, 1, 2, 3, 7, 8}
    packed, _ = pack(lats, m)
    assert packed.n_xtri == 1 and packed.n_unk == 0
    assert packed.xtri_mask.shape == (1, packed.n_nodes)


@pytest.mark.gpu
@pytest.mark.parametrize('k', [1, 3, 16])
@pytest.mark.parametrize('order', ['reg_a_b', 'b_mp_a', 'a_a'])
def test_several_trigram_scorers_match_ref_beam(gpu_decoder, k, order):
    lats, tri_a, tri_b = _lattices_and_scorers()
    mp = MorphemePreferenceScore({'Noun': {'x1': 0.5}})
    funcs = {'reg_a_b': BeamScoreFunctions(RegularizationScore(), tri_a, tri_b),
             'b_mp_a': BeamScoreFunctions(tri_b, mp, tri_a, RegularizationScore()),
             'a_a': BeamScoreFunctions(tri_a, tri_a)}[order]
    got = beam_search_batch(lats, funcs, beam_size=k)
    for (bindex, chars), matures in zip(lats, got):
        exp = ref_beam.beam_search(bindex, chars, funcs, beam_size=k)
        assert len(matures) == len(exp)
        for m, (path, score) in zip(matures, exp):
            assert float(m.score).hex() == float(score).hex()
            assert all(a is b or a == b for a, b in zip(m.sequences[1:-1], path[1:-1]))


@pytest.mark.gpu
def test_several_trigram_scorers_debug_dump(gpu_decoder):
    """debug=True (the trace kernel) with two trigram terms: its last
    position's best grown hypothesis is the decoder's best mature."""
    lats, tri_a, tri_b = _lattices_and_scorers(4)
    funcs = BeamScoreFunctions(tri_a, RegularizationScore(), tri_b)
    bindex, chars = lats[0]
    buf = io.StringIO()
    debug_dump(bindex, chars, funcs, beam_size=3, file=buf)
    text = buf.getvalue()
    assert 'End point = %d' % len(chars) in text
    best = beam_search(bindex, chars, funcs, beam_size=3)[0]
    exp = ref_beam.beam_search(bindex, chars, funcs, beam_size=3)[0]
    assert float(best.score).hex() == float(exp[1]).hex()
