"""Scoring-plugin protocol of the decoder.

Mirrors the reference plugin API (`lattice_tagger/beam/score_funcs.py`):

* ``BeamScoreFunction``      -- protocol: ``score(seq, word_k)`` / ``evaluate(seq)``
                                (`score_funcs.py:7-15`)
* ``BeamScoreFunctions``     -- ordered composite (`score_funcs.py:18-54`)
* ``RegularizationScore``    -- node-local length/unknown prior (`:57-73`)
* ``MorphemePreferenceScore``-- node-local morpheme bonus (`:75-88`)
* ``WordPreferenceScore``    -- node-local surface bonus (`:90-100`)
* ``SimpleTrigramFeatureScore`` -- second-order trigram feature score (`:102-144`)

The decoder (``beam_search``) never calls ``score`` per expansion: it
*lowers* the composite to device tables (see ``lowering.py``) and evaluates
it inside the HIP kernel.  The Python ``score`` / ``evaluate`` methods are
kept because they are part of the public plugin interface (gold-path scoring,
user code); they follow the reference arithmetic exactly.
"""

import numpy as np

from .tagset import BOS, EOS, Noun, Unk


class BeamScoreFunction:
    """Protocol for one additive term of the expansion score.

    Two kinds of user subclass are lowered to the device, in constructor
    order, like the built-in scorers:

    * ``node_local = True`` -- ``score(seq, word_k)`` reads ``word_k`` only:
      evaluated as ``score(None, w)`` once per lattice node (host side);
    * ``edge_local = True`` -- it reads ``seq.sequences[-1]`` and ``word_k``
      only: evaluated once per lattice edge (last word wj -> candidate w),
      host side, with a ``seq`` whose ``sequences`` ends in wj.

    A subclass that reads more of the path has no device lowering and is
    refused (``NotImplementedError``), never evaluated on a CPU path."""

    node_local = False
    edge_local = False

    def __call__(self, sequence, word_k):
        return self.score(sequence, word_k)

    def evaluate(self, seq):
        raise NotImplementedError('Inherit and implement evaluate function')

    def score(self, seq, word_k):
        raise NotImplementedError('Inherit and implement score function')


class BeamScoreFunctions:
    """Ordered sum of scoring plugins.

    The increment of an expansion is ``((0 + f1) + f2) + ...`` in constructor
    order (`score_funcs.py:50-54`); the HIP kernel reproduces that order.
    """

    def __init__(self, *functions):
        for func in functions:
            if not isinstance(func, _plugin_base_classes()):
                raise ValueError('functions must be instance of BeamScoreFunction')
        self.funcs = list(functions)

    def __call__(self, sequence, word_k):
        return self.score(sequence, word_k)

    def evaluate(self, seq):
        total = 0
        for func in self.funcs:
            total += func.evaluate(seq)
        return total

    def score(self, sequence, word_k):
        total = 0
        for func in self.funcs:
            total += func(sequence, word_k)
        return total


def _plugin_base_classes():
    """Our protocol class plus the reference's, when it is importable, so a
    composite may mix plugins from either package."""
    bases = [BeamScoreFunction]
    import sys
    ref = sys.modules.get('lattice_tagger.beam.score_funcs')
    if ref is not None and hasattr(ref, 'BeamScoreFunction'):
        bases.append(ref.BeamScoreFunction)
    return tuple(bases)


class RegularizationScore(BeamScoreFunction):
    """Node-local prior on word length (`score_funcs.py:57-73`)."""

    def __init__(self, unknown_penalty=-0.1, known_preference=0.2, syllable_penalty=-0.2):
        self.unknown_penalty = unknown_penalty
        self.known_preference = known_preference
        self.syllable_penalty = syllable_penalty

    def evaluate(self, seq):
        return sum(self.score(None, w) for w in seq.sequences)

    def score(self, seq, word_k):
        value = 0
        if word_k.tag0 == Unk:
            value += self.unknown_penalty * (word_k.len + 0.1)
        else:
            value += self.known_preference * word_k.len
        if word_k.len == 1 and word_k.tag0 == Noun:
            value += self.syllable_penalty
        return value


class MorphemePreferenceScore(BeamScoreFunction):
    """Node-local bonus looked up by (tag, morpheme) (`score_funcs.py:75-88`)."""

    def __init__(self, tag_to_morph=None):
        self.tag_to_morph = {} if tag_to_morph is None else tag_to_morph

    def evaluate(self, seq):
        return sum(self.score(None, w) for w in seq.sequences)

    def score(self, seq, word_k):
        value = self.tag_to_morph.get(word_k.tag0, {}).get(word_k.morph0, 0)
        if word_k.tag1 is not None:
            value += self.tag_to_morph.get(word_k.tag1, {}).get(word_k.morph1, 0)
        return value


class WordPreferenceScore(BeamScoreFunction):
    """Node-local bonus looked up by (tag, surface) (`score_funcs.py:90-100`)."""

    def __init__(self, tag_to_word=None):
        self.tag_to_word = {} if tag_to_word is None else tag_to_word

    def evaluate(self, seq):
        return sum(self.score(None, w) for w in seq.sequences)

    def score(self, seq, word_k):
        return self.tag_to_word.get(word_k.tag0, {}).get(word_k.word, 0)


class SimpleTrigramFeatureScore(BeamScoreFunction):
    """Sum of trained coefficients of the trigram features present in the
    encoder's feature dictionary (`score_funcs.py:102-144`).

    Lowered by ``lowering.lower_scorers`` to a device hash table keyed by
    interned feature tuples; the kernel repeats numpy's pairwise summation
    order over the present features.
    """

    def __init__(self, encoder=None, coefficients=None):
        self.set_encoder(encoder, coefficients)

    def set_encoder(self, encoder, coefficients=None):
        if encoder is None:
            self.num_features = 0
            self.coefficients = None
            self.encoder = None
            return self
        if not encoder.is_trained():
            raise ValueError('Encoder must be trained first')
        self.num_features = len(encoder.feature_dic)
        if coefficients is None:
            coefficients = np.zeros(self.num_features)
        if len(coefficients) != self.num_features:
            raise ValueError('Encoder and coefficients have different size features')
        self.coefficients = coefficients
        self.encoder = encoder
        return self

    def evaluate(self, seq):
        from .beam import Sequence
        partial = Sequence([seq.sequences[0]], 0)
        for word in seq.sequences:
            if word.tag0 == BOS or word.tag0 == EOS:
                continue
            partial = partial.add(word, self.score(partial, word))
        return partial.score

    def score(self, seq, word_k):
        path = seq.sequences
        word_i = path[-2] if len(path) > 1 else None
        idxs = self.encoder.encode_word(word_i, path[-1], word_k)
        if not idxs:
            return 0
        return self.coefficients[np.asarray(idxs, dtype=np.int64)].sum()
