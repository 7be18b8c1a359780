"""Trigram feature schema and encoder.

Mirrors `lattice_tagger/features/feature.py`:

* ``trigram_encoder(wi, wj, wk)`` -- the nine feature classes, in the order
  the scorer sums them (`feature.py:76-121`).
* ``SimpleTrigramEncoder`` -- filters generated features by membership in a
  trained ``feature_dic`` and maps them to coefficient indices
  (`feature.py:31-74`, `_filter` at `:28-29`).

The decoder evaluates this schema on the GPU: classes 0-3, 7 and 8 are probed
in a device hash table per expansion, classes 4-6 depend on one node only and
are resolved once per node while packing (``packer.py``).
"""

from .tagset import CONTEXTUAL_TAGS, Unk

# Number of tuple components after the class id, per feature class.
FEATURE_ARITY = {0: 3, 1: 2, 2: 3, 3: 2, 4: 1, 5: 3, 6: 1, 7: 3, 8: 2}
# Classes whose key depends on the hypothesis (probed in the kernel).
EXPANSION_CLASSES = (0, 1, 2, 3, 7, 8)
# Classes that depend on a single node (resolved per node on the host).
NODE_CLASSES = (4, 5, 6)


def trigram_encoder(word_i, word_j, word_k):
    """Candidate features of appending ``word_k`` after ``(word_i, word_j)``.

    ``word_i`` is None when ``word_j`` is the sentence-start node.
    """
    tj, tk = word_j.tag0, word_k.tag0
    feats = [
        (0, word_j.word, word_k.word, tk),
        (1, word_j.word, tk),
        (2, tj, word_k.word, tk),
        (3, tj, tk),
        (4, word_k.len),
        (5, word_k.word, tk, word_k.is_l),
    ]
    if tj == Unk:
        feats.append((6, min(8, word_j.len)))
    if word_i is not None:
        feats.append((7, word_i.word, word_j.word, word_k.word))
    if tk in CONTEXTUAL_TAGS:
        if tj in CONTEXTUAL_TAGS:
            feats.append((8, word_j.morph0, word_k.morph0))
        elif word_i is not None and word_i.tag0 in CONTEXTUAL_TAGS:
            feats.append((8, word_i.morph0, word_k.morph0))
    return feats


class WordsEncoder:
    """Base class of feature encoders (`feature.py:4-29`)."""

    def __init__(self, feature_dic=None):
        self.feature_dic = feature_dic

    def is_trained(self):
        return self.feature_dic is not None

    def set_feature_dic(self, feature_dic):
        self.feature_dic = feature_dic
        return self

    def encode_sequence(self, words, *args):
        raise NotImplementedError

    def encode_word(self, *args):
        raise NotImplementedError

    def transform_sequence(self, words, *args):
        raise NotImplementedError

    def transform_word(self, *args):
        raise NotImplementedError

    def _filter(self, features):
        dic = self.feature_dic
        return [f for f in features if f in dic]


class SimpleTrigramEncoder(WordsEncoder):
    """Trigram encoder over ``trigram_encoder`` (`feature.py:31-74`)."""

    def encode_sequence(self, words):
        if not self.is_trained():
            raise ValueError('Insert feature_dic first')
        dic = self.feature_dic
        return [[dic[f] for f in feats] for feats in self.transform_sequence(words)]

    def encode_word(self, word_i, word_j, word_k):
        dic = self.feature_dic
        return [dic[f] for f in self.transform_word(word_i, word_j, word_k)]

    def transform_sequence(self, words):
        # words = [BOS, w1, ..., wn, EOS]; one feature list per real word.
        out = []
        for pos in range(1, len(words) - 1):
            wi = words[pos - 2] if pos >= 2 else None
            out.append(self.transform_word(wi, words[pos - 1], words[pos]))
        return out

    def transform_word(self, word_i, word_j, word_k):
        feats = trigram_encoder(word_i, word_j, word_k)
        if self.is_trained():
            feats = self._filter(feats)
        return feats
