"""MI355X-native batched lattice decoder with the API of lovit/lattice_based_tagger.

Public surface (mirrors the reference's ``lattice_tagger.beam``,
``lattice_tagger.features`` and ``lattice_tagger.tagger``):

    beam_search, beam_search_batch, Beam, Sequence
    BeamScoreFunction, BeamScoreFunctions, RegularizationScore,
    MorphemePreferenceScore, WordPreferenceScore, SimpleTrigramFeatureScore
    WordsEncoder, SimpleTrigramEncoder, trigram_encoder
    Tagger, Word, tag constants
    evaluate_batch (BeamScoreFunctions.evaluate for many paths on the GPU)
    modelpack (trained-model files: save / load)

Decoding runs in hand-written HIP kernels for gfx950 (``csrc/``) behind the
C-ABI ``include/lattice_decode.h``; see DESIGN.md.
"""

from .tagset import *  # noqa: F401,F403
from .word import Word
from .score_funcs import (BeamScoreFunction, BeamScoreFunctions, RegularizationScore,
                          MorphemePreferenceScore, WordPreferenceScore,
                          SimpleTrigramFeatureScore)
from .feature import WordsEncoder, SimpleTrigramEncoder, trigram_encoder
from .beam import beam_search, beam_search_batch, Beam, Sequence, Decoder
from .tagger import Tagger, sentence_lookup, sentence_lookup_as_begin_index
from .evaluate import evaluate_batch

__version__ = '0.1.0'
