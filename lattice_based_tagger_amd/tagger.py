"""``Tagger`` -- the reference's public tagging API on the GPU decoder.

Mirrors `lattice_tagger/tagger/tagger.py:10-78`:
``Tagger(dictionary, lookup, encoder, score_funcs).tag(sent, beam_size=5,
ensure_normalize=True, debug=False) -> Sequence``.

Lattice construction (dictionary lookup) is outside the accelerated path:
the tagger drives whatever eojeol lookup it is given -- normally the
reference's own ``MorphemeLookup`` (`dictionary/lookup.py:99-132`), which it
builds from a reference ``MorphemeDictionary`` exactly as the reference
``Tagger.__init__`` does (`tagger.py:60`).  The sentence-level grouping into a
begin index restates `lookup.py:7-62` and `:344-369`.  Decoding runs through
``beam_search_batch`` on the device.
"""

import sys

from .beam import beam_search_batch
from .word import bos_word, eos_word


def sentence_lookup(sent, eojeol_lookup):
    """[BOS] + nodes of every eojeol (offset by the characters before it) +
    [EOS] (`lookup.py:52-62`)."""
    n = len(sent.replace(' ', ''))
    nodes = [bos_word()]
    offset = 0
    for eojeol in sent.split():
        nodes += eojeol_lookup(eojeol, offset)
        offset += len(eojeol)
    nodes.append(eos_word(n))
    return nodes


def sentence_lookup_as_begin_index(sent, eojeol_lookup):
    """(nodes, bindex) with bindex[b] = dictionary nodes beginning at b, in
    lookup order; bindex = [] when no eojeol produced a node
    (`lookup.py:357-369`)."""
    n = len(sent.replace(' ', ''))
    nodes = sentence_lookup(sent, eojeol_lookup)
    if len(nodes) <= 2:
        return nodes, []
    bindex = [[] for _ in range(n)]
    for w in nodes[1:-1]:
        bindex[w.b].append(w)
    return nodes, bindex


def _default_lookup(dictionary):
    ref = sys.modules.get('lattice_tagger.dictionary')
    if ref is None:
        try:
            import lattice_tagger.dictionary as ref       # the user's reference install
        except ImportError as exc:
            raise NotImplementedError(
                'no eojeol lookup: pass lookup=<callable(eojeol, offset) -> [Word]> or a '
                'lattice_tagger MorphemeDictionary') from exc
    return ref.MorphemeLookup(dictionary, flatten=False)


class Tagger:
    """Part-of-speech tagger over a morpheme lattice (`tagger.py:10-78`).

    ``dictionary``  a reference ``MorphemeDictionary`` (or the string
                    'base', which builds the reference BaseMorphemeDictionary)
    ``lookup``      optional callable ``(eojeol, offset) -> [Word]``; when not
                    callable the reference MorphemeLookup over ``dictionary``
                    is used, as the reference does
    ``score_funcs`` a ``BeamScoreFunctions`` composite (reference or mirror)
    ``device``      HIP device ordinal of the decoder
    """

    def __init__(self, dictionary='base', lookup='subword_lookup', encoder=None,
                 score_funcs=None, device=0):
        if callable(lookup):
            self.dictionary = dictionary
            self.eojeol_lookup = lookup
        else:
            if isinstance(dictionary, str):
                ref = sys.modules.get('lattice_tagger.dictionary')
                if ref is None:
                    import lattice_tagger.dictionary as ref
                dictionary = ref.BaseMorphemeDictionary()
            self.dictionary = dictionary
            self.eojeol_lookup = _default_lookup(dictionary)
        self.encoder = encoder
        self.score_funcs = score_funcs
        self.device = device

    def lattice(self, sent):
        chars = sent.replace(' ', '')
        _, bindex = sentence_lookup_as_begin_index(sent, self.eojeol_lookup)
        return bindex, chars

    def tag(self, sent, beam_size=5, ensure_normalize=True, debug=False):
        if debug:
            raise NotImplementedError('debug=True is not available from the device decoder')
        return self.tag_batch([sent], beam_size=beam_size)[0]

    def tag_batch(self, sents, beam_size=5):
        """Best ``Sequence`` per sentence, decoded in one device launch.
        Raises IndexError like ``tag`` when a non-empty sentence has no
        dictionary node at all (`beam.py:32`)."""
        lattices = [self.lattice(s) for s in sents]
        matures = beam_search_batch(lattices, self.score_funcs, beam_size=beam_size,
                                    device=self.device)
        return [m[0] for m in matures]
