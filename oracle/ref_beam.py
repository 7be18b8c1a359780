"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the reference decoder.

Restates, over lattice ``Word`` objects (any object with the fields
``word morph0 morph1 tag0 tag1 len b e is_l``):

* ``beam_search``  -- `lattice_tagger/beam/beam.py:5-61` (with ``Beam.append``
  `:83-86` and ``Sequence.add`` `:112-116`)
* the composite score and the four scorers -- `beam/score_funcs.py:50-54,
  65-73, 84-88, 99-100, 137-144`
* the trigram feature schema -- `features/feature.py:76-121` filtered as in
  `:28-29, 57-60, 70-74`
* numpy's pairwise float64 summation used by ``coefficients[idx].sum()``
  (`score_funcs.py:144`; order verified bit-exact on numpy 2.2.6 for 1..11
  terms)

Scorer objects are read through their public attributes only (class name +
parameters), so the oracle works with the reference's scorer classes and with
the build's mirror classes alike, without calling either's ``score``.

Parity is pinned by ``tests/golden/*.json.gz`` (outputs of the reference run
in the survey container); ``tests/test_oracle_golden.py`` checks this module
against them.
"""

CONTEXTUAL = {'Noun', 'Adverb', 'Adjective', 'Verb'}
UNK, NOUN, BOS, EOS = 'Unknown', 'Noun', 'BOS', 'EOS'


class OracleWord(tuple):
    """Minimal node type for synthesised Unknown/BOS/EOS nodes."""
    __slots__ = ()
    _fields = ('word', 'morph0', 'morph1', 'tag0', 'tag1', 'len', 'b', 'e', 'is_l')

    def __new__(cls, *fields):
        return tuple.__new__(cls, fields)

    word = property(lambda s: s[0])
    morph0 = property(lambda s: s[1])
    morph1 = property(lambda s: s[2])
    tag0 = property(lambda s: s[3])
    tag1 = property(lambda s: s[4])
    len = property(lambda s: s[5])
    b = property(lambda s: s[6])
    e = property(lambda s: s[7])
    is_l = property(lambda s: s[8])


def numpy_pairwise_sum(vals):
    """float64 sum in numpy's pairwise order for a contiguous array."""
    m = len(vals)
    if m < 8:
        acc = 0.0
        for v in vals:
            acc += v
        return acc
    r = [float(v) for v in vals[:8]]
    i = 8
    while i < m - (m % 8):
        for j in range(8):
            r[j] += vals[i + j]
        i += 8
    acc = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    while i < m:
        acc += vals[i]
        i += 1
    return acc


def trigram_features(wi, wj, wk):
    """Feature tuples in generation order (`features/feature.py:76-121`)."""
    out = [(0, wj.word, wk.word, wk.tag0), (1, wj.word, wk.tag0),
           (2, wj.tag0, wk.word, wk.tag0), (3, wj.tag0, wk.tag0), (4, wk.len),
           (5, wk.word, wk.tag0, wk.is_l)]
    if wj.tag0 == UNK:
        out.append((6, min(8, wj.len)))
    if wi is not None:
        out.append((7, wi.word, wj.word, wk.word))
    if wk.tag0 in CONTEXTUAL:
        if wj.tag0 in CONTEXTUAL:
            out.append((8, wj.morph0, wk.morph0))
        elif wi is not None and wi.tag0 in CONTEXTUAL:
            out.append((8, wi.morph0, wk.morph0))
    return out


def _scorer_value(func, path, wk):
    name = type(func).__name__
    if name == 'RegularizationScore':                      # score_funcs.py:65-73
        v = 0
        if wk.tag0 == UNK:
            v += func.unknown_penalty * (wk.len + 0.1)
        else:
            v += func.known_preference * wk.len
        if wk.len == 1 and wk.tag0 == NOUN:
            v += func.syllable_penalty
        return v
    if name == 'MorphemePreferenceScore':                  # score_funcs.py:84-88
        t = func.tag_to_morph
        v = t.get(wk.tag0, {}).get(wk.morph0, 0)
        if wk.tag1 is not None:
            v += t.get(wk.tag1, {}).get(wk.morph1, 0)
        return v
    if name == 'WordPreferenceScore':                      # score_funcs.py:99-100
        return func.tag_to_word.get(wk.tag0, {}).get(wk.word, 0)
    if name == 'SimpleTrigramFeatureScore':                # score_funcs.py:137-144
        wi = path[-2] if len(path) > 1 else None
        dic = func.encoder.feature_dic
        idx = [dic[f] for f in trigram_features(wi, path[-1], wk) if f in dic]
        if not idx:
            return 0
        coef = func.coefficients
        return numpy_pairwise_sum([float(coef[i]) for i in idx])
    if getattr(func, 'node_local', False) is True:           # a user plugin: the reference calls it
        return func.score(path, wk)                          # (score_funcs.py:50-54); it reads wk only
    if getattr(func, 'edge_local', False) is True:           # a user plugin of (seq.sequences[-1], wk)
        return func.score(_PathSeq(path), wk)
    raise TypeError('oracle has no restatement of scorer %r' % name)


class _PathSeq:
    """The hypothesis as a plugin sees it (``Sequence.sequences``)."""
    __slots__ = ('sequences',)

    def __init__(self, path):
        self.sequences = path


def composite_increment(funcs, path, wk):
    """``score = 0; score += f(seq, w)`` in constructor order
    (`score_funcs.py:50-54`)."""
    total = 0
    for f in funcs:
        total = total + _scorer_value(f, path, wk)
    return total


def beam_search(bindex, chars, score_functions, beam_size=5, max_len=8):
    """Returns ``[(path, score), ...]`` for the <= beam_size matures, best
    first.  ``path`` is the node list including the BOS and EOS sentinels.
    Follows `beam/beam.py:5-61`."""
    funcs = score_functions.funcs
    n = len(chars)
    bos = OracleWord(BOS, BOS, None, BOS, None, 0, 0, 0, False)
    eos = OracleWord(EOS, EOS, None, EOS, None, 0, n, n, False)
    # hypothesis = (score, path_tuple, num_unk)
    beams = [[(0, (bos,), 0)]]
    for e in range(1, n + 1):
        grown = []
        b_min = max(0, e - max_len)
        for b in range(b_min, e):
            cands = [w for w in bindex[b] if w.e == e]
            if not cands:
                sub = chars[b:e]
                cands = [OracleWord(sub, sub, None, UNK, None, e - b, b, e, False)]
            for score, path, num_unk in beams[b]:
                for w in cands:
                    if num_unk > 0 and w.tag0 == UNK and b_min < b:
                        continue
                    inc = composite_increment(funcs, path, w)
                    grown.append((score + inc, path + (w,),
                                  num_unk + 1 if w.tag0 == UNK else 0))
        # stable sort on -score, keep the first beam_size (beam.py:83-86)
        beams.append(sorted(grown, key=lambda h: -h[0])[:beam_size])
    return [(path + (eos,), score + 0) for score, path, _ in beams[-1]]


def count_ops(bindex, chars, score_functions, beam_size=5, max_len=8):
    """Reference-algorithm operation counts for one sentence: (expansions,
    candidate feature tuples generated by ``trigram_encoder``).  Used by the
    bench's algorithmic-byte model."""
    counter = {'x': 0, 'p': 0}
    funcs = score_functions.funcs
    has_tri = any(type(f).__name__ == 'SimpleTrigramFeatureScore' for f in funcs)
    n = len(chars)
    bos = OracleWord(BOS, BOS, None, BOS, None, 0, 0, 0, False)
    beams = [[(0, (bos,), 0)]]
    for e in range(1, n + 1):
        grown = []
        b_min = max(0, e - max_len)
        for b in range(b_min, e):
            cands = [w for w in bindex[b] if w.e == e]
            if not cands:
                sub = chars[b:e]
                cands = [OracleWord(sub, sub, None, UNK, None, e - b, b, e, False)]
            for score, path, num_unk in beams[b]:
                for w in cands:
                    if num_unk > 0 and w.tag0 == UNK and b_min < b:
                        continue
                    counter['x'] += 1
                    if has_tri:
                        wi = path[-2] if len(path) > 1 else None
                        counter['p'] += len(trigram_features(wi, path[-1], w))
                    inc = composite_increment(funcs, path, w)
                    grown.append((score + inc, path + (w,),
                                  num_unk + 1 if w.tag0 == UNK else 0))
        beams.append(sorted(grown, key=lambda h: -h[0])[:beam_size])
    return counter['x'], counter['p']
