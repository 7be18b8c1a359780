"""The `_ltpy` extension (csrc/lt_pyobj.c) that builds the returned Words and
paths in bulk: equal to the Python constructions it replaces, and refusing
out-of-range input without touching its output list."""

import numpy as np
import pytest

from lattice_based_tagger_amd import _pyobj
from lattice_based_tagger_amd.tagset import Unk
from lattice_based_tagger_amd.word import Word, bos_word, eos_word


@pytest.fixture(scope='module')
def ext():
    return _pyobj.load()


def test_words_equal_python(ext):
    rng = np.random.default_rng(0)
    uniq = (['가', '나다', ''], ['가', '라'], ['이'], ['Noun', 'Verb'], ['Josa'])
    n = 200
    codes = tuple(rng.integers(-1, len(u), size=n).astype(np.int32) for u in uniq)
    ln = rng.integers(1, 9, size=n).astype(np.int64)
    b = rng.integers(0, 300, size=n).astype(np.int64)
    e = b + ln
    isl = rng.integers(0, 2, size=n).astype(np.uint8)
    pos = rng.permutation(n + 5)[:n].astype(np.int64)
    out = ['x'] * (n + 5)
    ext.words(Word, out, pos, uniq, codes, (ln, b, e, isl))
    for i in range(n):
        vals = [None if c[i] < 0 else u[c[i]] for u, c in zip(uniq, codes)]
        exp = Word(*vals, int(ln[i]), int(b[i]), int(e[i]), bool(isl[i]))
        got = out[pos[i]]
        assert type(got) is Word and got == exp and str(got) == str(exp)
        assert type(got.is_l) is bool and type(got.b) is int
    assert sum(o == 'x' for o in out) == 5


def test_unknowns_and_paths(ext):
    chars = ['가나다라', '마바']
    out = [None] * 3
    ext.unknowns(Word, out, np.array([2, 0, 1], np.int64), chars, np.array([0, 1, 0], np.int64),
                 np.array([1, 0, 0], np.int64), np.array([2, 2, 1], np.int64), Unk)
    assert out == [Word('마바', '마바', None, Unk, None, 2, 0, 2, False),
                   Word('가', '가', None, Unk, None, 1, 0, 1, False),
                   Word('나다', '나다', None, Unk, None, 2, 1, 3, False)]
    bos = bos_word()
    eos = [eos_word(4), eos_word(2), eos_word(3)]
    paths = ext.paths(out, np.array([2, 2, 3], np.int64), bos, eos, np.array([1, 0, 1], np.uint8))
    assert paths == [[bos] + out[0:2] + [eos[0]], None, [bos, out[2], eos[2]]]


def test_refusals(ext):
    out = [None] * 2
    with pytest.raises(IndexError):
        ext.words(Word, out, np.array([0, 5], np.int64), ([], [], [], [], []),
                  tuple(np.full(2, -1, np.int32) for _ in range(5)),
                  (np.ones(2, np.int64), np.zeros(2, np.int64), np.ones(2, np.int64), np.zeros(2, np.uint8)))
    with pytest.raises(IndexError):                       # string code past the distinct strings
        ext.words(Word, out, np.array([0, 1], np.int64), (['a'], [], [], [], []),
                  (np.array([0, 1], np.int32),) + tuple(np.full(2, -1, np.int32) for _ in range(4)),
                  (np.ones(2, np.int64), np.zeros(2, np.int64), np.ones(2, np.int64), np.zeros(2, np.uint8)))
    assert out == [None, None]
    with pytest.raises(IndexError):                       # span past the sentence
        ext.unknowns(Word, out, np.array([0], np.int64), ['가'], np.array([0], np.int64),
                     np.array([0], np.int64), np.array([2], np.int64), Unk)
    with pytest.raises(IndexError):
        ext.paths(out, np.array([3], np.int64), bos_word(), [eos_word(1)], np.array([1], np.uint8))
    with pytest.raises(TypeError):
        ext.words(dict, out, np.zeros(0, np.int64), ([],) * 5, (np.zeros(0, np.int32),) * 5,
                  (np.zeros(0, np.int64),) * 3 + (np.zeros(0, np.uint8),))


def test_words_untracked_by_cyclic_gc(ext):
    """Words of str / int / bool / None cannot form cycles; CPython never
    untracks tuple subclasses by itself, so `_ltpy` does (a full collection
    after a 64K-sentence call otherwise walks 1-2 million of them)."""
    import gc
    uniq = (['가'], ['가'], ['이'], ['Noun'], ['Josa'])
    codes = tuple(np.zeros(3, np.int32) for _ in uniq)
    ints = (np.ones(3, np.int64), np.zeros(3, np.int64), np.ones(3, np.int64), np.zeros(3, np.uint8))
    out = [None] * 3
    ext.words(Word, out, np.arange(3, dtype=np.int64), uniq, codes, ints)
    assert not any(gc.is_tracked(w) for w in out)
    # a container field keeps the Word tracked
    uniq_c = (['가'], ['가'], [['x']], ['Noun'], ['Josa'])
    ext.words(Word, out, np.arange(3, dtype=np.int64), uniq_c, codes, ints)
    assert all(gc.is_tracked(w) for w in out)
    unk = [None] * 2
    ext.unknowns(Word, unk, np.arange(2, dtype=np.int64), ['가나다'], np.zeros(2, np.int64),
                 np.array([0, 1], np.int64), np.array([1, 2], np.int64), Unk)
    assert not any(gc.is_tracked(w) for w in unk) and unk[1].word == '나다'
