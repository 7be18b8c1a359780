"""Native lattice builder (include/lattice_lookup.h, lookup.NativeLexicon)
against the reference's own lattices.

* tests/golden/lookup.json.gz (made by make_golden.py with the reference's
  MorphemeLookup, PYTHONHASHSEED=0): sentences of the base and demo
  dictionaries, incl. eojeols whose lemma candidates depend on the
  {word[i:i+2], word[i:i+3]} set order (lemmatizer.py:107) and edge strings;
  the lattice must equal the reference's field for field, in node order;
* the str-hash / set-order reproduction against this interpreter's hash()
  and real sets (any hash seed);
* threads and batching do not change the lattices.
"""

import gzip
import json
import os
import random
from types import SimpleNamespace

import pytest

from lattice_based_tagger_amd import lookup as LK
from lattice_based_tagger_amd.native_packer import Unsupported

HERE = os.path.dirname(os.path.abspath(__file__))
ZERO_KEY = (0, 0)                      # PYTHONHASHSEED=0 (the fixture's)


def _fixture():
    with gzip.open(os.path.join(HERE, 'golden', 'lookup.json.gz'), 'rt', encoding='utf-8') as f:
        return json.load(f)


def fixture_dictionary(lex):
    """A MorphemeDictionary-shaped object from the fixture's restriction."""
    t2m = {t: set(lex['morphs'][t]) for t in lex['tags']}
    return SimpleNamespace(tag_to_morphs=t2m, verbs=set(lex['verbs']), adjectives=set(lex['adjectives']),
                           eomis=set(lex['eomis']),
                           rules={k: tuple(tuple(p) for p in v) for k, v in lex['rules']})


def fixture_lexicon(entry, key=ZERO_KEY):
    lex = entry['lexicon']
    return LK.NativeLexicon(fixture_dictionary(lex), lex['standalones'], lex['max_len'],
                            lex['prefer_exact_match'], hash_key=key)


@pytest.fixture(scope='module')
def fix():
    return _fixture()


@pytest.mark.parametrize('name', ['base', 'demo'])
def test_lattices_equal_reference(fix, name):
    entry = fix[name]
    lex = fixture_lexicon(entry)
    sents = entry['sentences']
    lat = lex.lookup(sents, n_threads=3)
    for s, (sent, exp) in enumerate(zip(sents, entry['lattices'])):
        got = [[list(w) for w in ws] for ws in lat.bindex(s)]
        assert got == exp, (name, sent)
        for ws in lat.bindex(s):
            for w in ws:
                assert type(w.is_l) is bool and type(w.len) is int
    assert any(lat.empty(s) for s in range(len(sents)))          # 'ㅋㅋㅋ': bindex == []


def test_set_order_matters_and_is_reproduced(fix):
    """The order-sensitive eojeols change lattices under another hash key."""
    entry = fix['base']
    sents = entry['sentences']
    idx = [i for i, s in enumerate(sents) if '겨우나' in s or '누우라고' in s]
    assert idx
    wrong = fixture_lexicon(entry, key=(1, 2)).lookup([sents[i] for i in idx])
    right = fixture_lexicon(entry).lookup([sents[i] for i in idx])
    diff = 0
    for j, i in enumerate(idx):
        assert [[list(w) for w in ws] for ws in right.bindex(j)] == entry['lattices'][i]
        diff += [[list(w) for w in ws] for ws in wrong.bindex(j)] != entry['lattices'][i]
    assert diff > 0


def test_str_hash_and_set_order_match_interpreter():
    key = LK.process_hash_key()
    rng = random.Random(3)
    alph = 'ab\xe9\xff가나했랬우니\U0001F600\U00010000'
    for _ in range(3000):
        a = ''.join(rng.choice(alph) for _ in range(rng.randint(0, 4)))
        b = a + ''.join(rng.choice(alph) for _ in range(rng.randint(0, 2)))
        assert LK.py_str_hash(a, key) == hash(a)
        assert LK.set2_order(a, b, key) == list({a, b})
    LK.self_check()


def test_zero_key_is_hash_seed_zero():
    # CPython with PYTHONHASHSEED=0: hash('a') is fixed
    assert LK.py_str_hash('', ZERO_KEY) == 0
    assert LK.py_str_hash('a', ZERO_KEY) == -7583489610679606711
    assert LK.py_str_hash('가나', ZERO_KEY) == LK.py_str_hash('가나', (0, 0))


def test_threads_and_batching_do_not_change_lattices(fix):
    entry = fix['base']
    lex = fixture_lexicon(entry)
    sents = entry['sentences'] * 3
    one = lex.lookup(sents, n_threads=1)
    many = lex.lookup(sents, n_threads=8)
    for s in range(len(sents)):
        assert one.bindex(s) == many.bindex(s)
    single = lex.lookup([sents[5]])
    assert single.bindex(0) == one.bindex(5)


def test_rejects_what_it_cannot_represent(fix):
    lex = fixture_lexicon(fix['demo'])
    with pytest.raises(Unsupported):
        lex.lookup([b'bytes'])
    d = fixture_dictionary(fix['demo']['lexicon'])
    d.tag_to_morphs['Noun'] = {1, 2}
    with pytest.raises(Unsupported):
        LK.NativeLexicon(d, ['Noun'], 0, hash_key=ZERO_KEY)


def test_tagger_native_lattice_matches_fixture(fix):
    """Tagger.lattice goes through the native builder for a supplied lexicon."""
    from lattice_based_tagger_amd import Tagger
    entry = fix['demo']
    t = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=fixture_lexicon(entry))
    for sent, exp in list(zip(entry['sentences'], entry['lattices']))[:10]:
        bindex, chars = t.lattice(sent)
        assert chars == sent.replace(' ', '')
        assert [[list(w) for w in ws] for ws in bindex] == exp


def test_tagger_raises_index_error_on_empty_lattice(fix):
    """'ㅋㅋㅋ' has no dictionary node: bindex == [] and Tagger.tag raises
    IndexError (lookup.py:362-363, beam.py:32) before any device work."""
    from lattice_based_tagger_amd import Tagger
    entry = fix['base']
    t = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=fixture_lexicon(entry))
    with pytest.raises(IndexError):
        t.tag_batch(['ㅋㅋㅋ'])


def test_words_bulk_equals_word(fix):
    import numpy as np
    entry = fix['demo']
    lat = fixture_lexicon(entry).lookup(entry['sentences'])
    idx = np.random.default_rng(1).integers(0, lat.n_words, 500)
    bulk = lat.words_bulk(idx)
    assert [tuple(w) for w in bulk] == [tuple(lat.word(int(i))) for i in idx]
    assert all(type(w.is_l) is bool for w in bulk)
    assert lat.words_bulk(np.zeros(0, dtype=np.int64)) == []


def test_words_bulk_strings_with_nul():
    """A dictionary word holding a NUL byte cannot travel NUL-separated: the
    coded gather refuses it and words_bulk slices that field instead."""
    import numpy as np
    from types import SimpleNamespace
    d = SimpleNamespace(tag_to_morphs={'Noun': {'a\x00b', 'c'}}, verbs=set(), adjectives=set(),
                        eomis=set(), rules={})
    lex = LK.NativeLexicon(d, [], 3, True, hash_key=ZERO_KEY)
    lat = lex.lookup(['a\x00b c', 'c'])
    idx = np.arange(lat.n_words, dtype=np.int64)
    bulk = lat.words_bulk(idx)
    assert [tuple(w) for w in bulk] == [tuple(lat.word(int(i))) for i in idx]
    assert any('\x00' in w.word for w in bulk)


def test_tagger_ignores_lookup_argument_like_the_reference(fix):
    """The reference Tagger ignores its ``lookup`` argument and always builds
    MorphemeLookup(dictionary) (tagger.py:57-62): a callable passed as
    ``lookup`` is never called and the lattices are the reference's.  The
    build's own extension keyword ``custom_lookup`` does use the callable."""
    from lattice_based_tagger_amd import Tagger
    entry = fix['demo']
    calls = []

    def f(eojeol, offset):
        calls.append(eojeol)
        return []

    with pytest.warns(UserWarning, match='custom_lookup'):   # (the caller is told which keyword uses it)
        t = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lookup=f, lexicon=fixture_lexicon(entry))
    for sent, exp in list(zip(entry['sentences'], entry['lattices']))[:10]:
        bindex, _ = t.lattice(sent)
        assert [[list(w) for w in ws] for ws in bindex] == exp
    assert calls == []
    t2 = Tagger(dictionary=fixture_dictionary(entry['lexicon']), custom_lookup=f)
    sent = entry['sentences'][0]
    assert t2.lattice(sent)[0] == []
    assert calls == sent.split()
    with pytest.raises(TypeError):
        Tagger(dictionary=fixture_dictionary(entry['lexicon']), custom_lookup='not callable')


@pytest.mark.parametrize('name', ['base', 'demo'])
def test_pack_lattices_equals_pack_desc(fix, name):
    """lt_packer_pack_lattices (the compact lattices, strings hashed as code
    points) gives exactly lt_packer_pack's arrays over the UTF-8 columns --
    for composites with and without preference scorers (which read the node
    strings), and for a model whose vocabulary holds some Unknown spans."""
    import numpy as np
    from golden_io import load
    from lattice_based_tagger_amd.beam import lowered_model
    from lattice_based_tagger_amd.native_packer import packer_for
    entry = fix[name]
    sents = list(entry['sentences']) + ['ㅋㅋ 가\t나다', '😀 이것은']
    lat = fixture_lexicon(entry).lookup([s for s in sents if s.split()], n_threads=3)
    seen, models = 0, set()
    for gname in ('base', 'demo', 'scorers'):
        for case in load(gname):
            model = lowered_model(case.funcs)
            if id(model) in models:
                continue
            models.add(id(model))
            npk = packer_for(model)
            if npk is None:
                continue
            a, _ = npk.pack_desc(lat.desc, lat, lat.chars, max_len=8)
            b, _ = npk.pack_lattices(lat, max_len=8)
            for f in ('sent_n', 'sent_node_off', 'sent_span_off', 'span_start', 'node_word', 'node_morph0',
                      'node_tag', 'node_mask'):
                assert np.array_equal(getattr(a, f), getattr(b, f)), (gname, f)
            for f in ('node_pre', 'node_f4', 'node_f5', 'node_f6', 'node_post'):
                assert np.array_equal(np.asarray(getattr(a, f)).view(np.uint64),
                                      np.asarray(getattr(b, f)).view(np.uint64)), (gname, f)
            seen += 1
    assert seen >= 5


def _lookup_textdesc(lex, sents):
    """The lattices through lt_lexicon_lookup with the split done in Python
    (sent.split(), sent.replace(' ', '')) -- the reference's own calls."""
    import ctypes as C
    import numpy as np
    eojs, sent_eoj, chars_l = [], [0], []
    for s in sents:
        e = s.split()
        eojs.extend(e)
        sent_eoj.append(len(eojs))
        chars_l.append(s.replace(' ', ''))

    def cps(strs):
        raw = ''.join(strs).encode('utf-32-le')
        return np.frombuffer(raw, np.uint32) if raw else np.zeros(1, np.uint32)

    def offs(strs):
        o = np.zeros(len(strs) + 1, np.int64)
        np.cumsum([len(x) for x in strs], out=o[1:])
        return o
    text, chars, eoj_off, char_off = cps(eojs), cps(chars_l), offs(eojs), offs(chars_l)
    sent_eoj = np.asarray(sent_eoj, np.int64)
    td = LK.TextDesc(len(sents), text.ctypes.data, eoj_off.ctypes.data, sent_eoj.ctypes.data, chars.ctypes.data,
                     char_off.ctypes.data)
    h = C.c_void_p()
    from lattice_based_tagger_amd import _capi
    _capi.check(lex.lib.lt_lexicon_lookup(lex.handle, C.byref(td), 2, C.byref(h)))
    return LK.NativeLattices(lex.lib, h), chars_l


def test_sentence_split_in_the_library_matches_python(fix):
    """lt_lexicon_lookup_sents splits like str.split() (every str.isspace()
    character) and strips only U+0020 like str.replace(' ', '')."""
    import numpy as np
    entry = fix['base']
    lex = fixture_lexicon(entry)
    spaces = [chr(c) for c in range(0x110000) if chr(c).isspace()]
    assert len(spaces) == 29
    rng = np.random.default_rng(3)
    words = [w for s in entry['sentences'] for w in s.split()][:300] + ['​', 'ㅋ­', '😀']
    sents = []
    for _ in range(200):
        parts = [words[i] for i in rng.integers(0, len(words), rng.integers(1, 6))]
        seps = [''.join(rng.choice(spaces, rng.integers(1, 3))) for _ in parts]
        lead = rng.choice(['', ' ', '\t', '　 '])
        sents.append(lead + ''.join(p + sp for p, sp in zip(parts, seps)))
    sents = [s for s in sents if s.split()]
    a = lex.lookup(sents, n_threads=3)
    b, chars_l = _lookup_textdesc(lex, sents)
    assert list(a.chars) == chars_l
    assert np.array_equal(a.sent_words, b.sent_words) and np.array_equal(a.slot_off, b.slot_off)
    idx = np.arange(a.n_words, dtype=np.int64)
    assert [tuple(w) for w in a.words_bulk(idx)] == [tuple(w) for w in b.words_bulk(idx)]


def test_unknowns_from_code_points_equal_str_slices(fix):
    import numpy as np
    from lattice_based_tagger_amd import _pyobj
    from lattice_based_tagger_amd.tagset import Unk
    from lattice_based_tagger_amd.word import Word
    lat = fixture_lexicon(fix['demo']).lookup(['가나다 라마', '😀a b', 'ㅋ'])
    chars = list(lat.chars)
    assert chars == ['가나다라마', '😀ab', 'ㅋ'] and lat.chars[-1] == 'ㅋ' and lat.chars[0:2] == chars[:2]
    sent = np.array([0, 1, 1, 2], np.int64)
    b = np.array([1, 0, 1, 0], np.int64)
    d = np.array([3, 2, 2, 1], np.int64)
    out1, out2 = [None] * 4, [None] * 4
    pos = np.arange(4, dtype=np.int64)
    ext = _pyobj.load()
    ext.unknowns(Word, out1, pos, chars, sent, b, d, Unk)
    ext.unknowns_cp(Word, out2, pos, lat.chars.cps, lat.chars.off, sent, b, d, Unk)
    assert out1 == out2 and [type(w.word) for w in out2] == [str] * 4
    with pytest.raises(IndexError):
        ext.unknowns_cp(Word, out2, pos[:1], lat.chars.cps, lat.chars.off, sent[2:3], b[:1], np.array([5], np.int64), Unk)
