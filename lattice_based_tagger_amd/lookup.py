"""Native lattice builder -- ``lt_lexicon_*`` of include/lattice_lookup.h.

SURVEY.md §8(f) #1.  ``NativeLexicon`` snapshots a reference
``MorphemeDictionary`` (tag -> morph sets in the dictionary's tag order, the
verb / adjective / eomi sets, the lemmatisation rules in their tuple order)
and the ``MorphemeLookup`` parameters (``standalones``, ``max_len``,
``prefer_exact_match``), and builds the begin-indexed lattices of whole
corpora in C++: exactly the lists ``sentence_lookup_as_begin_index(sent,
MorphemeLookup(dictionary))`` returns (`lattice_tagger/dictionary/lookup.py:
212-279, 344-369`), in the same node order.

The one order the Python objects do not carry is the iteration order of the
set ``{word[i:i+2], word[i:i+3]}`` in ``get_lemma_candidates``
(`dictionary/lemmatizer.py:107`), which follows CPython's str hash: the
library reproduces CPython 3.10's SipHash-2-4 str hash and 8-slot set
insertion, keyed by the running interpreter's hash secret (so results match
what the reference does in this process), or by an explicit key (fixtures
made with ``PYTHONHASHSEED=0`` use the zero key).  ``NativeLexicon`` checks
the reproduction against ``hash()`` and real sets when it is built and
raises ``Unsupported`` if it does not hold (another interpreter), so callers
fall back to the Python lookup.
"""

import ctypes as C
import random
import sys

import numpy as np

from . import _capi, _pyobj
from .native_packer import Strings, LatticeDesc, Unsupported, _StrTable, _ptr
from .word import Word


class LexiconDesc(C.Structure):
    _fields_ = [('tag', Strings), ('morph_off', C.c_void_p), ('morph', Strings),
                ('verbs', Strings), ('adjectives', Strings), ('eomis', Strings),
                ('rule_surface', Strings), ('rule_off', C.c_void_p),
                ('rule_stem', Strings), ('rule_eomi', Strings),
                ('standalones', Strings), ('max_len', C.c_int32), ('prefer_exact_match', C.c_int32),
                ('hash_k0', C.c_uint64), ('hash_k1', C.c_uint64)]


class TextDesc(C.Structure):
    _fields_ = [('n_sent', C.c_int32), ('text', C.c_void_p), ('eoj_off', C.c_void_p),
                ('sent_eoj', C.c_void_p), ('chars', C.c_void_p), ('char_off', C.c_void_p)]


class LatticeView(C.Structure):
    _fields_ = [('lattice', LatticeDesc), ('b', C.c_void_p), ('sent_words', C.c_void_p)]


class LatticeColumns(C.Structure):
    _fields_ = [('n_sent', C.c_int32), ('n_words', C.c_int64), ('chars', C.c_void_p), ('char_off', C.c_void_p),
                ('slot_off', C.c_void_p), ('sent_words', C.c_void_p), ('len', C.c_void_p), ('b', C.c_void_p),
                ('e', C.c_void_p), ('is_l', C.c_void_p)]


_SIGS = {
    'lt_lexicon_create': (C.c_int32, [C.c_void_p, C.POINTER(C.c_void_p)]),
    'lt_lexicon_destroy': (C.c_int32, [C.c_void_p]),
    'lt_lexicon_lookup': (C.c_int32, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    'lt_lexicon_lookup_sents': (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int,
                                            C.POINTER(C.c_void_p)]),
    'lt_lattices_view': (C.c_int32, [C.c_void_p, C.POINTER(LatticeView)]),
    'lt_lattices_columns': (C.c_int32, [C.c_void_p, C.POINTER(LatticeColumns)]),
    'lt_lattices_destroy': (C.c_int32, [C.c_void_p]),
    'lt_py_str_hash': (C.c_int64, [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64]),
    'lt_py_set2_second_first': (C.c_int, [C.c_int64, C.c_int64]),
    'lt_lattices_strings': (C.c_int32, [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p,
                                        C.c_int64, C.POINTER(C.c_int64)]),
    'lt_lattices_strings_coded': (C.c_int32, [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p,
                                              C.c_void_p, C.c_int64, C.POINTER(C.c_int64),
                                              C.POINTER(C.c_int64)]),
    'lt_lattices_field_bytes': (C.c_int64, [C.c_void_p, C.c_int]),
}


def _lib():
    lib = _capi.load()
    if not getattr(lib, '_lookup_sigs', False):
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        # short gathers: keep the GIL across them (see _capi.load)
        for name in ('lt_lattices_strings', 'lt_lattices_strings_coded', 'lt_lattices_field_bytes'):
            fn = getattr(lib.held, name)
            fn.restype, fn.argtypes = _SIGS[name]
        lib._lookup_sigs = True
    return lib


def process_hash_key():
    """(k0, k1) of this interpreter's str hash (CPython ``_Py_HashSecret``)."""
    if sys.implementation.name != 'cpython' or sys.hash_info.algorithm != 'siphash24' \
            or sys.hash_info.cutoff != 0:
        raise Unsupported('str hash is not CPython siphash24 without small-string cutoff')
    try:
        sec = (C.c_uint8 * 24).in_dll(C.pythonapi, '_Py_HashSecret')
    except (ValueError, AttributeError) as exc:
        raise Unsupported('interpreter hash secret not accessible') from exc
    raw = bytes(sec)
    return int.from_bytes(raw[0:8], 'little'), int.from_bytes(raw[8:16], 'little')


def _cps(s):
    return np.frombuffer(s.encode('utf-32-le'), dtype=np.uint32) if s else np.zeros(1, np.uint32)


def py_str_hash(s, key):
    """The library's restatement of CPython's hash(s) under ``key``."""
    a = _cps(s)
    return int(_lib().lt_py_str_hash(a.ctypes.data, len(s), key[0], key[1]))


def set2_order(a, b, key):
    """[a, b] or [b, a]: the iteration order of ``{a, b}`` the library assumes."""
    if a == b:
        return [a]
    second = _lib().lt_py_set2_second_first(py_str_hash(a, key), py_str_hash(b, key))
    return [b, a] if second else [a, b]


def self_check(samples=200, seed=0):
    """The library's str hash and two-element set order agree with this
    interpreter's (raises Unsupported otherwise)."""
    key = process_hash_key()
    rng = random.Random(seed)
    alphabets = ['abcxyz', '\xe9\xff\x80', '가나다라마바사아자하했랬', '\U0001F600\U00010000가a']
    for i in range(samples):
        al = alphabets[i % len(alphabets)] + (alphabets[(i + 1) % len(alphabets)] if i % 3 == 0 else '')
        a = ''.join(rng.choice(al) for _ in range(rng.randint(1, 3)))
        b = a + ''.join(rng.choice(al) for _ in range(rng.randint(0, 1)))
        if py_str_hash(a, key) != hash(a):
            raise Unsupported('str hash reproduction differs from hash() for %r' % a)
        if set2_order(a, b, key) != list({a, b}):
            raise Unsupported('set order reproduction differs for %r, %r' % (a, b))


_CHECKED = None


def _check_once():
    global _CHECKED
    if _CHECKED is None:
        try:
            self_check()
            _CHECKED = True
        except Unsupported as exc:
            _CHECKED = exc
    if _CHECKED is not True:
        raise _CHECKED


def _strs(values, what):
    values = list(values)
    if any(type(v) is not str for v in values):
        raise Unsupported('%s: non-string entries' % what)
    try:
        return _StrTable(values)
    except Unsupported as exc:
        raise Unsupported('%s: %s' % (what, exc))


class NativeLexicon:
    """C++ snapshot of a reference MorphemeDictionary + MorphemeLookup.

    ``dictionary``   object with ``tag_to_morphs`` (dict tag -> set of str),
                     ``verbs`` / ``adjectives`` / ``eomis`` and ``rules``
                     (dict surface -> sequence of (stem, eomi)), as the
                     reference ``MorphemeDictionary`` (`dictionary.py:287-302`)
    ``standalones``, ``max_len``, ``prefer_exact_match``: the MorphemeLookup's
    ``hash_key``     (k0, k1) whose str hash orders lemmatizer.py:107's set;
                     None = this interpreter's (checked against hash())
    """

    def __init__(self, dictionary, standalones, max_len, prefer_exact_match=True, hash_key=None):
        self.lib = _lib()
        if hash_key is None:
            _check_once()
            hash_key = process_hash_key()
        t2m = dictionary.tag_to_morphs
        if not isinstance(t2m, dict):
            raise Unsupported('tag_to_morphs is not a dict')
        tags = list(t2m.keys())
        if any(type(t) is not str for t in tags):
            raise Unsupported('non-string tag')
        if len(tags) > 64:
            raise Unsupported('more than 64 tags')
        morphs, off = [], [0]
        for t in tags:
            ms = t2m[t]
            morphs.extend(ms)
            off.append(len(morphs))
        rules = getattr(dictionary, 'rules', None)
        if not isinstance(rules, dict):
            raise Unsupported('rules is not a dict')
        rsurf, roff, rstem, reomi = [], [0], [], []
        for surf, pairs in rules.items():
            if type(surf) is not str:
                raise Unsupported('non-string rule surface')
            for pair in pairs:
                if not (isinstance(pair, tuple) and len(pair) == 2):
                    raise Unsupported('rule entries must be (stem, eomi) pairs')
                rstem.append(pair[0])
                reomi.append(pair[1])
            rsurf.append(surf)
            roff.append(len(rstem))
        if any(type(t) is not str for t in standalones):
            raise Unsupported('non-string standalone tag')
        keep = [_strs(tags, 'tags'), np.asarray(off, dtype=np.int64), _strs(morphs, 'morphs'),
                _strs(dictionary.verbs, 'verbs'), _strs(dictionary.adjectives, 'adjectives'),
                _strs(dictionary.eomis, 'eomis'), _strs(rsurf, 'rule surfaces'),
                np.asarray(roff, dtype=np.int64), _strs(rstem, 'rule stems'), _strs(reomi, 'rule eomis'),
                _strs(standalones, 'standalones')]
        desc = LexiconDesc(keep[0].c(), _ptr(keep[1]), keep[2].c(), keep[3].c(), keep[4].c(),
                           keep[5].c(), keep[6].c(), _ptr(keep[7]), keep[8].c(), keep[9].c(),
                           keep[10].c(), int(max_len), 1 if prefer_exact_match else 0,
                           int(hash_key[0]), int(hash_key[1]))
        h = C.c_void_p()
        _capi.check(self.lib.lt_lexicon_create(C.byref(desc), C.byref(h)))
        self.handle = h
        self.fingerprint = dictionary_fingerprint(dictionary)

    @classmethod
    def from_lookup(cls, eojeol_lookup, hash_key=None):
        """From a reference ``MorphemeLookup`` (`lookup.py:99-121`)."""
        if getattr(eojeol_lookup, 'flatten', False):
            raise Unsupported('flatten=True lookups')
        return cls(eojeol_lookup.dictionary, list(eojeol_lookup.standalones), eojeol_lookup.max_len,
                   eojeol_lookup.prefer_exact_match, hash_key=hash_key)

    def lookup(self, sents, n_threads=0):
        """NativeLattices of ``sents`` (str each).  The sentences travel as one
        UTF-32 buffer; the library splits the eojeols (``sent.split()``) and
        drops the spaces (``sent.replace(' ', '')``) on its threads."""
        sents = sents if type(sents) is list else list(sents)
        for s in sents:
            if type(s) is not str:
                raise Unsupported('sentences must be str')
        try:
            raw = ''.join(sents).encode('utf-32-le')
        except UnicodeEncodeError:
            raise Unsupported('text not encodable')
        text = np.frombuffer(raw, dtype=np.uint32) if raw else np.zeros(1, np.uint32)
        off = np.zeros(len(sents) + 1, dtype=np.int64)
        if sents:
            np.cumsum(np.fromiter(map(len, sents), dtype=np.int64, count=len(sents)), out=off[1:])
        h = C.c_void_p()
        _capi.check(self.lib.lt_lexicon_lookup_sents(self.handle, text.ctypes.data, off.ctypes.data, len(sents),
                                                     int(n_threads), C.byref(h)))
        return NativeLattices(self.lib, h)

    def close(self):
        if self.handle:
            self.lib.lt_lexicon_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dictionary_fingerprint(dictionary):
    """Cheap change detector of a dictionary's sets (``add`` grows a set in
    place, ``remove_words`` replaces it; `dictionary.py:244-262`)."""
    parts = [id(dictionary.tag_to_morphs)]
    for t, ms in dictionary.tag_to_morphs.items():
        parts += [t, id(ms), len(ms)]
    for name in ('verbs', 'adjectives', 'eomis', 'rules'):
        v = getattr(dictionary, name, None)
        parts += [id(v), len(v) if v is not None else -1]
    return tuple(parts)


def _gather_strings(blob, off, idx):
    """Strings blob[off[i]:off[i+1]] for i in idx (UTF-8), via one gather and
    one decode: the selected byte ranges are joined with NUL separators
    (falling back to per-string slicing when the blob itself holds NULs)."""
    if b'\0' in blob:
        return [blob[int(off[i]):int(off[i + 1])].decode('utf-8') for i in idx.tolist()]
    starts = off[idx]
    lens = off[idx + 1] - starts
    n = idx.size
    total = int(lens.sum())
    src = np.frombuffer(blob, dtype=np.uint8)
    out = np.zeros(total + n, dtype=np.uint8)              # NUL after every string
    dst_start = np.zeros(n, dtype=np.int64)
    np.cumsum(lens[:-1] + 1, out=dst_start[1:])
    if total:
        seg = np.repeat(np.arange(n), lens)
        cum = np.zeros(n, dtype=np.int64)
        np.cumsum(lens[:-1], out=cum[1:])
        within = np.arange(total, dtype=np.int64) - cum[seg]
        out[dst_start[seg] + within] = src[starts[seg] + within]
    return out.tobytes().decode('utf-8').split('\0')[:n]


class SentChars:
    """The sentences' decode characters as a sequence of str, decoded from a
    UTF-32 buffer on access (``cps``, ``off``: the buffer and the sentence
    offsets, for bulk consumers; NativeLattices hands it copies of its own,
    so it stays valid after the lattices are closed)."""

    def __init__(self, cps, off):
        self.cps, self.off = cps, off

    def __len__(self):
        return len(self.off) - 1

    def __getitem__(self, s):
        if isinstance(s, slice):
            return [self[i] for i in range(*s.indices(len(self)))]
        if s < 0:
            s += len(self)
        if not 0 <= s < len(self):
            raise IndexError(s)
        return self.cps[int(self.off[s]):int(self.off[s + 1])].tobytes().decode('utf-32-le')

    def __iter__(self):
        for s in range(len(self)):
            yield self[s]


class NativeLattices:
    """Lattices built by the library: columnar (``desc`` for lt_packer_pack)
    plus lazy ``Word`` materialisation and the reference-shaped ``bindex``."""

    def __init__(self, lib, handle):
        self.lib, self.handle = lib, handle
        c = LatticeColumns()
        _capi.check(lib.lt_lattices_columns(handle, C.byref(c)))
        S, N = c.n_sent, c.n_words

        def arr(p, ct, n, dt):
            if n == 0 or not p:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(n,))

        self.n_words = N
        self.sent_words = arr(c.sent_words, C.c_int64, S + 1, np.int64)
        self.char_off = arr(c.char_off, C.c_int64, S + 1, np.int64)
        self.slot_off = arr(c.slot_off, C.c_int64, int(self.char_off[-1]) + 1 if S else 1, np.int64)
        # node columns of the compact lattices (int32 / uint8 views, no copies)
        self._ints = {'len': arr(c.len, C.c_int32, N, np.int32), 'b': arr(c.b, C.c_int32, N, np.int32),
                      'e': arr(c.e, C.c_int32, N, np.int32), 'is_l': arr(c.is_l, C.c_uint8, N, np.uint8)}
        self._view = None
        self._cols = None
        # each sentence's characters (sent.replace(' ', '')), decoded on access;
        # copies (4 B per character), so the sequence outlives these lattices
        self.chars = SentChars(arr(c.chars, C.c_uint32, int(self.char_off[-1]) if S else 0, np.uint32).copy(),
                               self.char_off.copy())

    @property
    def desc(self):
        """The lattices as an lt_lattice_desc (UTF-8 columns, built by the
        library on first use: the native packer reads the compact lattices
        directly, lt_packer_pack_lattices)."""
        if self._view is None:
            v = LatticeView()
            _capi.check(self.lib.lt_lattices_view(self.handle, C.byref(v)))
            self._view = v
        return self._view.lattice

    def _int_columns(self):
        """len / b / e / is_l as views of the library's arrays (no copies)."""
        return self._ints

    def _columns(self):
        if self._cols is None:
            d, N = self.desc, self.n_words

            def strs(t):
                if N == 0:
                    return [], None
                off = np.ctypeslib.as_array(C.cast(t.off, C.POINTER(C.c_int64)), shape=(N + 1,))
                blob = C.string_at(t.data, int(off[-1])) if off[-1] else b''
                null = (np.ctypeslib.as_array(C.cast(t.null, C.POINTER(C.c_uint8)), shape=(N,))
                        if t.null else None)
                return (blob, off), null

            self._cols = {'word': strs(d.word), 'morph0': strs(d.morph0), 'morph1': strs(d.morph1),
                          'tag0': strs(d.tag0), 'tag1': strs(d.tag1)}
            self._cols.update(self._ints)
        return self._cols

    def word(self, i):
        """The Word of global node index i (as the reference builds it)."""
        c = self._columns()

        def s(name):
            (blob, off), null = c[name]
            if null is not None and null[i]:
                return None
            return blob[int(off[i]):int(off[i + 1])].decode('utf-8')
        return Word(s('word'), s('morph0'), s('morph1'), s('tag0'), s('tag1'), int(c['len'][i]),
                    int(c['b'][i]), int(c['e'][i]), bool(c['is_l'][i]))

    def __getitem__(self, i):
        return self.word(int(i))

    def words_bulk(self, idx):
        """[Word] of global node indices ``idx`` (int array)."""
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.int64))
        out = [None] * idx.size
        self.words_into(out, np.arange(idx.size, dtype=np.int64), idx)
        return out

    def words_into(self, out, pos, idx):
        """out[pos[i]] = the Word of global node idx[i].  Each string field
        comes back dictionary-coded from one C call (the distinct strings,
        decoded once, plus an int32 code per node), so a path's repeated tags
        and words share str objects; the Word tuples are built in C
        (`_ltpy.words`, csrc/lt_pyobj.c)."""
        self.words_from_coded(out, pos, self.words_coded(idx))

    def words_from_coded(self, out, pos, coded):
        """The object-building half of words_into (holds the GIL)."""
        if coded is None:
            return
        uniqs, codes_all, ints = coded
        _pyobj.load().words(Word, out, np.ascontiguousarray(pos, dtype=np.int64), uniqs, codes_all, ints)

    def words_coded(self, idx):
        """The string-coding half of words_into: every field's distinct
        strings and per-node codes, and the integer fields (C calls that
        release the GIL, numpy gathers; no per-node Python objects), so a
        pipeline can run it on a worker thread ahead of words_from_coded."""
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.int64))
        if idx.size == 0:
            return None
        uniqs, codes_all = [], []
        lib = self.lib                      # (CDLL: the GIL is released during each call)
        # one buffer for the five fields' distinct strings (paths repeat few
        # of them); a field that needs more is coded again into a larger one
        full = max(int(lib.lt_lattices_field_bytes(self.handle, f)) for f in range(5)) + idx.size
        cap = min(full, 1 << 20)
        buf = C.create_string_buffer(cap)
        used, n_u = C.c_int64(), C.c_int64()
        for f, name in enumerate(('word', 'morph0', 'morph1', 'tag0', 'tag1')):
            codes = np.empty(idx.size, dtype=np.int32)
            st = lib.lt_lattices_strings_coded(self.handle, f, idx.ctypes.data, idx.size,
                                               codes.ctypes.data, buf, cap, C.byref(used), C.byref(n_u))
            if st == -1 and used.value > cap:                   # LT_EINVAL: too small
                cap = int(used.value)
                buf = C.create_string_buffer(cap)
                st = lib.lt_lattices_strings_coded(self.handle, f, idx.ctypes.data, idx.size,
                                                   codes.ctypes.data, buf, cap, C.byref(used), C.byref(n_u))
            if st == _capi.LT_EUNSUPPORTED:                     # a NUL inside a string: slice each
                (blob, off), null = self._columns()[name]
                uniqs.append([blob[int(off[i]):int(off[i + 1])].decode('utf-8') for i in idx.tolist()])
                codes = np.arange(idx.size, dtype=np.int32)
                if null is not None:
                    codes[null[idx] != 0] = -1
                codes_all.append(codes)
                continue
            _capi.check(st)
            uniqs.append(C.string_at(buf, used.value).decode('utf-8').split('\0')[:n_u.value])
            codes_all.append(codes)
        ints = self._int_columns()
        isl = (ints['is_l'][idx] != 0).view(np.uint8)
        return (tuple(uniqs), tuple(codes_all),
                tuple(ints[f][idx].astype(np.int64) for f in ('len', 'b', 'e')) + (isl,))

    def empty(self, s):
        """True when sentence s has characters but no node: the reference's
        ``bindex == []`` (`lookup.py:362-363`)."""
        return self.sent_words[s + 1] == self.sent_words[s] and self.char_off[s + 1] > self.char_off[s]

    def bindex(self, s):
        """Sentence s's begin index as the reference returns it."""
        if self.sent_words[s + 1] == self.sent_words[s]:
            return []
        lo, hi = int(self.char_off[s]), int(self.char_off[s + 1])
        return [[self.word(i) for i in range(int(self.slot_off[g]), int(self.slot_off[g + 1]))]
                for g in range(lo, hi)]

    def close(self):
        if self.handle:
            self.lib.lt_lattices_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
