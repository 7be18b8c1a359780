"""Native (C++) lattice packer -- ``lt_packer_*`` of include/lattice_pack.h.

Same output as ``packer.pack`` (bit-identical arrays, tests/test_native_packer.py)
but the per-node work -- span grouping, Unknown synthesis, interning, the
node-local scorers and feature classes 4-6 -- runs in C++; Python only
flattens the ``Word`` fields into columns.  ``Unsupported`` is raised (and
``beam.beam_search_batch`` falls back to ``packer.pack``) whenever a value
could compare equal under Python semantics in a way the native tables do not
model: non-string words/morphemes/tags, non-integral lengths or end
positions, non-numeric scorer values, non-string preference keys.
"""

import ctypes as C
import math
import numbers

from itertools import chain
from operator import itemgetter

import numpy as np

from . import _capi
from .packer import PackedBatch, span_slots, unknown_word
from .tagset import Unk
from .word import Word, bos_word

KIND = {'RegularizationScore': 0, 'MorphemePreferenceScore': 1, 'WordPreferenceScore': 2}
FIELDS = ('word', 'morph0', 'morph1', 'tag0', 'tag1', 'len', 'b', 'e', 'is_l')     # Word, dictionary.py:169


class Unsupported(Exception):
    """The native packer cannot represent this input exactly."""


class Strings(C.Structure):
    _fields_ = [('data', C.c_void_p), ('off', C.c_void_p), ('null', C.c_void_p), ('n', C.c_int64)]


class PackerDesc(C.Structure):
    _fields_ = [('vocab', Strings), ('vocab_id', C.c_void_p), ('vmask', C.c_void_p),
                ('n_vmask', C.c_int64),
                ('n4', C.c_int64), ('c4_len', C.c_void_p), ('c4_coef', C.c_void_p),
                ('n6', C.c_int64), ('c6_len', C.c_void_p), ('c6_coef', C.c_void_p),
                ('c5_word', Strings), ('c5_tag', Strings), ('c5_isl', C.c_void_p),
                ('c5_coef', C.c_void_p),
                ('n_local', C.c_int32), ('local_kind', C.c_void_p), ('reg_params', C.c_void_p),
                ('n_pre', C.c_int32),
                ('pref_tag', Strings), ('pref_key', Strings), ('pref_scorer', C.c_void_p),
                ('pref_value', C.c_void_p), ('implicit_unk', C.c_int32)]


class LatticeDesc(C.Structure):
    _fields_ = [('n_sent', C.c_int32), ('chars', C.c_void_p), ('char_off', C.c_void_p),
                ('slot_off', C.c_void_p), ('n_words', C.c_int64),
                ('word', Strings), ('morph0', Strings), ('tag0', Strings), ('morph1', Strings),
                ('tag1', Strings), ('len', C.c_void_p), ('e', C.c_void_p), ('is_l', C.c_void_p)]


class Packed(C.Structure):
    _fields_ = [('batch', _capi.BatchDesc), ('node_src', C.c_void_p), ('owner', C.c_void_p)]


class _PackBlock:
    """Owns one lt_packer_pack result; the arrays handed out are views of it
    (numpy bases hold this object), so the block lives as long as any view."""

    def __init__(self, lib, out):
        self.lib, self.out = lib, out

    def view(self, p, ct, n, dt):
        if n == 0 or not p:
            return np.zeros(0, dtype=dt)
        buf = (ct * n).from_address(p)
        buf._block = self
        return np.frombuffer(buf, dtype=dt)

    def __del__(self):
        try:
            self.lib.lt_packed_release(C.byref(self.out))
        except Exception:
            pass


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


class _StrTable:
    """UTF-8 blob + offsets (+ None flags) of a sequence of str / None."""

    def __init__(self, values, nullable=False):
        values = values if isinstance(values, (list, tuple)) else list(values)
        types = set(map(type, values))
        bad = types - ({str, type(None)} if nullable else {str})
        if bad:
            raise Unsupported('non-string values of types %s' % sorted(t.__name__ for t in bad))
        null = None
        if nullable and type(None) in types:
            arr = np.array(values, dtype=object)
            isnull = np.equal(arr, None)
            null = isnull.astype(np.uint8)
            arr[isnull] = ''
            values = arr.tolist()
        elif nullable:
            null = np.zeros(len(values), dtype=np.uint8)
        try:
            enc = list(map(str.encode, values))
        except UnicodeEncodeError:
            raise Unsupported('string not encodable as UTF-8')
        self.blob = np.frombuffer(b''.join(enc) or b'\0', dtype=np.uint8)
        self.off = np.zeros(len(enc) + 1, dtype=np.int64)
        if enc:
            np.cumsum(np.fromiter(map(len, enc), dtype=np.int64, count=len(enc)), out=self.off[1:])
        self.null = null
        self.n = len(enc)

    def c(self):
        return Strings(_ptr(self.blob), _ptr(self.off), _ptr(self.null), self.n)


def _int_column(values, what, none_as=None):
    """int64 array of Python-equality integer values (``none_as`` for values
    equal to no integer, or Unsupported when none_as is None)."""
    if set(map(type, values)) <= {int, bool}:
        return np.fromiter(values, dtype=np.int64, count=len(values))
    out = []
    for v in values:
        x = _int_like(v)
        if x is None:
            if none_as is None:
                raise Unsupported('%s %r is not integral' % (what, v))
            x = none_as
        out.append(x)
    return np.asarray(out, dtype=np.int64)


def _int_like(v):
    """Python-equality integer value of v, or None if v equals no integer."""
    if type(v) is int or type(v) is bool:
        return int(v)
    if isinstance(v, numbers.Integral):
        return int(v)
    if isinstance(v, numbers.Real) and math.isfinite(v) and float(v) == int(v):
        return int(v)
    return None


def _number(v):
    """float of a scorer value; integers must be exact in float64 (Python adds
    them as ints before the final float conversion)."""
    if isinstance(v, numbers.Integral):
        if abs(int(v)) > 2 ** 53:
            raise Unsupported('integer scorer value beyond 2**53')
        return float(v)
    if isinstance(v, numbers.Real):
        return float(v)
    raise Unsupported('non-numeric scorer value %r' % (v,))


class NativePacker:
    """The lowered model in native tables (one per LoweredModel and
    ``implicit_unk`` setting: packer.pack's implicit Unknowns)."""

    def __init__(self, model, implicit_unk=True):
        self.lib = _capi.load()
        keep = []
        vocab = [(v, i) for v, i in model.vocab.items() if type(v) is str]
        vt = _StrTable([v for v, _ in vocab])
        vid = np.asarray([i for _, i in vocab], dtype=np.int32)
        vmask = np.ascontiguousarray(model.vmask, dtype=np.uint32)
        # node-local feature classes 4, 5, 6: {(cls, *comps): coef}
        c4, c5, c6 = {}, {}, {}
        if model.local is not None:
            items = model.local.items()
        elif model.feature_dic is not None:
            coef = model.coefficients
            items = ((f, float(coef[i])) for f, i in model.feature_dic.items()
                     if isinstance(f, tuple) and f and f[0] in (4, 5, 6) and type(f[0]) is not bool)
        else:
            items = ()
        for f, cf in items:
            cls = f[0]
            if cls in (4, 6) and len(f) == 2:
                v = _int_like(f[1])
                if v is not None:
                    (c4 if cls == 4 else c6).setdefault(v, cf)
            elif cls == 5 and len(f) == 4:
                w, t, isl = f[1], f[2], _int_like(f[3])
                if type(w) is str and type(t) is str and isl is not None:
                    c5.setdefault((w, t, isl), cf)
        self.c4 = (np.asarray(list(c4), dtype=np.int64), np.asarray(list(c4.values()), dtype=np.float64))
        self.c6 = (np.asarray(list(c6), dtype=np.int64), np.asarray(list(c6.values()), dtype=np.float64))
        c5k = list(c5)
        c5w, c5t = _StrTable([k[0] for k in c5k]), _StrTable([k[1] for k in c5k])
        c5i = np.asarray([k[2] for k in c5k], dtype=np.int64)
        c5c = np.asarray(list(c5.values()), dtype=np.float64)
        if getattr(model, 'edge_funcs', None):      # edge_local plugins: Python, per lattice edge
            raise Unsupported('edge_local scorers are evaluated per edge in Python')
        if getattr(model, 'n_xtri', 0):             # several trigram scorers: per-scorer node arrays
            raise Unsupported('several trigram scorers are packed by the Python packer')
        # node-local scorers in constructor order
        funcs = list(model.pre_funcs) + list(model.post_funcs)
        kinds, reg, ptag, pkey, pscorer, pval = [], [], [], [], [], []
        for s, f in enumerate(funcs):
            name = type(f).__name__
            if name not in KIND:                    # a node-local plugin of the user's: Python packer
                raise Unsupported('scorer %s is evaluated per node in Python' % name)
            kinds.append(KIND[name])
            if name == 'RegularizationScore':
                reg += [_number(f.unknown_penalty), _number(f.known_preference), _number(f.syllable_penalty)]
                continue
            reg += [0.0, 0.0, 0.0]
            table = f.tag_to_morph if name == 'MorphemePreferenceScore' else f.tag_to_word
            for tag, inner in table.items():
                if type(tag) is not str:
                    raise Unsupported('non-string preference tag %r' % (tag,))
                for key, val in inner.items():
                    if type(key) is not str:
                        raise Unsupported('non-string preference key %r' % (key,))
                    ptag.append(tag)
                    pkey.append(key)
                    pscorer.append(s)
                    pval.append(_number(val))
        kinds = np.asarray(kinds, dtype=np.int32)
        reg = np.asarray(reg, dtype=np.float64)
        pt, pk = _StrTable(ptag), _StrTable(pkey)
        ps = np.asarray(pscorer, dtype=np.int32)
        pv = np.asarray(pval, dtype=np.float64)
        keep += [vt, vid, vmask, c5w, c5t, c5i, c5c, kinds, reg, pt, pk, ps, pv, self.c4, self.c6]
        desc = PackerDesc(vt.c(), _ptr(vid), _ptr(vmask), vmask.size,
                          self.c4[0].size, _ptr(self.c4[0]), _ptr(self.c4[1]),
                          self.c6[0].size, _ptr(self.c6[0]), _ptr(self.c6[1]),
                          c5w.c(), c5t.c(), _ptr(c5i), _ptr(c5c),
                          len(funcs), _ptr(kinds), _ptr(reg), len(model.pre_funcs),
                          pt.c(), pk.c(), _ptr(ps), _ptr(pv), 1 if implicit_unk else 0)
        h = C.c_void_p()
        _capi.check(self.lib.lt_packer_create(C.byref(desc), C.byref(h)))
        self.handle = h
        self.model = model

    def pack(self, sentences, max_len=8):
        """-> (PackedBatch, node views) as packer.pack."""
        chars_l, slots = [], []
        for bindex, chars in sentences:
            n = len(chars)
            if len(bindex) < n:
                raise IndexError('list index out of range')
            if type(chars) is not str:
                raise Unsupported('chars must be a str')
            chars_l.append(chars)
            slots.append(bindex if len(bindex) == n else bindex[:n])
        # begin slots and their words flattened at C speed
        slot_lists = list(chain.from_iterable(slots))
        words = list(chain.from_iterable(slot_lists))
        char_off = np.zeros(len(chars_l) + 1, dtype=np.int64)
        np.cumsum(np.fromiter(map(len, chars_l), dtype=np.int64, count=len(chars_l)), out=char_off[1:])
        slot_off = np.zeros(len(slot_lists) + 1, dtype=np.int64)
        np.cumsum(np.fromiter(map(len, slot_lists), dtype=np.int64, count=len(slot_lists)),
                  out=slot_off[1:])
        text = ''.join(chars_l)
        try:
            cps = np.frombuffer(text.encode('utf-32-le'), dtype=np.uint32) if text else np.zeros(1, np.uint32)
        except UnicodeEncodeError:
            raise Unsupported('chars not encodable')
        # Word fields as columns: tuple-like Words (namedtuples in field order
        # word, morph0, morph1, tag0, tag1, len, b, e, is_l) transpose at C speed
        if words and len(set(map(type, words))) == 1 and isinstance(words[0], tuple) \
                and getattr(type(words[0]), '_fields', None) == FIELDS:
            # (itemgetter per field: 3x faster than the transpose zip(*words))
            cw, cm, cm1, ct, ct1, cl, ce, ci = (list(map(itemgetter(f), words)) for f in (0, 1, 2, 3, 4, 5, 7, 8))
        else:
            get = lambda f: [getattr(w, f) for w in words]
            cw, cm, cm1, ct, ct1, cl, ce, ci = (get('word'), get('morph0'), get('morph1'), get('tag0'),
                                                get('tag1'), get('len'), get('e'), get('is_l'))
        lens = _int_column(cl, 'len')
        isl = _int_column(ci, 'is_l')
        ends = _int_column(ce, 'e', none_as=-1)
        tw, tm, tt = _StrTable(cw), _StrTable(cm), _StrTable(ct)
        tm1, tt1 = _StrTable(cm1, nullable=True), _StrTable(ct1, nullable=True)
        desc = LatticeDesc(len(chars_l), _ptr(cps), _ptr(char_off), _ptr(slot_off), len(words),
                           tw.c(), tm.c(), tt.c(), tm1.c(), tt1.c(), _ptr(lens), _ptr(ends), _ptr(isl))
        return self.pack_desc(desc, words, chars_l, max_len)

    def pack_desc(self, desc, words, chars_l, max_len=8):
        """Pack columnar lattices (an lt_lattice_desc, e.g. the native lattice
        builder's); ``words[i]`` materialises global node i, ``chars_l`` are
        the sentences' characters.  -> (PackedBatch, node views)."""
        out = Packed()
        _capi.check(self.lib.lt_packer_pack(self.handle, C.byref(desc), int(max_len), C.byref(out)))
        return self._result(out, words, chars_l)

    def pack_lattices(self, lat, max_len=8):
        """pack_desc of the native lattice builder's lattices (lookup.NativeLattices),
        read in their compact form (lt_packer_pack_lattices): the same arrays
        without building the lattices' UTF-8 columns."""
        out = Packed()
        _capi.check(self.lib.lt_packer_pack_lattices(self.handle, lat.handle, int(max_len), C.byref(out)))
        return self._result(out, lat, lat.chars)

    def _result(self, out, words, chars_l):
        block = _PackBlock(self.lib, out)       # no copies: the arrays are views of the pack
        b = out.batch
        N, S, nspan, npost = b.n_nodes, b.n_sent, b.n_span, b.n_post
        arr = block.view
        batch = PackedBatch(
            max_len=int(b.max_len), n_post=int(npost), has_trigram=int(self.model.has_trigram),
            sent_n=arr(b.sent_n, C.c_int32, S, np.int32),
            sent_node_off=arr(b.sent_node_off, C.c_int64, S + 1, np.int64),
            sent_span_off=arr(b.sent_span_off, C.c_int64, S + 1, np.int64),
            span_start=arr(b.span_start, C.c_int32, nspan, np.int32),
            node_word=arr(b.node_word, C.c_int32, N, np.int32),
            node_morph0=arr(b.node_morph0, C.c_int32, N, np.int32),
            node_tag=arr(b.node_tag, C.c_int32, N, np.int32),
            node_mask=arr(b.node_mask, C.c_uint32, N, np.uint32),
            node_pre=arr(b.node_pre, C.c_double, N, np.float64),
            node_f4=arr(b.node_f4, C.c_double, N, np.float64),
            node_f5=arr(b.node_f5, C.c_double, N, np.float64),
            node_f6=arr(b.node_f6, C.c_double, N, np.float64),
            node_post=(arr(b.node_post, C.c_double, npost * N, np.float64).reshape(npost, N)
                       if npost else np.zeros((0, N))),
        )
        nu = int(b.n_unk)
        batch.unk_n = nu
        if nu:                                  # implicit Unknowns (lattice_decode.h n_unk)
            batch.unk_word = arr(b.unk_word, C.c_int32, nu, np.int32)
            batch.unk_morph0 = arr(b.unk_morph0, C.c_int32, nu, np.int32)
            batch.unk_tag = arr(b.unk_tag, C.c_int32, nu, np.int32)
            batch.unk_mask = arr(b.unk_mask, C.c_uint32, nu, np.uint32)
            batch.unk_pre = arr(b.unk_pre, C.c_double, nu, np.float64)
            batch.unk_f4 = arr(b.unk_f4, C.c_double, nu, np.float64)
            batch.unk_f5 = arr(b.unk_f5, C.c_double, nu, np.float64)
            batch.unk_f6 = arr(b.unk_f6, C.c_double, nu, np.float64)
            batch.unk_post = (arr(b.unk_post, C.c_double, npost * nu, np.float64).reshape(npost, nu)
                              if npost else np.zeros((0, nu)))
        src = arr(out.node_src, C.c_int64, N, np.int64)
        if S == 0:
            batch.sent_node_off = np.zeros(1, np.int64)
            batch.sent_span_off = np.zeros(1, np.int64)
        return batch, _Views(src, batch.sent_node_off, words, chars_l, span_slots(int(b.max_len)))

    def close(self):
        if self.handle:
            self.lib.lt_packer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Views:
    """Per-sentence node views of a pack (sentence s -> _NodeView), made on
    access: ``views[s][i]`` is the Word of sentence s's local node i."""

    def __init__(self, src, node_off, words, chars_l, S=8):
        self.src, self.node_off, self.words, self.chars_l = src, node_off, words, chars_l
        self.S = S

    def __len__(self):
        return len(self.node_off) - 1

    def __getitem__(self, s):
        if s < 0:
            s += len(self)
        if not 0 <= s < len(self):
            raise IndexError(s)
        return _NodeView(self.src, int(self.node_off[s]), int(self.node_off[s + 1]), self.words, self.chars_l, s,
                         self.S)

    def __iter__(self):
        for s in range(len(self)):
            yield self[s]


class _NodeView:
    """Lazy local-node -> Word object of one sentence (as packer.pack's lists;
    a negative index is the path code of an implicit Unknown)."""

    def __init__(self, src, lo, hi, words, chars_l, s, S=8):
        self.src, self.lo, self.hi, self.words = src, lo, hi, words
        self._chars_l, self._s, self.S = chars_l, s, S

    @property
    def chars(self):
        return self._chars_l[self._s]

    def __len__(self):
        return self.hi - self.lo

    def __getitem__(self, i):
        i = int(i)
        if i <= -2:
            return unknown_word(self.chars, i, self.S)
        if not 0 <= i < self.hi - self.lo:
            raise IndexError(i)
        v = int(self.src[self.lo + i])
        if v >= 0:
            return self.words[v]
        if v == -1:
            return bos_word()
        code = -2 - v
        b, d = code >> 32, (code & 0xFFFFFFFF) + 1
        sub = self.chars[b:b + d]
        return Word(sub, sub, None, Unk, None, d, b, b + d, False)


def packer_for(model, implicit_unk=True):
    """The model's NativePacker (cached on the LoweredModel), or None when
    the model cannot be represented natively."""
    cache = model.__dict__.setdefault('_native_packers', {})
    key = bool(implicit_unk)
    np_ = cache.get(key, False)
    if np_ is False:
        try:
            np_ = NativePacker(model, key)
        except Unsupported:
            np_ = None
        cache[key] = np_
    return np_
