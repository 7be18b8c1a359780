"""Drop-in ``beam_search`` backed by the MI355X decoder.

Same signature and result type as the reference decoder
``beam_search(bindex, chars, score_functions, beam_size=5, max_len=8,
debug=False)`` (`lattice_tagger/beam/beam.py:5-61`): a list of at most
``beam_size`` ``Sequence`` objects (best first, each ending in EOS).  The
work is done by ``liblt.so``: the scorer composite is lowered once
(``lowering.py``), the lattice is packed (``packer.py``) and decoded on the
GPU by the HIP kernel (``csrc/lt_decode.hip``).

``beam_search_batch`` decodes many sentences in one launch -- the intended
high-throughput entry point.
"""

import gc
import weakref

import os

import numpy as np

from . import _capi
from .lowering import LoweredModel
from .packer import pack
from .tagset import Unk
from .word import Word, bos_word, eos_word

__all__ = ['beam_search', 'beam_search_batch', 'Beam', 'Sequence', 'Decoder']


class Sequence:
    """A hypothesis: node path, score and trailing-unknown count
    (`beam.py:88-116`)."""

    def __init__(self, sequences, score, num_unk=0):
        self.sequences = sequences
        self.score = score
        self.num_unk = num_unk

    def add(self, node, score_increment):
        num_unk = self.num_unk + 1 if node.tag0 == 'Unknown' else 0
        return Sequence(list(self.sequences) + [node], self.score + score_increment, num_unk)

    def __repr__(self):
        body = '\n    '.join(str(w) for w in self.sequences)
        return 'Sequences(\n  words : [\n    {}\n  ]\n  score : {}\n  num unks in tails : {}\n)'.format(
            body, self.score, self.num_unk)

    __str__ = __repr__


class Beam:
    """Per-end-position hypothesis lists (`beam.py:64-86`).  Kept for API
    compatibility; the GPU decoder keeps its beams on the device."""

    def __init__(self, beam=None, k=5):
        self.k = k
        self.beam = beam if beam is not None else []

    def __getitem__(self, index):
        return self.beam[index]

    def append(self, candidates):
        self.beam.append(sorted(candidates, key=lambda x: -x.score)[:self.k])


# ---------------------------------------------------------------------------
# lowered-model cache: one LoweredModel per scorer composite
# ---------------------------------------------------------------------------
_model_cache = weakref.WeakKeyDictionary()


def _fingerprint(score_functions):
    parts = []
    for f in getattr(score_functions, 'funcs', []):
        parts.append(id(f))
        if type(f).__name__ == 'SimpleTrigramFeatureScore':
            enc = f.encoder
            dic = getattr(enc, 'feature_dic', None)
            coef = f.coefficients
            parts += [id(enc), id(dic), len(dic) if dic is not None else -1, id(coef),
                      coef.ctypes.data if isinstance(coef, np.ndarray) else 0]
    return tuple(parts)


def lowered_model(score_functions):
    """LoweredModel of a composite, cached while the composite is unchanged
    (same plugin objects, same feature_dic object and size, same
    coefficient array).  Call ``invalidate_model_cache`` after mutating a
    feature_dic or coefficients in place."""
    fp = _fingerprint(score_functions)
    try:
        hit = _model_cache.get(score_functions)
    except TypeError:
        hit = None
    if hit is not None and hit[0] == fp:
        return hit[1]
    model = LoweredModel(score_functions)
    try:
        _model_cache[score_functions] = (fp, model)
    except TypeError:
        pass
    return model


def invalidate_model_cache():
    _model_cache.clear()


class Decoder:
    """A device context plus the device-resident models it has seen."""

    _instances = {}

    def __init__(self, device=0):
        self.ctx = _capi.Context(device)
        self.device = device

    @classmethod
    def get(cls, device=0):
        dec = cls._instances.get(device)
        if dec is None:
            dec = cls._instances[device] = cls(device)
        return dec

    def device_model(self, model):
        dm = model._device_models.get(self.device)
        if dm is None:
            if getattr(model, 'image', None) is not None:      # model pack: no table build
                dm = _capi.DeviceModel.from_image(self.ctx, model.image)
            else:
                dm = _capi.DeviceModel(self.ctx, model.keys, model.coefs)
            model._device_models[self.device] = dm
        return dm

    # node records per launch (lt_batch_create takes < 2^31 B of 48 B records)
    MAX_NODES = 40_000_000

    def upload(self, model, packed, k):
        """Device batches of a PackedBatch, one per launch piece of at most
        MAX_NODES nodes, as (s0, s1, DeviceBatch).  Safe from a worker thread
        while this thread's caller decodes (lt_batch_create only queues
        copies on the context's stream), so uploads overlap decodes."""
        out = []
        try:
            for s0, s1 in packed.split(self.MAX_NODES):
                piece = packed if (s0, s1) == (0, packed.n_sent) else packed.slice(s0, s1)
                out.append((s0, s1, _capi.DeviceBatch(self.ctx, piece, max_k=k)))
        except BaseException:
            for _, _, db in out:
                db.close()
            raise
        return out

    def decode_packed(self, model, packed, k, uploaded=None):
        """Decode a PackedBatch (in launches of at most MAX_NODES nodes, or
        the pieces ``upload`` made of it); returns (count, length, score,
        codes, cum_n)."""
        dm = self.device_model(model)
        parts = []
        pieces = uploaded if uploaded is not None else packed.split(self.MAX_NODES)
        for piece in pieces:
            if uploaded is not None:
                db = piece[2]
            else:
                s0, s1 = piece
                sub = packed if (s0, s1) == (0, packed.n_sent) else packed.slice(s0, s1)
                db = _capi.DeviceBatch(self.ctx, sub, max_k=k)
            try:
                parts.append(db.decode(dm, k))
            finally:
                db.close()
        if uploaded is not None:
            for _, _, db in uploaded:
                db.close()
        if len(parts) == 1:
            count, length, score, codes = parts[0]
        else:
            count, length, score, codes = (np.concatenate([p[i] for p in parts]) for i in range(4))
        cum_n = np.zeros(packed.n_sent + 1, dtype=np.int64)
        np.cumsum(packed.sent_n, out=cum_n[1:])
        return count, length, score, codes, cum_n


def pack_lattices(sentences, model, max_len):
    """Native packer (``native_packer``) when the model and lattices are
    representable there, else the Python packer -- identical results."""
    if os.environ.get('LT_NATIVE_PACK', '1') != '0':
        from .native_packer import packer_for, Unsupported
        npk = packer_for(model)
        if npk is not None:
            try:
                return npk.pack(sentences, max_len)
            except Unsupported:
                pass
    return pack(sentences, model, max_len)


def _check_beam(beam_size):
    k = int(beam_size)
    if k < 0:
        raise NotImplementedError('negative beam_size is not supported')
    if k > _capi.LT_MAX_BEAM:
        raise NotImplementedError('beam_size > %d is not compiled in' % _capi.LT_MAX_BEAM)
    return k


def beam_search_batch(sentences, score_functions, beam_size=5, max_len=8, device=0):
    """Decode ``sentences`` = list of ``(bindex, chars)``; returns one list of
    matures per sentence, each as ``beam_search`` returns it."""
    sentences = list(sentences)
    k = _check_beam(beam_size)
    model = lowered_model(score_functions)
    packed, objs = pack_lattices(sentences, model, max_len)
    return decode_batch(packed, objs, [ch for _, ch in sentences], model, k, device)


def decode_batch(packed, objs, chars_list, model, k, device=0, best_only=False, uploaded=None):
    """Decode a packed batch and re-materialise the matures: ``objs[s][i]`` is
    the Word of sentence s's local node i, ``chars_list[s]`` its characters.
    ``best_only``: only the best mature of each sentence (what Tagger.tag
    returns, tagger.py:78).  ``uploaded``: ``Decoder.upload``'s device
    batches of ``packed`` (closed here)."""
    if k == 0:
        for _, _, db in uploaded or ():
            db.close()
        # beam_size=0 keeps no hypothesis past BOS (beam.py:85 slices to [])
        return [[Sequence([bos_word(), eos_word(0)], 0)] if len(ch) == 0 else []
                for ch in chars_list]
    count, length, score, codes, cum_n = Decoder.get(device).decode_packed(model, packed, k, uploaded)
    T = 1 if best_only else k
    if objs and hasattr(objs[0], 'src') and hasattr(objs[0], 'words'):      # native packer's views
        return _materialise_bulk(packed, objs, chars_list, k, T, count, length, score, codes, cum_n)
    out = []
    for s, chars in enumerate(chars_list):
        n = len(chars)
        nodes = objs[s]
        base = k * int(cum_n[s])
        matures = []
        for t in range(min(int(count[s]), T)):
            L = int(length[s, t])
            off = base + t * n
            path = [nodes[0]] + [nodes[c] for c in codes[off:off + L]] + [eos_word(n)]
            sc = float(score[s, t]) if n > 0 else 0
            matures.append(Sequence(path, sc, 0))
        out.append(matures)
    return out


def _materialise_bulk(*args):
    """decode_batch's result for lattices packed natively: every path node's
    Word is gathered in bulk (lookup.NativeLattices.words_bulk for native
    lattices, the caller's Word list otherwise).  The cyclic GC
    is paused meanwhile: millions of fresh tuples would otherwise trigger
    repeated full collections (4x the construction time)."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _materialise_bulk_body(*args)
    finally:
        if enabled:
            gc.enable()


def _materialise_bulk_body(packed, objs, chars_list, k, T, count, length, score, codes, cum_n):
    S = len(chars_list)
    n = np.asarray(packed.sent_n, dtype=np.int64)
    t = np.arange(T, dtype=np.int64)
    valid = t[None, :] < np.minimum(count, T)[:, None]                     # S x T
    L = np.where(valid, length[:, :T], 0).astype(np.int64)
    starts = k * cum_n[:-1, None] + t[None, :] * n[:, None]
    Lf = L.ravel()
    total = int(Lf.sum())
    seg = np.repeat(np.arange(Lf.size), Lf)
    first = np.zeros(Lf.size, dtype=np.int64)
    np.cumsum(Lf[:-1], out=first[1:])
    within = np.arange(total, dtype=np.int64) - first[seg]
    local = codes[starts.ravel()[seg] + within].astype(np.int64)
    glob = packed.sent_node_off[seg // T] + local
    src = objs[0].src[glob]
    lat = objs[0].words
    flat = [None] * total
    dic = np.flatnonzero(src >= 0)
    sel = src[dic]
    # native lattices build their Words in bulk; Word lists hand back the
    # caller's own objects (as the reference's paths hold them)
    words = lat.words_bulk(sel) if hasattr(lat, 'words_bulk') else [lat[i] for i in sel.tolist()]
    for j, w in zip(dic.tolist(), words):
        flat[j] = w
    unk = np.flatnonzero(src < 0)                      # synthesised Unknown nodes (BOS never on a path)
    if unk.size:
        code = -2 - src[unk]
        for j, b, d, s in zip(unk.tolist(), (code // 8).tolist(), (code % 8 + 1).tolist(),
                              (seg[unk] // T).tolist()):
            sub = chars_list[s][b:b + d]
            flat[j] = Word(sub, sub, None, Unk, None, d, b, b + d, False)
    # the sentinels are immutable tuples: one BOS, one EOS per sentence length
    bos, eos = bos_word(), {}
    if T == 1:                                          # best path only (Tagger.tag): one comprehension
        nl = n.tolist()
        for nch in set(nl):
            eos[nch] = eos_word(nch)
        L1 = L[:, 0]
        ends = np.cumsum(L1)
        return [[Sequence([bos] + flat[a:z] + [eos[nch]], sc if nch > 0 else 0, 0)] if c else []
                for a, z, nch, c, sc in zip((ends - L1).tolist(), ends.tolist(), nl,
                                            (np.minimum(count, 1) > 0).tolist(), score[:, 0].tolist())]
    out = []
    pos = 0
    cnt = np.minimum(count, T).tolist()
    Ll = L.tolist()
    sc = score.tolist()
    for s, nch in enumerate(n.tolist()):
        e = eos.get(nch)
        if e is None:
            e = eos[nch] = eos_word(nch)
        matures = []
        for tt in range(cnt[s]):
            ln = Ll[s][tt]
            matures.append(Sequence([bos] + flat[pos:pos + ln] + [e], sc[s][tt] if nch > 0 else 0, 0))
            pos += ln
        out.append(matures)
    return out


def beam_search(bindex, chars, score_functions, beam_size=5, max_len=8, debug=False):
    """Drop-in for the reference ``beam_search`` (`beam.py:5-61`)."""
    if debug:
        raise NotImplementedError('debug=True (per-position hypothesis dump) is not available '
                                  'from the device decoder')
    return beam_search_batch([(bindex, chars)], score_functions, beam_size, max_len)[0]
