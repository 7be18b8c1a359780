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
import os
import threading
import weakref

import numpy as np

from . import _capi, _pyobj
from .lowering import LoweredModel
from .packer import pack, span_slots
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


def _immutable(a):
    """True when no one can write into the array's memory: the array and
    every array it views are read-only and the memory itself is a read-only
    buffer (``bytes``, a read-only ``mmap`` -- a model pack's arrays).  An
    array that owns its memory is never immutable: numpy lets its owner set
    ``flags.writeable`` back to True, edit it, and clear the flag again."""
    while isinstance(a, np.ndarray):
        if a.flags.writeable:
            return False
        a = a.base
    if a is None:
        return False
    try:
        return memoryview(a).readonly
    except TypeError:
        return False


def _digest_array(a):
    """Content digest of a numpy array (in-place edits change it).  An array
    over read-only memory (``_immutable``) cannot change, so its identity
    stands in for the content and the per-call hash of the whole array
    (about 1 ms for 1M coefficients) is skipped; the cached model holds a
    reference to it, so its address cannot be reused while it is cached.
    (``invalidate_model_cache`` drops every lowered model.)"""
    if isinstance(a, np.ndarray) and _immutable(a):
        return ('ro', a.dtype.str, a.shape, a.__array_interface__['data'][0], a.strides, id(a))
    a = np.ascontiguousarray(a)
    try:
        import xxhash
        return (a.dtype.str, a.shape, xxhash.xxh3_64_intdigest(a.data))
    except ImportError:                 # pragma: no cover - xxhash ships with the image
        return (a.dtype.str, a.shape, int(np.bitwise_xor.reduce(a.view(np.uint8).reshape(-1))))


def _digest_table(t):
    """Content digest of a preference table {tag: {string: value}}."""
    try:
        return hash(tuple((tag, id(inner), hash(frozenset(inner.items())) if isinstance(inner, dict) else id(inner))
                          for tag, inner in t.items()))
    except TypeError:                   # unhashable values: identity only
        return id(t)


def _fingerprint(score_functions):
    """Everything the lowered model copies from the composite: the plugin
    objects, the regularisation coefficients, the preference tables'
    contents, the trigram's encoder / feature_dic (identity and size) and the
    coefficient array's contents (the reference reads all of them live on
    every call, score_funcs.py:63-105, 137-144).  A feature_dic edited in
    place without a size change is not detected: call
    ``invalidate_model_cache`` after that."""
    parts = []
    for f in getattr(score_functions, 'funcs', []):
        parts.append(id(f))
        name = type(f).__name__
        if name == 'RegularizationScore':
            parts += [f.unknown_penalty, f.known_preference, f.syllable_penalty,
                      type(f.unknown_penalty), type(f.known_preference), type(f.syllable_penalty)]
        elif name == 'MorphemePreferenceScore':
            parts += [id(f.tag_to_morph), _digest_table(f.tag_to_morph)]
        elif name == 'WordPreferenceScore':
            parts += [id(f.tag_to_word), _digest_table(f.tag_to_word)]
        elif name == 'SimpleTrigramFeatureScore':
            enc = f.encoder
            dic = getattr(enc, 'feature_dic', None)
            coef = f.coefficients
            parts += [id(enc), id(dic), len(dic) if dic is not None else -1, id(coef),
                      _digest_array(coef) if isinstance(coef, np.ndarray) else None]
    return tuple(parts)


def lowered_model(score_functions):
    """LoweredModel of a composite, cached while the composite is unchanged
    (``_fingerprint``).  Call ``invalidate_model_cache`` after editing a
    feature_dic in place."""
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
    """A device context plus the device-resident models it has seen.

    ``Decoder.get(device, slot)``: one per (device ordinal, slot); several
    slots on one device are independent contexts (streams, buffers), which
    is how a multi-device decode is exercised on a one-GPU machine."""

    _instances = {}
    _lock = threading.Lock()

    def __init__(self, device=0, slot=0):
        self.ctx = _capi.Context(device)
        self.device = device
        self.key = (int(device), int(slot))

    @classmethod
    def get(cls, device=0, slot=0):
        key = (int(device), int(slot))
        with cls._lock:
            dec = cls._instances.get(key)
            if dec is None:
                dec = cls._instances[key] = cls(device, slot)
        return dec

    def device_model(self, model):
        dm = model._device_models.get(self.key)
        if dm is None:
            image = getattr(model, 'image', None)           # model pack: no table build
            lib_hash = getattr(self.ctx._lib, 'lt_hash_version', None)
            if image is not None and lib_hash is not None and int(image.get('hash_version', 0)) != int(lib_hash()):
                image = None                                # a pack from another slot hash: rebuild
            if image is None and len(model.keys) and len(model._device_models):
                image = _built_image(model)                 # second device: build the table once
            if image is not None:
                dm = _capi.DeviceModel.from_image(self.ctx, image)
            else:
                dm = _capi.DeviceModel(self.ctx, model.keys, model.coefs)
            model._device_models[self.key] = dm
        return dm

    def upload(self, model, packed, k):
        """The PackedBatch on the device, as [(0, n_sent, DeviceBatch)] (a
        batch of any size: the library decodes it in launch pieces).  Safe
        from a worker thread while this thread's caller decodes
        (lt_batch_create only queues copies on the context's upload
        stream), so uploads overlap decodes."""
        return [(0, packed.n_sent, _capi.DeviceBatch(self.ctx, packed, max_k=k))]

    def decode_packed(self, model, packed, k, uploaded=None):
        """Decode a PackedBatch (or the device batches ``upload`` made of
        it); returns the batch's ``_capi.PackedResults``."""
        dm = self.device_model(model)
        dbs = [db for _, _, db in uploaded] if uploaded is not None else \
            [_capi.DeviceBatch(self.ctx, packed, max_k=k)]
        parts = []
        try:
            for db in dbs:
                parts.append(db.decode_packed(dm, k))
        finally:
            for db in dbs:
                db.close()
        return concat_results(parts)


def concat_results(parts):
    """One PackedResults of consecutive sentence ranges' PackedResults."""
    if len(parts) == 1:
        return parts[0]
    out = _capi.PackedResults.__new__(_capi.PackedResults)
    out.k = parts[0].k
    for f in ('count', 'length', 'score', 'codes'):
        setattr(out, f, np.concatenate([getattr(p, f) for p in parts]))
    out.off = np.zeros(out.length.size + 1, dtype=np.int64)
    np.cumsum(out.length.ravel(), out=out.off[1:])
    return out


def _built_image(model):
    """The model's device image (cuckoo + dense class-3 tables), built once
    on the host and uploaded to each further device without a rebuild."""
    with Decoder._lock:
        image = getattr(model, '_built_image', None)
        if image is None:
            im = _capi.ModelImage(model.keys, model.coefs)
            image = im.arrays()
            im.close()
            model._built_image = image
    return image


def decoders_for(devices):
    """Decoders of a device list; a repeated ordinal gets a context of its
    own (slot 0, 1, ... in order of appearance)."""
    seen = {}
    out = []
    for d in devices:
        d = int(d)
        out.append(Decoder.get(d, seen.get(d, 0)))
        seen[d] = seen.get(d, 0) + 1
    return out


def device_list(device):
    """``device`` as a tuple of ordinals (an int, or a sequence of them)."""
    if isinstance(device, (list, tuple)):
        if not device:
            raise ValueError('devices must not be empty')
        return tuple(int(d) for d in device)
    return (int(device),)


def decode_packed_devices(model, packed, k, devices):
    """Decode a PackedBatch over several devices: sentences
    are independent (beam.py:5-61 keeps no cross-sentence state), so the
    batch is cut into contiguous shards of about equal work -- sum of
    (n_s + 1) * k, ``dist.shard_range`` -- one per device, decoded
    concurrently (one host thread per device; the library calls release the
    GIL) and concatenated in input order.  Returns the batch's
    ``_capi.PackedResults``."""
    from concurrent.futures import ThreadPoolExecutor
    from .dist import shard_range
    decs = decoders_for(devices)
    if len(decs) == 1:
        return decs[0].decode_packed(model, packed, k)
    w = (np.asarray(packed.sent_n, dtype=np.int64) + 1) * k
    ranges = [shard_range(w, len(decs), r) for r in range(len(decs))]
    for dec in decs:                               # tables built before the threads start
        dec.device_model(model)

    def run(r):
        lo, hi = ranges[r]
        return decs[r].decode_packed(model, packed.slice(lo, hi), k)
    with ThreadPoolExecutor(max_workers=len(decs)) as ex:
        parts = list(ex.map(run, range(len(decs))))
    return concat_results(parts)


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
    if k > _capi.LT_MAX_BEAM_ANY:
        raise NotImplementedError('beam_size > %d is not supported' % _capi.LT_MAX_BEAM_ANY)
    return k


def beam_search_batch(sentences, score_functions, beam_size=5, max_len=8, device=0):
    """Decode ``sentences`` = list of ``(bindex, chars)``; returns one list of
    matures per sentence, each as ``beam_search`` returns it.  ``device``: a
    HIP device ordinal, or a sequence of them -- the batch is then split
    into one contiguous shard per entry, decoded concurrently, results in
    input order (``decode_packed_devices``)."""
    sentences = list(sentences)
    k = _check_beam(beam_size)
    model = lowered_model(score_functions)
    if int(max_len) < 1:
        # b_min = e - max_len >= e: no span, no expansion, beam[e] = [] for
        # e >= 1 (beam.py:29-31) and bindex is never read; an empty sentence
        # keeps [BOS] + EOS, which is its decode at any max_len
        out = [[] for _ in sentences]
        empty = [i for i, (_, ch) in enumerate(sentences) if len(ch) == 0]
        if empty:
            for i, m in zip(empty, beam_search_batch([sentences[i] for i in empty], score_functions,
                                                     beam_size, 1, device)):
                out[i] = m
        return out
    packed, objs = pack_lattices(sentences, model, max_len)
    return decode_batch(packed, objs, [ch for _, ch in sentences], model, k, device)


# ---------------------------------------------------------------------------
# score types: the reference's score is a Python sum whose type follows the
# increments -- BOS starts at int 0 (beam.py:21), each increment is
# ((0 + f1) + f2) + ... (score_funcs.py:50-54), the trigram term is int 0 for
# an empty feature set and a numpy.float64 sum otherwise
# (score_funcs.py:141-144), EOS adds int 0 (beam.py:60).  numpy.float64
# absorbs int and float, float absorbs int.
# ---------------------------------------------------------------------------
from .lowering import F_HAS4, F_HAS5  # noqa: E402

_TRI_LOCAL = F_HAS4 | F_HAS5          # a class-4/5 feature of wk: the trigram set is non-empty


def path_score_type(model, path):
    """Type of the reference score of ``path`` (BOS, words...; no EOS) under
    the lowered composite: the increments' values replayed on the host
    (node-local and edge plugins evaluated, trigram presence from the
    encoder), in constructor order (score_funcs.py:50-54)."""
    from .lowering import KIND_EDGE, KIND_TRI, EdgeSequence
    acc = 0
    for q in range(1, len(path)):
        wk, wj = path[q], path[q - 1]
        wi = None if q == 1 else path[q - 2]
        inc = 0
        for f in model.pre_funcs:
            inc = inc + f.score(None, wk)
        for kind, f in model.plan:
            if kind == KIND_TRI:                # (each trigram scorer's own encoder)
                inc = inc + (np.float64(0.0) if f.encoder.encode_word(wi, wj, wk) else 0)
            elif kind == KIND_EDGE:
                inc = inc + f.score(EdgeSequence(wj), wk)
            else:
                inc = inc + f.score(None, wk)
        acc = acc + inc
    return type(acc + 0)


def typed_score(kind, value):
    return kind(value) if kind is not float else float(value)


def score_kinds(model, n_paths, path_masks_any, path_words, need=None):
    """Types of n_paths scores.  ``path_masks_any[p]``: some word of path p
    has a class-4/5 trigram feature (its increment, and so the score, is a
    numpy.float64); the other paths are replayed (``path_words(p)``);
    ``need[p]`` false: not wanted (float)."""
    out = []
    for p in range(n_paths):
        if need is not None and not need[p]:
            out.append(float)
        elif model.trigram is not None and path_masks_any[p]:
            out.append(np.float64)
        else:
            out.append(path_score_type(model, path_words(p)))
    return out


def decode_batch(packed, objs, chars_list, model, k, device=0, best_only=False, uploaded=None,
                 decoder=None):
    """Decode a packed batch and re-materialise the matures: ``objs[s][i]`` is
    the Word of sentence s's local node i, ``chars_list[s]`` its characters.
    ``best_only``: only the best mature of each sentence (what Tagger.tag
    returns, tagger.py:78).  ``uploaded``: ``Decoder.upload``'s device
    batches of ``packed`` (closed here; made by ``decoder``, default
    ``Decoder.get(device)``)."""
    if k == 0:
        for _, _, db in uploaded or ():
            db.close()
        # beam_size=0 keeps no hypothesis past BOS (beam.py:85 slices to [])
        return [[Sequence([bos_word(), eos_word(0)], 0)] if len(ch) == 0 else []
                for ch in chars_list]
    devices = device_list(device)
    if decoder is not None or uploaded is not None or len(devices) == 1:
        dec = decoder if decoder is not None else Decoder.get(devices[0])
        res = dec.decode_packed(model, packed, k, uploaded)
    else:
        res = decode_packed_devices(model, packed, k, devices)
    T = 1 if best_only else k
    if objs and hasattr(objs[0], 'src') and hasattr(objs[0], 'words'):      # native packer's views
        return _materialise_bulk(packed, objs, chars_list, T, res, model)
    count, length, score, codes, off = res.count, res.length, res.score, res.codes, res.off
    out = []
    for s, chars in enumerate(chars_list):
        n = len(chars)
        nodes = objs[s]
        matures = []
        for t in range(min(int(count[s]), T)):
            a = int(off[s * k + t])
            cs = codes[a:a + int(length[s, t])]
            path = [nodes[0]] + [nodes[c] for c in cs]       # (a code <= -2: an implicit Unknown)
            if n > 0:
                hit = bool(np.any(packed.masks_of(s, cs) & _TRI_LOCAL))
                kind = score_kinds(model, 1, [hit], lambda _: path)[0]
                sc = typed_score(kind, score[s, t])
            else:
                sc = 0
            matures.append(Sequence(path + [eos_word(n)], sc, 0))
        out.append(matures)
    return out


def _materialise_bulk(*args):
    """decode_batch's result for lattices packed natively: every path node's
    Word is gathered in bulk (lookup.NativeLattices.words_bulk for native
    lattices, the caller's Word list otherwise).  The cyclic GC
    is paused meanwhile: millions of fresh tuples would otherwise trigger
    repeated full collections (4x the construction time)."""
    return materialise_prepared(prepare_bulk(*args))


def decode_prepared(packed, views, chars_list, model, k, best_only=False, uploaded=None, decoder=None):
    """The first half of decode_batch for natively packed lattices, meant for
    a pipeline's worker thread: the decode (the device; waits release the
    GIL), the path-node indices and the string coding of their Words (numpy
    and C calls, no per-word Python objects).  materialise_prepared builds
    the Sequences from it on the caller's thread."""
    dec = decoder if decoder is not None else Decoder.get(0)
    res = dec.decode_packed(model, packed, k, uploaded)
    return prepare_bulk(packed, views, chars_list, 1 if best_only else k, res, model)


def prepare_bulk(packed, objs, chars_list, T, res, model):
    """Everything of the materialisation but the Python objects (see
    decode_prepared): a dict materialise_prepared consumes."""
    count, length, score, codes, k = res.count, res.length, res.score, res.codes, res.k
    S = len(chars_list)
    n = np.asarray(packed.sent_n, dtype=np.int64)
    t = np.arange(T, dtype=np.int64)
    valid = t[None, :] < np.minimum(count, T)[:, None]                     # S x T
    L = np.where(valid, length[:, :T], 0).astype(np.int64)
    starts = res.off[np.arange(S, dtype=np.int64)[:, None] * k + t[None, :]]
    Lf = L.ravel()
    total = int(Lf.sum())
    seg = np.repeat(np.arange(Lf.size), Lf)
    first = np.zeros(Lf.size, dtype=np.int64)
    np.cumsum(Lf[:-1], out=first[1:])
    within = np.arange(total, dtype=np.int64) - first[seg]
    local = codes[starts.ravel()[seg] + within].astype(np.int64)
    glob = packed.sent_node_off[seg // T] + np.maximum(local, 0)
    src = objs[0].src[glob]
    pmask = np.asarray(packed.node_mask)[glob]
    imp = np.flatnonzero(local < 0)
    if imp.size:
        # implicit Unknowns (path code -2 - span entry): the node source code of
        # their span, -2 - (b << 32 | d - 1), and the canonical mask of d
        S = span_slots(packed.max_len)
        x = -2 - local[imp]
        d = S - x % S
        b = x // S + 1 - d
        src = src.copy()
        src[imp] = -2 - ((b << 32) | (d - 1))
        pmask[imp] = np.asarray(packed.unk_mask)[d - 1]
    lat = objs[0].words
    dic = np.flatnonzero(src >= 0)
    sel = src[dic]
    # native lattices: the strings coded here, the Words built in C later
    coded = lat.words_coded(sel) if dic.size and hasattr(lat, 'words_coded') else None
    unk = np.flatnonzero(src < 0)                      # synthesised Unknown nodes (BOS never on a path)
    return dict(packed=packed, chars_list=chars_list, T=T, model=model, count=count, length=length,
                score=score, n=n, L=L, Lf=Lf, first=first, seg=seg, src=src, pmask=pmask, total=total,
                lat=lat, dic=dic, sel=sel, coded=coded, unk=unk)


def materialise_prepared(prep):
    """The Sequences of prepare_bulk's result (the GIL-holding half: Word
    tuples built in C, paths, typed scores).  The cyclic GC is paused (see
    _materialise_bulk)."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _materialise_prepared_body(**prep)
    finally:
        if enabled:
            gc.enable()


def _materialise_prepared_body(packed, chars_list, T, model, count, length, score, n, L, Lf, first, seg, src,
                               pmask, total, lat, dic, sel, coded, unk):
    ext = _pyobj.load()
    flat = [None] * total
    # native lattices build their Words in C; Word lists hand back the
    # caller's own objects (as the reference's paths hold them)
    if dic.size:
        if coded is not None:
            lat.words_from_coded(flat, dic, coded)
        elif hasattr(lat, 'words_into'):
            lat.words_into(flat, dic, sel)
        else:
            ext.scatter(flat, dic, [lat[i] for i in sel.tolist()])
    if unk.size:
        code = -2 - src[unk]
        if hasattr(chars_list, 'cps'):                  # native lattices: straight from their UTF-32 buffer
            ext.unknowns_cp(Word, flat, unk, chars_list.cps, chars_list.off, seg[unk] // T, code >> 32,
                            (code & 0xFFFFFFFF) + 1, Unk)
        else:
            chars = chars_list if type(chars_list) is list else list(chars_list)
            ext.unknowns(Word, flat, unk, chars, seg[unk] // T, code >> 32, (code & 0xFFFFFFFF) + 1, Unk)
    # the sentinels are immutable tuples: one BOS, one EOS per sentence length
    bos, eos = bos_word(), {}
    vals = _typed_scores(model, pmask, seg, Lf, first, score[:, :T], n, T, bos, flat)
    if T == 1:                                          # best path only (Tagger.tag): paths cut in C
        nl = n.tolist()
        for nch in set(nl):
            eos[nch] = eos_word(nch)
        paths = ext.paths(flat, np.cumsum(L[:, 0]), bos, [eos[nch] for nch in nl],
                          (np.minimum(count, 1) > 0).view(np.uint8))
        return [[Sequence(p, sc, 0)] if p is not None else [] for p, sc in zip(paths, vals)]
    out = []
    pos = 0
    cnt = np.minimum(count, T).tolist()
    Ll = L.tolist()
    for s, nch in enumerate(n.tolist()):
        e = eos.get(nch)
        if e is None:
            e = eos[nch] = eos_word(nch)
        matures = []
        for tt in range(cnt[s]):
            ln = Ll[s][tt]
            matures.append(Sequence([bos] + flat[pos:pos + ln] + [e], vals[s * T + tt], 0))
            pos += ln
        out.append(matures)
    return out


def _typed_scores(model, pmask, seg, Lf, first, score, n, T, bos, flat):
    """Scores of the S x T paths (flattened) with the reference's types
    (path_score_type): numpy.float64 for every path with a class-4/5 trigram
    feature on some word (all of them in a trained model), the rest
    replayed; int 0 for an empty sentence.  ``pmask``: node_mask of every
    path word."""
    P = Lf.size
    hit = np.bincount(seg, weights=(pmask & _TRI_LOCAL) != 0,
                      minlength=P) > 0 if P else np.zeros(0, dtype=bool)
    flat_sc = score.reshape(-1)
    empty = np.repeat(n == 0, T)
    need = Lf > 0                                       # a mature of a non-empty sentence
    if model.trigram is not None and bool(np.all(hit | ~need)):
        vals = list(flat_sc)                            # numpy.float64 scalars
    else:
        kinds = score_kinds(model, P, hit.tolist(),
                            lambda p: [bos] + flat[int(first[p]):int(first[p] + Lf[p])], need.tolist())
        vals = [typed_score(kd, v) for kd, v in zip(kinds, flat_sc.tolist())]
    if empty.any():
        for p in np.flatnonzero(empty).tolist():
            vals[p] = 0
    return vals


def beam_search(bindex, chars, score_functions, beam_size=5, max_len=8, debug=False):
    """Drop-in for the reference ``beam_search`` (`beam.py:5-61`).  With
    ``debug=True`` the growns of every end position are printed as the
    reference prints them (`beam.py:53-57`), from the device trace."""
    if debug:
        debug_dump(bindex, chars, score_functions, beam_size, max_len)
    return beam_search_batch([(bindex, chars)], score_functions, beam_size, max_len)[0]


def debug_dump(bindex, chars, score_functions, beam_size=5, max_len=8, device=0, file=None):
    """Print, for each end position e, every hypothesis grown there -- sorted
    by score, ties in generation order -- exactly as the reference's
    ``debug=True`` branch (`beam.py:53-57`) does.  The expansions and beams
    come from the device trace (``lt_decode_trace``: the decoders' scoring
    code, every expansion kept); paths are rebuilt here from the beams'
    parent links."""
    import sys
    out = file or sys.stdout
    k = _check_beam(beam_size)
    model = lowered_model(score_functions)
    if int(max_len) < 1:                 # no span at any end position (beam.py:29-31)
        for e in range(1, len(chars) + 1):
            print('\n{}\nEnd point = {}, len(growns) = {}\n'.format('-' * 40, e, 0), file=out)
        return
    packed, objs = pack([(bindex, chars)], model, max_len)      # the Word objects, not views
    if len(chars) == 0:
        return
    # beam_size 0 keeps no hypothesis past BOS (beam.py:85 slices to []): the
    # growns of e are BOS's expansions (b = 0), which a beam-1 trace also
    # enumerates with the same scores and order
    kt = max(k, 1)
    dec = Decoder.get(device)
    dm = dec.device_model(model)
    db = _capi.DeviceBatch(dec.ctx, packed, max_k=kt)
    try:
        tr = db.trace(dm, kt)
    finally:
        db.close()
    nodes = objs[0]
    n = len(chars)
    S = span_slots(packed.max_len)
    paths = {(0, 0): (nodes[0],)}
    off = tr['exp_off']
    node_of = lambda v: v & 0x1FFFFF                # noqa: E731  (csrc/lt_common.h bpw_pack)
    span_of = lambda v: ((v >> 21) & 0x1FFFFF) + 1   # noqa: E731
    rank_of = lambda v: v >> 42                      # noqa: E731

    def word_of(v, e):
        # the expansion's word ending at e: a node, or (node field UNK_LOCAL,
        # lt_common.h) the implicit Unknown of its span
        x = node_of(v)
        return nodes[x] if x != 0x1FFFFF else nodes[-2 - ((e - 1) * S + (S - span_of(v)))]

    def path(pos, rank):
        got = paths.get((pos, rank))
        if got is None:
            v = int(tr['exp_link'][off[pos] + tr['beam_gen'][pos, rank]])
            got = path(pos - span_of(v), rank_of(v)) + (word_of(v, pos),)
            paths[(pos, rank)] = got
        return got

    for e in range(1, n + 1):
        a, m = int(off[e]), int(tr['exp_count'][e])
        growns = [g for g in range(m) if not tr['exp_skip'][a + g]
                  and (k > 0 or span_of(int(tr['exp_link'][a + g])) == e)]
        print('\n{}\nEnd point = {}, len(growns) = {}\n'.format('-' * 40, e, len(growns)), file=out)
        sc = tr['exp_score']
        for g in sorted(growns, key=lambda g: -sc[a + g]):      # stable: generation order on ties
            v = int(tr['exp_link'][a + g])
            words = list(path(e - span_of(v), rank_of(v)) + (word_of(v, e),))
            kind = path_score_type(model, words)
            num_unk = 0
            for w in reversed(words[1:]):
                if w.tag0 != Unk:
                    break
                num_unk += 1
            print(Sequence(words, typed_score(kind, sc[a + g]), num_unk), end='\n\n', file=out)
