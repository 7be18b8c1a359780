"""Lattice packer: ``bindex`` lists of ``Word`` nodes -> packed CSR batch.

Input is exactly what the reference decoder consumes
(`lattice_tagger/beam/beam.py:5`): per sentence ``bindex`` (a list indexed by
begin character of lists of nodes, as produced by
`dictionary/lookup.py:344-369`) and ``chars``.  Output is the device batch
layout described in DESIGN.md §Data layout:

* nodes of one sentence are stored in *expansion generation order*: local
  node 0 is BOS, then for every end position ``e`` and every begin
  ``b = e-d`` in ascending order (d = max_len..1) the span's candidates in
  ``bindex[b]`` order filtered by ``w.e == e`` (`beam.py:31-33`), or the
  synthesised Unknown node when that filter is empty (`beam.py:36-38`).
* ``span_start[(e-1)*S + (S-d)]`` is the local index of the first node of
  span (e-d, e); entry ``S*n`` closes the sentence.  ``S = span_slots(max_len)``:
  8 up to max_len 8 (the tuned kernels' layout), else max_len (the general
  kernel).  ``max_len`` is first clamped to ``max(8, longest sentence)``: a
  span never exceeds its sentence, so the decode is unchanged (`beam.py:29-30`).
* per node: interned ``word``/``morph0``/``tag0`` ids, the 21-bit
  mask/flag word (``lowering.py``), the node-local score terms and the
  coefficients of the node-local feature classes 4, 5 and 6.
* with ``edge_local`` plugins (``lowering.KIND_EDGE``): one value per lattice
  edge and plugin.  The hypotheses a candidate of span (b, e) extends end in
  the candidates of end position b (beam.py:41: ``beam[b]``), or in BOS for
  b = 0, so its predecessors are the contiguous local nodes
  ``[first(b), first(b+1))``; its values sit at ``edge_val[t][base + j]`` for
  predecessor local node j, ``node_edge_base = base`` (``sent_edge_off``
  delimits each sentence's block).

* several trigram scorers (``LoweredModel.trigrams``): scorer t >= 1's
  pre-filter mask + flags and class 4-6 coefficients of every node in the
  ``xtri_*`` arrays ([n_xtri][n_nodes], lattice_decode.h ABI 6); no implicit
  Unknowns then.

* implicit Unknowns (``implicit_unk``, lattice_decode.h ``n_unk``): the
  synthesised Unknown of a span is not stored as a node when its record
  equals the *canonical* record of its length d -- the record of an Unknown
  whose surface occurs in no key of the model and in no preference table
  (``unknown_records``).  Its span then holds no node, and the decoder takes
  the record from ``unk_*[d-1]``; a path through it reports the negative code
  ``-2 - span_entry`` (``unknown_word`` rebuilds its Word).  Most spans of a
  lattice are such spans.  Not with edge terms or user node-local plugins
  (whose values the canonical record could not stand for).

The packer never reorders candidates: duplicates, ``len != e-b`` nodes and
nodes filed under a begin slot other than their ``b`` field are kept exactly
as the reference would see them.
"""

import struct

import numpy as np

from . import lowering as L
from .tagset import BOS, CONTEXTUAL_TAGS, Unk
from .word import Word, bos_word

MAX_SPAN = 8            # span slots per end position in the tuned kernels' layout
MAX_LEN_ANY = 1 << 20   # LT_MAX_LEN_ANY (include/lattice_decode.h)


def span_slots(max_len):
    """Span slots per end position (csrc/lt_common.h span_slots)."""
    return MAX_SPAN if max_len <= MAX_SPAN else int(max_len)


def effective_max_len(max_len, lengths):
    """``max_len`` clamped to ``max(8, longest sentence)`` -- the same decode
    (a span never exceeds its sentence) with a smaller span table.  Raises
    NotImplementedError below 1 (the caller handles those) or past
    MAX_LEN_ANY."""
    max_len = int(max_len)
    if max_len < 1:
        raise NotImplementedError('max_len < 1 is handled by the caller')
    max_len = min(max_len, max([MAX_SPAN] + [int(n) for n in lengths]))
    if max_len > MAX_LEN_ANY:
        raise NotImplementedError('max_len > %d' % MAX_LEN_ANY)
    return max_len


class PackedBatch:
    """Host arrays of one packed batch (field names follow lt_batch_desc)."""

    def __init__(self, **arrays):
        self.__dict__.update(arrays)

    @property
    def n_sent(self):
        return int(self.sent_n.shape[0])

    @property
    def n_nodes(self):
        return int(self.node_word.shape[0])

    NODE_FIELDS = ('node_word', 'node_morph0', 'node_tag', 'node_mask', 'node_pre', 'node_f4',
                   'node_f5', 'node_f6')
    UNK_FIELDS = ('unk_word', 'unk_morph0', 'unk_tag', 'unk_mask', 'unk_pre', 'unk_f4', 'unk_f5',
                  'unk_f6', 'unk_post')

    XTRI_FIELDS = ('xtri_mask', 'xtri_f4', 'xtri_f5', 'xtri_f6')

    @property
    def n_unk(self):
        return int(getattr(self, 'unk_n', 0))

    @property
    def n_xtri(self):
        return int(getattr(self, 'xtri_n', 0))

    def _xtri_of(self, out, node_sel):
        """The further trigram scorers' node arrays of a sub-batch."""
        out['xtri_n'] = self.n_xtri
        if self.n_xtri:
            for f in self.XTRI_FIELDS:
                out[f] = getattr(self, f)[:, node_sel]

    def _unk_of(self, out):
        """The implicit-Unknown records (batch-wide) into a sub-batch's fields."""
        out['unk_n'] = self.n_unk
        if self.n_unk:
            for f in self.UNK_FIELDS:
                out[f] = getattr(self, f)

    def masks_of(self, s, codes):
        """node_mask of the path codes of sentence s (an implicit Unknown's
        from unk_mask)."""
        codes = np.asarray(codes, dtype=np.int64)
        m = np.asarray(self.node_mask)[self.sent_node_off[s] + np.maximum(codes, 0)]
        neg = codes < 0
        if neg.any():
            S = span_slots(self.max_len)
            m = m.copy()
            m[neg] = np.asarray(self.unk_mask)[S - 1 - ((-2 - codes[neg]) % S)]
        return m

    @property
    def n_edge(self):
        return int(getattr(self, 'edge_terms', 0))

    def _edges_of(self, out, node_sel, sent_sel):
        """Edge arrays of a sub-batch: sentences ``sent_sel`` (their nodes
        ``node_sel``), blocks rebuilt in the new order."""
        out['edge_terms'] = self.n_edge
        out['term_kinds'] = getattr(self, 'term_kinds', 0)
        out['n_terms'] = getattr(self, 'n_terms', 0)
        if not self.n_edge:
            return
        eoff = self.sent_edge_off
        cnt = (eoff[1:] - eoff[:-1])[sent_sel]
        new_off = np.zeros(len(cnt) + 1, dtype=np.int64)
        np.cumsum(cnt, out=new_off[1:])
        seg = np.repeat(np.arange(len(cnt), dtype=np.int64), cnt)
        ei = eoff[:-1][sent_sel][seg] + (np.arange(int(new_off[-1]), dtype=np.int64) - new_off[seg])
        out['edge_val'] = self.edge_val[:, ei]
        out['sent_edge_off'] = new_off
        nodes_per = np.diff(self.sent_node_off)[sent_sel]
        nseg = np.repeat(np.arange(len(cnt), dtype=np.int64), nodes_per)
        out['node_edge_base'] = self.node_edge_base[node_sel] - eoff[:-1][sent_sel][nseg] + new_off[nseg]

    def slice(self, s0, s1):
        """Sentences [s0, s1) as a batch of their own (views; offsets rebased)."""
        n0, n1 = int(self.sent_node_off[s0]), int(self.sent_node_off[s1])
        p0, p1 = int(self.sent_span_off[s0]), int(self.sent_span_off[s1])
        out = dict(max_len=self.max_len, n_post=self.n_post, has_trigram=self.has_trigram,
                   sent_n=self.sent_n[s0:s1],
                   sent_node_off=self.sent_node_off[s0:s1 + 1] - n0,
                   sent_span_off=self.sent_span_off[s0:s1 + 1] - p0,
                   span_start=self.span_start[p0:p1],
                   node_post=self.node_post[:, n0:n1] if self.n_post else np.zeros((0, n1 - n0)))
        for f in self.NODE_FIELDS:
            out[f] = getattr(self, f)[n0:n1]
        self._edges_of(out, np.arange(n0, n1), np.arange(s0, s1))
        self._unk_of(out)
        self._xtri_of(out, slice(n0, n1))
        return PackedBatch(**out)

    # backpointer bytes of one launch: lt_batch_create takes sum_s (n_s + 1) * k
    # 4-byte slots below 2^31 B
    MAX_BP_BYTES = (1 << 31) - 1

    def split(self, max_nodes, k=1):
        """[(s0, s1)] sentence ranges that fit one launch each: at most
        max_nodes nodes and fewer than 2^31 B of beam-k backpointers (a
        single larger sentence gets a range of its own)."""
        S = self.n_sent
        if S == 0:
            return [(0, 0)]
        cuts, s0 = [], 0
        off = self.sent_node_off
        bp = np.zeros(S + 1, dtype=np.int64)
        np.cumsum((np.asarray(self.sent_n, dtype=np.int64) + 1) * (4 * max(int(k), 1)), out=bp[1:])
        while s0 < S:
            s1 = int(np.searchsorted(off, off[s0] + max_nodes, side='right')) - 1
            s1b = int(np.searchsorted(bp, bp[s0] + self.MAX_BP_BYTES, side='right')) - 1
            s1 = min(max(min(s1, s1b), s0 + 1), S)
            cuts.append((s0, s1))
            s0 = s1
        return cuts

    def take(self, order):
        """Sentences ``order`` (indices, repeats allowed) as a new batch, in
        that order (copies; offsets rebuilt)."""
        order = np.asarray(order, dtype=np.int64)
        n_nodes = np.diff(self.sent_node_off)[order]
        n_span = np.diff(self.sent_span_off)[order]
        node_off = np.zeros(len(order) + 1, dtype=np.int64)
        np.cumsum(n_nodes, out=node_off[1:])
        span_off = np.zeros(len(order) + 1, dtype=np.int64)
        np.cumsum(n_span, out=span_off[1:])

        def gather_index(src_off, counts, dst_off):
            total = int(dst_off[-1])
            seg = np.repeat(np.arange(len(order), dtype=np.int64), counts)
            return src_off[order][seg] + (np.arange(total, dtype=np.int64) - dst_off[seg])
        ni = gather_index(self.sent_node_off[:-1], n_nodes, node_off)
        si = gather_index(self.sent_span_off[:-1], n_span, span_off)
        out = dict(max_len=self.max_len, n_post=self.n_post, has_trigram=self.has_trigram,
                   sent_n=self.sent_n[order], sent_node_off=node_off, sent_span_off=span_off,
                   span_start=self.span_start[si],
                   node_post=self.node_post[:, ni] if self.n_post else np.zeros((0, len(ni))))
        for f in self.NODE_FIELDS:
            out[f] = getattr(self, f)[ni]
        self._edges_of(out, ni, order)
        self._unk_of(out)
        self._xtri_of(out, ni)
        return PackedBatch(**out)


def _span_candidates(bindex_b, b, n, max_len):
    """Dict e -> candidates of bindex[b] ending at e, in bindex order."""
    groups = {}
    for w in bindex_b:
        groups.setdefault(w.e, []).append(w)
    return groups


def node_record(model, w, t=0):
    """Device fields of lattice node ``w``: interned word / morph0 / tag ids,
    pre-filter mask + flags, and the coefficients of the node-local feature
    classes 4, 5, 6 (None when absent) -- under trigram scorer t."""
    vocab = model.vocab
    vmask = model.vmasks[t] if t < len(model.vmasks) else model.vmask
    is_unk = w.tag0 == Unk
    wid = vocab.get(w.word, 0)
    mid = vocab.get(w.morph0, 0)
    tid = vocab.get(w.tag0, 0)
    m = L.node_mask_from_vocab(int(vmask[wid]), int(vmask[mid]), int(vmask[tid]))
    if is_unk:
        m |= L.F_UNK
    if w.tag0 in CONTEXTUAL_TAGS:
        m |= L.F_CTX
    c4, c5, c6 = model.node_local_features(w, is_unk, t)
    if c4 is not None:
        m |= L.F_HAS4
    if c5 is not None:
        m |= L.F_HAS5
    if c6 is not None:
        m |= L.F_HAS6
    return wid, mid, tid, m, c4, c5, c6


class _NoString:
    """A surface equal to no value of any key or table (the canonical
    Unknown's, ``unknown_records``)."""
    __slots__ = ()

    def __eq__(self, other):
        return self is other

    def __hash__(self):
        return 0x5EED


_NOSTR = _NoString()
KNOWN_NODE_SCORERS = ('RegularizationScore', 'MorphemePreferenceScore', 'WordPreferenceScore')


def implicit_unk_ok(model):
    """True when the model's Unknown records can stand for each other:
    no edge terms, and node-local terms only from the three built-in scorers
    (whose value for an Unknown depends on its length and on table entries
    for its surface -- which ``_same_record`` then sees)."""
    if getattr(model, 'n_edge', 0) or getattr(model, 'n_xtri', 0):
        return False
    return all(type(f).__name__ in KNOWN_NODE_SCORERS for f in list(model.pre_funcs) + list(model.post_funcs))


def _record(model, w):
    """(wid, mid, tid, mask, pre, f4, f5, f6, post, xtri) of node w, as pack
    stores it; xtri: (mask, f4, f5, f6) under each further trigram scorer."""
    wid, mid, tid, m, c4, c5, c6 = node_record(model, w)
    p, q = model.node_terms(w)
    x = []
    for t in range(1, getattr(model, 'n_xtri', 0) + 1):
        m_t, x4, x5, x6 = node_record(model, w, t)[3:]
        x.append((m_t, 0.0 if x4 is None else x4, 0.0 if x5 is None else x5, 0.0 if x6 is None else x6))
    return (wid, mid, tid, m, float(p), 0.0 if c4 is None else c4, 0.0 if c5 is None else c5,
            0.0 if c6 is None else c6, [float(v) for v in q], x)


def _bits(rec):
    """A record with its floats as bit patterns (exact equality, -0.0 kept)."""
    f = lambda v: struct.pack('<d', v)       # noqa: E731
    return rec[:4] + tuple(f(v) for v in rec[4:8]) + tuple(f(v) for v in rec[8])


def unknown_records(model, S):
    """The canonical implicit-Unknown records of span lengths d = 1..S: the
    record of Word(x, x, None, 'Unknown', None, d, ..., False) for a surface x
    equal to nothing the model holds (id 0, no class-5 feature, no
    preference-table value)."""
    return [_record(model, Word(_NOSTR, _NOSTR, None, Unk, None, d, 0, d, False)) for d in range(1, S + 1)]


def unknown_word(chars, code, S):
    """The Word of the implicit Unknown with path code ``code`` (<= -2) in a
    sentence of characters ``chars`` (beam.py:36-38)."""
    x = -2 - int(code)
    e = x // S + 1
    d = S - x % S
    b = e - d
    sub = chars[b:e]
    return Word(sub, sub, None, Unk, None, d, b, e, False)


class SentNodes(list):
    """Local node -> Word of one packed sentence (``pack``'s node_objects[s]);
    a negative index is a path code of an implicit Unknown (``unknown_word``),
    not Python's from-the-end indexing."""
    __slots__ = ('chars', 'S')

    def __getitem__(self, i):
        if not isinstance(i, slice) and i < 0:
            return unknown_word(self.chars, i, self.S)
        return list.__getitem__(self, i)


def pack(sentences, model, max_len=8, implicit_unk=True):
    """Pack ``sentences`` = iterable of ``(bindex, chars)``.

    Returns ``(PackedBatch, node_objects)`` where ``node_objects[s][i]`` is the
    Python node behind local node ``i`` of sentence ``s`` (the original
    object for dictionary nodes; ``node_objects[s][code]`` for the negative
    path code of an implicit Unknown).  Raises ``IndexError`` for a sentence
    whose ``bindex`` is shorter than its character count, as the reference
    does (`beam.py:32`).  ``implicit_unk``: leave out the Unknowns whose
    record is the canonical one of their length (module docstring).
    """
    sentences = list(sentences)
    max_len = effective_max_len(max_len, [len(chars) for _, chars in sentences])
    S = span_slots(max_len)
    n_post = model.n_post
    n_edge = model.n_edge
    edge_vals = [[] for _ in range(n_edge)]
    edge_base, edge_off = [], [0]
    implicit = bool(implicit_unk) and implicit_unk_ok(model)
    canon = unknown_records(model, S) if implicit else []
    canon_bits = [_bits(r) for r in canon]

    sent_n, node_off, span_off = [], [0], [0]
    span_start = []
    words, morphs, tags, masks = [], [], [], []
    pre, f4, f5, f6 = [], [], [], []
    post = [[] for _ in range(n_post)]
    n_x = getattr(model, 'n_xtri', 0)
    xcols = [([], [], [], []) for _ in range(n_x)]
    node_objects = []

    def add_record(rec):
        wid, mid, tid, m, p, c4, c5, c6, q, x = rec
        for cols, vals in zip(xcols, x):
            for col, v in zip(cols, vals):
                col.append(v)
        words.append(wid)
        morphs.append(mid)
        tags.append(tid)
        masks.append(m)
        pre.append(p)
        f4.append(c4)
        f5.append(c5)
        f6.append(c6)
        for j in range(n_post):
            post[j].append(q[j])

    for bindex, chars in sentences:
        n = len(chars)
        if len(bindex) < n:
            raise IndexError('list index out of range')
        objs = SentNodes([bos_word()])
        objs.chars, objs.S = chars, S
        base = len(words)
        add_record(_record(model, objs[0]))
        groups = [_span_candidates(bindex[b], b, n, max_len) for b in range(n)]
        for e in range(1, n + 1):
            for d in range(S, 0, -1):
                span_start.append(len(objs))
                b = e - d
                if d > max_len or b < 0:
                    continue
                cands = groups[b].get(e)
                if not cands:
                    w = Word(chars[b:e], chars[b:e], None, Unk, None, d, b, e, False)
                    rec = _record(model, w)
                    if implicit and _bits(rec) == canon_bits[d - 1]:
                        continue                            # implicit: no node
                    objs.append(w)
                    add_record(rec)
                    continue
                for w in cands:
                    objs.append(w)
                    add_record(_record(model, w))
        span_start.append(len(objs))
        if n_edge:
            _pack_edges(model, objs, span_start[len(span_start) - S * n - 1:], S, n,
                        edge_vals, edge_base, edge_off)
        sent_n.append(n)
        node_off.append(base + len(objs))
        span_off.append(len(span_start))
        node_objects.append(objs)

    u32 = lambda a: np.asarray(a, dtype=np.uint32)
    i32 = lambda a: np.asarray(a, dtype=np.int32)
    f64 = lambda a: np.asarray(a, dtype=np.float64)
    batch = PackedBatch(
        max_len=max_len, n_post=n_post, has_trigram=int(model.has_trigram),
        sent_n=i32(sent_n), sent_node_off=np.asarray(node_off, dtype=np.int64),
        sent_span_off=np.asarray(span_off, dtype=np.int64),
        span_start=i32(span_start),
        node_word=i32(words), node_morph0=i32(morphs), node_tag=i32(tags),
        node_mask=u32(masks), node_pre=f64(pre), node_f4=f64(f4),
        node_f5=f64(f5), node_f6=f64(f6),
        node_post=f64(post).reshape(n_post, -1) if n_post else np.zeros((0, len(words))),
        edge_terms=n_edge, term_kinds=int(model.term_kinds), n_terms=len(model.plan),
        unk_n=S if implicit else 0, xtri_n=n_x,
    )
    if n_x:
        batch.xtri_mask = u32([c[0] for c in xcols]).reshape(n_x, -1)
        batch.xtri_f4, batch.xtri_f5, batch.xtri_f6 = (f64([c[j] for c in xcols]).reshape(n_x, -1)
                                                        for j in (1, 2, 3))
    if implicit:
        col = lambda i: [r[i] for r in canon]      # noqa: E731
        batch.unk_word, batch.unk_morph0, batch.unk_tag = i32(col(0)), i32(col(1)), i32(col(2))
        batch.unk_mask = u32(col(3))
        batch.unk_pre, batch.unk_f4, batch.unk_f5, batch.unk_f6 = f64(col(4)), f64(col(5)), f64(col(6)), f64(col(7))
        batch.unk_post = (f64([[r[8][j] for r in canon] for j in range(n_post)]).reshape(n_post, S)
                          if n_post else np.zeros((0, S)))
    if n_edge:
        batch.edge_val = f64(edge_vals).reshape(n_edge, -1)
        batch.node_edge_base = np.asarray(edge_base, dtype=np.int64)
        batch.sent_edge_off = np.asarray(edge_off, dtype=np.int64)
    return batch, node_objects


def _pack_edges(model, objs, ss, S, n, edge_vals, edge_base, edge_off):
    """Edge values of one sentence (``objs``: its local nodes; ``ss``: its
    span_start entries, S per end position + the closing one): per local
    node, in node order, one value per predecessor and edge plugin
    (``model.edge_terms``).  Appends to the batch-wide lists."""
    first = [0] + [ss[(e - 1) * S] for e in range(1, n + 1)] + [ss[S * n]]
    pos = edge_off[-1]
    edge_base.append(pos)                       # BOS: no predecessor
    for e in range(1, n + 1):
        for slot in range(S):
            d = S - slot
            b = e - d
            lo_n, hi_n = ss[(e - 1) * S + slot], ss[(e - 1) * S + slot + 1]
            if lo_n == hi_n:
                continue
            lo, hi = (0, 1) if b == 0 else (first[b], first[b + 1])
            for k in range(lo_n, hi_n):
                edge_base.append(pos - lo)
                wk = objs[k]
                for j in range(lo, hi):
                    for t, v in enumerate(model.edge_terms(objs[j], wk)):
                        edge_vals[t].append(float(v))
                pos += hi - lo
    edge_off.append(pos)
