"""Synthetic lattices and trigram models for the benchmark configurations.

BASELINE.json configs 2-5 decode synthetic sentences with the statistics of
full-dictionary lattices: 20 eojeols of 2-5
characters, about 2.5 dictionary candidates per begin position spread over
spans of 1-8 characters, Unknown fill for empty spans (fan-in about 9 per end
position), 26 % exact-duplicate candidates, 2 % nodes whose ``len`` differs
from their span, tags uniform over the ten POS tags, word/morpheme ids
Zipf(1.1) over a 200K vocabulary.  The trigram model holds the features of
sampled real expansions plus random fill (1M keys at full size), with
N(0, 1) float64 coefficients; the composite is
``RegularizationScore() + SimpleTrigramFeatureScore``.

Two renderings of the same batch:

* ``pack_fast`` -- vectorised numpy, straight to the device batch layout
  (what ``bench.py`` uses; the lattice build is outside the timed region);
* ``to_words`` -- ``(bindex, chars)`` lattices of ``Word`` objects plus a
  ``feature_dic`` over Python tuples, the reference's own input form (used
  by tests on small batches, and by tests/golden/make_golden.py).
"""

import numpy as np

from . import lowering as Lw
from .tagset import POS_TAGS, CONTEXTUAL_TAGS, Noun, Unk, BOS

MAX_SPAN = 8
# probability that span length d (1..8) holds dictionary candidates
SPAN_P = np.array([0.60, 0.42, 0.16, 0.07, 0.04, 0.03, 0.02, 0.02])
EXTRA_LAMBDA = 0.85            # candidates per non-empty span = 1 + Poisson
DUP_RATE = 0.26
LEN_MISMATCH = 0.02


class IdSpace:
    """Interned-id layout of the synthetic vocabulary."""

    def __init__(self, vocab):
        self.vocab = vocab                      # word / morpheme ids 1..vocab
        self.tag0 = vocab + 1                   # POS tag t -> tag0 + t
        self.unk = vocab + 1 + len(POS_TAGS)    # 'Unknown'
        self.bos = vocab + 2 + len(POS_TAGS)    # 'BOS' (word, morph0 and tag of BOS)
        self.size = vocab + 3 + len(POS_TAGS)   # ids are < size

    def tag_id(self, t):
        return self.tag0 + t

    def render(self, vid):
        """Python value of an id (for the Word rendering)."""
        vid = int(vid)
        if 1 <= vid <= self.vocab:
            return 'x%d' % vid
        if self.tag0 <= vid < self.unk:
            return POS_TAGS[vid - self.tag0]
        if vid == self.unk:
            return Unk
        if vid == self.bos:
            return BOS
        raise ValueError(vid)


class RawLattices:
    """Dictionary nodes of S sentences in bindex order (numpy arrays)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _zipf_ids(rng, size, vocab, a):
    # inverse-CDF Zipf over 1..vocab (numpy's zipf is unbounded)
    ranks = np.arange(1, vocab + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -a)
    cdf /= cdf[-1]
    return (np.searchsorted(cdf, rng.random(size)) + 1).astype(np.int32)


def make_lattices(n_sent, seed=0, eojeols=20, eojeol_len=(2, 5), vocab=200_000, zipf_a=1.1,
                  extra_lambda=EXTRA_LAMBDA, dup_rate=DUP_RATE):
    rng = np.random.default_rng(seed)
    S = int(n_sent)
    elen = rng.integers(eojeol_len[0], eojeol_len[1] + 1, size=(S, eojeols), dtype=np.int32)
    sent_n = elen.sum(axis=1).astype(np.int32)
    T = int(sent_n.sum())
    sent_char_off = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(sent_n, out=sent_char_off[1:])
    char_sent = np.repeat(np.arange(S, dtype=np.int32), sent_n)
    char_pos = (np.arange(T, dtype=np.int64) - sent_char_off[char_sent]).astype(np.int32)
    # eojeol starts -> is_l
    starts = np.zeros(T, dtype=bool)
    e_off = np.concatenate([np.zeros((S, 1), np.int64), np.cumsum(elen, axis=1)[:, :-1]], axis=1)
    starts[(sent_char_off[:-1, None] + e_off).ravel()] = True
    chars = rng.integers(0, 11172, size=T, dtype=np.int32)

    # candidates per (char b, span d)
    remain = (sent_n[char_sent] - char_pos)[:, None]
    dd = np.arange(1, MAX_SPAN + 1, dtype=np.int32)[None, :]
    valid = dd <= remain
    nonempty = (rng.random((T, MAX_SPAN)) < SPAN_P[None, :]) & valid
    cnt = np.where(nonempty, 1 + rng.poisson(extra_lambda, size=(T, MAX_SPAN)), 0).astype(np.int32)

    N = int(cnt.sum())
    flat = np.repeat(np.arange(T * MAX_SPAN, dtype=np.int64), cnt.ravel())
    node_char = (flat // MAX_SPAN).astype(np.int64)
    node_d = (flat % MAX_SPAN + 1).astype(np.int32)
    span_first = np.zeros(T * MAX_SPAN + 1, dtype=np.int64)
    np.cumsum(cnt.ravel(), out=span_first[1:])
    idx_in_span = (np.arange(N, dtype=np.int64) - span_first[flat]).astype(np.int32)

    word = _zipf_ids(rng, N, vocab, zipf_a)
    morph = np.where(rng.random(N) < 0.7, word, _zipf_ids(rng, N, vocab, zipf_a)).astype(np.int32)
    tag = rng.integers(0, len(POS_TAGS), size=N, dtype=np.int32)
    length = np.where(rng.random(N) < LEN_MISMATCH,
                      rng.integers(1, 10, size=N, dtype=np.int32), node_d).astype(np.int32)
    is_l = starts[node_char].astype(np.int8)
    # exact duplicates of the span's first candidate
    dup = (idx_in_span > 0) & (rng.random(N) < dup_rate)
    first = span_first[flat]
    for arr in (word, morph, tag, length):
        arr[dup] = arr[first[dup]]

    # bindex order: all candidates of one begin position, shuffled
    key = rng.random(N)
    order = np.lexsort((key, node_char))
    return RawLattices(
        S=S, sent_n=sent_n, sent_char_off=sent_char_off, chars=chars,
        node_char=node_char[order], node_d=node_d[order], word=word[order], morph=morph[order],
        tag=tag[order], length=length[order], is_l=is_l[order], cnt=cnt, char_sent=char_sent,
        char_pos=char_pos, ids=IdSpace(vocab), vocab=vocab)


# ---------------------------------------------------------------------------
# packed layout (ids only) -- mirrors packer.pack on the same lattices
# ---------------------------------------------------------------------------
class FastLayout:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def layout(raw, implicit_unk=False):
    """Packed node order of ``raw`` (dictionary + Unknown nodes) without
    model-dependent columns.  ``implicit_unk``: the Unknowns are implicit
    (packer.py; every synthetic Unknown surface is in no key, so all of them
    are) -- only dictionary nodes are nodes."""
    S, T = raw.S, int(raw.sent_n.sum())
    n = raw.sent_n.astype(np.int64)
    span_base = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(8 * n + 1, out=span_base[1:])
    n_span = int(span_base[-1])
    # span slot of (char b, d): e = b + d, j = 8 - d
    cs = raw.char_sent.astype(np.int64)
    b = raw.char_pos.astype(np.int64)
    d = np.arange(1, MAX_SPAN + 1, dtype=np.int64)[None, :]
    valid = d <= (n[cs] - b)[:, None]
    slot = span_base[cs][:, None] + (b[:, None] + d - 1) * 8 + (8 - d)
    span_count = np.zeros(n_span, dtype=np.int64)
    span_count[slot[valid]] = (raw.cnt if implicit_unk else np.maximum(raw.cnt, 1))[valid]
    # local start of every span = 1 (BOS) + exclusive prefix inside the sentence
    incl = np.cumsum(span_count)
    excl = incl - span_count
    sent_of_span = np.repeat(np.arange(S, dtype=np.int64), 8 * n + 1)
    local = excl - excl[span_base[:-1]][sent_of_span] + 1
    nodes_per_sent = 1 + incl[span_base[1:] - 1] - excl[span_base[:-1]]
    node_off = np.zeros(S + 1, dtype=np.int64)
    np.cumsum(nodes_per_sent, out=node_off[1:])
    NT = int(node_off[-1])

    # dictionary nodes -> packed position
    nsent = cs[raw.node_char]
    nb = b[raw.node_char]
    nd = raw.node_d.astype(np.int64)
    nslot = span_base[nsent] + (nb + nd - 1) * 8 + (8 - nd)
    # rank inside the span in bindex order (raw nodes are in bindex order)
    o = np.argsort(nslot, kind='stable')
    ranks = np.empty(len(o), dtype=np.int64)
    sorted_slot = nslot[o]
    grp_start = np.r_[0, np.flatnonzero(np.diff(sorted_slot)) + 1]
    grp_len = np.diff(np.r_[grp_start, len(o)])
    ranks[o] = np.arange(len(o)) - np.repeat(grp_start, grp_len)
    dict_pos = node_off[nsent] + local[nslot] + ranks

    # Unknown nodes: valid spans without dictionary candidates
    unk_mask = valid & (raw.cnt == 0) & (not implicit_unk)
    uslot = slot[unk_mask]
    usent = np.broadcast_to(cs[:, None], valid.shape)[unk_mask]
    ub = np.broadcast_to(b[:, None], valid.shape)[unk_mask]
    ud = np.broadcast_to(d, valid.shape)[unk_mask]
    unk_pos = node_off[usent] + local[uslot]
    node_b = np.zeros(NT, dtype=np.int64)
    node_b[dict_pos] = nb
    node_b[unk_pos] = ub
    return FastLayout(node_b=node_b, S=S, n=n, span_base=span_base, n_span=n_span,
                      span_start=local.astype(np.int32), node_off=node_off, NT=NT,
                      dict_pos=dict_pos, unk_pos=unk_pos, unk_sent=usent, unk_b=ub, unk_d=ud,
                      bos_pos=node_off[:-1], implicit=bool(implicit_unk))


def node_columns(raw, lay):
    """Per packed node: word, morph0, tag ids, len, is_l, unk flag, b, e."""
    ids = raw.ids
    NT = lay.NT
    word = np.zeros(NT, dtype=np.int32)
    morph = np.zeros(NT, dtype=np.int32)
    tag = np.zeros(NT, dtype=np.int32)
    length = np.zeros(NT, dtype=np.int32)
    is_l = np.zeros(NT, dtype=np.int8)
    unk = np.zeros(NT, dtype=bool)
    p = lay.dict_pos
    word[p] = raw.word
    morph[p] = raw.morph
    tag[p] = ids.tag0 + raw.tag
    length[p] = raw.length
    is_l[p] = raw.is_l
    q = lay.unk_pos
    tag[q] = ids.unk            # Unknown word surfaces occur in no key -> id 0
    length[q] = lay.unk_d
    unk[q] = True
    r = lay.bos_pos
    word[r] = morph[r] = tag[r] = ids.bos
    return word, morph, tag, length, is_l, unk


# ---------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------
class SynthModel:
    """Trigram model in id space.

    keys4: dict len -> coef idx;  keys5: dict (word, tag, is_l) -> idx;
    keys6: dict v -> idx;  probed: uint32 [F, 4] (a, b, c, class) and idx.
    """

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _features_of(raw, lay, cols, k_nodes, j_nodes, i_nodes):
    """Feature rows (cls, a, b, c) of expansions (i, j, k); i = -1 for None."""
    word, morph, tag, length, is_l, unk = cols
    ids = raw.ids
    ctx_tags = np.array([ids.tag0 + POS_TAGS.index(t) for t in CONTEXTUAL_TAGS])
    kw_, kt, km = word[k_nodes], tag[k_nodes], morph[k_nodes]
    jw, jt, jm = word[j_nodes], tag[j_nodes], morph[j_nodes]
    has_i = i_nodes >= 0
    ii = np.where(has_i, i_nodes, 0)
    iw, it, im = word[ii], tag[ii], morph[ii]
    z = np.zeros_like(kw_)
    rows = [np.stack([np.full_like(kw_, 0), jw, kw_, kt], 1),
            np.stack([np.full_like(kw_, 1), jw, kt, z], 1),
            np.stack([np.full_like(kw_, 2), jt, kw_, kt], 1),
            np.stack([np.full_like(kw_, 3), jt, kt, z], 1),
            np.stack([np.full_like(kw_, 7), iw, jw, kw_], 1)[has_i]]
    kc = np.isin(kt, ctx_tags)
    jc = np.isin(jt, ctx_tags)
    ic = np.isin(it, ctx_tags) & has_i
    r8a = kc & jc
    r8b = kc & ~jc & ic
    rows.append(np.stack([np.full_like(kw_, 8), jm, km, z], 1)[r8a])
    rows.append(np.stack([np.full_like(kw_, 8), im, km, z], 1)[r8b])
    probed = np.concatenate(rows, 0)
    probed = probed[(probed[:, 1] != 0) & (probed[:, 2] != 0) &
                    ((probed[:, 3] != 0) | np.isin(probed[:, 0], [1, 3, 8]))]
    f4 = length[k_nodes]
    f5 = np.stack([kw_, kt, is_l[k_nodes].astype(np.int32)], 1)[kw_ != 0]
    f6 = np.minimum(8, length[j_nodes][unk[j_nodes]])
    return probed, f4, f5, f6


def _enc_rows(r):
    """(cls, a, b, c) rows with ids < 2**20 -> one int64 (exact, sortable)."""
    r = r.astype(np.int64)
    return (r[:, 0] << 60) | (r[:, 1] << 40) | (r[:, 2] << 20) | r[:, 3]


def _dec_rows(k):
    m = (1 << 20) - 1
    return np.stack([(k >> 60) & 15, (k >> 40) & m, (k >> 20) & m, k & m], 1)


def make_model(raw, lay=None, cols=None, seed=0, n_features=1_000_000, samples_per_char=0.1,
               fill=True):
    """Features of sampled real expansions + random fill up to n_features
    (sampled over the explicit layout, so the model does not depend on how
    the batch stores its Unknowns)."""
    if lay is None or lay.implicit:
        lay, cols = layout(raw), None
    if cols is None:
        cols = node_columns(raw, lay)
    rng = np.random.default_rng(seed + 7919)
    ids = raw.ids
    n = lay.n
    S = lay.S
    # sample (s, e) positions and a node ending there, then predecessors
    M = int(samples_per_char * n.sum())
    s = rng.integers(0, S, size=M)
    e = (rng.random(M) * n[s]).astype(np.int64) + 1
    def nodes_ending(s_, e_):
        # local node range of end position e_ (>= 1): spans (e_-1)*8 .. e_*8
        lo = lay.span_start[lay.span_base[s_] + (e_ - 1) * 8]
        hi = lay.span_start[lay.span_base[s_] + e_ * 8]
        pick = lo + (rng.random(len(s_)) * (hi - lo)).astype(np.int64)
        return lay.node_off[s_] + pick
    def begin_of(node, s_):
        return lay.node_b[node]
    k_nodes = nodes_ending(s, e)
    kb = begin_of(k_nodes, s)
    j_nodes = np.where(kb > 0, 0, lay.node_off[s])
    has_j = kb > 0
    j_nodes[has_j] = nodes_ending(s[has_j], kb[has_j])
    jb = np.zeros(M, dtype=np.int64)
    jb[has_j] = begin_of(j_nodes[has_j], s[has_j])
    i_nodes = np.full(M, -1, dtype=np.int64)
    i_nodes[has_j] = lay.node_off[s[has_j]]          # wi = BOS when wj starts at 0
    has_i2 = has_j & (jb > 0)
    i_nodes[has_i2] = nodes_ending(s[has_i2], jb[has_i2])
    probed, f4, f5, f6 = _features_of(raw, lay, cols, k_nodes, j_nodes, i_nodes)
    assert raw.ids.size < (1 << 20)
    probed = np.unique(_enc_rows(probed))
    n_local = len(np.unique(f4)) + len(np.unique(f5.astype(np.int64), axis=0)) + len(np.unique(f6))
    for _ in range(8):
        if not fill or n_features - n_local <= len(probed):
            break
        extra = int((n_features - n_local - len(probed)) * 1.15) + 16
        cls = rng.choice(np.array([0, 1, 2, 7, 8]), size=extra)
        wid = lambda: _zipf_ids(rng, extra, ids.vocab, 1.1).astype(np.int64)
        tid = lambda: ids.tag0 + rng.integers(0, len(POS_TAGS), size=extra)
        a = np.where(cls == 2, tid(), wid())
        bb = np.where(cls == 1, tid(), wid())
        c = np.where(np.isin(cls, [0, 2]), tid(), np.where(cls == 7, wid(), 0))
        probed = np.unique(np.concatenate([probed, _enc_rows(np.stack([cls, a, bb, c], 1))]))
    if fill and len(probed) > n_features - n_local:
        keep = np.sort(rng.choice(len(probed), size=max(n_features - n_local, 0), replace=False))
        probed = probed[keep]
    probed = _dec_rows(probed)
    f4u = np.unique(f4)
    f5u = np.unique(f5.astype(np.int64), axis=0)
    f6u = np.unique(f6)
    F = len(probed) + len(f4u) + len(f5u) + len(f6u)
    perm = rng.permutation(F)
    coef = rng.standard_normal(F)
    o = 0
    probed_idx = perm[o:o + len(probed)]; o += len(probed)
    idx4 = perm[o:o + len(f4u)]; o += len(f4u)
    idx5 = perm[o:o + len(f5u)]; o += len(f5u)
    idx6 = perm[o:o + len(f6u)]
    return SynthModel(
        F=F, coef=coef, probed=probed.astype(np.int64), probed_idx=probed_idx,
        keys4={int(v): int(i) for v, i in zip(f4u, idx4)},
        keys5_arr=f5u, idx5=idx5,
        keys6={int(v): int(i) for v, i in zip(f6u, idx6)},
        reg=(-0.1, 0.2, -0.2))


def _reg_terms(length, unk, tag_is_noun, reg):
    """RegularizationScore().score per node, Python arithmetic in float64
    (`score_funcs.py:65-73`): value = 0 + up*(len+0.1) | 0 + kp*len, then
    + sp for a one-syllable Noun."""
    up, kp, sp = reg
    L = length.astype(np.float64)
    v = np.where(unk, 0.0 + up * (L + 0.1), 0.0 + kp * L)
    v = np.where((length == 1) & tag_is_noun, v + sp, v)
    return 0.0 + v          # BeamScoreFunctions: 0 + reg


def pack_fast(raw, model, lay=None, cols=None, implicit_unk=True):
    """Device batch layout for ``raw`` under ``model`` (same arrays packer.pack
    would build from the Word rendering, up to a renaming of ids).
    ``implicit_unk``: Unknowns implicit (packer.py), else every Unknown a node."""
    from .packer import PackedBatch
    if lay is None or lay.implicit != bool(implicit_unk):
        lay, cols = layout(raw, implicit_unk), None
    if cols is None:
        cols = node_columns(raw, lay)
    word, morph, tag, length, is_l, unk = cols
    ids = raw.ids
    # vocabulary slot masks from the probed keys
    vmask = np.zeros(ids.size, dtype=np.uint32)
    pk = model.probed
    for cls in (0, 1, 2, 3, 7, 8):
        sel = pk[pk[:, 0] == cls]
        for pos in range(3):
            if (cls, pos) not in Lw.SLOT_BITS:
                continue
            np.bitwise_or.at(vmask, sel[:, 1 + pos], np.uint32(1 << Lw.SLOT_BITS[(cls, pos)]))
    mask = Lw.node_mask_from_vocab(vmask[word], vmask[morph], vmask[tag]).astype(np.uint32)
    ctx_ids = np.array([ids.tag0 + POS_TAGS.index(t) for t in CONTEXTUAL_TAGS])
    mask |= np.where(unk, Lw.F_UNK, 0).astype(np.uint32)
    mask |= np.where(np.isin(tag, ctx_ids), Lw.F_CTX, 0).astype(np.uint32)
    coef = model.coef
    f4 = np.zeros(lay.NT)
    f5 = np.zeros(lay.NT)
    f6 = np.zeros(lay.NT)
    i4 = np.array([model.keys4.get(int(v), -1) for v in range(0, 16)])
    lk = np.clip(length, 0, 15)
    h4 = i4[lk] >= 0
    f4[h4] = coef[i4[lk][h4]]
    mask |= np.where(h4, Lw.F_HAS4, 0).astype(np.uint32)
    # class 5 via sorted packed keys
    k5 = model.keys5_arr
    enc = lambda w, t, l: (w.astype(np.int64) << 20) | (t.astype(np.int64) << 1) | l.astype(np.int64)
    ek = enc(k5[:, 0], k5[:, 1], k5[:, 2]) if len(k5) else np.zeros(0, np.int64)
    so = np.argsort(ek)
    ek_s = ek[so]
    q = enc(word, tag, is_l)
    pos = np.searchsorted(ek_s, q)
    pos_c = np.minimum(pos, max(len(ek_s) - 1, 0))
    h5 = (len(ek_s) > 0) & (ek_s[pos_c] == q) & (word != 0)
    f5[h5] = coef[model.idx5[so[pos_c[h5]]]]
    mask |= np.where(h5, Lw.F_HAS5, 0).astype(np.uint32)
    i6 = np.array([model.keys6.get(int(v), -1) for v in range(0, 9)])
    l6 = np.clip(np.minimum(8, length), 0, 8)
    h6 = unk & (i6[l6] >= 0)
    f6[h6] = coef[i6[l6][h6]]
    mask |= np.where(h6, Lw.F_HAS6, 0).astype(np.uint32)
    pre = _reg_terms(length, unk, tag == ids.tag0 + POS_TAGS.index(Noun), model.reg)
    keys = np.stack([model.probed[:, 1], model.probed[:, 2], model.probed[:, 3],
                     model.probed[:, 0]], 1).astype(np.uint32)
    batch = PackedBatch(
        max_len=8, n_post=0, has_trigram=1, sent_n=raw.sent_n.astype(np.int32),
        sent_node_off=lay.node_off, sent_span_off=lay.span_base, span_start=lay.span_start,
        node_word=word, node_morph0=morph, node_tag=tag, node_mask=mask, node_pre=pre,
        node_f4=f4, node_f5=f5, node_f6=f6, node_post=np.zeros((0, lay.NT)), unk_n=0)
    if implicit_unk:
        # the canonical Unknown of each span length d (packer.unknown_records):
        # ids 0, tag 'Unknown', classes 4 / 6 of d, Regularization of d
        d = np.arange(1, MAX_SPAN + 1, dtype=np.int32)
        um = np.uint32(Lw.node_mask_from_vocab(int(vmask[0]), int(vmask[0]), int(vmask[ids.unk])) | Lw.F_UNK)
        u4 = i4[np.clip(d, 0, 15)]
        u6 = i6[np.minimum(8, d)]
        batch.unk_n = MAX_SPAN
        batch.unk_word = np.zeros(MAX_SPAN, np.int32)
        batch.unk_morph0 = np.zeros(MAX_SPAN, np.int32)
        batch.unk_tag = np.full(MAX_SPAN, ids.unk, np.int32)
        batch.unk_mask = (um | np.where(u4 >= 0, Lw.F_HAS4, 0) | np.where(u6 >= 0, Lw.F_HAS6, 0)).astype(np.uint32)
        batch.unk_pre = _reg_terms(d, np.ones(MAX_SPAN, bool), np.zeros(MAX_SPAN, bool), model.reg)
        batch.unk_f4 = np.where(u4 >= 0, coef[np.maximum(u4, 0)], 0.0)
        batch.unk_f5 = np.zeros(MAX_SPAN)
        batch.unk_f6 = np.where(u6 >= 0, coef[np.maximum(u6, 0)], 0.0)
        batch.unk_post = np.zeros((0, MAX_SPAN))
    return batch, keys, coef[model.probed_idx].astype(np.float64)


def widen_ids(packed, keys, offset=1 << 20):
    """The same batch and model with every interned id moved up by `offset`
    (id 0 -- "occurs in no key" -- stays 0).  Ids of 2^20 and more put the
    model in the wide table format (32 B slots, lattice_decode.h
    lt_model_desc.narrow = 0); id equality, hence every feature match and
    every result, is unchanged."""
    import copy
    wp = copy.copy(packed)
    shift = lambda a: np.where(np.asarray(a) != 0, np.asarray(a) + offset, 0).astype(np.asarray(a).dtype)  # noqa: E731
    for f in ('node_word', 'node_morph0', 'node_tag'):
        setattr(wp, f, shift(getattr(packed, f)))
    if getattr(packed, 'unk_n', 0):
        for f in ('unk_word', 'unk_morph0', 'unk_tag'):
            setattr(wp, f, shift(getattr(packed, f)))
    wk = np.array(keys, copy=True).reshape(-1, 4)
    wk[:, :3] = shift(wk[:, :3])
    return wp, wk


# ---------------------------------------------------------------------------
# Word rendering (reference input form)
# ---------------------------------------------------------------------------
def render_sentences(raw, sentences, word_cls=None):
    """``(bindex, chars)`` lattices of ``word_cls`` nodes for the given sentences."""
    from .word import Word
    word_cls = word_cls or Word
    R = raw.ids.render
    out = []
    node_sent = raw.char_sent[raw.node_char]
    starts = np.searchsorted(node_sent, np.arange(raw.S + 1))
    for s in sentences:
        n = int(raw.sent_n[s])
        c0 = int(raw.sent_char_off[s])
        chars = ''.join(chr(0xAC00 + int(c)) for c in raw.chars[c0:c0 + n])
        bindex = [[] for _ in range(n)]
        for t in range(int(starts[s]), int(starts[s + 1])):
            b = int(raw.node_char[t]) - c0
            d = int(raw.node_d[t])
            w = word_cls(R(raw.word[t]), R(raw.morph[t]), None, POS_TAGS[int(raw.tag[t])], None,
                         int(raw.length[t]), b, b + d, bool(raw.is_l[t]))
            bindex[b].append(w)
        out.append((bindex, chars))
    return out


def render_model(raw, model):
    """The model as ``(feature_dic over Python tuples, coefficients)``."""
    R = raw.ids.render
    dic = {}
    for row, i in zip(model.probed, model.probed_idx):
        cls = int(row[0])
        comps = [R(row[1]), R(row[2])] + ([R(row[3])] if cls in (0, 2, 7) else [])
        dic[(cls, *comps)] = int(i)
    for v, i in model.keys4.items():
        dic[(4, v)] = i
    for row, i in zip(model.keys5_arr, model.idx5):
        dic[(5, R(row[0]), R(row[1]), bool(row[2]))] = int(i)
    for v, i in model.keys6.items():
        dic[(6, v)] = i
    return dic, model.coef


def to_words(raw, model, word_cls=None, sentences=None):
    """Render sentences as ``(bindex, chars)`` over ``word_cls`` nodes and the
    model as ``(feature_dic, coefficients)``."""
    sentences = range(raw.S) if sentences is None else sentences
    dic, coef = render_model(raw, model)
    return render_sentences(raw, sentences, word_cls), dic, coef
