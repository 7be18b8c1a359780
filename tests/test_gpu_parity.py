"""Parity of the HIP decoder (through the C-ABI) with the reference.

* golden vectors of the reference itself (tests/golden) through the drop-in
  ``beam_search_batch`` / ``beam_search`` API: bit-exact paths (node identity)
  and float64 scores compared as float.hex() -- 0 ULP;
* the C restatement (oracle/lt_oracle.c) on synthetic batches of the bench
  shape, bit-exact, up to the full 64K-sentence config;
* size-independent properties at full size (determinism, path validity,
  sorted matures).
"""

import numpy as np
import pytest

from golden_io import MULTI_SETS, SETS, beams_of, load, path_matches
from lattice_based_tagger_amd import _capi, beam_search, beam_search_batch, synth
from oracle import lt_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', SETS + MULTI_SETS)
def test_golden_vectors_on_gpu(gpu_decoder, name):
    cases = load(name)
    groups = {}
    for c in cases:
        groups.setdefault((id(c.funcs), c.max_len), []).append(c)
    checked = 0
    for group in groups.values():
        ok = [c for c in group if not any('error' in e for e in c.expected.values())]
        for c in group:
            if c not in ok:
                with pytest.raises(IndexError):
                    beam_search(c.bindex, c.chars, c.funcs, beam_size=1, max_len=c.max_len)
        if not ok:
            continue
        for k in beams_of(ok):
            okk = [c for c in ok if str(k) in c.expected]
            got = beam_search_batch([(c.bindex, c.chars) for c in okk], okk[0].funcs,
                                    beam_size=k, max_len=okk[0].max_len)
            for c, matures in zip(okk, got):
                exp = c.expected[str(k)]['matures']
                assert len(matures) == len(exp), (c.tag, k)
                for m, (codes, shex, kind) in zip(matures, exp):
                    assert float(m.score).hex() == shex, (c.tag, k)
                    assert type(m.score).__name__ == kind, (c.tag, k, type(m.score), kind)
                    assert path_matches(c, codes, m.sequences[1:-1]), (c.tag, k)
                    checked += 1
    assert checked > 0


def test_single_sentence_drop_in(gpu_decoder):
    case = load('base')[0]          # config 1: one 10-eojeol sentence
    m = beam_search(case.bindex, case.chars, case.funcs, beam_size=5)
    exp = case.expected['5']['matures']
    assert [float(x.score).hex() for x in m] == [e[1] for e in exp]


def _synthetic(n_sent, seed, n_features, **kw):
    raw = synth.make_lattices(n_sent, seed=seed, **kw)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=seed, n_features=n_features)
    return synth.pack_fast(raw, sm, lay, cols)


def _gpu_decode(ctx, packed, keys, coefs, k):
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, packed, max_k=k)
    try:
        return db.decode(dm, k), db.count_ops(dm, k)
    finally:
        db.close()
        dm.close()


@pytest.mark.parametrize('k,n_sent', [(5, 8192), (16, 4096), (2, 2048), (3, 2048), (8, 2048), (32, 512),
                                       (33, 300), (64, 300), (100, 200), (256, 120)])
def test_kernel_matches_c_oracle_on_synthetic(gpu_decoder, k, n_sent):
    packed, keys, coefs = _synthetic(n_sent, seed=100 + k, n_features=1_000_000)
    (count, length, score, codes), (ex, tu, _, _) = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)
    o_count, o_len, o_score, o_codes, o_ex, o_tu = lt_oracle.decode(packed, keys, coefs, k,
                                                                    nthreads=16)
    assert np.array_equal(count, o_count)
    assert np.array_equal(length, o_len)
    assert np.array_equal(score.view(np.uint64), o_score.view(np.uint64))   # 0 ULP
    assert np.array_equal(codes, o_codes)
    assert (ex, tu) == (o_ex, o_tu)


@pytest.mark.parametrize('k', [1, 2, 5, 8, 16])
def test_dense_lattices_with_ties_match_c_oracle(gpu_decoder, k):
    """Dense lattices (about 30 candidates per end position, half of the extra
    ones exact duplicates of the span's first candidate, hence score ties):
    the k=1 kernel packs more candidates than lanes into several rounds per
    position with sentences straddling rounds; the beam kernel runs several
    chunks per position.  Bit-exact against the C restatement."""
    packed, keys, coefs = _synthetic(4096 if k == 1 else 1024, seed=300 + k, n_features=200_000,
                                     eojeols=6, extra_lambda=3.0, dup_rate=0.5)
    (count, length, score, codes), (ex, tu, _, _) = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)
    o_count, o_len, o_score, o_codes, o_ex, o_tu = lt_oracle.decode(packed, keys, coefs, k,
                                                                    nthreads=16)
    assert np.array_equal(count, o_count)
    assert np.array_equal(length, o_len)
    assert np.array_equal(score.view(np.uint64), o_score.view(np.uint64))
    assert np.array_equal(codes, o_codes)
    assert (ex, tu) == (o_ex, o_tu)


@pytest.fixture(scope='module')
def config3_batch():
    """BASELINE config 3 exactly as bench.py builds it: 65,536 synthetic
    sentences (seed 0), 1M-key trigram model."""
    import bench
    raw, lay, sm, packed, keys, coefs = bench.make_workload(65536, 0, 1_000_000)
    return packed, keys, coefs


@pytest.mark.parametrize('k', [1, 5, 16])
def test_config3_full_batch_matches_c_oracle(gpu_decoder, config3_batch, k):
    """The whole 64K-sentence bench batch, byte for byte against the C
    restatement: k=1 (the headline), k=5 (config 3 secondary, Tagger.tag's
    default) and k=16 (config 5) -- counts, lengths, score bits, codes and
    the reference-algorithm operation counts."""
    packed, keys, coefs = config3_batch
    (count, length, score, codes), (ex, tu, _, _) = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)
    o_count, o_len, o_score, o_codes, o_ex, o_tu = lt_oracle.decode(packed, keys, coefs, k, nthreads=16)
    assert np.array_equal(count, o_count)
    assert np.array_equal(length, o_len)
    assert np.array_equal(score.view(np.uint64), o_score.view(np.uint64))   # 0 ULP
    assert np.array_equal(codes, o_codes)
    assert (ex, tu) == (o_ex, o_tu)


@pytest.mark.parametrize('k', [1, 2, 5, 16, 300])
def test_class46_pair_escape_matches_c_oracle(gpu_decoder, k):
    """The node records hold their class-4/6 coefficients as an index into the
    batch's pair table (at most 126 distinct pairs, lt_common.h NodeRec); a
    batch with more sends the rest to the per-node escape array.  Here every
    node gets its own class-4 coefficient (and the implicit Unknowns keep
    theirs): the table fills, most nodes escape, and every kernel (k=1, the
    lane-group and one-wave beams, the general kernel at 300) still decodes
    byte-equal to the C restatement."""
    packed, keys, coefs = _synthetic(1024 if k <= 16 else 64, seed=4600 + k, n_features=200_000)
    rng = np.random.default_rng(k)
    packed.node_f4 = rng.standard_normal(len(packed.node_f4))
    packed.node_mask = (np.asarray(packed.node_mask, dtype=np.uint32) | np.uint32(1 << 18)).astype(np.uint32)
    (count, length, score, codes), (ex, tu, _, _) = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)
    o_count, o_len, o_score, o_codes, o_ex, o_tu = lt_oracle.decode(packed, keys, coefs, k, nthreads=16)
    assert np.array_equal(count, o_count)
    assert np.array_equal(length, o_len)
    assert np.array_equal(score.view(np.uint64), o_score.view(np.uint64))
    assert np.array_equal(codes, o_codes)
    assert (ex, tu) == (o_ex, o_tu)


@pytest.mark.parametrize('k', [1, 5, 16])
def test_wide_key_model_matches_narrow_and_oracle(gpu_decoder, k):
    """A model whose interned ids pass 2^20 (synth.widen_ids) lives in the
    wide table format (32 B slots, four 32-bit key compares): every kernel
    decodes it byte-equal to the same batch under the narrow model and to the
    C restatement, operation counts included."""
    packed, keys, coefs = _synthetic(2048 if k < 16 else 1024, seed=1700 + k, n_features=200_000)
    wp, wk = synth.widen_ids(packed, keys)
    narrow, n_ops = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)
    wide, w_ops = _gpu_decode(gpu_decoder.ctx, wp, wk, coefs, k)
    for a, b in zip(narrow, wide):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    assert n_ops[:2] == w_ops[:2]
    o = lt_oracle.decode(wp, wk, coefs, k, nthreads=16)
    assert np.array_equal(wide[0], o[0]) and np.array_equal(wide[1], o[1])
    assert np.array_equal(wide[2].view(np.uint64), o[2].view(np.uint64))
    assert np.array_equal(wide[3], o[3])
    assert (w_ops[0], w_ops[1]) == (o[4], o[5])


def test_long_sentences_cross_the_lds_backpointer_window(gpu_decoder):
    """k=1 keeps the backpointers of end positions < PK_BPL (87) in LDS and
    the rest in HBM: 40-eojeol sentences (about 140 characters) put most
    positions past the window; byte-equal to the C restatement."""
    packed, keys, coefs = _synthetic(8192, seed=4040, n_features=200_000, eojeols=40)
    assert float(np.mean(packed.sent_n)) > 120
    (count, length, score, codes), _ = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, 1)
    o = lt_oracle.decode(packed, keys, coefs, 1, nthreads=16)
    assert np.array_equal(count, o[0]) and np.array_equal(length, o[1])
    assert np.array_equal(score.view(np.uint64), o[2].view(np.uint64))
    assert np.array_equal(codes, o[3])


@pytest.mark.parametrize('case', ['long', 'dense', 'long_lazy', 'dense_lazy'])
def test_k1_schedule_long_and_dense(gpu_decoder, case):
    """The k=1 lane schedule (lt_internal.h k1_schedule): sentences advance
    independently, several end positions per macro-step.  'long': 90-eojeol
    sentences (about 300 characters) -- positions past the schedule kernels'
    LDS counts (K1_NCAP = 192: counts from the span table, placements in the
    backpointer rows) and past the kernel's LDS backpointer window; 'dense':
    about 64 candidates per end position, so positions above 64 candidates
    take several macro-steps alone.  '_lazy': the batch is created for beam 5
    and decoded at beam 1 (schedule counted on the device).  Byte-equal to
    the C restatement."""
    if case.startswith('long'):
        packed, keys, coefs = _synthetic(600, seed=5151, n_features=100_000, eojeols=90)
        assert int(packed.sent_n.max()) > 192
    else:
        packed, keys, coefs = _synthetic(300, seed=5252, n_features=100_000, eojeols=6,
                                         extra_lambda=45.0, dup_rate=0.4)
    dm = _capi.DeviceModel(gpu_decoder.ctx, keys, coefs)
    db = _capi.DeviceBatch(gpu_decoder.ctx, packed, max_k=5 if case.endswith('lazy') else 1)
    try:
        count, length, score, codes = db.decode(dm, 1)
    finally:
        db.close()
        dm.close()
    o = lt_oracle.decode(packed, keys, coefs, 1, nthreads=16)
    assert np.array_equal(count, o[0]) and np.array_equal(length, o[1])
    assert np.array_equal(score.view(np.uint64), o[2].view(np.uint64))
    assert np.array_equal(codes, o[3])


@pytest.mark.parametrize('case', ['bench', 'long', 'dense'])
def test_k1_fill_inside_decode(gpu_decoder, case):
    """A batch whose beam-1 schedule is not filled yet (lt_batch_reset_prep:
    the next decode rebuilds it; likewise a beam-5 batch's first beam-1 decode)
    has it filled by the decode kernel itself (DecodeParams.k1_fill,
    LT_K1_FUSED_FILL): each wave fills its own rows in its ring's LDS before
    decoding.  Byte-equal to the C restatement, and to the decode of the
    schedule the standalone fill built (at lt_batch_create), twice over."""
    if case == 'bench':
        packed, keys, coefs = _synthetic(4096, seed=6161, n_features=200_000)
    elif case == 'long':
        packed, keys, coefs = _synthetic(400, seed=6262, n_features=100_000, eojeols=90)
    else:
        packed, keys, coefs = _synthetic(300, seed=6363, n_features=100_000, eojeols=6,
                                         extra_lambda=45.0, dup_rate=0.4)
    dm = _capi.DeviceModel(gpu_decoder.ctx, keys, coefs)
    db = _capi.DeviceBatch(gpu_decoder.ctx, packed, max_k=1)
    try:
        first = db.decode(dm, 1)                 # schedule filled at lt_batch_create
        fused = []
        for _ in range(2):
            db.reset_prep()
            fused.append(db.decode(dm, 1))
    finally:
        db.close()
        dm.close()
    o = lt_oracle.decode(packed, keys, coefs, 1, nthreads=16)
    for count, length, score, codes in [first] + fused:
        assert np.array_equal(count, o[0]) and np.array_equal(length, o[1])
        assert np.array_equal(score.view(np.uint64), o[2].view(np.uint64))
        assert np.array_equal(codes, o[3])


def test_full_size_properties(gpu_decoder):
    """64K sentences, k=16: deterministic, sorted, and every path is a chain of
    spans from 0 to n made of the sentence's own nodes."""
    raw = synth.make_lattices(65536, seed=7)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=7)
    packed, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    k = 16
    dm = _capi.DeviceModel(gpu_decoder.ctx, keys, coefs)
    db = _capi.DeviceBatch(gpu_decoder.ctx, packed, max_k=k)
    r1 = db.decode(dm, k)
    r2 = db.decode(dm, k)
    for a, b in zip(r1, r2):
        assert np.array_equal(a, b)
    count, length, score, codes = r1
    assert np.all(count == k)
    assert np.all(np.diff(score, axis=1) <= 0)
    # span chain check on a sample: every path word's span entry x (a node's:
    # the entry whose node range holds it; an implicit Unknown's: from its
    # code -2 - x, and its span holds no node), spans chained from 0 to n
    n = packed.sent_n.astype(np.int64)
    cum = np.r_[0, np.cumsum(n)]
    rng = np.random.default_rng(0)
    n_imp = 0
    for s in rng.choice(len(n), size=200, replace=False):
        ss = packed.span_start[packed.sent_span_off[s]:packed.sent_span_off[s + 1]].astype(np.int64)
        for t in range(k):
            L = length[s, t]
            off = k * cum[s] + t * n[s]
            local = codes[off:off + L].astype(np.int64)
            imp = local <= -2
            x = np.where(imp, -2 - local, np.searchsorted(ss, local, side='right') - 1)
            assert np.all(ss[x[imp]] == ss[x[imp] + 1])            # implicit: an empty span
            assert np.all(ss[x[~imp]] <= local[~imp]) and np.all(local[~imp] < ss[x[~imp] + 1])
            e = x // 8 + 1
            d = 8 - x % 8
            b = e - d
            assert b[0] == 0 and e[-1] == n[s] and np.all(b[1:] == e[:-1])
            n_imp += int(imp.sum())
    assert n_imp > 0                       # the sample crosses implicit Unknowns
    db.close()
    dm.close()


def test_ragged_and_empty_batch(gpu_decoder):
    from golden_io import load as gl
    cases = [c for c in gl('edge') if c.model == 'edge_tri' and c.max_len == 8
             and not any('error' in e for e in c.expected.values())]
    # interleave empty and long sentences; results must not depend on batching
    lats = [(c.bindex, c.chars) for c in cases]
    funcs = cases[0].funcs
    together = beam_search_batch(lats, funcs, beam_size=5)
    for (b, ch), m in zip(lats, together):
        alone = beam_search_batch([(b, ch)], funcs, beam_size=5)[0]
        assert [float(x.score).hex() for x in m] == [float(x.score).hex() for x in alone]
    assert beam_search_batch([], funcs, beam_size=3) == []


@pytest.mark.parametrize('k', [1, 2, 5, 16])
def test_decode_in_several_launches(gpu_decoder, k):
    """A batch above the per-launch budget is decoded as several launch
    pieces writing one result array (lt_batch_pieces) -- forced here with
    the piece-size test hook -- with the results of one launch."""
    from lattice_based_tagger_amd import _capi as C
    lib = C.load()
    cases = [c for c in load('base') if c.bindex]
    lats = [(c.bindex, c.chars) for c in cases]
    whole = beam_search_batch(lats, cases[0].funcs, beam_size=k)
    packed, keys, coefs = _synthetic(300, seed=7, n_features=20_000, eojeols=6)
    one = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, k)[0]
    old = lib.lt_set_piece_bytes(100_000)
    try:
        pieces = beam_search_batch(lats, cases[0].funcs, beam_size=k)
        dm = C.DeviceModel(gpu_decoder.ctx, keys, coefs)
        db = C.DeviceBatch(gpu_decoder.ctx, packed, max_k=k)
        try:
            assert db.pieces > 3
            many = db.decode(dm, k)
            pk = db.decode_packed(dm, k)
        finally:
            db.close()
            dm.close()
    finally:
        lib.lt_set_piece_bytes(old)
    for a, b in zip(whole, pieces):
        assert [float(x.score).hex() for x in a] == [float(x.score).hex() for x in b]
        assert [[tuple(w) for w in x.sequences] for x in a] == [[tuple(w) for w in x.sequences] for x in b]
    for x, y in zip(one, many):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    for x, y in zip(pk.padded(packed.sent_n), one):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_half_wave_beam_kernel_multi_chunk(gpu_decoder):
    """k=2 runs lt_beam_hw in 16-lane groups (four sentences per wave).  Very
    dense lattices (about 64 candidates per end position) give positions with
    several expansion chunks per group, so the threshold-pruning path and the
    carried running top-k run in every group at once, with ties; results
    bit-exact against the C restatement."""
    from lattice_based_tagger_amd import _capi as C
    assert C.load().lt_kernel_name(2) == b'lt_beam_hw'
    packed, keys, coefs = _synthetic(257, seed=411, n_features=100_000, eojeols=5,
                                     extra_lambda=45.0, dup_rate=0.4)
    (count, length, score, codes), _ = _gpu_decode(gpu_decoder.ctx, packed, keys, coefs, 2)
    o = lt_oracle.decode(packed, keys, coefs, 2, nthreads=16)
    assert np.array_equal(count, o[0]) and np.array_equal(length, o[1])
    assert np.array_equal(score.view(np.uint64), o[2].view(np.uint64))
    assert np.array_equal(codes, o[3])


def test_recycled_batch_buffers(gpu_decoder):
    """Batch buffers are recycled through the context (lt_batch_destroy keeps
    small arenas): decoding batches of alternating sizes and beams -- a large
    one after a small one reuses nothing, a small one after a large one runs
    in the large one's arena with stale data around it -- gives each batch the
    C restatement's results, bit for bit."""
    ctx = gpu_decoder.ctx
    small = _synthetic(40, seed=901, n_features=20_000)
    large = _synthetic(600, seed=902, n_features=20_000)
    ref = {}
    for name, (packed, keys, coefs) in (('s', small), ('l', large)):
        for k in (1, 5):
            o = lt_oracle.decode(packed, keys, coefs, k, nthreads=16)
            ref[name, k] = (o[0], o[1], o[2].view(np.uint64), o[3])
    for name, k in [('l', 5), ('s', 1), ('l', 1), ('s', 5), ('s', 1), ('l', 5), ('s', 5)]:
        packed, keys, coefs = small if name == 's' else large
        count, length, score, codes = _gpu_decode(ctx, packed, keys, coefs, k)[0]
        for x, y in zip((count, length, score.view(np.uint64), codes), ref[name, k]):
            assert np.array_equal(x, y), (name, k)
