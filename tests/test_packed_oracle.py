"""Host packing (packer.py, lowering.py) + the C restatement (oracle/lt_oracle.c)
reproduce the reference's golden vectors, and the vectorised synthetic packer
(synth.pack_fast) builds the same batch as packer.pack on the Word rendering."""

import numpy as np
import pytest

from golden_io import SETS, beams_of, load, path_matches
from lattice_based_tagger_amd import lowering, packer, synth
from lattice_based_tagger_amd import score_funcs as SF, feature as FE
from oracle import lt_oracle, ref_beam


def _groups(cases):
    out = {}
    for c in cases:
        out.setdefault((id(c.funcs), c.max_len), []).append(c)
    return out.values()


@pytest.mark.parametrize('name', SETS)
def test_c_oracle_on_packed_golden(name):
    for group in _groups(load(name, packable=True)):
        model = lowering.LoweredModel(group[0].funcs)
        ok_cases = []
        for c in group:
            try:
                packer.pack([(c.bindex, c.chars)], model, c.max_len)
                ok_cases.append(c)
            except IndexError:
                assert all(e.get('error') == 'IndexError' for e in c.expected.values())
        if not ok_cases:
            continue
        pk, objs = packer.pack([(c.bindex, c.chars) for c in ok_cases], model, ok_cases[0].max_len)
        cum = np.r_[0, np.cumsum(pk.sent_n)]
        for k in beams_of(ok_cases):
            count, length, score, codes, _, _ = lt_oracle.decode(pk, model.keys, model.coefs, k)
            for s, c in enumerate(ok_cases):
                if str(k) not in c.expected:
                    continue
                exp = c.expected[str(k)]['matures']
                assert count[s] == len(exp), (c.tag, k)
                n = len(c.chars)
                for t, (ecodes, shex, _) in enumerate(exp):
                    L = int(length[s, t])
                    off = k * cum[s] + t * n
                    words = [objs[s][x] for x in codes[off:off + L]]
                    assert float(score[s, t]).hex() == shex, (c.tag, k, t)
                    assert path_matches(c, ecodes, words), (c.tag, k, t)


def test_pack_fast_equals_word_packer():
    raw = synth.make_lattices(30, seed=5, eojeols=7)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=5, n_features=5000)
    sents, dic, coef = synth.to_words(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    lm = lowering.LoweredModel(funcs)
    pk, _ = packer.pack(sents, lm)
    fb, fkeys, fcoefs = synth.pack_fast(raw, sm, lay, cols)
    # identical structure
    for f in ('sent_n', 'sent_node_off', 'sent_span_off', 'span_start'):
        assert np.array_equal(getattr(pk, f), getattr(fb, f)), f
    for f in ('node_pre', 'node_f4', 'node_f5', 'node_f6'):
        assert np.array_equal(getattr(pk, f), getattr(fb, f)), f
    flag_bits = np.uint32(0x1F0000)
    assert np.array_equal(pk.node_mask & flag_bits, fb.node_mask & flag_bits)
    # identical decode (ids differ by renaming only)
    for k in (1, 4, 16):
        a = lt_oracle.decode(pk, lm.keys, lm.coefs, k)
        b = lt_oracle.decode(fb, fkeys, fcoefs, k)
        for x, y in zip(a[:4], b[:4]):
            assert np.array_equal(x, y)
        assert a[4:] == b[4:]


def test_c_oracle_counts_match_python_oracle():
    raw = synth.make_lattices(12, seed=8, eojeols=5)
    sm = synth.make_model(raw, seed=8, n_features=2000)
    sents, dic, coef = synth.to_words(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    lm = lowering.LoweredModel(funcs)
    pk, _ = packer.pack(sents, lm)
    for k in (1, 5):
        ex = tu = 0
        for b, c in sents:
            x, p = ref_beam.count_ops(b, c, funcs, k)
            ex += x
            tu += p
        res = lt_oracle.decode(pk, lm.keys, lm.coefs, k)
        assert (res[4], res[5]) == (ex, tu)


def test_packer_rejects_short_bindex():
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore())
    lm = lowering.LoweredModel(funcs)
    with pytest.raises(IndexError):
        packer.pack([([], 'abc')], lm)


def test_unsupported_scorer_raises():
    class Custom(SF.BeamScoreFunction):
        def score(self, seq, w):
            return 1.0
    with pytest.raises(NotImplementedError):
        lowering.LoweredModel(SF.BeamScoreFunctions(Custom()))


def test_batch_split_and_slice_preserve_results():
    """Decoding a batch in sentence-range pieces (Decoder.decode_packed over
    PackedBatch.split/slice) gives the whole batch's results."""
    raw = synth.make_lattices(300, seed=5, eojeols=7)
    sm = synth.make_model(raw, seed=5, n_features=5000)
    packed, keys, coefs = synth.pack_fast(raw, sm)
    full = lt_oracle.decode(packed, keys, coefs, 3)
    cuts = packed.split(packed.n_nodes // 7)
    assert len(cuts) >= 7 and cuts[0][0] == 0 and cuts[-1][1] == packed.n_sent
    assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
    parts = [lt_oracle.decode(packed.slice(s0, s1), keys, coefs, 3) for s0, s1 in cuts]
    for i in range(4):
        got = np.concatenate([p[i] for p in parts])
        assert np.array_equal(got.view(np.uint8), np.asarray(full[i]).view(np.uint8))
    assert packed.split(1) == [(s, s + 1) for s in range(packed.n_sent)]


@pytest.mark.parametrize('k', [33, 64, 100, 256])
def test_c_oracle_matches_python_oracle_at_large_beams(k):
    """Beams above the golden vectors' k = 16: the C restatement equals the
    pure-Python one (pinned to the reference by the golden vectors, and
    generic in k like beam.py:64-86) on every mature, so the device's
    big-beam kernels have an oracle."""
    raw = synth.make_lattices(10, seed=21 + k, eojeols=4)
    sm = synth.make_model(raw, seed=21, n_features=3000)
    sents, dic, coef = synth.to_words(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    lm = lowering.LoweredModel(funcs)
    pk, objs = packer.pack(sents, lm)
    count, length, score, codes, _, _ = lt_oracle.decode(pk, lm.keys, lm.coefs, k)
    cum = np.concatenate([[0], np.cumsum(pk.sent_n.astype(np.int64))])
    n_full = 0
    for s, (b, c) in enumerate(sents):
        got = ref_beam.beam_search(b, c, funcs, k)
        assert int(count[s]) == len(got)
        n_full += len(got) == k
        for t, (path, sc) in enumerate(got):
            assert float(sc).hex() == float(score[s, t]).hex()
            L = int(length[s, t])
            off = k * cum[s] + t * len(c)
            assert [tuple(w) for w in path[1:-1]] == [tuple(objs[s][x]) for x in codes[off:off + L]]
    assert n_full > 0


def test_widened_ids_decode_identically():
    """synth.widen_ids moves every interned id past 2^20 (the wide, 32 B slot
    table format on the device): the C restatement decodes the widened batch
    and model exactly as the original -- the premise of the wide-key GPU
    parity test and bench entry."""
    raw = synth.make_lattices(200, seed=5)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=5, n_features=20_000)
    packed, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    wp, wk = synth.widen_ids(packed, keys)
    assert int(wk[:, :3].max()) >= (1 << 20) and int(wp.node_word.max()) >= (1 << 20)
    for k in (1, 5):
        a = lt_oracle.decode(packed, keys, coefs, k)
        b = lt_oracle.decode(wp, wk, coefs, k)
        for x, y in zip(a[:4], b[:4]):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
        assert a[4:] == b[4:]
