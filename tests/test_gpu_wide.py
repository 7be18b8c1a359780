"""The general kernel (lt_beam_wide, csrc/lt_decode.hip): the configurations
beyond the tuned kernels' layouts -- max_len > 8 (`beam.py:5,29-30` accepts
any) and beam_size > 256.  The golden set `wide` (reference run here, spans up
to 20 with dictionary nodes of 9-16 characters, beams of 300, max_len < 1)
goes through the drop-in API in test_gpu_parity; here the device is checked
byte for byte against the C restatement (oracle/lt_oracle.c, pinned to the
`wide` vectors in test_packed_oracle) on synthetic batches with long nodes,
and the batch-level behaviours (launch pieces, mixed beams on one batch).
"""
import random

import numpy as np
import pytest

from lattice_based_tagger_amd import (BeamScoreFunctions, RegularizationScore, SimpleTrigramEncoder,
                                      SimpleTrigramFeatureScore, Word, _capi, beam_search_batch, synth)
from lattice_based_tagger_amd.beam import lowered_model, pack_lattices
from oracle import lt_oracle, ref_beam

pytestmark = pytest.mark.gpu


def _lattices(n, seed, long_nodes=4):
    """Synthetic Word lattices (synth.render_sentences) plus dictionary nodes
    of 9-16 characters, and a trigram model over them."""
    raw = synth.make_lattices(n, seed=seed, eojeols=8)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=seed, n_features=100_000)
    dic, coef = synth.render_model(raw, sm)
    sents = synth.render_sentences(raw, range(raw.S))
    rng = random.Random(seed)
    for bindex, chars in sents:
        for _ in range(long_nodes):
            L = rng.randint(9, 16)
            if len(chars) <= L:
                break
            b = rng.randrange(0, len(chars) - L + 1)
            bindex[b].append(Word(chars[b:b + L], chars[b:b + L], None, rng.choice(['Noun', 'Verb']), None,
                                  L, b, b + L, rng.random() < 0.5))
    funcs = BeamScoreFunctions(RegularizationScore(),
                               SimpleTrigramFeatureScore(SimpleTrigramEncoder(dic), coef))
    return sents, funcs


def _device_vs_oracle(dec, packed, model, k):
    dm = dec.device_model(model)
    db = _capi.DeviceBatch(dec.ctx, packed, max_k=k)
    try:
        count, length, score, codes = db.decode(dm, k)
        ex, tu, _, _ = db.count_ops(dm, k)           # the general kernel's COUNT variant
    finally:
        db.close()
    o_count, o_len, o_score, o_codes, o_ex, o_tu = lt_oracle.decode(packed, model.keys, model.coefs, k,
                                                                    nthreads=16)
    assert (ex, tu) == (o_ex, o_tu)                    # reference-algorithm operation counts
    assert np.array_equal(count, o_count)
    assert np.array_equal(length, o_len)
    assert np.array_equal(score.view(np.uint64), o_score.view(np.uint64))    # 0 ULP
    assert np.array_equal(codes, o_codes)
    return count


@pytest.mark.parametrize('max_len,k,n', [(12, 1, 2048), (12, 5, 1024), (20, 2, 512), (16, 300, 48),
                                         (8, 300, 48), (9, 1000, 8)])
def test_wide_kernel_matches_c_oracle(gpu_decoder, max_len, k, n):
    sents, funcs = _lattices(n, seed=500 + k + max_len)
    model = lowered_model(funcs)
    packed, _ = pack_lattices(sents, model, max_len)
    assert packed.max_len == max_len
    count = _device_vs_oracle(gpu_decoder, packed, model, k)
    if k > 256:
        assert count.max() == k        # the beams are full: selection is exercised


def test_wide_matches_python_restatement(gpu_decoder):
    """Node identity + score bits + score type against oracle/ref_beam.py."""
    sents, funcs = _lattices(24, seed=77)
    for max_len, k, part in ((11, 3, sents), (14, 260, sents[:4])):
        got = beam_search_batch(part, funcs, beam_size=k, max_len=max_len)
        for (bindex, chars), matures in zip(part, got):
            exp = ref_beam.beam_search(bindex, chars, funcs, k, max_len)
            assert len(matures) == len(exp)
            for m, (path, score) in zip(matures, exp):
                assert float(m.score).hex() == float(score).hex()
                assert [tuple(w) for w in m.sequences] == [tuple(w) for w in path]


def test_wide_batch_in_launch_pieces(gpu_decoder):
    """A wide batch cut into several launch pieces (small piece limit) decodes
    as one; the scratch is shared by the pieces in stream order."""
    sents, funcs = _lattices(256, seed=91)
    model = lowered_model(funcs)
    packed, _ = pack_lattices(sents, model, 8)      # max_len 8: k <= 256 on the tuned kernels
    lib = _capi.load()
    old = lib.lt_set_piece_bytes(1 << 20)
    try:
        dm = gpu_decoder.device_model(model)
        db = _capi.DeviceBatch(gpu_decoder.ctx, packed, max_k=300)
        assert lib.lt_batch_pieces(db.handle) > 1
        try:
            for k in (1, 5, 300):              # tuned and general kernels on one wide-k batch
                got = db.decode(dm, k)
                o = lt_oracle.decode(packed, model.keys, model.coefs, k, nthreads=16)
                assert np.array_equal(got[0], o[0]) and np.array_equal(got[1], o[1])
                assert np.array_equal(got[2].view(np.uint64), o[2].view(np.uint64))
                assert np.array_equal(got[3], o[3])
        finally:
            db.close()
    finally:
        lib.lt_set_piece_bytes(old)


def test_max_len_below_one(gpu_decoder):
    """No span: beam[e] = [] for e >= 1 and bindex is never read (beam.py:29-31);
    an empty sentence keeps [BOS, EOS]."""
    sents, funcs = _lattices(4, seed=3)
    got = beam_search_batch(sents + [([], 'ㅋㅋ'), ([], '')], funcs, beam_size=5, max_len=0)
    assert got[:5] == [[], [], [], [], []]
    assert len(got[5]) == 1 and got[5][0].score == 0 and type(got[5][0].score) is int
