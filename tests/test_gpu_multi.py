"""Compact results, pipelined result copies and multi-device decoding
(SURVEY §8(d) timed region, §8(e) partitioning), on the one GPU of the test
box.

* the packed result slab (lt_results.hip) equals the padded results of the
  same decode and the C oracle, including empty and ragged batches;
* decodes launched back to back with their result copies in flight (two
  result slots, copy stream) deliver every step's results intact;
* a batch split over two contexts of GPU 0 (``device=(0, 0)``: two shards,
  two streams, concurrent host threads) equals the one-device decode;
* config 4's 1,048,576-sentence batch decodes on one GPU (launch pieces of
  ``PackedBatch.split``), every sentence byte-equal to the C oracle.
"""

import types

import numpy as np
import pytest

from lattice_based_tagger_amd import _capi, beam_search_batch, synth
from lattice_based_tagger_amd.beam import Decoder, decode_packed_devices, decoders_for
from oracle import lt_oracle

pytestmark = pytest.mark.gpu


def _workload(n_sent, seed, n_features, **kw):
    raw = synth.make_lattices(n_sent, seed=seed, **kw)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=seed, n_features=n_features)
    return raw, sm, synth.pack_fast(raw, sm, lay, cols)


def _model(keys, coefs):
    """The part of a LoweredModel the Decoder uses."""
    return types.SimpleNamespace(keys=keys, coefs=coefs, _device_models={}, image=None)


def _same(a, b):
    return all(np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
               for x, y in zip(a, b))


@pytest.mark.parametrize('k', [1, 2, 5, 16])
def test_packed_results_equal_padded_and_oracle(gpu_decoder, k):
    _, _, (packed, keys, coefs) = _workload(700, 11 + k, 30_000, eojeols=7)
    ctx = gpu_decoder.ctx
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, packed, max_k=16)
    try:
        pk = db.decode_packed(dm, k)
        pad = db.decode(dm, k)
        assert pk.n_sent == packed.n_sent and pk.k == k
        assert _same(pk.padded(packed.sent_n), pad)
        assert int(pk.off[-1]) == pk.codes.size == int(pk.length.sum())
        oc, ol, osc, ocodes, _, _ = lt_oracle.decode(packed, keys, coefs, k)
        assert _same(pk.padded(packed.sent_n), (oc, ol, osc, ocodes))
    finally:
        db.close()
        dm.close()


def test_packed_results_empty_and_tiny_batches(gpu_decoder):
    _, _, (packed, keys, coefs) = _workload(5, 3, 2_000, eojeols=3)
    ctx = gpu_decoder.ctx
    dm = _capi.DeviceModel(ctx, keys, coefs)
    try:
        for s0, s1 in ((0, 0), (0, 1), (2, 5)):
            piece = packed.slice(s0, s1)
            db = _capi.DeviceBatch(ctx, piece, max_k=5)
            try:
                for k in (1, 5):
                    pk = db.decode_packed(dm, k)
                    assert pk.n_sent == s1 - s0
                    assert _same(pk.padded(piece.sent_n), db.decode(dm, k))
            finally:
                db.close()
    finally:
        dm.close()


def test_back_to_back_decodes_with_copies_in_flight(gpu_decoder):
    """Steps queued without host waits (bench.py's timed loop): decode i+1
    writes the other result slot while step i's results are copied; two
    batches alternate so every step's copy is checked."""
    _, _, (pa, keys, coefs) = _workload(3000, 21, 50_000)
    _, _, (pb, _, _) = _workload(2000, 22, 50_000)
    ctx = _capi.Context(0)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    da = _capi.DeviceBatch(ctx, pa, max_k=5)
    db = _capi.DeviceBatch(ctx, pb, max_k=5)
    try:
        ref = {id(da): da.decode_packed(dm, 5), id(db): db.decode_packed(dm, 5)}
        for b in (da, db):
            for _ in range(5):                   # five steps, nothing synchronised
                b.launch(dm, 5)
                b.fetch_packed()
            ctx.sync()
            got = b.results_packed()
            r = ref[id(b)]
            assert _same((got.count, got.length, got.score, got.codes), (r.count, r.length, r.score, r.codes))
        # padded and packed fetches of the same decode agree while both are in flight
        da.launch(dm, 5)
        da.fetch()
        da.fetch_packed()
        ctx.sync()
        assert _same(da.results_packed().padded(pa.sent_n), da.results(5))
        assert len(ctx.kernel_ms_recent(100)) == 2 + 10 + 1
    finally:
        da.close()
        db.close()
        dm.close()
        ctx.close()


@pytest.mark.parametrize('k', [1, 5])
def test_two_contexts_equal_one_device(gpu_decoder, k):
    _, _, (packed, keys, coefs) = _workload(6000, 31, 100_000)
    model = _model(keys, coefs)
    one = Decoder.get(0).decode_packed(model, packed, k)
    two = decode_packed_devices(model, packed, k, (0, 0))
    assert [d.key for d in decoders_for((0, 0))] == [(0, 0), (0, 1)]
    assert _same((two.count, two.length, two.score, two.codes, two.off),
                 (one.count, one.length, one.score, one.codes, one.off))
    three = decode_packed_devices(model, packed, k, (0, 0, 0))
    assert _same((three.codes, three.score), (one.codes, one.score))


def test_beam_search_batch_over_two_contexts(gpu_decoder):
    from lattice_based_tagger_amd import feature as FE, score_funcs as SF
    raw, sm, _ = _workload(300, 41, 20_000, eojeols=6)
    sents, dic, coef = synth.to_words(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    for k in (1, 5):
        one = beam_search_batch(sents, funcs, beam_size=k)
        two = beam_search_batch(sents, funcs, beam_size=k, device=(0, 0))
        assert len(one) == len(two) == len(sents)
        for a, b in zip(one, two):
            assert [float(m.score).hex() for m in a] == [float(m.score).hex() for m in b]
            # the caller's own Word objects (Unknown nodes are synthesised per call)
            key = lambda w: (tuple(w), w.tag0 == 'Unknown' or id(w))   # noqa: E731
            assert [[key(w) for w in m.sequences[1:-1]] for m in a] == \
                [[key(w) for w in m.sequences[1:-1]] for m in b]


def test_config4_million_sentences_on_one_gpu(gpu_decoder):
    """1,048,576 sentences (the 64K generated lattices in 16 seeded
    permutations, as bench.py --sentences 1048576 builds them) as one device
    batch: the library decodes it in launch pieces (each below 2^31 B of
    node records); every sentence equals the C oracle's decode of its
    lattice, in the packed and the padded result layouts."""
    _, _, (base, keys, coefs) = _workload(65536, 5, 1_000_000)
    rng = np.random.default_rng(99)
    order = np.concatenate([rng.permutation(base.n_sent) for _ in range(16)])
    big = base.take(order)
    assert big.n_sent == 1 << 20
    dec = Decoder.get(0)
    dm = dec.device_model(_model(keys, coefs))
    db = _capi.DeviceBatch(dec.ctx, big, max_k=1)
    del big
    try:
        assert db.pieces > 2                    # launch pieces below 2^31 B of node records each
        got = db.decode_packed(dm, 1)
        padded = db.decode(dm, 1)               # the padded layout of the same batch
    finally:
        db.close()
    assert _same(got.padded(base.sent_n[order]), padded)
    oc, ol, osc, ocodes, _, _ = lt_oracle.decode(base, keys, coefs, 1, nthreads=16)
    assert np.array_equal(got.count, oc[order])
    assert np.array_equal(got.length[:, 0], ol[order, 0])
    assert np.array_equal(got.score[:, 0].view(np.uint64), osc[order, 0].view(np.uint64))
    cum = np.zeros(base.n_sent + 1, dtype=np.int64)
    np.cumsum(base.sent_n, out=cum[1:])
    L = ol[:, 0].astype(np.int64)[order]
    seg = np.repeat(order, L)
    within = np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L)
    assert np.array_equal(got.codes, ocodes[cum[seg] + within])
