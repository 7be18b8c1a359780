"""RCCL result gather (include/lattice_decode.h "multi-GPU result gather") on
the one GPU of the test box: a single-rank communicator gathers the decode
results of a ragged batch to itself as a packed slab, and the gathered
block must equal the batch's own results byte for byte (and the C
oracle's).  The multi-rank path
is the same code with nranks > 1 (bench.py --gpus N at round end); the gloo
exchange of the communicator id is covered on the CPU in test_dist.py."""

import numpy as np
import pytest

from lattice_based_tagger_amd import _capi, synth
from oracle import lt_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('k', [1, 5])
def test_single_rank_gather_equals_local_results(gpu_decoder, k):
    raw = synth.make_lattices(300, seed=7, eojeols=9)
    sm = synth.make_model(raw, seed=7, n_features=20_000)
    packed, keys, coefs = synth.pack_fast(raw, sm)
    ctx = _capi.Context(0)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    db = _capi.DeviceBatch(ctx, packed, max_k=16)
    comm = _capi.Comm(ctx, 1, 0, _capi.comm_unique_id())
    try:
        comm.prepare(db, k, root=0)
        with pytest.raises(_capi.LTError):
            comm.launch(db)                     # nothing decoded yet
        db.launch(dm, k)
        comm.launch(db)
        db.fetch()
        comm.sync()
        comm.fetch()
        ctx.sync()
        assert comm.gather_ms() >= 0.0
        local = db.results(k)
        got = comm.view(0)                      # rank 0's slab, packed
        assert got.n_sent == packed.n_sent
        for x, y in zip(got.padded(packed.sent_n), local):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
        oc, ol, osc, ocodes, _, _ = lt_oracle.decode(packed, keys, coefs, k)
        pc, pl, ps, pcodes = got.padded(packed.sent_n)
        assert np.array_equal(pc, oc) and np.array_equal(pl, ol)
        assert np.array_equal(ps.view(np.uint64), osc.view(np.uint64))
        assert np.array_equal(pcodes, ocodes)
        # pipelined: two more decode + gather rounds reuse both slots
        for _ in range(2):
            db.launch(dm, k)
            comm.launch(db)
            comm.fetch()
        comm.sync()
        ctx.sync()
        again = comm.view(0)
        for x, y in zip(again.padded(packed.sent_n), local):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
        # a decode of another beam cannot be gathered with this preparation
        db.launch(dm, 1 if k != 1 else 2)
        with pytest.raises(_capi.LTError):
            comm.launch(db)
        ctx.sync()
    finally:
        comm.close()
        db.close()
        dm.close()
        ctx.close()
