"""Multi-process (world_size 2 and 3, CPU) coverage of the sharding path: shard
ranges tile the batch, per-rank decodes of the shards reassemble to the
single-process decode, and the torch-free host group's (dist.HostGroup, TCP)
barrier/max/sum/gather/id broadcast work.  The processes are started with the
standard library's multiprocessing and never import torch.  The per-rank
decode here is the C restatement (oracle) standing in for the device, which
the CPU container does not have."""

import os
import socket

import numpy as np
import pytest
import multiprocessing as mp
import sys

from lattice_based_tagger_amd import dist, synth


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_range_tiles_and_balances():
    rng = np.random.default_rng(0)
    w = rng.integers(40, 100, size=1001)
    for world in (1, 2, 3, 8):
        cuts = [dist.shard_range(w, world, r) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(w)
        for (a, b), (c, d) in zip(cuts, cuts[1:]):
            assert b == c and a <= b
        loads = [w[a:b].sum() for a, b in cuts]
        assert max(loads) - min(loads) <= 2 * w.max()
    assert dist.shard_range([], 4, 3) == (0, 0)


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from oracle import lt_oracle
    g = dist.HostGroup()
    raw = synth.make_lattices(96, seed=11, eojeols=6)
    sm = synth.make_model(raw, seed=11, n_features=4000)
    packed, keys, coefs = synth.pack_fast(raw, sm)
    lo, hi = dist.shard_range(packed.sent_n, g.ranks.world, g.ranks.rank)
    count, length, score, codes, ex, tu = lt_oracle.decode(packed, keys, coefs, 2, s0=lo, s1=hi)
    cum = np.concatenate([[0], np.cumsum(packed.sent_n.astype(np.int64))])
    mine = (lo, hi, count[lo:hi].copy(), length[lo:hi].copy(), score[lo:hi].copy(),
            codes[2 * cum[lo]:2 * cum[hi]].copy())
    g.barrier()
    no_torch = 'torch' not in sys.modules
    total = g.sum(float(hi - lo))
    mx = g.max(float(rank))
    parts = g.gather(mine)
    if rank == 0:
        full = lt_oracle.decode(packed, keys, coefs, 2)
        ok = total == len(packed.sent_n) and mx == world - 1 and no_torch
        got_count = np.concatenate([p[2] for p in parts])
        got_len = np.concatenate([p[3] for p in parts])
        got_score = np.concatenate([p[4] for p in parts])
        got_codes = np.concatenate([p[5] for p in parts])
        ok = ok and np.array_equal(got_count, full[0]) and np.array_equal(got_len, full[1])
        ok = ok and np.array_equal(got_score.view(np.uint64), full[2].view(np.uint64))
        ok = ok and np.array_equal(got_codes, full[3])
        out_q.put(bool(ok))
    g.close()


def test_two_rank_host_group_shards_reassemble():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def _id_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    d = bench.Dist(world)
    uid = bytes(range(128)) if rank == 0 else None       # stands in for lt_comm_unique_id()
    got = d.broadcast_bytes(uid)
    out_q.put((rank, got == bytes(range(128)), d.max(float(rank)), d.sum(1.0), d.min(float(rank)),
               'torch' not in sys.modules))
    d.close()


def test_bench_dist_shares_the_communicator_id():
    """bench.py's host group hands rank 0's RCCL id to every rank (TCP, no
    torch imported)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_id_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True, 1.0, 2.0, 0.0, True), (1, True, 1.0, 2.0, 0.0, True)]


def _al16(x):
    return (x + 15) // 16 * 16


def _slab_layout(n_sent, k, chars):
    """Section offsets of a slab (lattice_decode.h "compact results",
    lt_internal.h slab_layout): 32 B header, then 16 B aligned count,
    length, score and codes; capacity for `chars` characters."""
    count = 32
    length = count + _al16(4 * n_sent)
    score = length + _al16(4 * n_sent * k)
    codes = score + _al16(8 * n_sent * k)
    return count, length, score, codes, codes + _al16(4 * chars * k)


def _write_slab(res, chars):
    """A rank's PackedResults as the bytes of its slab, padded to the
    capacity of its shard (what lt_gather_launch sends)."""
    S, k = res.n_sent, res.k
    c0, l0, s0, d0, cap = _slab_layout(S, k, chars)
    buf = np.zeros(cap, dtype=np.uint8)
    used = d0 + _al16(4 * res.codes.size)
    buf[:32] = np.frombuffer(np.array([S, k], np.int32).tobytes() +
                             np.array([res.codes.size, used, 0], np.int64).tobytes(), np.uint8)
    buf[c0:c0 + 4 * S] = res.count.astype(np.int32).view(np.uint8)
    buf[l0:l0 + 4 * S * k] = res.length.astype(np.int32).ravel().view(np.uint8)
    buf[s0:s0 + 8 * S * k] = res.score.astype(np.float64).ravel().view(np.uint8)
    buf[d0:d0 + 4 * res.codes.size] = res.codes.astype(np.int32).view(np.uint8)
    return buf


def _strong_worker(rank, world, port, total, out_q):
    """bench.py's strong-scaling path on the CPU: the seeded batch (in
    seeded permutations past the generated lattices, as config 4 builds
    it), this rank's shard (``shard_of``), its decode (the C restatement
    standing in for the device), the per-rank results gathered to rank 0
    (the TCP host group here, RCCL in bench.py) and rank 0's byte-for-byte check against
    a single-process decode (``check_results``)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from oracle import lt_oracle
    d = bench.Dist(world)
    k = 2
    raw, lay, sm, packed, keys, coefs = bench.make_workload(64, 13, 5000)
    order = bench.batch_order(total, packed.n_sent, 13)
    lo, hi, piece = bench.shard_of(packed, order, k, world, rank)
    res = lt_oracle.decode(piece, keys, coefs, k)[:4]
    mine = bench.padded_as_packed(res, piece.sent_n, k)
    parts = d.gather(mine)
    # the RCCL path's bytes: every rank's slab (padded to its capacity), laid
    # out by the root at stride cap = the largest capacity, as the receive
    # slot of lt_gather_launch holds them, and read back with lt_slab_parse
    # (lt_gather_view) -- the reassembly that runs only at N > 1 on a node
    slabs = d.gather(_write_slab(mine, int(np.sum(piece.sent_n))))
    if rank == 0:
        from lattice_based_tagger_amd import _capi
        ref = bench.padded_as_packed(lt_oracle.decode(packed, keys, coefs, k)[:4], packed.sent_n, k)
        idx = np.arange(packed.n_sent) if order is None else order
        ok = bench.check_results(parts, ref, idx)
        try:                                   # a wrong reassembly is caught
            bench.check_results(parts[::-1], ref, idx)
            caught = False
        except AssertionError:
            caught = True
        cap = max(x.size for x in slabs)
        recv = np.zeros(cap * world, dtype=np.uint8)
        for q, x in enumerate(slabs):
            recv[q * cap:q * cap + x.size] = x
        views = [_capi.parse_slab(recv[q * cap:(q + 1) * cap]) for q in range(world)]
        ok = ok and bench.check_results(views, ref, idx)
        bad = recv[:cap].copy()
        bad[16:24] = np.frombuffer(np.int64(cap + 16).tobytes(), np.uint8)   # used bytes past the slot
        try:
            _capi.parse_slab(bad)
            caught = False
        except _capi.LTError:
            pass
        out_q.put((ok, caught, all(p.n_sent > 0 for p in parts), [p.n_sent for p in parts]))
    d.close()


@pytest.mark.parametrize('world,total', [(2, 64), (3, 200)])
def test_bench_strong_split_reassembles(world, total):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, caught, nonempty, sizes = q.get(timeout=10)
    assert ok and caught and nonempty and sum(sizes) == total
