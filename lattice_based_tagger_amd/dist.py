"""Multi-GPU sharding of the decode (one process per GPU).

``beam_search`` has no cross-sentence state (`lattice_tagger/beam/beam.py:5-61`
decodes one sentence; `Tagger.tag` is per sentence, `tagger/tagger.py:68-78`),
so sentences shard across GPUs with no data-path collective: each rank decodes
a contiguous shard on its own device.  The host group below (TCP sockets, no
torch: the reference has no torch dependency) is used for the barrier /
max-over-ranks timing of the benchmark, to hand rank 0's RCCL unique id to
the other ranks, and, when a caller wants all results on one host without the
RCCL gather, for an object gather after the decode.

``shard_range`` balances shards by characters (decode work is linear in the
sentence length).
"""

import os
import pickle
import socket
import struct
import time

import numpy as np


class Ranks:
    """RANK / WORLD_SIZE / LOCAL_RANK from the environment (torchrun sets them)."""

    def __init__(self, env=None):
        env = os.environ if env is None else env
        self.rank = int(env.get('RANK', 0))
        self.world = int(env.get('WORLD_SIZE', 1))
        self.local = int(env.get('LOCAL_RANK', self.rank))


def shard_range(weights, world, rank):
    """Contiguous [lo, hi) of items for ``rank`` so that every shard carries about
    1/world of the total weight (greedy prefix split).  Shards tile [0, n)."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if world <= 1:
        return 0, n
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0] + [int(np.searchsorted(cum, total * r / world, side='left')) for r in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return int(cuts[rank]), int(cuts[rank + 1])


def host_port(env=None):
    """The host group's TCP port: LT_HOST_PORT, else MASTER_PORT -- plus one
    under torchrun, whose agent keeps its own store on MASTER_PORT."""
    env = os.environ if env is None else env
    if env.get('LT_HOST_PORT'):
        return int(env['LT_HOST_PORT'])
    port = int(env.get('MASTER_PORT', 29500))
    return port + 1 if env.get('TORCHELASTIC_RUN_ID') or env.get('TORCHELASTIC_USE_AGENT_STORE') else port


def _send(sock, data):
    sock.sendall(struct.pack('<Q', len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        r = sock.recv_into(view[got:], n - got)
        if r == 0:
            raise ConnectionError('host group: peer closed the connection')
        got += r
    return bytes(buf)


def _recv(sock):
    (n,) = struct.unpack('<Q', _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class HostGroup:
    """Host-side coordination of the ranks over TCP (never on the data path):
    a star around rank 0, which listens on MASTER_ADDR:host_port() and takes
    one connection per other rank.  Every collective is one round: each rank
    sends its part to rank 0, rank 0 answers each with the result.  All ranks
    call the collectives in the same order (as with any process group)."""

    def __init__(self, ranks=None, timeout=600.0):
        self.ranks = ranks or Ranks()
        self.peers = []                   # rank 0: sockets of ranks 1..world-1, in rank order
        self.sock = None                  # other ranks: the connection to rank 0
        if self.ranks.world <= 1:
            return
        addr = os.environ.get('MASTER_ADDR', '127.0.0.1')
        port = host_port()
        if self.ranks.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.ranks.world)
            srv.settimeout(timeout)
            got = {}
            try:
                while len(got) < self.ranks.world - 1:
                    c, _ = srv.accept()
                    c.settimeout(timeout)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack('<i', _recv_exact(c, 4))
                    if not 0 < r < self.ranks.world or r in got:
                        c.close()
                        raise RuntimeError('host group: unexpected rank %d' % r)
                    got[r] = c
            finally:
                srv.close()
            self.peers = [got[r] for r in range(1, self.ranks.world)]
        else:
            t_end = time.monotonic() + timeout
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > t_end:
                        raise
                    time.sleep(0.05)                # rank 0 not listening yet
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack('<i', self.ranks.rank))
            self.sock = s

    # one round: every rank's payload to rank 0, fn(list of payloads in rank
    # order) -> per-rank replies (or one reply for all)
    def _round(self, payload, fn):
        if self.ranks.world <= 1:
            out = fn([payload])
            return out[0] if isinstance(out, list) else out
        if self.ranks.rank == 0:
            parts = [payload] + [_recv(c) for c in self.peers]
            out = fn(parts)
            replies = out if isinstance(out, list) else [out] * self.ranks.world
            for c, rep in zip(self.peers, replies[1:]):
                _send(c, rep)
            return replies[0]
        _send(self.sock, payload)
        return _recv(self.sock)

    def barrier(self):
        self._round(b'', lambda parts: b'')

    def _reduce(self, v, op):
        out = self._round(struct.pack('<d', float(v)),
                          lambda parts: struct.pack('<d', op(struct.unpack('<d', p)[0] for p in parts)))
        return struct.unpack('<d', out)[0]

    def max(self, v):
        return self._reduce(v, max)

    def min(self, v):
        return self._reduce(v, min)

    def sum(self, v):
        return self._reduce(v, lambda xs: float(np.sum(list(xs))))

    def broadcast_bytes(self, data):
        """Rank 0's bytes on every rank (the RCCL unique id)."""
        return self._round(bytes(data) if self.ranks.rank == 0 else b'', lambda parts: parts[0])

    def gather(self, obj, dst=0):
        """Per-rank objects (this process's own results) on rank 0, as a list
        in rank order; None elsewhere."""
        if dst != 0:
            raise ValueError('host group: gathers go to rank 0')
        blob = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        if self.ranks.world <= 1:
            return [obj]
        if self.ranks.rank == 0:
            parts = [blob] + [_recv(c) for c in self.peers]
            for c in self.peers:
                _send(c, b'')
            return [pickle.loads(p) for p in parts]
        _send(self.sock, blob)
        _recv(self.sock)
        return None

    def close(self):
        for c in self.peers:
            c.close()
        self.peers = []
        if self.sock is not None:
            self.sock.close()
            self.sock = None
