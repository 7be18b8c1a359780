"""Multi-GPU sharding of the decode (one process per GPU).

``beam_search`` has no cross-sentence state (`lattice_tagger/beam/beam.py:5-61`
decodes one sentence; `Tagger.tag` is per sentence, `tagger/tagger.py:68-78`),
so sentences shard across GPUs with no data-path collective: each rank decodes
a contiguous shard on its own device.  The process group (``gloo``, host only)
is used for the barrier / max-over-ranks timing of the benchmark and, when a
caller wants all results on one host, for an object gather after the decode.

``shard_range`` balances shards by characters (decode work is linear in the
sentence length).
"""

import os

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


class HostGroup:
    """gloo process group for host-side coordination (never on the data path)."""

    def __init__(self, ranks=None):
        self.ranks = ranks or Ranks()
        self.pg = None
        if self.ranks.world > 1:
            import torch.distributed as dist
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            if not dist.is_initialized():
                dist.init_process_group('gloo', rank=self.ranks.rank, world_size=self.ranks.world)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def _reduce(self, v, op):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.pg.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v):
        return self._reduce(v, self.pg.ReduceOp.MAX if self.pg else None)

    def sum(self, v):
        return self._reduce(v, self.pg.ReduceOp.SUM if self.pg else None)

    def gather(self, obj, dst=0):
        """Gather picklable per-rank results on ``dst`` (list in rank order)."""
        if not self.pg:
            return [obj]
        out = [None] * self.ranks.world if self.ranks.rank == dst else None
        self.pg.gather_object(obj, out, dst=dst)
        return out

    def close(self):
        if self.pg and self.pg.is_initialized():
            self.pg.destroy_process_group()
