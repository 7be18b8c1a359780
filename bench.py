#!/usr/bin/env python3
"""Benchmark of the MI355X lattice decoder (BASELINE.json metric).

One step = one decode of a 64K-sentence synthetic batch (BASELINE.json config
3: 20 eojeols x 2-5 characters, full-dictionary lattice statistics, 1M-key
trigram model, RegularizationScore + SimpleTrigramFeatureScore, beam k=1 =
Viterbi) that is already resident in HBM: decode kernel (incl. backtrace),
results written to HBM, stream sync.  Lattice build, packing and H2D happen
before the timed region.  The PCIe-inclusive rate (results copied to pinned
host memory every step) is measured separately and reported as
``pcie_inclusive_sentences_per_s`` -- never as ``value``.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--k 1] [--sentences 65536]

N > 1 is launched by torch.distributed.run (one process per GPU); each rank
decodes its own 64K-sentence shard (weak scaling, no data-path collective),
ranks are timed between barriers and the max over ranks is reported.
Rank 0 prints one JSON line.
"""

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# Load the HIP library before anything that could pull another HIP runtime in.
from lattice_based_tagger_amd import _capi, synth  # noqa: E402

METRIC = 'sentences/sec Viterbi decode, 64K-sentence batch; achieved HBM GB/s vs 8 TB/s'
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--k', type=int, default=1, help='beam size (1 = Viterbi headline)')
    ap.add_argument('--sentences', type=int, default=65536)
    ap.add_argument('--features', type=int, default=1_000_000)
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='budget of the pure-Python CPU baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--gather', type=int, default=None,
                    help='1: gather every rank\'s results to rank 0 with RCCL inside each step '
                         '(default: on when WORLD_SIZE > 1)')
    return ap.parse_args()


class Dist:
    """Rank bookkeeping; gloo process group for barrier / max (host only)."""

    def __init__(self, want):
        self.rank = int(os.environ.get('RANK', 0))
        self.world = int(os.environ.get('WORLD_SIZE', 1))
        self.local = int(os.environ.get('LOCAL_RANK', 0))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist          # after liblt is loaded
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            dist.init_process_group('gloo', rank=self.rank, world_size=self.world)
            self.pg = dist
        if want != self.world and self.rank == 0:
            print('warning: --gpus %d but WORLD_SIZE %d' % (want, self.world), file=sys.stderr)

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, v):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def min(self, v):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MIN)
        return float(t.item())

    def sum(self, v):
        if not self.pg:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def broadcast_bytes(self, data):
        """Rank 0's bytes on every rank (gloo; host only)."""
        if not self.pg:
            return data
        obj = [data]
        self.pg.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def make_workload(n_sent, seed, n_features):
    raw = synth.make_lattices(n_sent, seed=seed)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=seed, n_features=n_features)
    packed, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    return raw, lay, sm, packed, keys, coefs


def reachable_dict_nodes(raw):
    """Dictionary candidates on spans <= 8 inside the sentence (all generated ones)."""
    return int(len(raw.word))


def algorithmic_bytes(raw, packed, tuples, length, k):
    """B = 32*N + 8*(8n+1) + 4*8n + 24*P + 8*T*N + sum_matures (4*(L+1)+8),
    summed over the batch (N dictionary nodes, n chars, P trigram feature tuples
    of the reference algorithm, T = 1 node-local term, L words per mature)."""
    n = packed.sent_n.astype(np.int64)
    N = reachable_dict_nodes(raw)
    T = 1
    out = int(np.sum(4 * (length[length > 0] + 1) + 8)) if k else 0
    out += int(np.sum(length == 0) * 0)
    return 32 * N + int(np.sum(8 * (8 * n + 1) + 4 * 8 * n)) + 24 * tuples + 8 * T * N + out


def cpu_baseline(raw, sm, budget_s):
    """Pure-Python restatement of the reference beam_search (oracle/ref_beam.py,
    1 core) on the first sentences of the same batch, ~budget_s seconds."""
    from lattice_based_tagger_amd import score_funcs as SF, feature as FE
    from oracle import ref_beam
    dic, coef = synth.render_model(raw, sm)
    funcs = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                  SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    done = 0
    dt = 0.0
    chunk = 256
    while dt < budget_s and done < raw.S:
        sents = synth.render_sentences(raw, range(done, min(done + chunk, raw.S)))
        t0 = time.perf_counter()
        for bindex, chars in sents:
            ref_beam.beam_search(bindex, chars, funcs, beam_size=1)
            done += 1
            if dt + time.perf_counter() - t0 >= budget_s:
                break
        dt += time.perf_counter() - t0
    return {'value': done / dt, 'unit': 'sentences/s', 'cores': 1, 'kind': 'port',
            'sample': '%d sentences (first of the 64K batch, %.1f chars avg), k=1, '
                      'oracle/ref_beam.py pure-Python restatement of beam.py:5-61, %.1f s'
                      % (done, float(raw.sent_n[:done].mean()), dt)}


_POOL = {}


def _pool_worker(args):
    """One process of cpu_baseline_pool: render and decode sentences lo..hi
    step `step` with the pure-Python restatement; returns (count, decode s)."""
    lo, hi, step = args
    from oracle import ref_beam
    raw, funcs = _POOL['raw'], _POOL['funcs']
    idx = list(range(lo, hi, step))
    sents = synth.render_sentences(raw, idx)
    t0 = time.perf_counter()
    for bindex, chars in sents:
        ref_beam.beam_search(bindex, chars, funcs, beam_size=1)
    return len(idx), time.perf_counter() - t0


def cpu_baseline_pool(raw, sm, procs, budget_s):
    """The pure-Python restatement (as cpu_baseline) on `procs` host cores at
    once: multiprocessing (fork, before this process touches the GPU), each
    worker a strided share of the batch prefix; rate = sentences / the
    slowest worker's decode time."""
    import multiprocessing as mp
    from lattice_based_tagger_amd import score_funcs as SF, feature as FE
    dic, coef = synth.render_model(raw, sm)
    _POOL['raw'] = raw
    _POOL['funcs'] = SF.BeamScoreFunctions(SF.RegularizationScore(),
                                           SF.SimpleTrigramFeatureScore(FE.SimpleTrigramEncoder(dic), coef))
    n = int(min(raw.S, 500 * procs * budget_s))
    with mp.get_context('fork').Pool(procs) as pool:
        res = pool.map(_pool_worker, [(r, n, procs) for r in range(procs)])
    _POOL.clear()
    done = sum(c for c, _ in res)
    slow = max(t for _, t in res)
    return {'value': done / slow, 'unit': 'sentences/s', 'cores': procs, 'kind': 'port',
            'sample': 'first %d sentences of the batch, k=1, oracle/ref_beam.py pure-Python restatement '
                      'of beam.py:5-61 in %d processes (one per host core of the job), slowest '
                      'worker %.1f s' % (done, procs, slow)}


def cpu_baseline_c(packed, keys, coefs, k, budget_s):
    """The C restatement (oracle/lt_oracle.c: sorted-key binary search, OpenMP
    over sentences) on the host cores available to this job, on a bounded
    prefix of the same batch sized to about budget_s seconds."""
    from oracle import lt_oracle
    threads = max(1, min(int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1)), 64))
    S = len(packed.sent_n)
    n = min(S, 2048)
    t0 = time.perf_counter()
    lt_oracle.decode(packed, keys, coefs, k, 0, n, nthreads=threads)
    dt = time.perf_counter() - t0
    if dt < budget_s and n < S:
        n = int(min(S, n * max(1.0, budget_s / max(dt, 1e-3))))
        t0 = time.perf_counter()
        lt_oracle.decode(packed, keys, coefs, k, 0, n, nthreads=threads)
        dt = time.perf_counter() - t0
    return {'value': n / dt, 'unit': 'sentences/s', 'cores': threads, 'kind': 'port',
            'sample': 'first %d sentences of the batch, k=%d, oracle/lt_oracle.c (C restatement of '
                      'beam.py:5-61, OpenMP over sentences, %d threads; includes its per-call '
                      'sorted-key model build), %.2f s' % (n, k, threads, dt)}


def traffic_from_profiles(kernel, k, sentences, features, seed):
    """HBM bytes per launch of this configuration from the newest committed PMC
    summary (profiles/*traffic*.json, written by tools/traffic_summary.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench,
    FETCH_SIZE doubled per the gfx950 correction), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*traffic*.json'))):
        try:
            entries = json.load(open(f))
        except (OSError, ValueError):
            continue
        for e in entries:
            if (e.get('kernel'), e.get('k'), e.get('sentences'), e.get('features'), e.get('seed')) == \
                    (kernel, k, sentences, features, seed):
                best = (e['traffic_bytes_per_launch'], os.path.relpath(f, ROOT))
    return best


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    a = parse()
    lib = _capi.load()          # liblt binds its HIP runtime before torch (gloo) is imported
    d = Dist(a.gpus)
    t_gen = time.perf_counter()
    raw, lay, sm, packed, keys, coefs = make_workload(a.sentences, a.seed + 1000 * d.rank, a.features)
    t_gen = time.perf_counter() - t_gen
    host_cores = max(1, min(int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1)), 64))
    pool_baseline = None
    if not a.no_cpu_baseline and d.world == 1:
        # forked workers: before this process initialises the GPU
        pool_baseline = cpu_baseline_pool(raw, sm, host_cores, a.cpu_seconds / 2)
    ndev = lib.lt_device_count()
    if ndev < 1:
        raise SystemExit('bench.py: no HIP device visible')
    # one GPU per local rank; a launcher that shows each rank only its own
    # GPU (or a rehearsal with more ranks than GPUs) maps round-robin
    ctx = _capi.Context(d.local % ndev)
    dm = _capi.DeviceModel(ctx, keys, coefs)
    t_up = time.perf_counter()
    db = _capi.DeviceBatch(ctx, packed, max_k=a.k)          # H2D, outside the timed region
    t_up = time.perf_counter() - t_up
    expansions, tuples, probes = db.count_ops(dm, a.k)

    # result gather to rank 0 over RCCL/xGMI (the path's one exchange step)
    gather = d.world > 1 if a.gather is None else bool(a.gather)
    comm, gather_error = None, None
    if gather:
        try:
            uid = d.broadcast_bytes(_capi.comm_unique_id() if d.rank == 0 else None)
            comm = _capi.Comm(ctx, d.world, d.rank, uid)
            comm.prepare(db, a.k, root=0)
        except (_capi.LTError, OSError) as exc:      # reported in the JSON line, never silent
            gather_error = '%s: %s' % (type(exc).__name__, exc)
            print('bench.py: result gather disabled on rank %d: %s' % (d.rank, gather_error),
                  file=sys.stderr)
        if d.min(0.0 if gather_error else 1.0) < 1.0:  # every rank gathers, or none does
            if comm:
                comm.close()
            comm = None
            gather_error = gather_error or 'failed on another rank'

    def step():
        db.launch(dm, a.k)
        if comm:
            comm.launch(db)
        ctx.sync()

    for _ in range(max(1, a.warmup)):
        step()

    d.barrier()
    ctx.sync()
    kern_ms, gather_ms = [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        kern_ms.append(ctx.kernel_ms())
    if comm:
        comm.sync()
        gather_ms.append(comm.gather_ms())
    ctx.sync()
    if comm:
        comm.sync()
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    total_sent = d.sum(float(a.sentences * a.steps))

    # PCIe-inclusive rate (results to pinned host memory each step), untimed above
    pcie_steps = max(3, a.steps // 4)
    ctx.sync()
    tp = time.perf_counter()
    for _ in range(pcie_steps):
        db.launch(dm, a.k)
        db.fetch()
        ctx.sync()
    tp = time.perf_counter() - tp
    pcie_rate = d.sum(float(a.sentences * pcie_steps)) / d.max(tp)

    count, length, score, codes = db.results(a.k)
    gather_info = {'error': gather_error} if gather_error else None
    if comm:
        # the last gather delivered every rank's results of the same batch
        step()
        db.fetch()
        ctx.sync()
        comm.sync()
        count, length, score, codes = db.results(a.k)
        if d.rank == 0:
            comm.fetch()
            ctx.sync()
            g0 = comm.view(0)
            for x, y in zip(g0, (count, length, score, codes)):
                assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8)), \
                    'gathered rank-0 block differs from the local results'
            got = [comm.view(r) for r in range(d.world)]
            assert all(int(g[0].shape[0]) == a.sentences and int((g[0] > 0).sum()) == a.sentences
                       for g in got), 'gathered result blocks incomplete'
        gather_info = {'collective': 'ncclGather x4 in one group (RCCL), root 0, on its own '
                                     'stream: gather of step i overlaps decode of step i+1',
                       'rccl': (lib.lt_comm_library() or b'?').decode(),
                       'last_gather_ms': float(np.mean(gather_ms)) if gather_ms else None,
                       'in_timed_region': True}
    kernel = (lib.lt_kernel_name(a.k) or b'?').decode()
    traffic = traffic_from_profiles(kernel, a.k, a.sentences, a.features, a.seed)
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    B = algorithmic_bytes(raw, packed, tuples, length, a.k)
    achieved = B / avg_kernel_s / 1e9

    if d.rank == 0:
        line = {
            'metric': METRIC,
            'value': total_sent / elapsed,
            'unit': 'sentences/s',
            'n_gpus': d.world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (lattice_based_tagger_amd/synth.py, seed %d + 1000*rank)' % a.seed,
            'config': {
                'workload': 'config3: %d synthetic sentences/GPU, 20 eojeols x 2-5 chars, '
                            'full-dictionary lattice stats, %d-key trigram model, '
                            'Regularization+SimpleTrigram scorers, beam k=%d, max_len 8'
                            % (a.sentences, a.features, a.k),
                'sentences_per_gpu': a.sentences,
                'beam': a.k,
                'max_len': 8,
                'chars_per_sentence': float(packed.sent_n.mean()),
                'dict_nodes_per_sentence': reachable_dict_nodes(raw) / a.sentences,
                'parallelism': 'dp%d' % d.world,
            },
            'roofline': {
                'bound': 'hbm',
                'achieved': achieved,
                'peak': HBM_PEAK_GBS,
                'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS,
                'traffic': traffic[0] if traffic else None,
                'traffic_unit': 'HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)',
                'traffic_source': traffic[1] if traffic else None,
                'kernel': kernel,
                'algorithmic_bytes_per_launch': B,
                'avg_kernel_ms': avg_kernel_s * 1e3,
            },
            'ops_per_launch': {'expansions': expansions, 'feature_tuples': tuples,
                               'table_probes': probes},
            'kernel_only_sentences_per_s': a.sentences / avg_kernel_s,
            'pcie_inclusive_sentences_per_s': pcie_rate,
            'gather': gather_info,
            'host': {'gen_s': t_gen, 'h2d_s': t_up, 'nproc': os.cpu_count(), 'cpu': cpu_model(),
                     'visible_gpus': ndev},
        }
        if not a.no_cpu_baseline and d.world == 1:
            line['cpu_baseline'] = cpu_baseline(raw, sm, a.cpu_seconds)
            line['cpu_baseline_c'] = cpu_baseline_c(packed, keys, coefs, a.k, a.cpu_seconds / 2)
            line['cpu_baseline_pool'] = pool_baseline
        else:
            line['cpu_baseline'] = None
        print(json.dumps(line), flush=True)
    if comm:
        comm.close()
    db.close()
    dm.close()
    ctx.close()
    d.close()


if __name__ == '__main__':
    main()
