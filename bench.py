#!/usr/bin/env python3
"""Benchmark of the MI355X lattice decoder (BASELINE.json metric).

One step = one decode of the batch that is already resident in HBM, with
its results delivered to pinned host memory (kernel(s) +
backtrace + D2H of results inside the timed region): decode kernel (incl.
backtrace), results packed on the device (lt_results.hip) and their used
bytes copied to the host on a copy stream -- step i's copy runs under step
i+1's decode (two result slots per batch).  Lattice build, packing and H2D
happen before the timed region.

The default workload is BASELINE.json config 3: a 64K-sentence synthetic
batch (20 eojeols x 2-5 characters, full-dictionary lattice statistics,
1M-key trigram model, RegularizationScore + SimpleTrigramFeatureScore,
beam k=1 = Viterbi).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--k 1] [--sentences 65536]
                    [--scaling strong|weak]

N > 1 is launched by torch.distributed.run (one process per GPU).  Strong
scaling (default, the north star's "64K batch at 1, 2, 4 and 8 GPUs"): every
rank builds the same seeded batch and decodes one contiguous shard of it
(``dist.shard_range`` on sum (n+1)*k); each step ends with one RCCL gather
of every rank's packed results to rank 0 over xGMI and rank 0's D2H of all
of them.  ``--sentences 1048576`` is config 4 (the 64K generated lattices
in 16 seeded permutations).  ``--scaling weak``: each rank its own
64K-sentence batch.  Ranks are timed between barriers, the max over ranks
is reported; rank 0 checks the gathered results against a single-process
decode of the batch and prints one JSON line.
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
from lattice_based_tagger_amd import _capi, synth, lowering as Lw  # noqa: E402

METRIC = 'sentences/sec Viterbi decode, 64K-sentence batch; achieved HBM GB/s vs 8 TB/s'
HBM_PEAK_GBS = 8000.0
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles
# per SIMD (16 lanes wide; f64 adds at the same rate on CDNA4), 2.4 GHz
SIMDS = 1024
CLOCK_HZ = 2.4e9
VALU_PEAK_PER_S = SIMDS * CLOCK_HZ / 4
# the byte model's revision (roofline.byte_model_version): 2 = round 5 on,
# one slot load per probe must-move for the tuned beams (both issued);
# 1 = rounds 1-4, every issued slot load
BYTE_MODEL_VERSION = 2
# batch layout of this revision (implicit Unknowns, lattice_decode.h ABI 5): PMC
# traffic summaries are only matched to a run of the same layout
LAYOUT = 'abi5-rec32'


BASE_SENTENCES = 65536         # lattices generated per seed (config 3); larger batches permute them


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--k', type=int, default=1, help='beam size (1 = Viterbi headline)')
    ap.add_argument('--sentences', type=int, default=65536,
                    help='batch size (strong: whole batch; weak: per rank)')
    ap.add_argument('--scaling', choices=('strong', 'weak'), default='strong')
    ap.add_argument('--features', type=int, default=1_000_000)
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='budget of the pure-Python CPU baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-check', action='store_true', help='skip the post-run result check')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--gather', type=int, default=None,
                    help='1: gather every rank\'s results to rank 0 with RCCL inside each step '
                         '(default: on when WORLD_SIZE > 1; a failed RCCL setup then fails the run); '
                         '0: local delivery -- every rank copies its own shard\'s compact results to '
                         'pinned host memory over its own PCIe link, no RCCL (labelled in the JSON line)')
    ap.add_argument('--d2h', choices=('padded', 'packed'), default=None,
                    help='result delivery without the gather: padded arrays (the N=1 default) or the '
                         'compact slab (lt_result_fetch_packed; the default of --gather 0 at N > 1)')
    ap.add_argument('--no-wide-keys', dest='wide_keys', action='store_false',
                    help='skip the wide-key (ids >= 2^20) model entry under "extra"')
    ap.add_argument('--extra-k', default='5,16',
                    help='beams timed after the headline on the same batch (single GPU), reported under '
                         '"extra": BASELINE config 3 secondary (k=5) and config 5 (k=16); "" for none')
    return ap.parse_args()


class Dist(object):
    """Rank bookkeeping; barrier / max / sum / the RCCL id over the torch-free
    host group (lattice_based_tagger_amd/dist.py HostGroup: TCP, host only)."""

    def __init__(self, want):
        from lattice_based_tagger_amd.dist import HostGroup, Ranks
        r = Ranks()
        self.rank, self.world, self.local = r.rank, r.world, r.local
        self.g = HostGroup(r) if self.world > 1 else None
        if want != self.world and self.rank == 0:
            print('warning: --gpus %d but WORLD_SIZE %d' % (want, self.world), file=sys.stderr)

    def barrier(self):
        if self.g:
            self.g.barrier()

    def max(self, v):
        return self.g.max(v) if self.g else v

    def min(self, v):
        return self.g.min(v) if self.g else v

    def sum(self, v):
        return self.g.sum(v) if self.g else v

    def broadcast_bytes(self, data):
        """Rank 0's bytes on every rank (host only)."""
        return self.g.broadcast_bytes(data) if self.g else data

    def gather(self, obj):
        """Per-rank objects on rank 0 (list in rank order), None elsewhere."""
        return self.g.gather(obj) if self.g else [obj]

    def close(self):
        if self.g:
            self.g.close()


def make_workload(n_sent, seed, n_features):
    raw = synth.make_lattices(n_sent, seed=seed)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=seed, n_features=n_features)
    packed, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    return raw, lay, sm, packed, keys, coefs


def batch_order(total, base, seed):
    """Sentence order of a `total`-sentence batch over `base` generated
    lattices: identity when total <= base, else seeded permutations of the
    base lattices back to back (config 4's 1M batch = 16 permutations of
    the 64K lattices)."""
    if total <= base:
        return None
    rng = np.random.default_rng(seed + 4242)
    reps = -(-total // base)
    return np.concatenate([rng.permutation(base) for _ in range(reps)])[:total].astype(np.int64)


def shard_of(packed, order, k, world, rank):
    """Rank's contiguous shard [lo, hi) of the batch (balanced on (n+1)*k,
    SURVEY §8(e)) and its PackedBatch."""
    from lattice_based_tagger_amd.dist import shard_range
    n = np.asarray(packed.sent_n, dtype=np.int64)
    w = (n if order is None else n[order]) + 1
    lo, hi = shard_range(w * k, world, rank)
    if order is None:
        piece = packed if (lo, hi) == (0, packed.n_sent) else packed.slice(lo, hi)
    else:
        piece = packed.take(order[lo:hi])
    return lo, hi, piece


def algorithmic_bytes(piece, n_dict, tuples, length, count, k):
    """B = 32*N + 8*(8n+1) + 4*8n + 24*P + 8*T*N + sum_matures (4*(L+1)+8),
    summed over the launch's sentences (N dictionary nodes, n chars, P trigram
    feature tuples of the reference algorithm, T = 1 node-local term, L words
    per mature)."""
    n = np.asarray(piece.sent_n, dtype=np.int64)
    T = 1
    valid = np.arange(length.shape[1])[None, :] < count[:, None]
    out = int(np.sum(np.where(valid, 4 * (length.astype(np.int64) + 1) + 8, 0)))
    return 32 * n_dict + int(np.sum(8 * (8 * n + 1) + 4 * 8 * n)) + 24 * tuples + 8 * T * n_dict + out


PK_BPL = 96                    # k=1: end positions whose backpointers stay in LDS (lt_decode.hip)


def must_move_loads(table_loads, k):
    """Feature-table slot loads a kernel of this design cannot avoid, from the
    counting launch's issued loads: one per table probe past the node
    pre-filter, plus the secondary slot where the primary is flagged (a
    cuckoo key displaced to its second slot).  k=1 and the general kernel
    issue exactly that (primary first, secondary on a flag).  The tuned beam
    kernels load both slots of every probe in one round trip (the flag-free
    copy, lt_model.d_plain), so half their issued loads -- one per probe --
    is the lower bound; the other half is counted as issued, not as must-move
    (flagged primaries are about 1 in 5 probes, so this undercounts slightly)."""
    return table_loads if (k == 1 or k > 256) else table_loads // 2


def kernel_bytes(piece, table_loads, k, prep_bytes, blocks, d3, n_pairs=1):
    """The bytes the decode kernel moves per launch (the roofline's byte
    model, given the slot loads ``table_loads``; with must_move_loads a lower
    bound for this table layout): every node record once (32 B; the
    implicit Unknowns' records are staged from one 256 B block per workgroup,
    and at k=1 the class-4/6 pair table, ``n_pairs`` x 16 B, per workgroup),
    the k=1 lane schedule (``prep_bytes``) or, for beams, the span starts; the
    per-sentence offsets; 16 B per feature-table slot load (counted by the
    counting launch past the node pre-filter); the dense
    class-3 table staged per workgroup (``blocks`` x 8 KiB, where the model
    has one, ``d3``, and the kernel stages it); backpointers
    written and read back in HBM (k=1: only positions past the LDS window);
    the padded results written."""
    S = piece.n_sent
    n = np.asarray(piece.sent_n, dtype=np.int64)
    chars = int(n.sum())
    if k == 1:
        meta = 32 * S + prep_bytes                              # order, sent_n, node_off, bp_off, cum_n
        bp = 8 * int(np.maximum(n - PK_BPL + 1, 0).sum())       # write + backtrace read past the window
    else:
        meta = 40 * S + 4 * int(len(piece.span_start))
        bp = 4 * int(((n + 1) * k).sum()) + 4 * chars * k      # written per (position, rank), read on paths
    results = 16 * S * k + 4 * chars * k                        # count, length, score; padded codes
    stage = blocks * (256 + (16 * n_pairs if k == 1 else 0) + (8192 if d3 and k <= 4 else 0))
    return 32 * piece.n_nodes + meta + 16 * table_loads + stage + bp + results


def pair_count(batch):
    """Entries of the batch's class-4/6 pair table (lt_capi.cpp PairTable):
    the distinct (f4, f6) pairs of the nodes and implicit Unknowns, absent
    coefficients -0.0, plus the both-absent entry."""
    def pairs(mask, f4, f6):
        mask = np.asarray(mask, dtype=np.uint32)
        a = np.where(mask & Lw.F_HAS4, np.asarray(f4, dtype=np.float64), -0.0).view(np.uint64)
        b = np.where(mask & Lw.F_HAS6, np.asarray(f6, dtype=np.float64), -0.0).view(np.uint64)
        return np.stack([a, b], 1)
    x = [pairs(batch.node_mask, batch.node_f4, batch.node_f6), np.array([[1 << 63, 1 << 63]], dtype=np.uint64)]
    if getattr(batch, 'unk_n', 0):
        x.append(pairs(batch.unk_mask, batch.unk_f4, batch.unk_f6))
    return min(len(np.unique(np.concatenate(x), axis=0)), 127)


def has_dense3(keys):
    """The model gets a dense class-3 table (lt_capi.cpp build_dense3): its
    class-3 keys' tag values are at most 32."""
    keys = np.asarray(keys).reshape(-1, 4)
    c3 = keys[keys[:, 3] == 3]
    return 0 < len(np.unique(c3[:, :2])) <= 32


def workgroups(k, n_sent):
    """Workgroups of the decode launch (lt_decode.hip launch_k): each stages
    the dense class-3 table and the implicit-Unknown records."""
    if k == 1:
        return -(-n_sent // (8 * 8))                   # W = 8 sentences per wave, 8 waves per block (narrow keys)
    if k <= 8:
        wpb = 1 if k >= 5 else 4                       # HW8_WPB (k = 5..8, KT = 8), HW_WPB below
        return -(-n_sent // ((64 // (16 if k <= 3 else 32)) * wpb))
    return -(-n_sent // (1 if k <= 16 else 2))


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
    """Fabric bytes per launch of this configuration from the newest committed
    PMC summary of this batch layout (profiles/*traffic*.json, written by
    tools/traffic_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench, FETCH_SIZE doubled per the gfx950
    correction; Infinity-Cache hits included), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*traffic*.json'))):
        try:
            entries = json.load(open(f))
        except (OSError, ValueError):
            continue
        for e in entries:
            if (e.get('kernel'), e.get('k'), e.get('sentences'), e.get('features'), e.get('seed'),
                    e.get('layout')) == (kernel, k, sentences, features, seed, LAYOUT):
                best = (e['traffic_bytes_per_launch'], os.path.relpath(f, ROOT))
    return best


def decode_src_sha():
    """sha256 of the decode kernels' source (first 16 hex digits): ties a
    committed counter summary to the build it was measured on."""
    import hashlib
    p = os.path.join(ROOT, 'lattice_based_tagger_amd', 'csrc', 'lt_decode.hip')
    try:
        return hashlib.sha256(open(p, 'rb').read()).hexdigest()[:16]
    except OSError:
        return None


def issue_from_profiles(kernel, k, sentences, features, seed, kernel_s, expansions):
    """The VALU issue roofline of this configuration from the newest committed
    SQ counter summary of this batch layout (profiles/**/sq_summary*.json,
    tools/sq_summary.py over tools/gpu_sq_ab.sh): VALU wave-instructions per
    launch over this run's kernel time against the VALU issue peak, and the
    VALU busy fraction (SQ_ACTIVE_INST_VALU x 4 cycles / (SIMDs x kernel
    cycles)).  same_build: the summary's source hash equals this tree's
    lt_decode.hip.  None without a summary."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', '**', 'sq_summary*.json'), recursive=True)):
        try:
            entries = json.load(open(f))
        except (OSError, ValueError):
            continue
        for e in entries:
            if (e.get('kernel'), e.get('k'), e.get('sentences'), e.get('features'), e.get('seed'),
                    e.get('layout')) == (kernel, k, sentences, features, seed, LAYOUT):
                if best is None or e.get('src_sha') == decode_src_sha() or best[0].get('src_sha') != decode_src_sha():
                    best = (e, os.path.relpath(f, ROOT))
    if best is None:
        return None
    e, src = best
    c = e['counters_per_launch']
    valu = c.get('SQ_INSTS_VALU')
    act = c.get('SQ_ACTIVE_INST_VALU', valu)
    if not valu:
        return None
    out = {'bound': 'valu', 'achieved': valu / kernel_s, 'peak': VALU_PEAK_PER_S,
           'unit': 'VALU wave-instructions/s', 'frac': valu / kernel_s / VALU_PEAK_PER_S,
           'valu_busy': act * 4 / (SIMDS * CLOCK_HZ * kernel_s),
           'valu_per_launch': valu, 'valu_per_expansion': valu / expansions if expansions else None,
           'source': src, 'same_build': e.get('src_sha') == decode_src_sha()}
    if c.get('SQ_LDS_IDX_ACTIVE'):
        out['lds_conflict_frac'] = c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']
    return out


def roofline_bound(hbm_frac, traffic_frac, issue):
    """The resource the kernel runs closest to its peak on: 'valu' when the
    VALU busy fraction exceeds both the must-move byte fraction and the
    measured fabric-traffic fraction, else 'hbm'."""
    b = max(hbm_frac, traffic_frac or 0.0)
    return 'valu' if issue and issue['valu_busy'] > b else 'hbm'


def gather_ceiling(table_bytes):
    """Random 16 B gather ceiling of the MI355X for a table of table_bytes:
    the newest committed tools/gather_ceiling run (profiles/*/gather_ceiling.jsonl:
    uniformly random 16 B loads, 4-16 in flight per lane, every CU busy), the
    row of the smallest measured table at least this large, best over the
    loads in flight.  (loads/s, source) or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*', 'gather_ceiling*.jsonl')))
    if not files:
        return None
    rows = []
    for line in open(files[-1]):
        try:
            rows.append(json.loads(line))
        except ValueError:
            pass
    fit = [r for r in rows if r.get('table_bytes', 0) >= table_bytes]
    if not fit:
        return None
    tb = min(r['table_bytes'] for r in fit)
    return max(r['loads_per_s'] for r in fit if r['table_bytes'] == tb), os.path.relpath(files[-1], ROOT), tb


def probe_rate(table_loads, kernel_s, keys, slots, traffic=None):
    """The feature-table probes against the measured random-gather ceiling
    for the model's table size (tools/gather_ceiling.hip): the probes are
    spread 16 B loads, each L2 miss moves a 128 B line, so the roofline that
    binds them is a line rate, not HBM bytes.
      ratio_to_uniform_ceiling
                  issued slot loads per second / the uniform-random ceiling;
                  above 1.0 = cache reuse beyond uniform random (line groups,
                  Zipf-popular words, the hypotheses of one beam) -- so not a
                  roofline fraction (kept out of `roofline` since round 6)
      fabric_frac the kernel's L2-miss traffic (PMC, roofline.traffic) per
                  second / the ceiling's line rate (loads/s x 128 B)"""
    keys = np.asarray(keys).reshape(-1, 4)
    narrow = keys.size == 0 or int(keys[:, :3].max()) < (1 << 20)
    table_bytes = int(slots) * (16 if narrow else 32)
    rate = table_loads / kernel_s
    ceil = gather_ceiling(table_bytes)
    line_gbps = ceil[0] * 128 / 1e9 if ceil else None
    fabric_gbps = traffic / kernel_s / 1e9 if traffic else None
    return {'loads_per_s': rate, 'table_bytes': table_bytes,
            'ceiling_loads_per_s': ceil[0] if ceil else None,
            'ratio_to_uniform_ceiling': rate / ceil[0] if ceil else None,
            'ceiling_line_GBps': line_gbps,
            'fabric_GBps': fabric_gbps,
            'fabric_frac': fabric_gbps / line_gbps if (line_gbps and fabric_gbps) else None,
            'ceiling_source': ('%s (table of %d B)' % (ceil[1], ceil[2])) if ceil else None}


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
    strong = a.scaling == 'strong'
    k = a.k
    t_gen = time.perf_counter()
    seed = a.seed if strong else a.seed + 1000 * d.rank
    base_n = min(a.sentences, BASE_SENTENCES)
    raw, lay, sm, packed, keys, coefs = make_workload(base_n, seed, a.features)
    order = batch_order(a.sentences, base_n, seed)
    if strong:
        lo, hi, piece = shard_of(packed, order, k, d.world, d.rank)
    else:
        lo, hi = 0, a.sentences
        piece = packed if order is None else packed.take(order)
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
    db = _capi.DeviceBatch(ctx, piece, max_k=k)          # H2D, outside the timed region
    t_up = time.perf_counter() - t_up
    host_sched_ms = db.host_sched_ms()
    expansions, tuples, probes, table_loads = db.count_ops(dm, k)

    # result gather to rank 0 over RCCL/xGMI (the path's one exchange step)
    gather = d.world > 1 if a.gather is None else bool(a.gather)
    comm, gather_error = None, None
    if gather:
        try:
            uid = d.broadcast_bytes(_capi.comm_unique_id() if d.rank == 0 else None)
            comm = _capi.Comm(ctx, d.world, d.rank, uid)
            comm.prepare(db, k, root=0)
        except (_capi.LTError, OSError) as exc:
            gather_error = '%s: %s' % (type(exc).__name__, exc)
            print('bench.py: RCCL result gather failed on rank %d: %s' % (d.rank, gather_error),
                  file=sys.stderr)
        if d.min(0.0 if gather_error else 1.0) < 1.0:
            # the step includes the gather: without it there is
            # no valid multi-GPU number -- fail the run on every rank (--gather 0
            # is the explicit, labelled opt-out)
            if comm:
                comm.close()
            print('bench.py: rank %d exits: the RCCL gather could not be set up (%s); '
                  'run with --gather 0 to time the shards without the exchange'
                  % (d.rank, gather_error or 'failed on another rank'), file=sys.stderr)
            d.close()
            sys.exit(3)
    root = d.rank == 0
    d2h_mode = a.d2h or ('packed' if (d.world > 1 and not comm) else 'padded')

    def step():
        db.launch(dm, k)
        if comm:
            comm.launch(db)            # pack into the send slot + ncclGather (own stream)
            if root:
                comm.fetch()           # every rank's used bytes -> pinned host (copy stream)
        elif d2h_mode == 'packed':
            db.fetch_packed()          # compact slab on the device, its used bytes -> pinned host
        else:
            db.fetch()                 # DMA of the results -> pinned host (copy stream)

    def drain():
        ctx.sync()
        if comm:
            comm.sync()
            ctx.sync()

    for _ in range(max(1, a.warmup)):
        step()
    drain()

    d.barrier()
    drain()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    kern = ctx.kernel_ms_recent(a.steps)
    gather_ms = comm.gather_ms() if comm else None

    # fresh batch (k=1): the same step on a batch whose device preparation
    # (the lane schedule) is not built yet -- what every new chunk of
    # Tagger.tag_batch costs; lt_batch_reset_prep makes the next decode
    # rebuild it on the decode stream
    fresh = None
    if k == 1:
        def fresh_step():
            db.reset_prep()
            step()
        for _ in range(max(1, a.warmup)):
            fresh_step()
        drain()
        d.barrier()
        drain()
        tf0 = time.perf_counter()
        for _ in range(a.steps):
            fresh_step()
        drain()
        tf1 = time.perf_counter()
        d.barrier()
        fel = d.max(tf1 - tf0)
        fresh = {'value': total_sent_of(a, d, strong) / fel, 'unit': 'sentences/s',
                 'ms_per_step': fel / a.steps * 1e3, 'prep_ms_last': db.prep_ms(),
                 'prep_bytes': db.prep_bytes(), 'host_sched_ms': host_sched_ms,
                 'step': 'lane-schedule build (lt_k1_sched) + decode + result D2H of a batch not decoded '
                         'before, batch resident in HBM (H2D excluded, as the headline)'}
    total_sent = total_sent_of(a, d, strong)

    # results of the timed region's last step, checked (untimed)
    check = None
    if comm and root:
        got = [comm.view(r) for r in range(d.world)]
    elif not comm:
        got = [db.results_packed() if d2h_mode == 'packed' else padded_as_packed(db.results(k), piece.sent_n, k)]
    else:
        got = None
    mine = db.decode(dm, k)                                   # padded layout, this rank's shard
    if got is not None:
        mine_pk = got[0]
        assert all(np.array_equal(x, y) for x, y in zip(mine_pk.padded(piece.sent_n), mine)), \
            'packed results differ from the padded results of the same decode'
    if root and got is not None and not a.no_check:
        ref_db = _capi.DeviceBatch(ctx, packed, max_k=k)            # the whole (base) batch here
        ref = ref_db.decode_packed(dm, k)
        ref_db.close()
        base_idx = np.arange(packed.n_sent) if order is None else order
        if strong and comm:                  # every rank's shard: the whole batch
            check_results(got, ref, base_idx)
            what = 'all %d sentences of the batch, gathered from %d ranks over RCCL' % (a.sentences, d.world)
        elif strong:                         # this rank's shard only (no gather)
            check_results(got, ref, base_idx[lo:hi])
            what = ('all %d sentences of the batch' % a.sentences if d.world == 1 else
                    'rank 0 shard [%d, %d) of the batch (no gather)' % (lo, hi))
        else:                                # weak: rank 0's own batch, other blocks complete
            check_results(got[:1], ref, base_idx, (got, a.sentences) if comm else None)
            what = 'rank 0 batch of %d sentences%s' % (a.sentences, ', %d gathered blocks complete'
                                                        % len(got) if comm else '')
        check = {'what': what + ': equal to a single-process decode byte for byte', 'ok': True}
    count, length = mine[0], mine[1]
    kernel = (lib.lt_kernel_name(k) or b'?').decode()
    traffic = traffic_from_profiles(kernel, k, piece.n_sent, a.features, a.seed) \
        if (d.world == 1 or not strong) else None
    avg_kernel_s = float(np.mean(kern)) / 1e3
    nd = dict_nodes(raw, order, lo, hi)
    B = algorithmic_bytes(piece, nd, tuples, length, count, k)
    KB = kernel_bytes(piece, must_move_loads(table_loads, k), k, db.prep_bytes() if k == 1 else 0,
                      workgroups(k, piece.n_sent), has_dense3(keys), pair_count(piece))
    achieved = KB / avg_kernel_s / 1e9
    # the roofline's byte model is what the kernel must move: it cannot run
    # faster than HBM moves it
    assert achieved <= HBM_PEAK_GBS, 'byte model above the HBM peak: %.0f GB/s' % achieved
    issue = issue_from_profiles(kernel, k, piece.n_sent, a.features, a.seed, avg_kernel_s, expansions) \
        if (d.world == 1 or not strong) else None
    traffic_frac = traffic[0] / avg_kernel_s / 1e9 / HBM_PEAK_GBS if traffic else None
    al = lambda x: (x + 15) // 16 * 16                      # noqa: E731
    if comm or d2h_mode == 'packed':
        d2h = sum(32 + al(4 * g.n_sent) + al(4 * g.length.size) + al(8 * g.length.size) +
                  al(4 * g.codes.size) for g in got) if got is not None else None
    else:
        d2h = 4 * piece.n_sent * (1 + 3 * k) + 4 * int(np.sum(piece.sent_n)) * k

    extra = None
    extra_ks = [int(x) for x in a.extra_k.split(',') if x.strip()]
    if d.world == 1 and extra_ks:
        extra = {}
        for kx in extra_ks:
            if kx != k:
                extra['k%d' % kx] = time_beam(ctx, dm, piece, raw, order, lo, hi, kx, a, keys)
        if a.wide_keys:
            # the same batch and model with every id moved past 2^20: the wide
            # table format (32 B slots), at the largest extra beam
            wpiece, wkeys = synth.widen_ids(piece, keys)
            wdm = _capi.DeviceModel(ctx, wkeys, coefs)
            kw = max(extra_ks)
            extra['k%d_wide_keys' % kw] = time_beam(ctx, wdm, wpiece, raw, order, lo, hi, kw, a, wkeys,
                                                    with_traffic=False)
            extra['k%d_wide_keys' % kw]['model'] = ('the same model with every interned id + 2^20 '
                                                    '(synth.widen_ids): the wide table format, 32 B slots')
            wdm.close()

    if root:
        wl = ('config3' if a.sentences == 65536 else 'config4' if a.sentences == 1048576 else 'custom')
        line = {
            'metric': METRIC,
            'value': total_sent / elapsed,
            'unit': 'sentences/s',
            'n_gpus': d.world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3,
            'higher_is_better': True,
            'scaling': a.scaling,
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (lattice_based_tagger_amd/synth.py, seed %d%s)%s' % (
                a.seed, '' if strong else ' + 1000*rank',
                '' if order is None else '; %d generated lattices in seeded permutations' % base_n),
            'config': {
                'workload': '%s: %d synthetic sentences%s, 20 eojeols x 2-5 chars, '
                            'full-dictionary lattice stats, %d-key trigram model, '
                            'Regularization+SimpleTrigram scorers, beam k=%d, max_len 8; '
                            'step = decode + result D2H%s'
                            % (wl, a.sentences, ' split over %d GPUs' % d.world if strong else ' per GPU',
                               a.features, k, ' + RCCL gather to rank 0' if comm else ''),
                'sentences': a.sentences if strong else a.sentences * d.world,
                'sentences_rank0': piece.n_sent,
                'beam': k,
                'max_len': 8,
                'chars_per_sentence': float(np.mean(piece.sent_n)),
                'dict_nodes_per_sentence': nd / max(piece.n_sent, 1),
                'parallelism': 'dp%d' % d.world,
            },
            'roofline': {
                'bound': roofline_bound(achieved / HBM_PEAK_GBS, traffic_frac, issue),
                'achieved': achieved,
                'peak': HBM_PEAK_GBS,
                'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS,
                'traffic': traffic[0] if traffic else None,
                'traffic_unit': 'fabric bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE: HBM and '
                                'Infinity-Cache hits)',
                'traffic_source': traffic[1] if traffic else None,
                'traffic_frac': traffic_frac,
                'issue': issue,
                'kernel': kernel,
                'bytes_per_launch': KB,
                'byte_model_version': BYTE_MODEL_VERSION,
                'avg_kernel_ms': avg_kernel_s * 1e3,
                'launch': 'rank 0 shard' if d.world > 1 else 'whole batch',
                'frac_note': 'achieved = bytes the kernel must move per launch (bench.kernel_bytes: node records '
                             'once, lane schedule, offsets, 16 B per feature-table slot load a kernel of this '
                             'table layout cannot avoid (bench.must_move_loads), staged '
                             'tables, HBM backpointers, results) / average kernel time (HIP events over the '
                             'timed steps); issue = VALU wave-instructions per launch (committed SQ counter '
                             'summary, same_build: of this source) / the same time against the VALU issue '
                             'peak (1,024 SIMDs, 2.4 GHz, 4 cycles each); bound = the larger of the byte, '
                             'fabric-traffic and VALU-busy fractions',
                'layout': LAYOUT,
            },
            'work_equivalent': {'bytes_per_launch': B, 'GBps': B / avg_kernel_s / 1e9,
                                'note': 'SURVEY 8(d) bytes (24 B per reference feature tuple, most never '
                                        'loaded: node pre-filter, class 3 in LDS, classes 4-6 per node) / '
                                        'kernel time -- a work rate, not a memory measurement (exceeds '
                                        'the HBM peak)'},
            'probe_rate': probe_rate(table_loads, avg_kernel_s, keys, dm.slots, traffic[0] if traffic else None),
            'ops_per_launch': {'expansions': expansions, 'feature_tuples': tuples,
                               'table_probes': probes, 'table_slot_loads': table_loads},
            'kernel_only_sentences_per_s': piece.n_sent / avg_kernel_s,
            'fresh_batch': fresh,
            'd2h': {'bytes_per_step': d2h, 'in_timed_region': True, 'mode': 'root' if comm else d2h_mode,
                    'how': ('rank 0: every rank\'s packed results (gathered slabs), used bytes to '
                            'pinned host memory on a copy stream' if comm else
                            'this rank\'s compact result slab (packed on the device), used bytes to '
                            'pinned host memory on a copy stream' if d2h_mode == 'packed' else
                            'padded results by DMA to pinned host memory on a copy stream') +
                           ', under the next decode'},
            'gather': ({'collective': 'one ncclGather of packed result slabs (RCCL), root 0, on its '
                                      'own stream: gather of step i overlaps decode of step i+1',
                        'rccl': (lib.lt_comm_library() or b'?').decode(),
                        'last_gather_ms': gather_ms, 'in_timed_region': True} if comm else
                       {'mode': 'local',
                        'disabled': '--gather 0: every rank decodes its shard and copies its own compact '
                                    'results to pinned host memory over its own PCIe link (no RCCL); the '
                                    'results end in N processes of one node, not in rank 0 (the north '
                                    'star\'s single gather is the default mode)'}
                       if d.world > 1 else None),
            'check': check,
            'host': {'gen_s': t_gen, 'h2d_s': t_up, 'sched_ms': host_sched_ms, 'nproc': os.cpu_count(),
                     'cpu': cpu_model(), 'visible_gpus': ndev,
                     'note': 'h2d_s = lt_batch_create (validation, records, the k=1 schedule on the host '
                             'threads -- sched_ms of it -- uploads, the schedule fill), outside the timed region'},
        }
        if extra is not None:
            line['extra'] = extra
        if not a.no_cpu_baseline and d.world == 1:
            line['cpu_baseline'] = cpu_baseline(raw, sm, a.cpu_seconds)
            line['cpu_baseline_c'] = cpu_baseline_c(packed, keys, coefs, k, a.cpu_seconds / 2)
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


def total_sent_of(a, d, strong):
    """Sentences all ranks decode in a.steps steps."""
    return float(a.sentences * a.steps) if strong else d.sum(float(a.sentences * a.steps))


def time_beam(ctx, dm, piece, raw, order, lo, hi, k, a, keys, with_traffic=True):
    """The headline's step (decode + result D2H on the copy stream, batch
    resident in HBM) at beam k on the same batch, same warmup / steps, one
    GPU: BASELINE config 3's k=5 secondary and config 5 (k=16).  Results
    are bit-checked against lt_oracle.c in tests/test_gpu_parity.py."""
    lib = _capi.load()
    db = _capi.DeviceBatch(ctx, piece, max_k=k)                 # H2D, outside the timed region
    try:
        expansions, tuples, probes, table_loads = db.count_ops(dm, k)
        for _ in range(max(1, a.warmup)):
            db.launch(dm, k)
            db.fetch()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            db.launch(dm, k)
            db.fetch()
        ctx.sync()
        elapsed = time.perf_counter() - t0
        kern = ctx.kernel_ms_recent(a.steps)
        count, length = db.results(k)[:2]
    finally:
        db.close()
    kernel = (lib.lt_kernel_name(k) or b'?').decode()
    avg_kernel_s = float(np.mean(kern)) / 1e3
    B = algorithmic_bytes(piece, dict_nodes(raw, order, lo, hi), tuples, length, count, k)
    blocks, d3 = workgroups(k, piece.n_sent), has_dense3(keys)
    KB = kernel_bytes(piece, must_move_loads(table_loads, k), k, 0, blocks, d3)
    KI = kernel_bytes(piece, table_loads, k, 0, blocks, d3)              # as issued (both cuckoo slots)
    assert KI / avg_kernel_s / 1e9 <= HBM_PEAK_GBS, 'issued byte model above the HBM peak'
    traffic = traffic_from_profiles(kernel, k, piece.n_sent, a.features, a.seed) if with_traffic else None
    traffic_frac = traffic[0] / avg_kernel_s / 1e9 / HBM_PEAK_GBS if traffic else None
    issue = issue_from_profiles(kernel, k, piece.n_sent, a.features, a.seed, avg_kernel_s, expansions) \
        if with_traffic else None
    return {
        'beam': k,
        'value': piece.n_sent * a.steps / elapsed,
        'unit': 'sentences/s',
        'ms_per_step': elapsed / a.steps * 1e3,
        'step': 'decode + result D2H (pinned, copy stream), batch resident in HBM',
        'kernel': kernel,
        'avg_kernel_ms': avg_kernel_s * 1e3,
        'kernel_only_sentences_per_s': piece.n_sent / avg_kernel_s,
        'roofline': {'bound': roofline_bound(KB / avg_kernel_s / 1e9 / HBM_PEAK_GBS, traffic_frac, issue),
                     'achieved': KB / avg_kernel_s / 1e9, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': KB / avg_kernel_s / 1e9 / HBM_PEAK_GBS,
                     'bytes_per_launch': KB,
                     'byte_model_version': BYTE_MODEL_VERSION,
                     'issued_bytes_per_launch': KI,
                     'issued_frac': KI / avg_kernel_s / 1e9 / HBM_PEAK_GBS,
                     'traffic': traffic[0] if traffic else None,
                     'traffic_source': traffic[1] if traffic else None,
                     'traffic_frac': traffic_frac,
                     'issue': issue},
        'work_equivalent': {'bytes_per_launch': B, 'GBps': B / avg_kernel_s / 1e9},
        'probe_rate': probe_rate(table_loads, avg_kernel_s, keys, dm.slots, traffic[0] if traffic else None),
        'ops_per_launch': {'expansions': expansions, 'feature_tuples': tuples,
                           'table_probes': probes, 'table_slot_loads': table_loads},
    }


def padded_as_packed(res, sent_n, k):
    """PackedResults of padded results (count, length, score, codes)."""
    count, length, score, codes = res
    n = np.asarray(sent_n, dtype=np.int64)
    cum = np.zeros(len(n) + 1, dtype=np.int64)
    np.cumsum(n, out=cum[1:])
    out = _capi.PackedResults.__new__(_capi.PackedResults)
    out.k = k
    t = np.arange(k)[None, :]
    valid = t < count[:, None]
    out.count, out.length = count, np.where(valid, length, 0).astype(np.int32)
    out.score = np.where(valid, score, 0.0)
    L = out.length.ravel().astype(np.int64)
    out.off = np.zeros(L.size + 1, dtype=np.int64)
    np.cumsum(L, out=out.off[1:])
    e = np.repeat(np.arange(L.size, dtype=np.int64), L)
    j = np.arange(int(L.sum()), dtype=np.int64) - out.off[e]
    out.codes = codes[k * cum[e // k] + (e % k) * n[e // k] + j]
    return out


def dict_nodes(raw, order, lo, hi):
    """Dictionary nodes of the batch's sentences [lo, hi)."""
    per = np.bincount(raw.char_sent[raw.node_char], minlength=raw.S).astype(np.int64)
    return int(per[lo:hi].sum() if order is None else per[order[lo:hi]].sum())


def check_results(got, ref, idx, n_blocks_complete=None):
    """Rank 0: results delivered to the host by the timed region's last step
    -- ``got``: PackedResults blocks, consecutive in the batch -- against
    ``ref``, a single-process decode of the generated (base) batch; ``idx``:
    the base sentence of every row of the concatenated blocks.
    ``n_blocks_complete``: (blocks, sentences each) that must be complete
    besides (weak scaling: the other ranks' batches)."""
    from lattice_based_tagger_amd.beam import concat_results
    whole = concat_results(got)
    idx = np.asarray(idx, dtype=np.int64)
    assert whole.n_sent == len(idx), 'got %d of %d sentences' % (whole.n_sent, len(idx))
    k = ref.k
    L = ref.length.ravel().astype(np.int64)
    sel = (idx[:, None] * k + np.arange(k)[None, :]).ravel()
    seg = np.repeat(sel, L[sel])
    first = np.repeat(np.cumsum(L[sel]) - L[sel], L[sel])
    exp_codes = ref.codes[ref.off[seg] + np.arange(int(L[sel].sum())) - first]
    ok = (np.array_equal(whole.count, ref.count[idx]) and np.array_equal(whole.length, ref.length[idx]) and
          np.array_equal(whole.score.view(np.uint64), ref.score[idx].view(np.uint64)) and
          np.array_equal(whole.codes, exp_codes))
    assert ok, 'results differ from the single-process decode'
    if n_blocks_complete:
        blocks, each = n_blocks_complete
        assert len(blocks) and all(b.n_sent == each for b in blocks), 'gathered result blocks incomplete'
    return True


if __name__ == '__main__':
    main()
