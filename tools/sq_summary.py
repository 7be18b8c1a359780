"""SQ counter summary of the decode kernels for bench.py's issue roofline.

Reads the per-dispatch tables tools/gpu_sq_ab.sh wrote (<dir>/<tag>_k<k>.txt,
tools/pmc_table.py format, the counting launch dropped) and writes a JSON list
with one entry per (kernel, k): VALU / LDS / SALU instructions per launch, LDS
bank-conflict and LDS-array cycles, VALU active cycles, and the source hash of
the build the counters came from (sha256 of csrc/lt_decode.hip, its first 16
hex digits), so that bench.py can tell whether they match the library it runs.

    python tools/sq_summary.py gpurun_out/r6b/sq base profiles/r06/sq_summary.json [--src-sha SHA]

The workload is tools/prof_decode.py's: the bench batch (65,536 sentences,
1M-key model, seed 0).
"""
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def src_sha():
    p = os.path.join(ROOT, 'lattice_based_tagger_amd', 'csrc', 'lt_decode.hip')
    return hashlib.sha256(open(p, 'rb').read()).hexdigest()[:16]


def main():
    d, tag, out = sys.argv[1:4]
    sha = sys.argv[sys.argv.index('--src-sha') + 1] if '--src-sha' in sys.argv else src_sha()
    import bench
    entries = []
    for f in sorted(os.listdir(d)):
        m = re.match(re.escape(tag) + r'_k(\d+)\.txt$', f)
        if not m:
            continue
        k = int(m.group(1))
        # the decode kernel of beam k (lt_decode.hip kernel_name_for); the
        # table also holds the counting launch's kernel (lt_beam_pk's COUNT
        # variant for k = 2..8), which is not the decode
        kernel = 'lt_viterbi_pk' if k <= 1 else 'lt_beam_hw' if k <= 8 else 'lt_beam_pk'
        ctr = {}
        for line in open(os.path.join(d, f)):
            t = line.split()
            if len(t) < 4 or re.sub(r'<.*', '', t[0]) != kernel:
                continue
            ctr[t[1]] = float(t[3].split('=')[1])
        if not ctr:
            continue
        entries.append({'kernel': kernel, 'k': k, 'sentences': 65536, 'features': 1_000_000, 'seed': 0,
                        'layout': bench.LAYOUT, 'src_sha': sha, 'counters_per_launch': ctr,
                        'source': os.path.relpath(os.path.join(d, f), ROOT)})
    os.makedirs(os.path.dirname(out) or '.', exist_ok=True)
    json.dump(entries, open(out, 'w'), indent=1)
    print('%d entries -> %s' % (len(entries), out))


if __name__ == '__main__':
    main()
