"""Lane use of the k=1 lane schedules on the bench lattices (CPU model).

Counts the macro-steps of the beam-1 decode for a sample of the bench batch
(synth.make_lattices, seed 0) under
  * the lockstep schedule of rounds 1-4: the W sentences of a wave at the same
    end position, ceil(sum of their candidates / 64) macro-steps per position;
  * the independent schedule of round 5 (lt_internal.h k1_schedule): at every
    macro-step the sentences are taken by priority (more end positions left
    first, then the lower index) while their candidates fit the lanes left.
Candidates of a sentence at end position e: every span's nodes, one implicit
Unknown for an empty span within max_len (lt_internal.h k1_candidates).

    python tools/k1_sched_model.py [--sentences 16384]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from lattice_based_tagger_amd import synth  # noqa: E402


def runs_of(raw):
    n = raw.sent_n.astype(np.int64)
    first = np.r_[0, np.cumsum(n)[:-1]]
    out = []
    for s in range(raw.S):
        c = np.maximum(raw.cnt[first[s]:first[s] + n[s]], 1)   # (position, span length): candidates
        out.append(np.array([sum(c[e - d, d - 1] for d in range(1, min(e, 8) + 1)) for e in range(1, n[s] + 1)]))
    return out


def lockstep(runs, w):
    steps = 0
    for w0 in range(0, len(runs), w):
        grp = runs[w0:w0 + w]
        m = np.zeros((len(grp), max(len(r) for r in grp)), dtype=np.int64)
        for i, r in enumerate(grp):
            m[i, :len(r)] = r
        steps += int(np.ceil(m.sum(0) / 64).sum())
    return steps


def independent(runs, w):
    steps = 0
    for w0 in range(0, len(runs), w):
        grp = runs[w0:w0 + w]
        pos = [0] * len(grp)
        while any(pos[i] < len(grp[i]) for i in range(len(grp))):
            live = sorted((i for i in range(len(grp)) if pos[i] < len(grp[i])),
                          key=lambda i: (-(len(grp[i]) - pos[i]), i))
            room = 64
            for r, i in enumerate(live):
                x = int(grp[i][pos[i]])
                if x > 64:
                    if r == 0:                      # a dense position, alone
                        steps += (x + 63) // 64 - 1
                        pos[i] += 1
                        break
                elif x <= room:
                    room -= x
                    pos[i] += 1
                if room == 0:
                    break
            steps += 1
    return steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sentences', type=int, default=16384)
    a = ap.parse_args()
    raw = synth.make_lattices(a.sentences, seed=0)
    runs = runs_of(raw)
    order = np.argsort(-raw.sent_n, kind='stable')           # the decoder's order: longest first
    runs = [runs[i] for i in order]
    lanes = sum(int(r.sum()) for r in runs)
    for w in (6, 8):
        for name, f in (('lockstep', lockstep), ('independent', independent)):
            st = f(runs, w)
            print('W=%d %-11s macro-steps %8d  lanes used %.3f' % (w, name, st, lanes / (64.0 * st)))


if __name__ == '__main__':
    main()
