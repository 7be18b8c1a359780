"""L2 hit-rate model of the k=1 feature-table probes under alternative slot
layouts (CPU only; a design aid, not a measurement).

The probe stream: every dictionary node of a synthetic batch as w_k, with a
random node ending at its begin as w_j and one ending at w_j's begin as w_i
(the k=1 best path is one such node; word statistics are the same), the
feature keys of classes 0, 1, 2, 7, 8 after the node pre-filter (class 3 is
the LDS table).  Each key's probe count is its popularity; a layout maps keys
to 128 B lines; the L2 hit rate of an independent-reference stream over line
popularities p_i with C lines of capacity follows Che's approximation
(h = sum p_i (1 - exp(-p_i T)), sum (1 - exp(-p_i T)) = C).

    python tools/cache_model.py [sentences] [l2_lines]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from lattice_based_tagger_amd import synth, lowering as Lw   # noqa: E402


def che_hit(pop, C):
    p = pop[pop > 0].astype(np.float64)
    p /= p.sum()
    if len(p) <= C:
        return 1.0
    lo, hi = 0.0, 1.0
    while np.sum(1 - np.exp(-p * hi)) < C:
        hi *= 2
    for _ in range(60):
        T = 0.5 * (lo + hi)
        if np.sum(1 - np.exp(-p * T)) < C:
            lo = T
        else:
            hi = T
    return float(np.sum(p * (1 - np.exp(-p * lo))))


def probe_stream(S, seed=0):
    raw = synth.make_lattices(S, seed=seed)
    model = synth.make_model(raw, seed=seed)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    rng = np.random.default_rng(seed + 1)
    n = lay.n

    def ending(s_, e_):
        lo = lay.span_start[lay.span_base[s_] + (e_ - 1) * 8]
        hi = lay.span_start[lay.span_base[s_] + e_ * 8]
        return lay.node_off[s_] + lo + (rng.random(len(s_)) * (hi - lo)).astype(np.int64)

    k_nodes = lay.dict_pos
    s = raw.char_sent[raw.node_char].astype(np.int64)
    kb = lay.node_b[k_nodes]
    j = lay.node_off[s].copy()
    hj = kb > 0
    j[hj] = ending(s[hj], kb[hj])
    jb = np.where(hj, lay.node_b[j], 0)
    i = np.full(len(k_nodes), -1, np.int64)
    i[hj] = lay.node_off[s[hj]]
    hi2 = hj & (jb > 0)
    i[hi2] = ending(s[hi2], jb[hi2])
    probed, _, _, _ = synth._features_of(raw, lay, cols, k_nodes, j, i)
    probed = probed[probed[:, 0] != 3]
    # pre-filter: every component occurs in its key slot in some model key
    pk = model.probed
    ok = np.ones(len(probed), bool)
    for cls in (0, 1, 2, 7, 8):
        sel = probed[:, 0] == cls
        mk = pk[pk[:, 0] == cls]
        for pos in range(3):
            if (cls, pos) not in Lw.SLOT_BITS:
                continue
            ok[sel] &= np.isin(probed[sel, 1 + pos], mk[:, 1 + pos])
    probed = probed[ok]
    keys = synth._enc_rows(probed)
    model_keys = synth._enc_rows(pk)
    return keys, model_keys, pk


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    keys, model_keys, pk = probe_stream(S)
    uk, cnt = np.unique(keys, return_counts=True)
    present = np.isin(uk, model_keys)
    print('probes %d  distinct %d  present %.3f of probes' % (len(keys), len(uk), cnt[present].sum() / cnt.sum()))
    slots = 1 << 22
    lines = slots // 8
    rng = np.random.default_rng(5)
    # current layout: a key (present or absent) lands on a uniform random line
    line = rng.integers(0, lines, size=len(uk))
    pop = np.bincount(line, weights=cnt, minlength=lines)
    print('uniform hash, %d lines: L2 hit %.3f' % (lines, che_hit(pop, C)))
    # tiered: keys whose max component id < 2^t go to a dense region
    comps = synth._dec_rows(uk)
    V = 200_000                          # synth vocabulary: word ids 1..V, tags above
    word_only = lambda c: np.where(c > V, 0, c)
    mx = np.max(word_only(comps[:, 1:]), axis=1)
    mk = synth._dec_rows(model_keys)
    mmx = np.max(word_only(mk[:, 1:]), axis=1)
    for t in (8, 10, 11, 12, 13, 14):
        hot = mx < (1 << t)
        n_hot_keys = int(np.sum(mmx < (1 << t)))
        hot_lines = max(1, int(np.ceil(n_hot_keys / 8 / 0.7)))
        l2 = np.where(hot, rng.integers(0, hot_lines, size=len(uk)),
                      hot_lines + rng.integers(0, lines, size=len(uk)))
        pop = np.bincount(l2, weights=cnt, minlength=hot_lines + lines)
        print('tier ids < 2^%d: %d model keys (%.1f MB at load 0.7), %.3f of probes hot -> L2 hit %.3f'
              % (t, n_hot_keys, hot_lines * 128 / 1e6, cnt[hot].sum() / cnt.sum(), che_hit(pop, C)))


if __name__ == '__main__':
    main()
