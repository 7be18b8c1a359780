"""User scoring plugins (CPU, no GPU): the reference's composite accepts any
BeamScoreFunction and calls it with the whole hypothesis
(`lattice_tagger/beam/score_funcs.py:7-15, 35-39, 50-54`).  A plugin that
declares ``edge_local = True`` reads only ``seq.sequences[-1]`` and the
appended word, so the build evaluates it once per lattice edge on the host
(packer.py) and the device adds the value in constructor order.

* the lowering's term plan follows the constructor order;
* every packed edge value is the plugin's own value for that (wj, wk);
* sub-batches (``slice``, ``take``) keep each node's values;
* a plugin with neither declaration is still refused loudly.
The decode itself is checked against the reference's vectors in
tests/test_gpu_plugins.py (and the pure-Python restatement in
tests/test_oracle_golden.py)."""

import numpy as np
import pytest

from golden_io import EdgeTableScore, load
from lattice_based_tagger_amd import BeamScoreFunctions, RegularizationScore, lowering
from lattice_based_tagger_amd.beam import lowered_model
from lattice_based_tagger_amd.packer import pack
from lattice_based_tagger_amd.score_funcs import BeamScoreFunction


def _cases(model_name):
    return [c for c in load('plugins') if c.model == model_name and c.chars]


def test_term_plan_follows_constructor_order():
    case = _cases('edge_first_last')[0]
    m = lowered_model(case.funcs)
    kinds = [k for k, _ in m.plan]
    # EdgeTable(morph0), Regularization, Trigram, WordPreference, EdgeTable(tag0):
    # no leading node-local scorer, so every scorer is a planned term
    assert kinds == [lowering.KIND_EDGE, lowering.KIND_NODE, lowering.KIND_TRI,
                     lowering.KIND_NODE, lowering.KIND_EDGE]
    assert m.pre_funcs == [] and m.n_post == 2 and m.n_edge == 2
    assert m.term_kinds == sum(k << (2 * t) for t, k in enumerate(kinds))
    mid = lowered_model(_cases('edge_mid')[0].funcs)
    assert [k for k, _ in mid.plan] == [lowering.KIND_EDGE, lowering.KIND_TRI]
    assert len(mid.pre_funcs) == 1


def test_packed_edge_values_are_the_plugins():
    cases = _cases('edge_first_last')[:4]
    funcs = cases[0].funcs
    model = lowered_model(funcs)
    packed, objs = pack([(c.bindex, c.chars) for c in cases], model)
    assert packed.n_edge == 2 and packed.edge_val.shape[0] == 2
    S = 8
    checked = 0
    for s, c in enumerate(cases):
        n = len(c.chars)
        ss = packed.span_start[packed.sent_span_off[s]:packed.sent_span_off[s + 1]]
        first = [0] + [int(ss[(e - 1) * S]) for e in range(1, n + 1)] + [int(ss[S * n])]
        g0 = int(packed.sent_node_off[s])
        for e in range(1, n + 1):
            for slot in range(S):
                b = e - (S - slot)
                for k in range(int(ss[(e - 1) * S + slot]), int(ss[(e - 1) * S + slot + 1])):
                    lo, hi = (0, 1) if b == 0 else (first[b], first[b + 1])
                    base = int(packed.node_edge_base[g0 + k])
                    assert packed.sent_edge_off[s] <= base + lo and base + hi <= packed.sent_edge_off[s + 1]
                    for j in range(lo, hi):
                        seq = lowering.EdgeSequence(objs[s][j])
                        for t, f in enumerate(model.edge_funcs):
                            assert packed.edge_val[t, base + j] == float(f.score(seq, objs[s][k]))
                            checked += 1
    assert checked > 1000


def test_sub_batches_keep_edge_values():
    cases = _cases('edge_mid')[:6]
    model = lowered_model(cases[0].funcs)
    packed, _ = pack([(c.bindex, c.chars) for c in cases], model)
    order = [4, 1, 1, 5]
    for sub, sel in ((packed.slice(2, 5), [2, 3, 4]), (packed.take(order), order)):
        for i, s in enumerate(sel):
            n0, n1 = packed.sent_node_off[s], packed.sent_node_off[s + 1]
            m0 = sub.sent_node_off[i]
            for v in range(n1 - n0):
                a = packed.node_edge_base[n0 + v] - packed.sent_edge_off[s]
                b = sub.node_edge_base[m0 + v] - sub.sent_edge_off[i]
                assert a == b
            e0, e1 = packed.sent_edge_off[s], packed.sent_edge_off[s + 1]
            f0, f1 = sub.sent_edge_off[i], sub.sent_edge_off[i + 1]
            assert np.array_equal(packed.edge_val[:, e0:e1], sub.edge_val[:, f0:f1])


def test_path_dependent_plugin_is_refused():
    class PathLength(BeamScoreFunction):       # reads the whole path: no declaration
        def score(self, seq, word_k):
            return len(seq.sequences)

    with pytest.raises(NotImplementedError):
        lowered_model(BeamScoreFunctions(RegularizationScore(), PathLength()))
    # an edge plugin is accepted anywhere in the composite
    lowered_model(BeamScoreFunctions(EdgeTableScore({}), RegularizationScore()))
