"""The CPU oracle (oracle/ref_beam.py, a restatement of beam/beam.py:5-61) is
pinned against the reference's own outputs (tests/golden)."""

import pytest

from golden_io import MULTI_SETS, PLUGIN_SETS, SETS, load, path_matches
from oracle import ref_beam


@pytest.mark.parametrize('name', SETS + PLUGIN_SETS + MULTI_SETS)
def test_ref_beam_matches_reference(name):
    n_checked = 0
    for case in load(name):
        for k, exp in case.expected.items():
            k = int(k)
            if 'error' in exp:
                with pytest.raises(Exception) as ei:
                    ref_beam.beam_search(case.bindex, case.chars, case.funcs, k, case.max_len)
                assert type(ei.value).__name__ == exp['error']
                continue
            got = ref_beam.beam_search(case.bindex, case.chars, case.funcs, k, case.max_len)
            assert len(got) == len(exp['matures']), (case.tag, k)
            for (path, score), (codes, shex, _) in zip(got, exp['matures']):
                assert float(score).hex() == shex, (case.tag, k)
                assert path_matches(case, codes, list(path[1:-1])), (case.tag, k)
            n_checked += 1
    assert n_checked > 0


def test_dense_set_exercises_pairwise_branch():
    """The dense fixture must contain expansions with 8 or 9 present features
    (numpy's pairwise branch)."""
    hist = {}
    for case in load('dense'):
        dic = case.funcs.funcs[1].encoder.feature_dic
        for codes, _, _ in case.expected['16']['matures']:
            path = [ref_beam.OracleWord('BOS', 'BOS', None, 'BOS', None, 0, 0, 0, False)]
            for code in codes:
                w = case.node(code)
                if w is None:
                    b, e = code[1], code[2]
                    sub = case.chars[b:e]
                    w = ref_beam.OracleWord(sub, sub, None, 'Unknown', None, e - b, b, e, False)
                wi = path[-2] if len(path) > 1 else None
                m = sum(1 for f in ref_beam.trigram_features(wi, path[-1], w) if f in dic)
                hist[m] = hist.get(m, 0) + 1
                path.append(w)
    assert hist.get(8, 0) + hist.get(9, 0) > 0, hist


def test_config1_is_a_ten_eojeol_sentence():
    case = load('base')[0]
    assert case.tag == 'config1'
    assert case.expected['1']['matures']
