"""BeamScoreFunctions.evaluate against the reference's own
values: tests/golden/*.json.gz record ``funcs.evaluate(m)`` of every mature
the reference returned (make_golden.py).  CPU: the restated scorers; GPU:
``evaluate_batch`` (lt_evaluate) over all matures of a set in one launch."""

import pytest

from golden_io import MULTI_SETS, PLUGIN_SETS, SETS, load
from lattice_based_tagger_amd import evaluate_batch
from lattice_based_tagger_amd.word import Word, bos_word, eos_word


def _paths(name):
    """(funcs, sequence words [BOS, ..., EOS], expected hex) per mature."""
    out = []
    for c in load(name):
        for k, exp in c.expected.items():
            if 'matures' not in exp:
                continue
            for (codes, _, _), ev in zip(exp['matures'], exp['evaluate']):
                if isinstance(ev, dict):
                    continue
                words = [bos_word()]
                for code in codes:
                    if code[0] == 'U':
                        b, e = code[1], code[2]
                        sub = c.chars[b:e]
                        words.append(Word(sub, sub, None, 'Unknown', None, e - b, b, e, False))
                    else:
                        words.append(c.node(code))
                words.append(eos_word(len(c.chars)))
                out.append((c.funcs, words, ev[0]))
    return out


class _Seq:
    def __init__(self, words):
        self.sequences = words


@pytest.mark.parametrize('name', SETS + PLUGIN_SETS + MULTI_SETS)
def test_cpu_evaluate_matches_reference(name):
    paths = _paths(name)
    assert paths
    for funcs, words, hexv in paths:
        assert float(funcs.evaluate(_Seq(words))).hex() == hexv


@pytest.mark.gpu
@pytest.mark.parametrize('name', SETS + MULTI_SETS)
def test_gpu_evaluate_batch_matches_reference(gpu_decoder, name):
    groups = {}
    for funcs, words, hexv in _paths(name):
        groups.setdefault(id(funcs), (funcs, []))[1].append((words, hexv))
    checked = 0
    for funcs, items in groups.values():
        got = evaluate_batch([w for w, _ in items], funcs)
        for v, (_, hexv) in zip(got, items):
            assert float(v).hex() == hexv
            checked += 1
    assert checked > 0
