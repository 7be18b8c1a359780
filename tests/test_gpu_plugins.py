"""User scoring plugins of (wj, wk) on the device (`score_funcs.py:7-15,
50-54`): the reference's own vectors (tests/golden/plugins.json.gz, made by
make_golden.py with the plugin inside the reference's composite) through the
drop-in API -- every tuned kernel (k = 1, 5, 16), the general kernel
(max_len 12, k = 300), launch pieces, evaluate and the score types."""

import numpy as np
import pytest

from golden_io import beams_of, load, path_matches
from lattice_based_tagger_amd import beam_search, beam_search_batch, evaluate_batch
from lattice_based_tagger_amd.word import Word, bos_word, eos_word

pytestmark = pytest.mark.gpu


def _groups():
    groups = {}
    for c in load('plugins'):
        groups.setdefault((id(c.funcs), c.max_len), []).append(c)
    return list(groups.values())


def _check(cases, k):
    got = beam_search_batch([(c.bindex, c.chars) for c in cases], cases[0].funcs, beam_size=k,
                            max_len=cases[0].max_len)
    n = 0
    for c, matures in zip(cases, got):
        exp = c.expected[str(k)]['matures']
        assert len(matures) == len(exp), (c.tag, k)
        for m, (codes, shex, kind) in zip(matures, exp):
            assert float(m.score).hex() == shex, (c.tag, k)
            assert type(m.score).__name__ == kind, (c.tag, k, type(m.score), kind)
            assert path_matches(c, codes, m.sequences[1:-1]), (c.tag, k)
            n += 1
    return n


def test_plugin_vectors_on_gpu(gpu_decoder):
    checked = 0
    for group in _groups():
        for k in beams_of(group):
            checked += _check([c for c in group if str(k) in c.expected], k)
    assert checked > 500


def test_plugin_vectors_in_several_launch_pieces(gpu_decoder):
    """Edge values are sliced per launch piece (lt_batch_create rebases each
    node's edge base to its piece's block)."""
    from lattice_based_tagger_amd import _capi
    lib = _capi.load()
    old = lib.lt_set_piece_bytes(60_000)
    try:
        for group in _groups():
            if group[0].max_len == 8:
                _check(group, 5)
    finally:
        lib.lt_set_piece_bytes(old)


def test_plugin_single_sentence_and_debug(gpu_decoder):
    case = [c for c in load('plugins') if c.model == 'edge_first_last'][0]
    exp = case.expected['5']['matures']
    for debug in (False, True):
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            got = beam_search(case.bindex, case.chars, case.funcs, beam_size=5, debug=debug)
        assert [float(m.score).hex() for m in got] == [e[1] for e in exp]


def test_plugin_evaluate_matches_reference(gpu_decoder):
    checked = 0
    for group in _groups():
        paths, want = [], []
        for c in group:
            for k, exp in c.expected.items():
                for (codes, _, _), ev in zip(exp['matures'], exp['evaluate']):
                    if isinstance(ev, dict):
                        continue
                    words = [bos_word()]
                    for code in codes:
                        if code[0] == 'U':
                            sub = c.chars[code[1]:code[2]]
                            words.append(Word(sub, sub, None, 'Unknown', None, code[2] - code[1], code[1],
                                              code[2], False))
                        else:
                            words.append(c.node(code))
                    words.append(eos_word(len(c.chars)))
                    paths.append(words)
                    want.append(ev[0])
        got = evaluate_batch(paths, group[0].funcs)
        for v, h in zip(got, want):
            assert float(v).hex() == h
            checked += 1
    assert checked > 500
