"""The static rule behind the decoders' dead implicit Unknowns
(lt_internal.h k1_unk_dead, lt_decode.hip cnt_live): an Unknown candidate of
span (b, e) with b > b_min is skipped after every hypothesis of beam[b] when
no dictionary word ends at b -- every hypothesis of beam[b] then ends in a
synthesised Unknown, so its num_unk is positive (beam.py:43-45,
Sequence.add :112-113).  The k=1 lane schedule gives such a candidate no
lane and the beam kernels give its span slot no expansions.

Checked here on the reference's own cases (tests/golden) at every beam of
their fixtures, through a copy of the oracle's loop (oracle/ref_beam.py,
beam.py:5-61) that records, for each synthesised Unknown, whether any of its
expansions was scored."""

import pytest

from golden_io import MULTI_SETS, PLUGIN_SETS, SETS, load
from oracle import ref_beam


def _dead_unknowns_scored(bindex, chars, funcs, beam_size, max_len):
    """Runs the reference loop; returns (statically dead Unknown candidates,
    how many of them had an expansion scored)."""
    n = len(chars)
    bos = ref_beam.OracleWord('BOS', 'BOS', None, 'BOS', None, 0, 0, 0, False)
    beams = [[(0, (bos,), 0)]]
    # position b holds a dictionary candidate (a word of bindex[a] ending at
    # b, a in [b_min(b), b))
    def has_word_ending(b):
        return any(w.e == b for a in range(max(0, b - max_len), b) for w in bindex[a])
    dead = scored = 0
    for e in range(1, n + 1):
        grown = []
        b_min = max(0, e - max_len)
        for b in range(b_min, e):
            cands = [w for w in bindex[b] if w.e == e]
            synth = not cands
            if synth:
                sub = chars[b:e]
                cands = [ref_beam.OracleWord(sub, sub, None, 'Unknown', None, e - b, b, e, False)]
            is_dead = synth and b > b_min and not has_word_ending(b)
            dead += is_dead
            for score, path, num_unk in beams[b]:
                for w in cands:
                    if num_unk > 0 and w.tag0 == 'Unknown' and b_min < b:
                        continue
                    scored += is_dead
                    inc = ref_beam.composite_increment(funcs.funcs, path, w)
                    grown.append((score + inc, path + (w,), num_unk + 1 if w.tag0 == 'Unknown' else 0))
        beams.append(sorted(grown, key=lambda h: -h[0])[:beam_size])
    return dead, scored


@pytest.mark.parametrize('name', SETS + PLUGIN_SETS + MULTI_SETS)
def test_statically_dead_unknowns_are_never_scored(name):
    total_dead = 0
    for case in load(name):
        for k, exp in case.expected.items():
            if 'error' in exp or case.max_len < 1:
                continue
            dead, scored = _dead_unknowns_scored(case.bindex, case.chars, case.funcs, int(k), case.max_len)
            assert scored == 0, (case.tag, k)
            total_dead += dead
    if name in ('base', 'synth', 'wide'):
        assert total_dead > 0                   # the rule has cases to hold on
