"""The lowered-model cache follows the composite's contents (no GPU): the
reference reads the scorers' coefficients and tables live on every call
(score_funcs.py:63-105, 137-144), so a changed value must not decode with
the old tables."""

import numpy as np

from golden_io import load
from lattice_based_tagger_amd import beam
from lattice_based_tagger_amd.packer import pack


def _funcs():
    case = [c for c in load('demo') if c.bindex][0]
    return case, case.funcs


def test_cache_hits_while_unchanged():
    _, funcs = _funcs()
    beam.invalidate_model_cache()
    assert beam.lowered_model(funcs) is beam.lowered_model(funcs)


def test_scalar_table_and_coefficient_edits_relower():
    case, funcs = _funcs()
    beam.invalidate_model_cache()
    by = {type(f).__name__: f for f in funcs.funcs}
    m0 = beam.lowered_model(funcs)
    p0, _ = pack([(case.bindex, case.chars)], m0)
    reg = by['RegularizationScore']
    old = reg.unknown_penalty
    reg.unknown_penalty = old - 1.0
    try:
        m1 = beam.lowered_model(funcs)
        assert m1 is not m0
        p1, _ = pack([(case.bindex, case.chars)], m1)
        assert not np.array_equal(p0.node_pre, p1.node_pre)
    finally:
        reg.unknown_penalty = old
    tri = by['SimpleTrigramFeatureScore']
    m2 = beam.lowered_model(funcs)
    tri.coefficients[0] += 1.0               # in place
    try:
        m3 = beam.lowered_model(funcs)
        assert m3 is not m2
    finally:
        tri.coefficients[0] -= 1.0
    for name, attr in (('MorphemePreferenceScore', 'tag_to_morph'), ('WordPreferenceScore', 'tag_to_word')):
        f = by.get(name)
        if f is None:
            continue
        table = getattr(f, attr)
        m4 = beam.lowered_model(funcs)
        tag = next(iter(table)) if table else 'Noun'
        inner = table.setdefault(tag, {})
        inner['__probe__'] = 1.5                 # in-place edit of an inner dict
        try:
            assert beam.lowered_model(funcs) is not m4
        finally:
            del inner['__probe__']


def test_read_only_coefficients_skip_the_content_hash():
    """Coefficients over read-only memory (bytes, a read-only mmap: a model
    pack) cannot change, so their identity is their fingerprint (no per-call
    hash of the array).  An array that owns its memory is hashed even when
    read-only: its owner can set writeable back, edit it and clear the flag
    again; a read-only view of a writeable array likewise."""
    frozen = np.frombuffer(np.arange(1000, dtype=np.float64).tobytes(), dtype=np.float64)
    assert not frozen.flags.writeable
    assert beam._digest_array(frozen)[0] == 'ro'
    owned = np.arange(1000, dtype=np.float64)
    owned.flags.writeable = False
    d0 = beam._digest_array(owned)
    assert d0[0] != 'ro'
    owned.flags.writeable = True
    owned[7] = 123.0
    owned.flags.writeable = False
    assert beam._digest_array(owned) != d0
    base = np.arange(1000, dtype=np.float64)
    view = base[:]
    view.flags.writeable = False
    d1 = beam._digest_array(view)
    assert d1[0] != 'ro'
    base[3] = -1.0
    assert beam._digest_array(view) != d1


def test_flipped_writeable_flag_relowers_the_model():
    """Flip a read-only owned coefficient array writeable, edit it, flip it
    back: the next call lowers the model again (no stale scores)."""
    from golden_io import load
    case = load('synth')[0]
    tri = [f for f in case.funcs.funcs if type(f).__name__ == 'SimpleTrigramFeatureScore'][0]
    coef = tri.coefficients
    coef.flags.writeable = False
    try:
        m1 = beam.lowered_model(case.funcs)
        assert beam.lowered_model(case.funcs) is m1
        coef.flags.writeable = True
        coef[0] += 1.0
        coef.flags.writeable = False
        m2 = beam.lowered_model(case.funcs)
        assert m2 is not m1
        assert m2.coefs is not None
    finally:
        coef.flags.writeable = True
        coef[0] -= 1.0
