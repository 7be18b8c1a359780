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
    """A read-only coefficient array cannot change, so its identity is its
    fingerprint (no per-call hash of the array); a read-only view of a
    writeable array is still hashed (the owner can write through)."""
    owned = np.arange(1000, dtype=np.float64)
    owned.flags.writeable = False
    assert beam._digest_array(owned)[0] == 'ro'
    base = np.arange(1000, dtype=np.float64)
    view = base[:]
    view.flags.writeable = False
    d0 = beam._digest_array(view)
    assert d0[0] != 'ro'
    base[3] = -1.0
    assert beam._digest_array(view) != d0
