"""beam_search(debug=True): the per-position dump of every grown hypothesis
(`lattice_tagger/beam/beam.py:53-57`) printed from the device trace
(lt_decode_trace) equals, character for character, what the REFERENCE printed
for the same lattices (tests/golden/debug.json.gz, made by
tests/golden/make_debug_golden.py from the reference itself)."""
import contextlib
import gzip
import io
import json
import os

import numpy as np
import pytest

import golden_io
from lattice_based_tagger_amd import beam_search, _capi
from lattice_based_tagger_amd.beam import Decoder, lowered_model
from lattice_based_tagger_amd.packer import pack

pytestmark = pytest.mark.gpu

DUMPS = json.load(gzip.open(os.path.join(golden_io.GOLDEN, 'debug.json.gz'), 'rt', encoding='utf-8'))
_SETS = {}


def _case(name, idx):
    if name not in _SETS:
        _SETS[name] = golden_io.load(name)
    return _SETS[name][idx]


@pytest.mark.parametrize('dump', DUMPS, ids=['%s-%d-k%d' % (d['set'], d['index'], d['beam']) for d in DUMPS])
def test_debug_dump_equals_reference(gpu_decoder, dump):
    case = _case(dump['set'], dump['index'])
    buf = io.StringIO()
    err = msg = None
    with contextlib.redirect_stdout(buf):
        try:
            got = beam_search(case.bindex, case.chars, case.funcs, beam_size=dump['beam'],
                              max_len=case.max_len, debug=True)
        except Exception as exc:
            err, msg = type(exc).__name__, str(exc)
    assert err == dump['error'], msg
    assert buf.getvalue() == dump['stdout']
    if err is None:
        # the returned matures are the decoder's, unchanged by debug
        plain = beam_search(case.bindex, case.chars, case.funcs, beam_size=dump['beam'], max_len=case.max_len)
        assert [float(m.score).hex() for m in got] == [float(m.score).hex() for m in plain]


@pytest.mark.parametrize('k', [1, 4])
def test_trace_beams_equal_decoder(gpu_decoder, k):
    """The trace's final beam (its own top-k selection) equals the optimised
    kernels' matures: node paths and 0-ULP scores."""
    from lattice_based_tagger_amd import synth
    raw = synth.make_lattices(64, seed=11, eojeols=6)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=11, n_features=20_000)
    packed, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    dec = Decoder.get(0)
    dm = _capi.DeviceModel(dec.ctx, keys, coefs)
    db = _capi.DeviceBatch(dec.ctx, packed, max_k=k)
    try:
        count, length, score, codes = db.decode(dm, k)
        tr = db.trace(dm, k)
    finally:
        db.close()
        dm.close()
    n = np.asarray(packed.sent_n)
    off = tr['exp_off']
    for s in range(len(n)):
        pe = int(tr['pos_off'][s] + n[s])
        assert int(tr['beam_count'][pe]) == int(count[s])
        for r in range(int(count[s])):
            g = int(tr['beam_gen'][pe, r])
            assert tr['exp_score'][off[pe] + g].view(np.uint64) == score[s, r].view(np.uint64)
