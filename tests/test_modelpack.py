"""Model pack format: lowering parity of a packed model with
the in-memory one, file integrity, and (GPU) decode parity through the
golden vectors with the device table uploaded from the pack's image."""

import numpy as np
import pytest

from golden_io import SETS, load, path_matches
from lattice_based_tagger_amd import _capi, beam_search_batch, modelpack
from lattice_based_tagger_amd.lowering import LoweredModel
from lattice_based_tagger_amd.score_funcs import BeamScoreFunctions, SimpleTrigramFeatureScore


def _packed_funcs(funcs, tmp_path, name):
    out, path = [], None
    for f in funcs.funcs:
        if isinstance(f, SimpleTrigramFeatureScore):
            path = str(tmp_path / ('%s.ltm' % name))
            modelpack.save(path, f)
            f = modelpack.load(path)
        out.append(f)
    return BeamScoreFunctions(*out), path


def _models(name):
    seen = {}
    for c in load(name):
        seen.setdefault(id(c.funcs), c)
    return list(seen.values())


@pytest.mark.parametrize('name', ['demo', 'scorers', 'edge', 'dense'])
def test_packed_lowering_matches(tmp_path, name):
    for j, case in enumerate(_models(name)):
        funcs = case.funcs
        if not any(isinstance(f, SimpleTrigramFeatureScore) for f in funcs.funcs):
            continue
        pf, _ = _packed_funcs(funcs, tmp_path, '%s_%d' % (name, j))
        a, b = LoweredModel(funcs), LoweredModel(pf)
        assert a.vocab == b.vocab
        for x, y in ((a.vmask, b.vmask), (a.keys, b.keys)):
            assert np.array_equal(x, y)
        assert np.array_equal(a.coefs.view(np.uint64), b.coefs.view(np.uint64))
        assert b.image is not None or len(b.keys) == 0
        # node-local classes 4-6 and the reference-protocol scorer, on every node
        tri_a = [f for f in funcs.funcs if isinstance(f, SimpleTrigramFeatureScore)][0]
        tri_b = [f for f in pf.funcs if isinstance(f, SimpleTrigramFeatureScore)][0]
        assert tri_a.encoder.feature_dic == tri_b.encoder.feature_dic
        for ws in case.bindex:
            for w in ws:
                for unk in (False, True):
                    assert a.node_local_features(w, unk) == b.node_local_features(w, unk)


def test_image_is_deterministic_and_file_checked(tmp_path):
    case = _models('demo')[0]
    tri = [f for f in case.funcs.funcs if isinstance(f, SimpleTrigramFeatureScore)][0]
    p1, p2 = str(tmp_path / 'a.ltm'), str(tmp_path / 'b.ltm')
    modelpack.save(p1, tri)
    modelpack.save(p2, tri)
    assert open(p1, 'rb').read() == open(p2, 'rb').read()
    im = modelpack.ModelPack(p1).image
    lm = LoweredModel(case.funcs)
    fresh = _capi.ModelImage(lm.keys, lm.coefs).arrays()
    assert np.array_equal(np.asarray(im['table']), fresh['table'])
    assert (im['seed'], im['slots'], im['narrow'], im['d3mul']) == \
        (fresh['seed'], fresh['slots'], fresh['narrow'], fresh['d3mul'])
    # a flipped byte in a blob is detected
    raw = bytearray(open(p1, 'rb').read())
    raw[-1] ^= 0xFF
    bad = str(tmp_path / 'bad.ltm')
    open(bad, 'wb').write(bytes(raw))
    with pytest.raises(ValueError):
        modelpack.ModelPack(bad)
    with pytest.raises(ValueError):
        open(bad, 'r+b').write(b'NOTAPACK')
        modelpack.ModelPack(bad)


@pytest.mark.gpu
@pytest.mark.parametrize('name', SETS)
def test_packed_model_decodes_golden_vectors(gpu_decoder, tmp_path, name):
    cases = load(name, packable=True)
    groups = {}
    for c in cases:
        groups.setdefault((id(c.funcs), c.max_len), []).append(c)
    checked = 0
    for gi, group in enumerate(groups.values()):
        ok = [c for c in group if not any('error' in e for e in c.expected.values())]
        if not ok:
            continue
        pf, path = _packed_funcs(ok[0].funcs, tmp_path, '%s_%d' % (name, gi))
        if path is None:
            continue
        for k in (1, 5):
            got = beam_search_batch([(c.bindex, c.chars) for c in ok], pf, beam_size=k,
                                    max_len=ok[0].max_len)
            for c, matures in zip(ok, got):
                if str(k) not in c.expected:
                    continue
                exp = c.expected[str(k)]['matures']
                assert len(matures) == len(exp)
                for m, (codes, shex, _) in zip(matures, exp):
                    assert float(m.score).hex() == shex
                    assert path_matches(c, codes, m.sequences[1:-1])
                    checked += 1
    assert checked > 0 or name == 'base'


@pytest.mark.parametrize('name', ['demo', 'base', 'scorers', 'dense'])
def test_dense_class3_table_uses_a_bit_window(name):
    """The dense class-3 table's index (lt_common.h d3_index) is a bit window
    v[off, off + 5) of the interned tag id when one separates the model's
    class-3 tag values (d3_window: the kernels then take it as one bit-field
    extract): true for the reference's tag set, interned first."""
    from lattice_based_tagger_amd import synth
    for case in _models(name)[:3]:
        lm = LoweredModel(case.funcs)
        if not lm.has_trigram:
            continue
        mul = _capi.ModelImage(lm.keys, lm.coefs).arrays()['d3mul']
        if mul:
            assert mul & (mul - 1) == 0 and mul <= 1 << 27, (case.tag, hex(mul))
    raw = synth.make_lattices(256, seed=3)
    lay = synth.layout(raw)
    cols = synth.node_columns(raw, lay)
    sm = synth.make_model(raw, lay, cols, seed=3, n_features=20_000)
    _, keys, coefs = synth.pack_fast(raw, sm, lay, cols)
    mul = _capi.ModelImage(keys, coefs).arrays()['d3mul']
    assert mul and mul & (mul - 1) == 0
