"""End-to-end Tagger on the device with native lattices: sentences (text) ->
native lattice builder (lookup.NativeLexicon, restricted reference
dictionaries of tests/golden/lookup.json.gz) -> native packer -> HIP decode.
The best sequence of every sentence must be the reference's (scores as
float.hex, nodes field for field) from the reference-made golden sets
'base' (Regularization + trigram) and 'demo' (all four scorers), at
k = 1, 5, 16."""

import pytest

from golden_io import load
from lattice_based_tagger_amd import Tagger
from test_lookup import _fixture, fixture_dictionary, fixture_lexicon

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name,chunk', [('base', None), ('demo', None), ('base', 16)])
def test_tagger_native_lattices_match_reference(gpu_decoder, name, chunk, monkeypatch):
    if chunk:                                   # several pipeline chunks (lookup/pack overlapped)
        monkeypatch.setattr(Tagger, 'CHUNK', chunk)
    entry = _fixture()[name]
    cases = load(name)
    by_chars = {c.chars: c for c in cases}
    sents = [s for s in entry['sentences'] if s.replace(' ', '') in by_chars
             and by_chars[s.replace(' ', '')].bindex]
    assert len(sents) >= (101 if name == 'base' else 40)
    tagger = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=fixture_lexicon(entry),
                    score_funcs=cases[0].funcs)
    for k in (1, 5, 16):
        best = tagger.tag_batch(sents, beam_size=k)
        for sent, seq in zip(sents, best):
            c = by_chars[sent.replace(' ', '')]
            codes, shex, kind = c.expected[str(k)]['matures'][0]
            assert float(seq.score).hex() == shex, (sent, k)
            assert type(seq.score).__name__ == kind, (sent, k)
            words = seq.sequences[1:-1]
            assert len(words) == len(codes), (sent, k)
            for code, w in zip(codes, words):
                if code[0] == 'U':
                    b, e = code[1], code[2]
                    sub = c.chars[b:e]
                    assert tuple(w) == (sub, sub, None, 'Unknown', None, e - b, b, e, False)
                else:
                    assert tuple(w) == tuple(c.node(code)), (sent, k)
    one = tagger.tag(sents[0], beam_size=5)
    assert float(one.score).hex() == by_chars[sents[0].replace(' ', '')].expected['5']['matures'][0][1]


def test_tagger_pipeline_error_in_a_later_chunk(gpu_decoder, monkeypatch):
    """A sentence without any dictionary node in the fourth pipeline chunk
    raises the reference's IndexError from tag_batch (the chunks before it
    already decoded), and the tagger decodes correctly afterwards -- nothing
    in flight is left behind."""
    monkeypatch.setattr(Tagger, 'CHUNK', 8)
    entry = _fixture()['base']
    cases = load('base')
    by_chars = {c.chars: c for c in cases}
    sents = [s for s in entry['sentences'] if s.replace(' ', '') in by_chars
             and by_chars[s.replace(' ', '')].bindex][:48]
    tagger = Tagger(dictionary=fixture_dictionary(entry['lexicon']), lexicon=fixture_lexicon(entry),
                    score_funcs=cases[0].funcs)
    bad = sents[:27] + ['ㅋㅋㅋ'] + sents[27:]
    with pytest.raises(IndexError):
        tagger.tag_batch(bad, beam_size=5)
    best = tagger.tag_batch(sents, beam_size=5)
    for sent, seq in zip(sents, best):
        shex = by_chars[sent.replace(' ', '')].expected['5']['matures'][0][1]
        assert float(seq.score).hex() == shex, sent
