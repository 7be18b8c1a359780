"""``Tagger`` -- the reference's public tagging API on the GPU decoder.

Mirrors `lattice_tagger/tagger/tagger.py:10-78`:
``Tagger(dictionary, lookup, encoder, score_funcs).tag(sent, beam_size=5,
ensure_normalize=True, debug=False) -> Sequence``.

Lattice construction: with a reference ``MorphemeDictionary`` (the
reference ``Tagger.__init__`` builds ``MorphemeLookup(dictionary)``,
`tagger.py:60`) the lattices of a whole batch come from the native lattice
builder (``lookup.NativeLexicon``, C++), which restates
``morpheme_lookup`` and the lemmatizer node for node; a custom ``lookup``
callable (or a dictionary subclass overriding the lookup methods) runs in
Python, grouped into a begin index as `lookup.py:7-62, 344-369` do.
Decoding runs on the device.
"""

import gc
import sys
import time

from .beam import beam_search_batch
from .tagset import Adjective, Adverb, Determiner, Exclamation, Noun, Number, Verb
from .word import bos_word, eos_word


def sentence_lookup(sent, eojeol_lookup):
    """[BOS] + nodes of every eojeol (offset by the characters before it) +
    [EOS] (`lookup.py:52-62`)."""
    n = len(sent.replace(' ', ''))
    nodes = [bos_word()]
    offset = 0
    for eojeol in sent.split():
        nodes += eojeol_lookup(eojeol, offset)
        offset += len(eojeol)
    nodes.append(eos_word(n))
    return nodes


def sentence_lookup_as_begin_index(sent, eojeol_lookup):
    """(nodes, bindex) with bindex[b] = dictionary nodes beginning at b, in
    lookup order; bindex = [] when no eojeol produced a node
    (`lookup.py:357-369`)."""
    n = len(sent.replace(' ', ''))
    nodes = sentence_lookup(sent, eojeol_lookup)
    if len(nodes) <= 2:
        return nodes, []
    bindex = [[] for _ in range(n)]
    for w in nodes[1:-1]:
        bindex[w.b].append(w)
    return nodes, bindex


# MorphemeLookup defaults (lookup.py:104-105) -- the lookup Tagger builds
# (tagger.py:60)
STANDALONES = (Noun, Adverb, Exclamation, Determiner, Number)

# the reference MorphemeDictionary methods the native lattice builder restates
_REF_METHODS = {'lookup': 'MorphemeDictionary.lookup', 'check': 'WordDictionary.check',
                'get_tags': 'WordDictionary.get_tags', 'lemmatize': 'MorphemeDictionary.lemmatize'}


def find_max_len(dictionary, standalones):
    """MorphemeLookup._find_max_len (`lookup.py:123-132`)."""
    keep = set(standalones)
    keep.add(Verb)
    keep.add(Adjective)
    max_len = 0
    for tag, morphs in dictionary.tag_to_morphs.items():
        if tag not in keep:
            continue
        max_len = max(max_len, max(len(m) for m in morphs))
    return max_len


def plain_morpheme_dictionary(dictionary):
    """True when ``dictionary`` answers lookups with the reference
    MorphemeDictionary's own methods (no subclass overrides), so the native
    lattice builder restates it exactly."""
    for name, qual in _REF_METHODS.items():
        f = getattr(type(dictionary), name, None)
        if f is None or getattr(f, '__qualname__', None) != qual or \
                not str(getattr(f, '__module__', '')).endswith('dictionary.dictionary'):
            return False
    return True


def _default_lookup(dictionary):
    ref = sys.modules.get('lattice_tagger.dictionary')
    if ref is None:
        try:
            import lattice_tagger.dictionary as ref       # the user's reference install
        except ImportError as exc:
            raise NotImplementedError(
                'no eojeol lookup: pass custom_lookup=<callable(eojeol, offset) -> [Word]> or a '
                'lattice_tagger MorphemeDictionary') from exc
    return ref.MorphemeLookup(dictionary, flatten=False)


class Tagger:
    """Part-of-speech tagger over a morpheme lattice (`tagger.py:10-78`).

    ``dictionary``  a reference ``MorphemeDictionary`` (or the string
                    'base', which builds the reference BaseMorphemeDictionary)
    ``lookup``, ``encoder``  accepted and ignored, as in the reference
                    (`tagger.py:57-62`: the lattices always come from
                    ``MorphemeLookup(dictionary, flatten=False)``)
    ``score_funcs`` a ``BeamScoreFunctions`` composite (reference or mirror)
    ``custom_lookup`` (extension, not in the reference) a callable
                    ``(eojeol, offset) -> [Word]`` that builds the lattices
                    instead of MorphemeLookup
    ``device``      HIP device ordinal of the decoder, or a sequence of
                    ordinals: ``tag_batch`` then deals its chunks to the
                    devices in turn (one context per entry; results in
                    input order)
    ``lexicon``     a prebuilt ``lookup.NativeLexicon`` (optional; used as
                    given -- the caller rebuilds it after changing the
                    dictionary)
    ``native_lookup`` build lattices with the native lattice builder
                    (``lookup.NativeLexicon``, C++) when the dictionary is a
                    plain reference MorphemeDictionary; otherwise (or when
                    False) the Python MorphemeLookup runs
    """

    def __init__(self, dictionary='base', lookup='subword_lookup', encoder=None,
                 score_funcs=None, device=0, lexicon=None, native_lookup=True, lookup_threads=0,
                 custom_lookup=None):
        if callable(lookup):
            # the reference ignores lookup (tagger.py:57-62) and so does this
            # Tagger; a caller handing a callable most likely wants it used
            import warnings
            warnings.warn('Tagger ignores lookup= as the reference does (tagger.py:57-62); pass '
                          'custom_lookup=<callable(eojeol, offset) -> [Word]> to build the lattices with it',
                          stacklevel=2)
        self._lexicon = lexicon
        self._lexicon_given = lexicon is not None     # used as given, never rebuilt
        self._eojeol_lookup = None
        self.lookup_threads = lookup_threads
        self.last_stats = None                     # tag_batch's stage times of its last pipelined call
        if custom_lookup is not None:
            if not callable(custom_lookup):
                raise TypeError('custom_lookup must be a callable (eojeol, offset) -> [Word]')
            self.dictionary = dictionary
            self._eojeol_lookup = custom_lookup
            self.native = lexicon is not None
        else:
            if isinstance(dictionary, str):
                ref = sys.modules.get('lattice_tagger.dictionary')
                if ref is None:
                    import lattice_tagger.dictionary as ref
                dictionary = ref.BaseMorphemeDictionary()
            if lexicon is None and not hasattr(dictionary, 'rules'):
                raise ValueError('dictionary must be MorphemeDictionary')      # lookup.py:101-102
            self.dictionary = dictionary
            self.native = lexicon is not None or (native_lookup and plain_morpheme_dictionary(dictionary))
        self.encoder = encoder
        self.score_funcs = score_funcs
        self.device = device

    @property
    def eojeol_lookup(self):
        if self._eojeol_lookup is None:
            self._eojeol_lookup = _default_lookup(self.dictionary)
        return self._eojeol_lookup

    def native_lexicon(self):
        """The NativeLexicon in use (rebuilt when the dictionary changed), or
        None when lattices are built in Python."""
        if not self.native:
            return None
        from .lookup import NativeLexicon, dictionary_fingerprint
        from .native_packer import Unsupported
        lex = self._lexicon
        if lex is not None and (self._lexicon_given or
                                dictionary_fingerprint(self.dictionary) == lex.fingerprint):
            return lex
        try:
            standalones = list(STANDALONES)
            lex = NativeLexicon(self.dictionary, standalones, find_max_len(self.dictionary, standalones),
                                prefer_exact_match=True)
        except Unsupported:
            self.native = False
            return None
        self._lexicon = lex
        return lex

    def lattice(self, sent):
        chars = sent.replace(' ', '')
        lex = self.native_lexicon()
        if lex is not None:
            return lex.lookup([sent], n_threads=1).bindex(0), chars
        _, bindex = sentence_lookup_as_begin_index(sent, self.eojeol_lookup)
        return bindex, chars

    def tag(self, sent, beam_size=5, ensure_normalize=True, debug=False):
        if debug:                                   # tagger.py:75-76 passes debug to beam_search
            bindex, chars = self.lattice(sent)
            return beam_search(bindex, chars, self.score_funcs, beam_size=beam_size, debug=True)[0]
        return self.tag_batch([sent], beam_size=beam_size)[0]

    # sentences per pipeline chunk of tag_batch
    CHUNK = 4096
    # pipeline stages of tag_batch: 4 (decode + path preparation on a worker)
    # or 3 (the caller decodes and materialises; rounds 2-5); LT_TAGGER_STAGES
    STAGES = int(__import__('os').environ.get('LT_TAGGER_STAGES', '4'))

    def tag_batch(self, sents, beam_size=5):
        """Best ``Sequence`` per sentence.  Raises IndexError like ``tag``
        when a non-empty sentence has no dictionary node at all
        (`beam.py:32`).  With native lattices the batch runs as a
        four-stage pipeline over chunks of CHUNK sentences: one worker
        thread builds and packs chunk i+3 (C++, outside the GIL), a second
        uploads chunk i+2 (node records, host-to-device copies), a third
        decodes chunk i+1 and prepares its paths (path-node indices, the
        dictionary-coded strings of their Words: numpy and C calls that
        release the GIL), while this thread builds chunk i's Sequences (the
        only stage that needs the GIL throughout).  The cyclic GC is paused
        meanwhile (millions of fresh tuples, no cycles)."""
        sents = list(sents)
        lex = self.native_lexicon()
        if lex is None:
            lattices = [self.lattice(s) for s in sents]
            matures = beam_search_batch(lattices, self.score_funcs, beam_size=beam_size,
                                        device=self.device)
            return [m[0] for m in matures]
        self.last_stats = None
        enabled = gc.isenabled()
        gc.disable()
        try:
            out = self._tag_native(lex, sents, beam_size)
            if self.last_stats is not None and 't_end' in self.last_stats:
                self.last_stats['teardown_s'] = time.perf_counter() - self.last_stats.pop('t_end')
            return out
        finally:
            if enabled:
                gc.enable()

    @staticmethod
    def _pipeline3(chunks, lat0, front, upload, finish):
        """The three-stage pipeline (builder, uploader, the caller decoding
        and materialising)."""
        from collections import deque
        from concurrent.futures import ThreadPoolExecutor
        out = []
        with ThreadPoolExecutor(max_workers=1) as builder, ThreadPoolExecutor(max_workers=1) as uploader:
            stages = deque()

            def feed(i):
                if i < len(chunks):
                    stages.append(uploader.submit(upload, i, builder.submit(front, chunks[i],
                                                                            lat0 if i == 0 else None)))
            feed(0)
            feed(1)
            try:
                for i in range(len(chunks)):
                    lat, packed, views, dbs = stages.popleft().result()
                    feed(i + 2)
                    out += finish(i, lat, packed, views, dbs)
            finally:
                for f in stages:                   # an error: drop what is still in flight
                    f.cancel()
                    if not f.cancelled():
                        try:
                            for _, _, db in f.result()[3] or ():
                                db.close()
                        except BaseException:
                            pass
        return out

    def _tag_native(self, lex, sents, beam_size):
        from collections import deque
        from concurrent.futures import ThreadPoolExecutor
        from .beam import (_check_beam, decode_batch, decode_prepared, decoders_for, device_list, lowered_model,
                           materialise_prepared)
        from .native_packer import packer_for
        k = _check_beam(beam_size)
        chunks = [sents[i:i + self.CHUNK] for i in range(0, len(sents), self.CHUNK)] or [[]]

        def lookup(chunk):
            lat = lex.lookup(chunk, n_threads=self.lookup_threads)
            for s in range(len(chunk)):
                if lat.empty(s):
                    raise IndexError('list index out of range')        # beam.py:32 on bindex == []
            return lat

        t_call = time.perf_counter()
        lat0 = lookup(chunks[0])                   # (the reference raises before scoring)
        lat0_s = time.perf_counter() - t_call
        model = lowered_model(self.score_funcs)
        npk = packer_for(model)
        decs = None
        if npk is not None and k > 0:
            decs = decoders_for(device_list(self.device))
            for dec in decs:                       # built here, before any worker uses it
                dec.device_model(model)

        def decoder(i):                            # chunk i's device
            return decs[i % len(decs)] if decs else None

        def front(chunk, lat=None):
            lat = lat if lat is not None else lookup(chunk)
            if npk is None:
                return lat, None, None
            packed, views = npk.pack_lattices(lat, max_len=8)
            return lat, packed, views

        def upload(i, fut):
            lat, packed, views = fut.result()
            dec = decoder(i)
            dbs = dec.upload(model, packed, k) if dec is not None and packed is not None else None
            return lat, packed, views, dbs

        def finish(i, lat, packed, views, dbs):
            if packed is None:
                lattices = [(lat.bindex(s), lat.chars[s]) for s in range(len(chunks[i]))]
                matures = beam_search_batch(lattices, self.score_funcs, beam_size=k, device=self.device)
            else:
                matures = decode_batch(packed, views, lat.chars, model, k, best_only=True,
                                       uploaded=dbs, decoder=decoder(i))
            return [m[0] for m in matures]

        if len(chunks) == 1:                       # nothing to overlap (Tagger.tag): no worker threads
            lat, packed, views = front(chunks[0], lat0)
            dec = decoder(0)
            dbs = dec.upload(model, packed, k) if dec is not None and packed is not None else None
            return finish(0, lat, packed, views, dbs)
        if self.STAGES == 3:
            return self._pipeline3(chunks, lat0, front, upload, finish)

        def decode(i, fut):                        # the decode stage (worker): device + path preparation
            lat, packed, views, dbs = fut.result()
            if packed is None or dbs is None:      # (Python-packed composites: the caller decodes)
                return i, lat, packed, views, dbs, None
            return i, lat, packed, views, None, decode_prepared(packed, views, lat.chars, model, k,
                                                                best_only=True, uploaded=dbs,
                                                                decoder=decoder(i))

        out = []
        # where the caller's time goes (last_stats): blocked on the decode
        # stage, building Sequences; the builder's own lookup + pack time
        st = {'chunks': len(chunks), 'lat0_s': lat0_s, 'wait_s': 0.0, 'objects_s': 0.0, 'front_s': 0.0,
              'first_chunk_s': 0.0}
        self.last_stats = st

        def front_timed(chunk, lat=None):
            t = time.perf_counter()
            r = front(chunk, lat)
            st['front_s'] += time.perf_counter() - t
            return r
        with ThreadPoolExecutor(max_workers=1) as builder, ThreadPoolExecutor(max_workers=1) as uploader, \
                ThreadPoolExecutor(max_workers=1) as decoding:
            stages = deque()

            def feed(i):
                if i < len(chunks):
                    up = uploader.submit(upload, i, builder.submit(front_timed, chunks[i], lat0 if i == 0 else None))
                    stages.append((up, decoding.submit(decode, i, up)))
            feed(0)
            feed(1)
            feed(2)
            try:
                for i in range(len(chunks)):
                    _, dfut = stages.popleft()
                    t = time.perf_counter()
                    _, lat, packed, views, dbs, prep = dfut.result()
                    t1 = time.perf_counter()
                    st['wait_s'] += t1 - t
                    if i == 0:
                        st['first_chunk_s'] = t1 - t_call
                    feed(i + 3)
                    if prep is None:
                        out += finish(i, lat, packed, views, dbs)
                    else:
                        out += [m[0] for m in materialise_prepared(prep)]
                    st['objects_s'] += time.perf_counter() - t1
            finally:
                for up, dfut in stages:            # an error: drop what is still in flight
                    dfut.cancel()
                    if dfut.cancelled():           # (its batches were not handed to a decode)
                        up.cancel()
                        if not up.cancelled():
                            try:
                                for _, _, db in up.result()[3] or ():
                                    db.close()
                            except BaseException:
                                pass
                    else:
                        try:
                            dfut.result()
                        except BaseException:
                            pass
                st['loop_s'] = time.perf_counter() - t_call
        t = time.perf_counter()
        st['inside_s'] = t - t_call
        # the last chunk's lattice, pack and prepared paths (its decode
        # future holds them) and chunk 0's lattice, released here and timed:
        # after a phase that freed gigabytes this release took 0.17-0.23 s
        # (profiles/r06/tagger_calls/)
        lat = packed = views = dbs = prep = dfut = lat0 = None
        st['t_end'] = time.perf_counter()
        st['release_s'] = st['t_end'] - t
        return out
