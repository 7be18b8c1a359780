"""Model pack format: a trained trigram model as one memory-mappable file.

SURVEY.md §8(f) #3.  The reference's model is ``scan_features``' output
(``idx_to_feature`` / ``feature_to_idx``, `features/utils.py:50-55`) plus a
coefficient vector, bound at run time by
``SimpleTrigramFeatureScore.set_encoder`` (`beam/score_funcs.py:106-125`).
Every run then re-interns the feature vocabulary and rebuilds the device hash
table.  A pack stores the result of that work once:

* the features in index order and the coefficients (so the reference-protocol
  scorer -- encoder + coefficients -- can be rebuilt exactly);
* the lowered model: interned component vocabulary (id order), per-id key-slot
  masks, the probed keys and their coefficients, the node-local classes 4/5/6
  (features with their coefficient index);
* the device image: the built cuckoo table and dense class-3 table
  (``lt_image_build``), uploaded by ``lt_model_create_from_image`` -- no table
  build at load time.

File layout: ``b'LTMODEL1'``, u64 header length, a JSON header, then 64-byte
aligned blobs (numpy arrays, memory-mapped on load; JSON sections stored as
UTF-8 blobs).  The header carries an xxh64 checksum of every blob.

    pack = modelpack.save('model.ltm', trigram_scorer)
    scorer = modelpack.load('model.ltm')        # a SimpleTrigramFeatureScore
    funcs = BeamScoreFunctions(RegularizationScore(), scorer)
"""

import json
import os

import numpy as np

from . import _capi
from .feature import SimpleTrigramEncoder
from .lowering import LoweredModel
from .score_funcs import SimpleTrigramFeatureScore

MAGIC = b'LTMODEL1'
VERSION = 1
_ALIGN = 64
_JSON_SCALARS = (str, int, float, bool, type(None))


def _check_json(values, what):
    for v in values:
        if not isinstance(v, _JSON_SCALARS):
            raise NotImplementedError('%s component %r (%s) cannot be stored in a model pack'
                                      % (what, v, type(v).__name__))


def _digest(buf):
    import xxhash
    return xxhash.xxh64(buf).hexdigest()


def save(path, scorer):
    """Write the trigram scorer ``scorer`` (a SimpleTrigramFeatureScore with a
    trained SimpleTrigramEncoder and float64 coefficients) to ``path``."""
    if scorer.encoder is None:
        raise ValueError('scorer has no encoder')
    lm = LoweredModel(_Composite([scorer]))
    dic = scorer.encoder.feature_dic
    coef = np.ascontiguousarray(scorer.coefficients, dtype=np.float64)
    n = coef.shape[0]
    feats = [None] * n
    for f, i in dic.items():
        i = int(i)
        if not 0 <= i < n or feats[i] is not None:
            raise NotImplementedError('feature_dic must map features to distinct indices 0..%d' % (n - 1))
        if not isinstance(f, tuple):
            raise NotImplementedError('feature %r is not a tuple' % (f,))
        _check_json(f, 'feature')
        feats[i] = list(f)
    if any(f is None for f in feats):
        raise NotImplementedError('feature_dic does not cover every coefficient index')
    vocab = [None] * len(lm.vocab)
    for v, i in lm.vocab.items():
        vocab[i - 1] = v
    _check_json(vocab, 'vocabulary')
    image = _capi.ModelImage(lm.keys, lm.coefs).arrays() if len(lm.keys) else None

    local = [[i, f] for i, f in enumerate(feats)
             if f and f[0] in (4, 5, 6) and not isinstance(f[0], bool)]
    blobs = {
        'features': json.dumps(feats, ensure_ascii=False).encode('utf-8'),
        'local': json.dumps(local, ensure_ascii=False).encode('utf-8'),
        'vocab': json.dumps(vocab, ensure_ascii=False).encode('utf-8'),
        'coefficients': coef,
        'keys': np.ascontiguousarray(lm.keys, dtype=np.uint32),
        'coefs': np.ascontiguousarray(lm.coefs, dtype=np.float64),
        'vmask': np.ascontiguousarray(lm.vmask, dtype=np.uint32),
    }
    meta = {'version': VERSION, 'n_features': n, 'n_keys': int(len(lm.keys)),
            'vocab_size': len(vocab), 'image': None}
    if image is not None:
        blobs['table'] = image['table']
        if image['d3mul']:
            blobs['d3'] = image['d3']
        meta['image'] = {k: image[k] for k in ('hash_version', 'narrow', 'seed', 'slots', 'd3mul')}
    entries, payload, off = {}, [], 0
    for name, b in blobs.items():
        raw = b if isinstance(b, bytes) else b.tobytes()
        pad = (-off) % _ALIGN
        payload.append(b'\0' * pad)
        off += pad
        entries[name] = {'offset': off, 'nbytes': len(raw),
                         'dtype': 'bytes' if isinstance(b, bytes) else b.dtype.str,
                         'shape': None if isinstance(b, bytes) else list(b.shape),
                         'xxh64': _digest(raw)}
        payload.append(raw)
        off += len(raw)
    meta['blobs'] = entries
    header = json.dumps(meta).encode('utf-8')
    head_len = len(MAGIC) + 8 + len(header)
    data_start = head_len + (-head_len) % _ALIGN
    meta_bytes = header + b' ' * (data_start - head_len)
    tmp = path + '.tmp'
    with open(tmp, 'wb') as fh:
        fh.write(MAGIC)
        fh.write(np.uint64(len(meta_bytes)).tobytes())
        fh.write(meta_bytes)
        for p in payload:
            fh.write(p)
    os.replace(tmp, path)
    return path


class ModelPack:
    """A loaded (memory-mapped) model pack."""

    def __init__(self, path, verify=True):
        self.path = path
        with open(path, 'rb') as fh:
            if fh.read(len(MAGIC)) != MAGIC:
                raise ValueError('%s is not a model pack' % path)
            hlen = int(np.frombuffer(fh.read(8), dtype=np.uint64)[0])
            meta = json.loads(fh.read(hlen).decode('utf-8'))
        if meta.get('version') != VERSION:
            raise ValueError('unsupported model pack version %r' % meta.get('version'))
        self.meta = meta
        base = len(MAGIC) + 8 + hlen
        self._mm = np.memmap(path, dtype=np.uint8, mode='r')
        self._base = base
        if verify:
            for name, e in meta['blobs'].items():
                if _digest(self._raw(name)) != e['xxh64']:
                    raise ValueError('model pack %s: blob %s is corrupt' % (path, name))

    def _raw(self, name):
        e = self.meta['blobs'][name]
        o = self._base + e['offset']
        return self._mm[o:o + e['nbytes']]

    def array(self, name):
        e = self.meta['blobs'][name]
        if e['dtype'] == 'bytes':
            return bytes(self._raw(name))
        return self._raw(name).view(np.dtype(e['dtype'])).reshape(e['shape'])

    def json(self, name):
        return json.loads(bytes(self._raw(name)).decode('utf-8'))

    @property
    def image(self):
        im = self.meta['image']
        if im is None:
            return None
        return dict(im, table=self.array('table'),
                    d3=self.array('d3') if im['d3mul'] else np.zeros(0, np.float64))

    def lowered_parts(self):
        """(vocab dict, vmask, keys, coefs, local) -- the LoweredModel fields,
        ``local`` = {(cls, *components): coefficient} of classes 4, 5, 6."""
        vocab = {v: i + 1 for i, v in enumerate(self.json('vocab'))}
        coef = self.array('coefficients')
        local = {tuple(f): float(coef[i]) for i, f in self.json('local')}
        return vocab, self.array('vmask'), self.array('keys'), self.array('coefs'), local


class PackedTrigramFeatureScore(SimpleTrigramFeatureScore):
    """``SimpleTrigramFeatureScore`` backed by a model pack.  The encoder and
    coefficients (reference protocol: ``score``, ``evaluate``) are rebuilt
    from the pack on first use; the device path uses the pack directly."""

    def __init__(self, pack):
        self.pack = pack
        self.num_features = pack.meta['n_features']
        self._encoder = None
        self.coefficients = pack.array('coefficients')

    @property
    def encoder(self):
        if self._encoder is None:
            feats = self.pack.json('features')
            enc = SimpleTrigramEncoder({tuple(f): i for i, f in enumerate(feats)})
            self._encoder = enc
        return self._encoder

    @encoder.setter
    def encoder(self, enc):
        self._encoder = enc


def load(path, verify=True):
    """Memory-map a model pack; returns a ``PackedTrigramFeatureScore``."""
    return PackedTrigramFeatureScore(ModelPack(path, verify=verify))


class _Composite:
    def __init__(self, funcs):
        self.funcs = funcs
