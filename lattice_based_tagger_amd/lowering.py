"""Lowering of a ``BeamScoreFunctions`` composite to the device model.

The reference scores every expansion by calling each plugin in order
(`lattice_tagger/beam/score_funcs.py:50-54`).  The build splits the
composite into

* node-local terms -- ``RegularizationScore`` (`:65-73`),
  ``MorphemePreferenceScore`` (`:84-88`) and ``WordPreferenceScore``
  (`:99-100`) depend on the appended node only.  They are evaluated once per
  lattice node while packing.  Terms in front of the trigram scorer are
  pre-summed in constructor order into ``pre`` (exact: the same left-to-right
  additions); terms after it stay separate (``post``) because f64 addition is
  not associative.
* the trigram term -- ``SimpleTrigramFeatureScore`` (`:137-144`).  Feature
  classes 0-3, 7 and 8 depend on the hypothesis and are probed per expansion
  in a device hash table; classes 4-6 depend on one node and are resolved per
  node by the packer.

Feature tuples are matched exactly as Python tuple membership does
(`features/feature.py:28-29`): every component value that occurs in a key of
``feature_dic`` is interned into one id space through a Python dict, so two
values receive the same id iff they compare (and hash) equal.  Id 0 means "occurs
in no key", which makes every feature containing it absent.

User plugins: a ``BeamScoreFunction`` subclass whose score depends on the
appended node only may declare ``node_local = True``; its ``score(None, w)``
is then evaluated once per lattice node (like the three built-in node-local
scorers) and summed in constructor order.  A plugin that declares it but reads
``seq`` gets ``None`` and fails loudly.

Several trigram scorers (round 6): each ``SimpleTrigramFeatureScore`` of the
composite is its own term, summed in its own numpy order and added in
constructor order (`score_funcs.py:50-54`).  Their keys share one interned id
space and one device table, the key class of scorer t carrying ``16 * t``
(``XTRI_CLASS_STRIDE``); scorer t >= 1 gets its own node masks and class
4-6 coefficients (``xtri_*`` batch arrays, lattice_decode.h ABI 6), and the
batch decodes on the general kernel.

Unsupported composites (a plugin of any other class, non-float64 or NaN
coefficients, +inf and -inf terms together) raise: there is no CPU fallback
decoder.
"""

import numpy as np

from .feature import FEATURE_ARITY, EXPANSION_CLASSES
from .tagset import POS_TAGS, Unk, BOS, EOS

TAG_IDS_FIRST = POS_TAGS + (Unk, BOS, EOS)

# ---------------------------------------------------------------------------
# Node mask bits (shared with csrc/lt_decode.hip and oracle/lt_oracle.c).
# Bits 0-15: "this node's component occurs at key slot X" (exact pre-filter).
# ---------------------------------------------------------------------------
K0B, K0C, K1B, K2B, K2C, K3B, K7C, K8B = (1 << i for i in range(8))
J0A, J1A, J2A, J3A, J7B, J8A = (1 << i for i in range(8, 14))
I7A, I8A = 1 << 14, 1 << 15
F_UNK = 1 << 16      # tag0 == 'Unknown'
F_CTX = 1 << 17      # tag0 in {Noun, Adverb, Adjective, Verb}
F_HAS4 = 1 << 18     # (4, len) in feature_dic
F_HAS5 = 1 << 19     # (5, word, tag0, is_l) in feature_dic
F_HAS6 = 1 << 20     # tag0 == Unk and (6, min(8, len)) in feature_dic

# Key slots: (class, component position) -> bit in the vocabulary mask.
SLOT_BITS = {
    (0, 0): 0, (0, 1): 1, (0, 2): 2,
    (1, 0): 3, (1, 1): 4,
    (2, 0): 5, (2, 1): 6, (2, 2): 7,
    (3, 0): 8, (3, 1): 9,
    (7, 0): 10, (7, 1): 11, (7, 2): 12,
    (8, 0): 13, (8, 1): 14,
}


def node_mask_from_vocab(vm_word, vm_morph, vm_tag):
    """Node pre-filter bits from the vocabulary slot masks of the node's word,
    morph0 and tag0 ids.  Works on ints and on numpy uint32 arrays."""
    def has(vm, cls, pos):
        return (vm >> SLOT_BITS[(cls, pos)]) & 1
    m = (has(vm_word, 0, 1) * K0B | has(vm_tag, 0, 2) * K0C |
         has(vm_tag, 1, 1) * K1B | has(vm_word, 2, 1) * K2B |
         has(vm_tag, 2, 2) * K2C | has(vm_tag, 3, 1) * K3B |
         has(vm_word, 7, 2) * K7C | has(vm_morph, 8, 1) * K8B |
         has(vm_word, 0, 0) * J0A | has(vm_word, 1, 0) * J1A |
         has(vm_tag, 2, 0) * J2A | has(vm_tag, 3, 0) * J3A |
         has(vm_word, 7, 1) * J7B | has(vm_morph, 8, 0) * J8A |
         has(vm_word, 7, 0) * I7A | has(vm_morph, 8, 0) * I8A)
    return m


# kinds of the scorers after the leading node-local ones (lt_batch_desc.term_kinds)
KIND_TRI, KIND_NODE, KIND_EDGE = 0, 1, 2
MAX_TERMS = 32
# several trigram scorers: scorer t's keys carry class + 16 * t (lattice_decode.h
# LT_XTRI_CLASS_STRIDE); at most LT_MAX_TRI of them
XTRI_CLASS_STRIDE = 16
MAX_TRI = 8


class EdgeSequence:
    """The hypothesis an ``edge_local`` plugin sees: its last word only
    (the plugin declares that it reads nothing else of the Sequence)."""
    __slots__ = ('sequences',)

    def __init__(self, wj, path=None):
        self.sequences = (wj,) if path is None else path


NODE_LOCAL_SCORERS = ('RegularizationScore', 'MorphemePreferenceScore',
                      'WordPreferenceScore')
TRIGRAM_SCORER = 'SimpleTrigramFeatureScore'
PACKED_TRIGRAM_SCORER = 'PackedTrigramFeatureScore'      # modelpack.py
ENCODER_CLASSES = ('SimpleTrigramEncoder',)


class _ClassIndex:
    """Python-equality lookup of a feature class id (True == 1 etc.)."""
    table = {c: c for c in range(9)}


class LoweredModel:
    """Host-side description of one scorer composite.

    Attributes
    ----------
    pre_funcs : the leading node-local plugins (summed per node on the host)
    plan : [(kind, func)] every later scorer in constructor order, kind
           KIND_TRI (the trigram), KIND_NODE (a node-local plugin: a
           node_post row) or KIND_EDGE (an ``edge_local`` plugin: an edge_val
           row, one value per lattice edge)
    post_funcs, edge_funcs : the KIND_NODE / KIND_EDGE plugins of ``plan``
    trigram : the first SimpleTrigramFeatureScore or None
    trigrams : every trigram scorer, in constructor order (trigrams[0] is
               ``trigram``); keys / coefs hold all of them, scorer t's classes
               offset by 16 * t, vmasks[t] / locals[t] its pre-filter masks and
               node-local classes
    vocab : dict value -> id (1-based) over every key component
    vmask : uint32[len(vocab)+1] key-slot bits per id
    keys : uint32[F, 4] (a, b, c, class) of the probed classes
    coefs : float64[F]
    feature_dic, coefficients : the trigram's tables (node-local classes)
    """

    def __init__(self, score_functions):
        funcs = list(getattr(score_functions, 'funcs', None) or [])
        if not hasattr(score_functions, 'funcs'):
            raise NotImplementedError(
                'beam_search expects a BeamScoreFunctions composite')
        self.pre_funcs, self.post_funcs, self.edge_funcs = [], [], []
        self.plan = []
        self.trigram = None
        self.trigrams = []
        for f in funcs:
            name = type(f).__name__
            if name in (TRIGRAM_SCORER, PACKED_TRIGRAM_SCORER):
                if self.trigrams and (name == PACKED_TRIGRAM_SCORER or
                                      type(self.trigrams[0]).__name__ == PACKED_TRIGRAM_SCORER):
                    raise NotImplementedError('a model pack scorer cannot be combined with another trigram scorer')
                if len(self.trigrams) >= MAX_TRI:
                    raise NotImplementedError('more than %d trigram scorers' % MAX_TRI)
                if self.trigram is None:
                    self.trigram = f
                self.trigrams.append(f)
                self.plan.append((KIND_TRI, f))
            elif name in NODE_LOCAL_SCORERS or getattr(f, 'node_local', False) is True:
                if self.plan:
                    self.plan.append((KIND_NODE, f))
                    self.post_funcs.append(f)
                else:
                    self.pre_funcs.append(f)
            elif getattr(f, 'edge_local', False) is True:
                # reads only seq.sequences[-1] and word_k: one value per lattice
                # edge (wj, wk), evaluated on the host
                self.plan.append((KIND_EDGE, f))
                self.edge_funcs.append(f)
            else:
                raise NotImplementedError(
                    'scorer %s has no device lowering (supported: %s, %s, and any '
                    'BeamScoreFunction that declares node_local = True or edge_local = True)'
                    % (name, ', '.join(NODE_LOCAL_SCORERS), TRIGRAM_SCORER))
        if len(self.plan) > MAX_TERMS:
            raise NotImplementedError('more than %d scorers after the leading node-local ones' % MAX_TERMS)
        _warn_slow_path(self)
        self.vocab = {}
        self.vmask = np.zeros(1, dtype=np.uint32)
        self.keys = np.zeros((0, 4), dtype=np.uint32)
        self.coefs = np.zeros(0, dtype=np.float64)
        self.feature_dic = None
        self.coefficients = None
        self.local = None           # packed models: {(cls, *comps): coef} of classes 4-6
        self.image = None           # packed models: prebuilt device image
        self.vmasks, self.feature_dics, self.coefficient_arrays = [], [], []
        if self.trigram is not None:
            if type(self.trigram).__name__ == PACKED_TRIGRAM_SCORER:
                self._lower_pack(self.trigram.pack)
            else:
                self._lower_trigrams()
        self._device_models = {}

    @property
    def n_post(self):
        return len(self.post_funcs)

    @property
    def n_edge(self):
        return len(self.edge_funcs)

    @property
    def term_kinds(self):
        """The plan's kinds, 2 bits per term (lt_batch_desc.term_kinds)."""
        return sum(kind << (2 * t) for t, (kind, _) in enumerate(self.plan))

    @property
    def has_trigram(self):
        return self.trigram is not None

    @property
    def n_xtri(self):
        """Trigram scorers past the first (lattice_decode.h n_xtri)."""
        return max(len(self.trigrams) - 1, 0)

    def _lower_trigrams(self):
        vocab = self.vocab
        # the tag set first: ids 1..13, distinct in their low four bits -- the
        # slot inside a key's line group (lt_common.h, HASH_VERSION 5)
        for t in TAG_IDS_FIRST:
            vocab[t] = len(vocab) + 1
        parts = [self._lower_trigram(tri, t) for t, tri in enumerate(self.trigrams)]
        # one id space for every scorer: the masks sized to the final vocabulary
        self.vmasks = []
        for slot_pairs in (p[2] for p in parts):
            vmask = np.zeros(len(vocab) + 1, dtype=np.uint32)
            if slot_pairs:
                sp = np.asarray(slot_pairs, dtype=np.int64)
                np.bitwise_or.at(vmask, sp[:, 0], (np.uint32(1) << sp[:, 1].astype(np.uint32)))
            self.vmasks.append(vmask)
        self.vmask = self.vmasks[0]
        self.keys = np.concatenate([p[0] for p in parts]).reshape(-1, 4)
        self.coefs = np.concatenate([p[1] for p in parts])
        self.feature_dic = self.feature_dics[0]
        self.coefficients = self.coefficient_arrays[0]

    def _lower_trigram(self, tri, t=0):
        """Keys (class + 16 t), coefficients and the (id, slot bit) pairs of
        the pre-filter masks of trigram scorer t."""
        enc = tri.encoder
        if enc is None:
            raise AttributeError("'NoneType' object has no attribute 'encode_word'")
        if type(enc).__name__ not in ENCODER_CLASSES:
            raise NotImplementedError('encoder %s has no device lowering' % type(enc).__name__)
        coef = tri.coefficients
        if not isinstance(coef, np.ndarray) or coef.dtype != np.float64 or coef.ndim != 1:
            raise NotImplementedError('coefficients must be a 1-D float64 numpy array')
        if np.isnan(coef).any():
            raise NotImplementedError('NaN coefficients: the order Python\'s sort gives NaN scores '
                                      'is not reproduced')
        if np.isposinf(coef).any() and np.isneginf(coef).any():
            raise NotImplementedError('+inf and -inf coefficients together: their sum is a NaN, whose '
                                      'order in Python\'s sort is not reproduced')
        dic = enc.feature_dic
        self.feature_dics.append(dic)
        self.coefficient_arrays.append(coef)
        vocab = self.vocab
        keys, coefs, slot_pairs = [], [], []
        cls_of = _ClassIndex.table
        n_coef = coef.shape[0]
        for key, idx in dic.items():
            if not isinstance(key, tuple) or not key:
                continue
            try:
                cls = cls_of.get(key[0])
            except TypeError:
                cls = None
            if cls is None or cls not in EXPANSION_CLASSES:
                continue
            if len(key) != FEATURE_ARITY[cls] + 1:
                continue        # can never equal a generated feature
            ids = []
            for pos, comp in enumerate(key[1:]):
                vid = vocab.get(comp)
                if vid is None:
                    vid = len(vocab) + 1
                    vocab[comp] = vid
                ids.append(vid)
                slot_pairs.append((vid, SLOT_BITS[(cls, pos)]))
            ids += [0] * (3 - len(ids))
            i = int(idx)
            if not -n_coef <= i < n_coef:
                raise IndexError('feature index %d out of range for %d coefficients' % (i, n_coef))
            keys.append((ids[0], ids[1], ids[2], cls + XTRI_CLASS_STRIDE * t))
            coefs.append(coef[i])
        return (np.asarray(keys, dtype=np.uint32).reshape(-1, 4), np.asarray(coefs, dtype=np.float64),
                slot_pairs)

    def _lower_pack(self, pack):
        """A model pack already holds the lowered tables and the device image."""
        self.vocab, self.vmask, self.keys, self.coefs, self.local = pack.lowered_parts()
        self.vmasks = [self.vmask]
        self.image = pack.image
        self.coefficients = pack.array('coefficients')

    # -- node-local helpers (used by the packer) ---------------------------
    def node_terms(self, w):
        """(pre, [post...]) for appending node ``w``: the node-local plugins'
        values summed as ``BeamScoreFunctions.score`` does."""
        pre = 0
        for f in self.pre_funcs:
            pre = pre + f.score(None, w)
        return pre, [f.score(None, w) for f in self.post_funcs]

    def edge_terms(self, wj, wk):
        """[value...] of the edge_local plugins for appending ``wk`` to a
        hypothesis whose last word is ``wj`` (score_funcs.py:50-54 calls
        ``f(seq, wk)``; such a plugin reads only ``seq.sequences[-1]``)."""
        seq = EdgeSequence(wj)
        return [f.score(seq, wk) for f in self.edge_funcs]

    def node_local_features(self, w, is_unk, t=0):
        """Coefficients (or None) of feature classes 4, 5 and 6 for node w
        under trigram scorer t."""
        if self.local is not None:
            loc = self.local
            return (loc.get((4, w.len)), loc.get((5, w.word, w.tag0, w.is_l)),
                    loc.get((6, min(8, w.len))) if is_unk else None)
        dic = self.feature_dics[t] if t < len(self.feature_dics) else None
        if dic is None:
            return None, None, None
        coef = self.coefficient_arrays[t]
        i4 = dic.get((4, w.len))
        i5 = dic.get((5, w.word, w.tag0, w.is_l))
        i6 = dic.get((6, min(8, w.len))) if is_unk else None
        return (None if i4 is None else float(coef[i4]),
                None if i5 is None else float(coef[i5]),
                None if i6 is None else float(coef[i6]))


_WARNED = set()


def _warn_slow_path(model):
    """One warning per composite shape whose plugins take the slow host path
    (INTEGRATION.md "edge-local plugins"): an edge_local plugin is evaluated in
    Python once per lattice edge, and any user plugin turns the implicit
    Unknown records off (every Unknown a node record of its own, about 3.5x
    the records on dictionary lattices) and the native packer off (the Python
    packer, about 70x slower).  The decode itself stays on the device."""
    user = [type(f).__name__ for f in list(model.pre_funcs) + list(model.post_funcs)
            if type(f).__name__ not in NODE_LOCAL_SCORERS]
    edge = [type(f).__name__ for f in model.edge_funcs]
    if not (user or edge):
        return
    sig = (tuple(user), tuple(edge))
    if sig in _WARNED:
        return
    _WARNED.add(sig)
    import warnings
    what = ', '.join(['%s (edge_local)' % n for n in edge] + ['%s (node_local)' % n for n in user])
    warnings.warn('lattice_based_tagger_amd: scorer plugin(s) %s: packed by the Python packer%s, '
                  'without implicit Unknown records (each Unknown its own node record); the decode '
                  'stays on the GPU, the host packing is about 70x slower than the native packer'
                  % (what, ', their values evaluated per lattice edge in Python' if edge else ''),
                  RuntimeWarning, stacklevel=4)


def lower_scorers(score_functions):
    return LoweredModel(score_functions)
