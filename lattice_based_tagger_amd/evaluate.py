"""Batch ``BeamScoreFunctions.evaluate`` on the GPU.

The reference scores a given path (e.g. a gold sequence for training) with
``BeamScoreFunctions.evaluate(seq)`` (`beam/score_funcs.py:44-48`):

    total = 0;  total += func.evaluate(seq)   for func in constructor order

* node-local scorers (`:62-63, 81-82, 96-97`): ``sum(score(None, w) for w in
  seq.sequences)`` -- every word, BOS and EOS included, left to right;
* ``edge_local`` plugins: their own ``evaluate(seq)`` (user code, on the host),
  entered as that scorer's value of the path;
* ``SimpleTrigramFeatureScore`` (`:127-135`): replays the path with
  ``Sequence.add`` from ``Sequence([seq.sequences[0]], 0)``, skipping words
  tagged BOS/EOS; each increment is the trigram score of the word after its
  replayed predecessors.

``evaluate_batch`` computes exactly that for many paths in one launch
(``lt_evaluate``): one GPU lane per word computes its trigram increment with
the decoder's probe code; one lane per path forms the sums in the reference's
order.  The node-local scorers' per-word values are the host's (the scorer
objects are Python); the ids, pre-filter masks and node-local feature
coefficients come from the same lowering as the decoder.
"""

import ctypes as C

import numpy as np

from . import _capi
from .beam import Decoder, lowered_model
from .lowering import EdgeSequence, NODE_LOCAL_SCORERS, TRIGRAM_SCORER, PACKED_TRIGRAM_SCORER
from .packer import node_record
from .tagset import BOS, EOS


class PathsDesc(C.Structure):
    _fields_ = [('n_paths', C.c_int32), ('n_words', C.c_int64), ('path_off', C.c_void_p),
                ('word', C.c_void_p), ('morph0', C.c_void_p), ('tag', C.c_void_p),
                ('mask', C.c_void_p), ('f4', C.c_void_p), ('f5', C.c_void_p), ('f6', C.c_void_p),
                ('prev1', C.c_void_p), ('prev2', C.c_void_p), ('n_terms', C.c_int32),
                ('terms', C.c_void_p), ('trigram_pos', C.c_int32), ('trigram_scorer', C.c_int32)]


def _words_of(seq):
    return list(seq.sequences) if hasattr(seq, 'sequences') else list(seq)


def evaluate_batch(sequences, score_functions, device=0):
    """``[score_functions.evaluate(seq) for seq in sequences]`` on the GPU.

    ``sequences``: ``Sequence`` objects (e.g. ``beam_search`` matures) or lists
    of words ``[BOS, w1, ..., EOS]``.  Returns a list of Python floats.

    A composite with several trigram scorers is evaluated one scorer per
    launch (each launch's total is that scorer's E_t exactly: 0 + E_t), and
    the totals are summed here in constructor order, as
    ``BeamScoreFunctions.evaluate`` does (`score_funcs.py:44-48`)."""
    funcs = list(score_functions.funcs)
    model = lowered_model(score_functions)
    sequences = list(sequences)
    if len(model.trigrams) > 1:
        per = []
        t = 0
        for f in funcs:
            if type(f).__name__ in (TRIGRAM_SCORER, PACKED_TRIGRAM_SCORER):
                per.append(_evaluate_launch(sequences, model, [f], device, scorer=t))
                t += 1
            else:
                per.append(_evaluate_launch(sequences, model, [f], device))
        out = []
        for p in range(len(sequences)):
            total = 0
            for v in per:
                total += v[p]
            out.append(float(total))
        return out
    return _evaluate_launch(sequences, model, funcs, device)


def _evaluate_launch(sequences, model, funcs, device, scorer=0):
    """One lt_evaluate launch: the scorers ``funcs`` (at most one trigram
    scorer, the composite's ``scorer``-th) over ``sequences``."""
    trigram_pos = -1
    local = []
    for pos, f in enumerate(funcs):
        if type(f).__name__ in (TRIGRAM_SCORER, PACKED_TRIGRAM_SCORER):
            trigram_pos = pos
        else:
            local.append(f)
    cols = {k: [] for k in ('word', 'morph', 'tag', 'mask', 'f4', 'f5', 'f6', 'p1', 'p2')}
    terms = [[] for _ in local]
    path_off = [0]
    for seq in sequences:
        words = _words_of(seq)
        if not words:
            raise IndexError('list index out of range')      # seq.sequences[0]
        base = len(cols['word'])
        replay = [base]                                       # Sequence([seq.sequences[0]])
        for idx, w in enumerate(words):
            wid, mid, tid, m, c4, c5, c6 = node_record(model, w, scorer)
            cols['word'].append(wid)
            cols['morph'].append(mid)
            cols['tag'].append(tid)
            cols['mask'].append(m)
            cols['f4'].append(0.0 if c4 is None else c4)
            cols['f5'].append(0.0 if c5 is None else c5)
            cols['f6'].append(0.0 if c6 is None else c6)
            for t, f in enumerate(local):
                # (LoweredModel's precedence: a plugin declaring node_local as
                # well is lowered -- and evaluated -- as node-local)
                if (getattr(f, 'edge_local', False) is True and getattr(f, 'node_local', False) is not True
                        and type(f).__name__ not in NODE_LOCAL_SCORERS):
                    # an edge plugin's own evaluate(seq) (user code, host), as one
                    # value of the path: ((0 + E) + -0.0) + ... == E
                    sq = seq if hasattr(seq, 'sequences') else EdgeSequence(None, words)
                    terms[t].append(float(f.evaluate(sq)) if idx == 0 else -0.0)
                else:
                    terms[t].append(float(f.score(None, w)))
            if w.tag0 == BOS or w.tag0 == EOS:
                cols['p1'].append(-2)
                cols['p2'].append(-1)
            else:
                cols['p1'].append(replay[-1])
                cols['p2'].append(replay[-2] if len(replay) > 1 else -1)
                replay.append(base + idx)
        path_off.append(len(cols['word']))

    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    f64 = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    i64 = lambda a: np.ascontiguousarray(a, dtype=np.int64)
    arrs = {
        'path_off': i64(path_off), 'word': i32(cols['word']), 'morph0': i32(cols['morph']),
        'tag': i32(cols['tag']), 'mask': np.ascontiguousarray(cols['mask'], dtype=np.uint32),
        'f4': f64(cols['f4']), 'f5': f64(cols['f5']), 'f6': f64(cols['f6']),
        'prev1': i64(cols['p1']), 'prev2': i64(cols['p2']),
        'terms': f64(terms).reshape(-1) if local else np.zeros(0, np.float64),
    }
    n_paths = len(path_off) - 1
    ptr = lambda a: a.ctypes.data if a.size else None
    desc = PathsDesc(n_paths, len(cols['word']), ptr(arrs['path_off']), ptr(arrs['word']),
                     ptr(arrs['morph0']), ptr(arrs['tag']), ptr(arrs['mask']), ptr(arrs['f4']),
                     ptr(arrs['f5']), ptr(arrs['f6']), ptr(arrs['prev1']), ptr(arrs['prev2']),
                     len(local), ptr(arrs['terms']), trigram_pos, scorer)
    out = np.zeros(n_paths, dtype=np.float64)
    dec = Decoder.get(device)
    dm = dec.device_model(model)
    _capi.check(dec.ctx._lib.lt_evaluate(dec.ctx.handle, dm.handle, C.byref(desc),
                                         out.ctypes.data if n_paths else None))
    return [float(x) for x in out]
