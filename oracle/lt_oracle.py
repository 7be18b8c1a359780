"""TEST INFRASTRUCTURE ONLY -- ctypes loader of the C restatement
(``oracle/lt_oracle.c`` -> ``oracle/build/liblt_oracle.so``).

``decode(packed, keys, coefs, k)`` decodes a packed batch (the arrays of
``include/lattice_decode.h``'s ``lt_batch_desc``) on the CPU and returns the
same ``(count, length, score, codes)`` layout as the device decoder, plus the
reference-algorithm counts (expansions, trigram feature tuples).
"""

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'build', 'liblt_oracle.so')


class _ModelDesc(C.Structure):
    _fields_ = [('n_keys', C.c_int64), ('keys', C.c_void_p), ('coefs', C.c_void_p)]


class _BatchDesc(C.Structure):
    # include/lattice_decode.h lt_batch_desc (ABI 6); edge terms and further
    # trigram terms unused here (ref_beam.py restates those composites)
    _fields_ = [('n_sent', C.c_int32), ('max_len', C.c_int32), ('n_post', C.c_int32),
                ('has_trigram', C.c_int32), ('n_nodes', C.c_int64), ('n_span', C.c_int64)] + [
        (f, C.c_void_p) for f in ('sent_n', 'sent_node_off', 'sent_span_off', 'span_start',
                                  'node_word', 'node_morph0', 'node_tag', 'node_mask',
                                  'node_pre', 'node_f4', 'node_f5', 'node_f6', 'node_post')] + [
        ('n_edge', C.c_int32), ('n_terms', C.c_int32), ('term_kinds', C.c_uint64),
        ('n_edges', C.c_int64), ('sent_edge_off', C.c_void_p), ('node_edge_base', C.c_void_p),
        ('edge_val', C.c_void_p), ('n_unk', C.c_int32)] + [
        (f, C.c_void_p) for f in ('unk_word', 'unk_morph0', 'unk_tag', 'unk_mask', 'unk_pre',
                                  'unk_f4', 'unk_f5', 'unk_f6', 'unk_post')] + [
        ('n_xtri', C.c_int32)] + [(f, C.c_void_p) for f in ('xtri_mask', 'xtri_f4', 'xtri_f5', 'xtri_f6')]


_lib = None


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        lib.lto_decode.restype = C.c_int
        lib.lto_decode.argtypes = [C.POINTER(_ModelDesc), C.POINTER(_BatchDesc), C.c_int, C.c_int,
                                   C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                   C.c_int]
        _lib = lib
    return _lib


_DT = {'sent_n': np.int32, 'sent_node_off': np.int64, 'sent_span_off': np.int64,
       'span_start': np.int32, 'node_word': np.int32, 'node_morph0': np.int32,
       'node_tag': np.int32, 'node_mask': np.uint32, 'node_pre': np.float64,
       'node_f4': np.float64, 'node_f5': np.float64, 'node_f6': np.float64}
_UNK_DT = {'unk_word': np.int32, 'unk_morph0': np.int32, 'unk_tag': np.int32, 'unk_mask': np.uint32,
           'unk_pre': np.float64, 'unk_f4': np.float64, 'unk_f5': np.float64, 'unk_f6': np.float64}


def decode(packed, keys, coefs, k, s0=0, s1=None, nthreads=1):
    if int(getattr(packed, 'xtri_n', 0)):
        raise NotImplementedError('lt_oracle.c restates one trigram term; oracle/ref_beam.py restates '
                                  'composites with several')
    lib = load()
    arr = {f: np.ascontiguousarray(getattr(packed, f), dtype=dt) for f, dt in _DT.items()}
    n_post = int(packed.n_post)
    post = np.ascontiguousarray(packed.node_post, dtype=np.float64) if n_post else None
    S = arr['sent_n'].shape[0]
    s1 = S if s1 is None else s1
    bd = _BatchDesc(S, int(packed.max_len), n_post, int(packed.has_trigram),
                    arr['node_word'].shape[0], arr['span_start'].shape[0],
                    *[arr[f].ctypes.data for f in _DT], None if post is None else post.ctypes.data)
    n_unk = int(getattr(packed, 'n_unk', 0))
    if n_unk:                    # implicit Unknowns (lattice_decode.h n_unk)
        unk = {f: np.ascontiguousarray(getattr(packed, f), dtype=dt) for f, dt in _UNK_DT.items()}
        unk['unk_post'] = np.ascontiguousarray(packed.unk_post, dtype=np.float64).reshape(n_post, n_unk)
        bd.n_unk = n_unk
        for f, a in unk.items():
            setattr(bd, f, a.ctypes.data if a.size else None)
    keys = np.ascontiguousarray(keys, dtype=np.uint32).reshape(-1, 4)
    coefs = np.ascontiguousarray(coefs, dtype=np.float64)
    md = _ModelDesc(keys.shape[0], keys.ctypes.data, coefs.ctypes.data)
    count = np.zeros(S, dtype=np.int32)
    length = np.zeros(S * k, dtype=np.int32)
    score = np.zeros(S * k, dtype=np.float64)
    codes = np.full(int(arr['sent_n'].astype(np.int64).sum()) * k, -1, dtype=np.int32)
    ex, tu, hi = C.c_int64(), C.c_int64(), C.c_int64()
    rc = lib.lto_decode(C.byref(md), C.byref(bd), int(k), int(s0), int(s1), count.ctypes.data,
                        length.ctypes.data, score.ctypes.data, codes.ctypes.data,
                        C.byref(ex), C.byref(tu), C.byref(hi), int(nthreads))
    if rc != 0:
        raise RuntimeError('lto_decode failed')
    decode.last_present = hi.value
    return count, length.reshape(S, k), score.reshape(S, k), codes, ex.value, tu.value
