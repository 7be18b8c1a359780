"""ctypes binding of ``liblt.so`` (include/lattice_decode.h).

The library is the product path: if it is missing or no GPU is visible the
calls raise -- there is no CPU fallback decoder.
"""

import ctypes as C
import os
import threading

import numpy as np

from ._build import LIB

LT_OK = 0
ABI_VERSION = 6           # include/lattice_decode.h LT_ABI_VERSION
LT_MAX_BEAM = 256          # tuned kernels (lattice_decode.h)
LT_MAX_BEAM_ANY = 1 << 20  # the general kernel lt_beam_wide
LT_EUNSUPPORTED = -4
_STATUS = {-1: 'LT_EINVAL', -2: 'LT_EHIP', -3: 'LT_ENOMEM', -4: 'LT_EUNSUPPORTED', -5: 'LT_ERCCL'}

EXPORTED_SYMBOLS = (
    'lt_abi_version', 'lt_hash_version', 'lt_last_error', 'lt_device_count', 'lt_ctx_create', 'lt_ctx_destroy',
    'lt_sync', 'lt_model_create', 'lt_model_destroy', 'lt_model_slots', 'lt_batch_create',
    'lt_batch_destroy', 'lt_batch_code_slots', 'lt_batch_pieces', 'lt_set_piece_bytes', 'lt_batch_reset_prep',
    'lt_batch_prep_ms', 'lt_batch_prep_bytes', 'lt_batch_host_sched_ms', 'lt_batch_prepare_k1',
    'lt_decode_launch', 'lt_last_kernel_ms',
    'lt_kernel_ms_recent', 'lt_kernel_name',
    'lt_result_fetch', 'lt_result_view', 'lt_decode', 'lt_count_ops',
    'lt_result_fetch_packed', 'lt_result_view_packed', 'lt_slab_parse',
    'lt_image_build', 'lt_image_view', 'lt_image_destroy', 'lt_model_create_from_image',
    'lt_evaluate', 'lt_decode_trace',
    'lt_comm_library', 'lt_comm_unique_id', 'lt_comm_create', 'lt_comm_destroy', 'lt_gather_prepare',
    'lt_gather_launch', 'lt_gather_sync', 'lt_gather_fetch', 'lt_gather_view', 'lt_last_gather_ms',
)
LT_COMM_ID_BYTES = 128


class LTError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__('%s (%d): %s' % (_STATUS.get(status, 'LT_ERROR'), status, msg))
        self.status = status


class ModelDesc(C.Structure):
    _fields_ = [('n_keys', C.c_int64), ('keys', C.c_void_p), ('coefs', C.c_void_p)]


class BatchDesc(C.Structure):
    _fields_ = [('n_sent', C.c_int32), ('max_len', C.c_int32), ('n_post', C.c_int32),
                ('has_trigram', C.c_int32), ('n_nodes', C.c_int64), ('n_span', C.c_int64),
                ('sent_n', C.c_void_p), ('sent_node_off', C.c_void_p),
                ('sent_span_off', C.c_void_p), ('span_start', C.c_void_p),
                ('node_word', C.c_void_p), ('node_morph0', C.c_void_p), ('node_tag', C.c_void_p),
                ('node_mask', C.c_void_p), ('node_pre', C.c_void_p), ('node_f4', C.c_void_p),
                ('node_f5', C.c_void_p), ('node_f6', C.c_void_p), ('node_post', C.c_void_p),
                ('n_edge', C.c_int32), ('n_terms', C.c_int32), ('term_kinds', C.c_uint64),
                ('n_edges', C.c_int64), ('sent_edge_off', C.c_void_p), ('node_edge_base', C.c_void_p),
                ('edge_val', C.c_void_p), ('n_unk', C.c_int32)] + [
        (f, C.c_void_p) for f in ('unk_word', 'unk_morph0', 'unk_tag', 'unk_mask', 'unk_pre', 'unk_f4',
                                  'unk_f5', 'unk_f6', 'unk_post')] + [
        ('n_xtri', C.c_int32)] + [(f, C.c_void_p) for f in ('xtri_mask', 'xtri_f4', 'xtri_f5', 'xtri_f6')]


class Result(C.Structure):
    _fields_ = [('count', C.POINTER(C.c_int32)), ('length', C.POINTER(C.c_int32)),
                ('score', C.POINTER(C.c_double)), ('codes', C.POINTER(C.c_int32))]


class PackedView(C.Structure):
    _fields_ = [('n_sent', C.c_int32), ('k', C.c_int32), ('n_codes', C.c_int64),
                ('count', C.POINTER(C.c_int32)), ('length', C.POINTER(C.c_int32)),
                ('score', C.POINTER(C.c_double)), ('codes', C.POINTER(C.c_int32))]


def _arr(p, n, dt):
    if n == 0:
        return np.zeros(0, dtype=dt)
    return np.ctypeslib.as_array(p, shape=(n,)).copy()


class PackedResults:
    """Compact results of one decode (a slab, lattice_decode.h "compact
    results"): ``count`` [S], ``length`` / ``score`` [S, k] (0 past count),
    ``codes`` the paths' node codes back to back, sentence-major, best
    mature first; ``off`` [S*k + 1] where mature (s, t) starts in ``codes``."""

    def __init__(self, v):
        S, k = int(v.n_sent), int(v.k)
        self.k = k
        self.count = _arr(v.count, S, np.int32)
        self.length = _arr(v.length, S * k, np.int32).reshape(S, k)
        self.score = _arr(v.score, S * k, np.float64).reshape(S, k)
        self.codes = _arr(v.codes, int(v.n_codes), np.int32)
        self.off = np.zeros(S * k + 1, dtype=np.int64)
        np.cumsum(self.length.ravel(), out=self.off[1:])

    @property
    def n_sent(self):
        return int(self.count.shape[0])

    def padded(self, sent_n):
        """(count, length, score, codes) in the padded layout of
        ``lt_result`` (codes of mature t of sentence s at k*cum_n[s] + t*n_s,
        -1 past the path)."""
        k = self.k
        n = np.asarray(sent_n, dtype=np.int64)
        cum = np.zeros(len(n) + 1, dtype=np.int64)
        np.cumsum(n, out=cum[1:])
        codes = np.full(int(cum[-1]) * k, -1, dtype=np.int32)
        L = self.length.ravel().astype(np.int64)
        if L.sum():
            e = np.repeat(np.arange(L.size, dtype=np.int64), L)
            s, t = e // k, e % k
            j = np.arange(int(L.sum()), dtype=np.int64) - self.off[e]
            codes[k * cum[s] + t * n[s] + j] = self.codes
        return self.count.copy(), self.length.copy(), self.score.copy(), codes


_lib = None
_lock = threading.Lock()


def load(path=None):
    """Load liblt.so (built in-tree by ``_build.build``).  Raises if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # LT_LIBRARY: an alternative in-tree build (kernel A/B experiments)
        path = path or os.environ.get('LT_LIBRARY') or LIB
        if not os.path.exists(path):
            raise RuntimeError('liblt.so not built (%s); run __graft_entry__.build()' % path)
        lib = C.CDLL(path)
        vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        sig = {
            'lt_abi_version': (C.c_int, []),
            'lt_last_error': (C.c_char_p, []),
            'lt_device_count': (C.c_int, []),
            'lt_ctx_create': (i32, [C.c_int, C.POINTER(vp)]),
            'lt_ctx_destroy': (i32, [vp]),
            'lt_sync': (i32, [vp]),
            'lt_model_create': (i32, [vp, C.POINTER(ModelDesc), C.POINTER(vp)]),
            'lt_model_destroy': (i32, [vp]),
            'lt_model_slots': (i64, [vp]),
            'lt_batch_create': (i32, [vp, C.POINTER(BatchDesc), C.c_int, C.POINTER(vp)]),
            'lt_batch_destroy': (i32, [vp]),
            'lt_batch_code_slots': (i64, [vp, C.c_int]),
            'lt_batch_pieces': (i32, [vp]),
            'lt_set_piece_bytes': (i64, [i64]),
            'lt_batch_reset_prep': (i32, [vp]),
            'lt_batch_prep_ms': (i32, [vp, C.POINTER(C.c_float)]),
            'lt_batch_prep_bytes': (i64, [vp]),
            'lt_batch_host_sched_ms': (C.c_double, [vp]),
            'lt_batch_prepare_k1': (i32, [vp]),
            'lt_decode_launch': (i32, [vp, vp, vp, C.c_int]),
            'lt_last_kernel_ms': (i32, [vp, C.POINTER(C.c_float)]),
            'lt_kernel_ms_recent': (i32, [vp, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int)]),
            'lt_kernel_name': (C.c_char_p, [C.c_int]),
            'lt_image_build': (i32, [vp, C.POINTER(vp)]),
            'lt_image_view': (i32, [vp, vp]),
            'lt_image_destroy': (i32, [vp]),
            'lt_model_create_from_image': (i32, [vp, vp, C.POINTER(vp)]),
            'lt_evaluate': (i32, [vp, vp, vp, vp]),
            'lt_decode_trace': (i32, [vp, vp, vp, C.c_int, vp]),
            'lt_result_fetch': (i32, [vp, vp]),
            'lt_result_view': (i32, [vp, C.POINTER(Result)]),
            'lt_result_fetch_packed': (i32, [vp, vp]),
            'lt_result_view_packed': (i32, [vp, C.POINTER(PackedView)]),
            'lt_slab_parse': (i32, [vp, C.c_uint64, C.POINTER(PackedView)]),
            'lt_decode': (i32, [vp, vp, vp, C.c_int, C.POINTER(Result)]),
            'lt_count_ops': (i32, [vp, vp, vp, C.c_int, C.POINTER(i64), C.POINTER(i64),
                                   C.POINTER(i64), C.POINTER(i64)]),
            'lt_comm_library': (C.c_char_p, []),
            'lt_hash_version': (C.c_uint32, []),
            'lt_comm_unique_id': (i32, [C.c_char_p]),
            'lt_comm_create': (i32, [vp, C.c_int, C.c_int, C.c_char_p, C.POINTER(vp)]),
            'lt_comm_destroy': (i32, [vp]),
            'lt_gather_prepare': (i32, [vp, vp, C.c_int, C.c_int]),
            'lt_gather_launch': (i32, [vp, vp]),
            'lt_gather_sync': (i32, [vp]),
            'lt_gather_fetch': (i32, [vp]),
            'lt_gather_view': (i32, [vp, C.c_int, C.POINTER(PackedView)]),
            'lt_last_gather_ms': (i32, [vp, C.POINTER(C.c_float)]),
        }
        for name, (res, args) in sig.items():
            if name in OPTIONAL_CALLS and not hasattr(lib, name):
                continue                    # (an older experiment build; see OPTIONAL_CALLS)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.lt_abi_version() != ABI_VERSION:
            raise RuntimeError('%s has ABI %d, this package needs %d (rebuild it)'
                               % (path, lib.lt_abi_version(), ABI_VERSION))
        # Calls that only queue work or copy a few bytes, bound a second time
        # through PyDLL (the GIL stays held): a CDLL call releases the GIL
        # and must win it back from whichever pipeline thread runs Python --
        # up to a switch interval (5 ms) per call -- which costs more than
        # these calls do.
        held = C.PyDLL(path)
        for name in HELD_CALLS:
            fn = getattr(held, name)
            fn.restype, fn.argtypes = sig[name]
        lib.held = held
        _lib = lib
        return lib


# entry points an A/B build of an earlier revision may lack (tools/gpu_ab.sh)
OPTIONAL_CALLS = ('lt_hash_version', 'lt_batch_host_sched_ms', 'lt_batch_prepare_k1')

# lt_* entry points that return in microseconds (see load)
HELD_CALLS = ('lt_decode_launch', 'lt_result_fetch', 'lt_result_view', 'lt_result_fetch_packed',
              'lt_result_view_packed')


def check(status):
    if status != LT_OK:
        msg = load().lt_last_error().decode('utf-8', 'replace')
        raise LTError(status, msg)


def _ptr(a):
    return None if a is None else a.ctypes.data


def parse_slab(buf):
    """PackedResults of a slab held in host memory (``buf``: a contiguous
    uint8 array whose size is the slab's capacity), checked by
    lt_slab_parse -- how the root reads every rank's slab of a gather."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    v = PackedView()
    check(load().lt_slab_parse(buf.ctypes.data, buf.size, C.byref(v)))
    return PackedResults(v)


class Context:
    """One device + one HIP stream (lt_ctx)."""

    def __init__(self, device=0):
        lib = load()
        h = C.c_void_p()
        check(lib.lt_ctx_create(int(device), C.byref(h)))
        self.handle = h
        self.device = device
        self._lib = lib

    def sync(self):
        check(self._lib.lt_sync(self.handle))

    def kernel_ms(self):
        v = C.c_float()
        check(self._lib.lt_last_kernel_ms(self.handle, C.byref(v)))
        return float(v.value)

    def kernel_ms_recent(self, n):
        """Device times (ms) of the last min(n, 64) decode kernels, oldest
        first (after sync)."""
        buf = (C.c_float * max(int(n), 1))()
        got = C.c_int()
        check(self._lib.lt_kernel_ms_recent(self.handle, int(n), buf, C.byref(got)))
        return [float(buf[i]) for i in range(got.value)]

    def close(self):
        if self.handle:
            self._lib.lt_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ModelImageView(C.Structure):
    _fields_ = [('hash_version', C.c_uint32), ('narrow', C.c_int32), ('seed', C.c_uint32),
                ('slots', C.c_int64),
                ('table', C.c_void_p), ('table_bytes', C.c_int64),
                ('d3mul', C.c_uint32), ('d3', C.c_void_p)]


class ModelImage:
    """Host-side model image (lt_image): the built cuckoo table and dense
    class-3 table of a key set, without a GPU.  ``arrays()`` copies them out
    (for a model file); ``DeviceModel.from_image`` uploads them."""

    def __init__(self, keys, coefs, lib=None):
        lib = lib or load()
        keys = np.ascontiguousarray(keys, dtype=np.uint32).reshape(-1, 4)
        coefs = np.ascontiguousarray(coefs, dtype=np.float64)
        desc = ModelDesc(keys.shape[0], _ptr(keys), _ptr(coefs))
        h = C.c_void_p()
        check(lib.lt_image_build(C.byref(desc), C.byref(h)))
        self.handle, self._lib = h, lib

    def arrays(self):
        v = ModelImageView()
        check(self._lib.lt_image_view(self.handle, C.byref(v)))
        table = np.frombuffer((C.c_uint8 * v.table_bytes).from_address(v.table), dtype=np.uint8).copy()
        d3 = (np.frombuffer((C.c_double * 1024).from_address(v.d3), dtype=np.float64).copy()
              if v.d3mul else np.zeros(0, dtype=np.float64))
        return {'hash_version': int(v.hash_version), 'narrow': int(v.narrow), 'seed': int(v.seed),
                'slots': int(v.slots),
                'd3mul': int(v.d3mul), 'table': table, 'd3': d3}

    def close(self):
        if self.handle:
            self._lib.lt_image_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceModel:
    """Hash table of the probed feature classes on one device (lt_model)."""

    def __init__(self, ctx, keys, coefs):
        keys = np.ascontiguousarray(keys, dtype=np.uint32).reshape(-1, 4)
        coefs = np.ascontiguousarray(coefs, dtype=np.float64)
        desc = ModelDesc(keys.shape[0], _ptr(keys), _ptr(coefs))
        h = C.c_void_p()
        check(ctx._lib.lt_model_create(ctx.handle, C.byref(desc), C.byref(h)))
        self.handle = h
        self.ctx = ctx
        self.slots = ctx._lib.lt_model_slots(h)

    @classmethod
    def from_image(cls, ctx, image):
        """Upload a model image: a dict as returned by ``ModelImage.arrays``
        (arrays may be memory-mapped from a model file)."""
        table = np.ascontiguousarray(image['table'], dtype=np.uint8)
        d3 = np.ascontiguousarray(image['d3'], dtype=np.float64)
        if image['d3mul'] and d3.size != 1024:
            raise ValueError('dense class-3 table must hold 1024 coefficients')
        v = ModelImageView(int(image.get('hash_version', 1)), int(image['narrow']),
                           int(image['seed']), int(image['slots']),
                           table.ctypes.data, table.nbytes, int(image['d3mul']),
                           d3.ctypes.data if image['d3mul'] else None)
        h = C.c_void_p()
        check(ctx._lib.lt_model_create_from_image(ctx.handle, C.byref(v), C.byref(h)))
        self = cls.__new__(cls)
        self.handle, self.ctx = h, ctx
        self.slots = ctx._lib.lt_model_slots(h)
        return self

    def close(self):
        if self.handle:
            self.ctx._lib.lt_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TraceDesc(C.Structure):
    _fields_ = [('pos_off', C.c_void_p), ('exp_off', C.c_void_p), ('n_exp', C.c_int64),
                ('beam_count', C.c_void_p), ('beam_gen', C.c_void_p), ('exp_count', C.c_void_p),
                ('exp_score', C.c_void_p), ('exp_node', C.c_void_p), ('exp_skip', C.c_void_p),
                ('exp_link', C.c_void_p)]


class DeviceBatch:
    """A packed batch resident on the device (lt_batch)."""

    FIELDS = ('sent_n', 'sent_node_off', 'sent_span_off', 'span_start', 'node_word',
              'node_morph0', 'node_tag', 'node_mask', 'node_pre', 'node_f4', 'node_f5',
              'node_f6')
    UNK_DTYPES = {'unk_word': np.int32, 'unk_morph0': np.int32, 'unk_tag': np.int32, 'unk_mask': np.uint32,
                  'unk_pre': np.float64, 'unk_f4': np.float64, 'unk_f5': np.float64, 'unk_f6': np.float64}
    DTYPES = {'sent_n': np.int32, 'sent_node_off': np.int64, 'sent_span_off': np.int64,
              'span_start': np.int32, 'node_word': np.int32, 'node_morph0': np.int32,
              'node_tag': np.int32, 'node_mask': np.uint32, 'node_pre': np.float64,
              'node_f4': np.float64, 'node_f5': np.float64, 'node_f6': np.float64}

    def __init__(self, ctx, packed, max_k):
        arr = {f: np.ascontiguousarray(getattr(packed, f), dtype=self.DTYPES[f])
               for f in self.FIELDS}
        n_post = int(packed.n_post)
        post = np.ascontiguousarray(packed.node_post, dtype=np.float64) if n_post else None
        self.n_sent = int(arr['sent_n'].shape[0])
        self.sent_n = arr['sent_n']
        self._span_start, self._span_off = arr['span_start'], arr['sent_span_off']
        self.cum_n = np.zeros(self.n_sent + 1, dtype=np.int64)
        np.cumsum(self.sent_n, out=self.cum_n[1:])
        n_edge = int(getattr(packed, 'edge_terms', 0))
        edges = (None, None, None)
        if n_edge:                   # edge_local plugins (lowering.KIND_EDGE)
            edges = (np.ascontiguousarray(packed.sent_edge_off, dtype=np.int64),
                     np.ascontiguousarray(packed.node_edge_base, dtype=np.int64),
                     np.ascontiguousarray(packed.edge_val, dtype=np.float64))
        n_unk = int(getattr(packed, 'n_unk', 0))
        unk = ()
        if n_unk:                    # implicit Unknowns (lattice_decode.h n_unk)
            unk = tuple(np.ascontiguousarray(getattr(packed, f), dtype=self.UNK_DTYPES[f])
                        for f in self.UNK_DTYPES) + (
                np.ascontiguousarray(packed.unk_post, dtype=np.float64) if n_post else None,)
        n_xtri = int(getattr(packed, 'xtri_n', 0))
        xtri = ()
        if n_xtri:                   # further trigram scorers (lattice_decode.h n_xtri, ABI 6)
            xtri = (np.ascontiguousarray(packed.xtri_mask, dtype=np.uint32),) + tuple(
                np.ascontiguousarray(getattr(packed, f), dtype=np.float64) for f in ('xtri_f4', 'xtri_f5', 'xtri_f6'))
        self._keep = (post,) + edges + unk + xtri
        plan = n_edge or n_xtri      # the term plan is read with edge terms or several trigram terms
        desc = BatchDesc(
            self.n_sent, int(packed.max_len), n_post, int(packed.has_trigram),
            int(arr['node_word'].shape[0]), int(arr['span_start'].shape[0]),
            *[_ptr(arr[f]) for f in self.FIELDS], _ptr(post),
            n_edge, int(getattr(packed, 'n_terms', 0)) if plan else 0,
            int(getattr(packed, 'term_kinds', 0)) if plan else 0,
            int(edges[2].shape[1]) if n_edge else 0, *[_ptr(x) for x in edges],
            n_unk, *([_ptr(x) for x in unk] if n_unk else [None] * 9),
            n_xtri, *([_ptr(x) for x in xtri] if n_xtri else [None] * 4))
        self.n_unk = n_unk
        h = C.c_void_p()
        check(ctx._lib.lt_batch_create(ctx.handle, C.byref(desc), int(max_k), C.byref(h)))
        self.handle = h
        self.ctx = ctx
        self.max_k = int(max_k)
        self.max_len = int(packed.max_len)

    @property
    def pieces(self):
        """Kernel launches per decode (lattice_decode.h lt_batch_pieces)."""
        return int(self.ctx._lib.lt_batch_pieces(self.handle))

    def launch(self, model, k):
        check(self.ctx._lib.held.lt_decode_launch(self.ctx.handle, model.handle, self.handle, int(k)))

    def reset_prep(self):
        """Forget the device preparation (the k=1 lane schedule): the next
        beam-1 decode rebuilds it -- a fresh-batch step for benchmarks."""
        check(self.ctx._lib.lt_batch_reset_prep(self.handle))

    def prep_bytes(self):
        """Bytes of the device preparation (lane schedules + wave offsets)."""
        return int(self.ctx._lib.lt_batch_prep_bytes(self.handle))

    def prep_ms(self):
        """Device time (ms) of the batch's last preparation (after sync)."""
        v = C.c_float()
        check(self.ctx._lib.lt_batch_prep_ms(self.handle, C.byref(v)))
        return float(v.value)

    def host_sched_ms(self):
        """Wall time (ms) lt_batch_create spent on the host half of the
        beam-1 schedule (steps and placements); None from a library without
        the call."""
        fn = getattr(self.ctx._lib, 'lt_batch_host_sched_ms', None)
        return float(fn(self.handle)) if fn else None

    def prepare_k1(self):
        """Build the beam-1 schedule of a batch created for larger beams now
        (lattice_decode.h lt_batch_prepare_k1), off the launch path."""
        check(self.ctx._lib.lt_batch_prepare_k1(self.handle))

    def fetch(self):
        check(self.ctx._lib.held.lt_result_fetch(self.ctx.handle, self.handle))

    def results(self, k):
        """numpy copies of (count, length, score, codes) after fetch + sync."""
        v = Result()
        check(self.ctx._lib.held.lt_result_view(self.handle, C.byref(v)))
        S = self.n_sent
        nc = int(self.cum_n[-1]) * k

        def arr(p, n, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(p, shape=(n,)).copy()
        return (arr(v.count, S, np.int32), arr(v.length, S * k, np.int32).reshape(S, k),
                arr(v.score, S * k, np.float64).reshape(S, k), arr(v.codes, nc, np.int32))

    def fetch_packed(self):
        check(self.ctx._lib.held.lt_result_fetch_packed(self.ctx.handle, self.handle))

    def results_packed(self):
        """PackedResults of the last fetch_packed (after sync)."""
        v = PackedView()
        check(self.ctx._lib.held.lt_result_view_packed(self.handle, C.byref(v)))
        return PackedResults(v)

    def decode(self, model, k):
        self.launch(model, k)
        self.fetch()
        self.ctx.sync()
        return self.results(k)

    def decode_packed(self, model, k):
        self.launch(model, k)
        self.fetch_packed()
        self.ctx.sync()
        return self.results_packed()

    def trace(self, model, k):
        """Every expansion of every end position (lt_decode_trace), as a dict
        of arrays: pos_off (positions of sentence s: pos_off[s] + e),
        exp_off, beam_count, beam_gen [positions, k], exp_count, exp_score,
        exp_node, exp_skip, exp_link (per expansion: node | span-1 << 21 |
        parent rank << 42, csrc/lt_common.h bpw_pack)."""
        n = self.sent_n.astype(np.int64)
        pos_off = np.zeros(self.n_sent + 1, dtype=np.int64)
        np.cumsum(n + 1, out=pos_off[1:])
        P = int(pos_off[-1])
        # slots of position e of sentence s: k x (candidates ending at e)
        span = np.ascontiguousarray(self._span_start, dtype=np.int64)
        span_off = self._span_off
        S = 8 if self.max_len <= 8 else int(self.max_len)          # span slots per position
        bound = np.zeros(P, dtype=np.int64)
        for s in range(self.n_sent):
            ns = int(n[s])
            if ns:
                a = span[span_off[s]:span_off[s] + S * ns + 1]
                cnt = np.diff(a).reshape(ns, S)
                if self.n_unk:       # an empty in-range span holds its implicit Unknown
                    e = np.arange(1, ns + 1)[:, None]
                    d = S - np.arange(S)[None, :]
                    cnt = np.where((cnt == 0) & (d <= np.minimum(e, self.max_len)), 1, cnt)
                bound[pos_off[s] + 1:pos_off[s] + 1 + ns] = cnt.sum(axis=1) * int(k)
        exp_off = np.zeros(P + 1, dtype=np.int64)
        np.cumsum(bound, out=exp_off[1:])
        n_exp = int(exp_off[-1])
        out = {'pos_off': pos_off, 'exp_off': exp_off,
               'beam_count': np.zeros(P, dtype=np.int32), 'beam_gen': np.zeros((P, int(k)), dtype=np.uint32),
               'exp_count': np.zeros(P, dtype=np.int32), 'exp_score': np.zeros(max(n_exp, 1), dtype=np.float64),
               'exp_node': np.zeros(max(n_exp, 1), dtype=np.uint32), 'exp_skip': np.zeros(max(n_exp, 1), dtype=np.uint8),
               'exp_link': np.zeros(max(n_exp, 1), dtype=np.uint64)}
        desc = TraceDesc(*[_ptr(out[f]) for f in ('pos_off', 'exp_off')], n_exp,
                         *[_ptr(out[f]) for f in ('beam_count', 'beam_gen', 'exp_count', 'exp_score',
                                                 'exp_node', 'exp_skip', 'exp_link')])
        check(self.ctx._lib.lt_decode_trace(self.ctx.handle, model.handle, self.handle, int(k), C.byref(desc)))
        return out

    def count_ops(self, model, k):
        """(expansions, feature tuples, probes, table loads) of beam k."""
        x, p, q, t = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(self.ctx._lib.lt_count_ops(self.ctx.handle, model.handle, self.handle, int(k),
                                         C.byref(x), C.byref(p), C.byref(q), C.byref(t)))
        return x.value, p.value, q.value, t.value

    def close(self):
        if self.handle:
            self.ctx._lib.lt_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    """A fresh RCCL communicator id (bytes) -- created on one rank, shared
    with the others by the caller (e.g. a gloo broadcast)."""
    buf = C.create_string_buffer(LT_COMM_ID_BYTES)
    check(load().lt_comm_unique_id(buf))
    return buf.raw


class Comm:
    """RCCL communicator of one rank (lt_comm): gathers every rank's decode
    results to a root rank (include/lattice_decode.h, "multi-GPU result
    gather").  All methods but ``view``/``gather_ms`` are collective."""

    def __init__(self, ctx, nranks, rank, uid):
        if len(uid) != LT_COMM_ID_BYTES:
            raise ValueError('communicator id must be %d bytes' % LT_COMM_ID_BYTES)
        h = C.c_void_p()
        check(ctx._lib.lt_comm_create(ctx.handle, int(nranks), int(rank), bytes(uid), C.byref(h)))
        self.handle, self.ctx = h, ctx
        self.nranks, self.rank = int(nranks), int(rank)
        self.k = 0

    def prepare(self, batch, k, root=0):
        check(self.ctx._lib.lt_gather_prepare(self.handle, batch.handle, int(k), int(root)))
        self.k, self.root = int(k), int(root)

    def launch(self, batch):
        check(self.ctx._lib.lt_gather_launch(self.handle, batch.handle))

    def sync(self):
        check(self.ctx._lib.lt_gather_sync(self.handle))

    def fetch(self):
        check(self.ctx._lib.lt_gather_fetch(self.handle))

    def gather_ms(self):
        v = C.c_float()
        check(self.ctx._lib.lt_last_gather_ms(self.handle, C.byref(v)))
        return float(v.value)

    def view(self, r):
        """Root, after fetch + sync: rank r's PackedResults."""
        v = PackedView()
        check(self.ctx._lib.lt_gather_view(self.handle, int(r), C.byref(v)))
        return PackedResults(v)

    def close(self):
        if self.handle:
            self.ctx._lib.lt_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
