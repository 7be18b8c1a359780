"""Loader of the `_ltpy` CPython extension (csrc/lt_pyobj.c), built in-tree by
``_build.build`` next to liblt.so.  There is no Python fallback: a missing
extension raises, like a missing liblt.so."""

import importlib.machinery
import importlib.util
import os
import threading

_mod = None
_lock = threading.Lock()


def load():
    global _mod
    if _mod is None:
        with _lock:
            if _mod is None:
                from ._build import PYOBJ as path             # (per-interpreter name, EXT_SUFFIX)
                if not os.path.exists(path):
                    raise ImportError('lattice_based_tagger_amd: %s is missing -- run '
                                      '__graft_entry__.build() (python -m lattice_based_tagger_amd._build)' % path)
                loader = importlib.machinery.ExtensionFileLoader('_ltpy', path)
                spec = importlib.util.spec_from_file_location('_ltpy', path, loader=loader)
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
                _mod = mod
    return _mod
