"""Build of the in-tree HIP library ``lattice_based_tagger_amd/_lib/liblt.so``.

``hipcc --offload-arch=gfx950`` cross-compiles without a GPU, so this runs in
the CPU container and the resulting ``.so`` travels to the GPU box with the
repository snapshot.  ``-ffp-contract=off`` keeps every float64 add/mul a
separate IEEE operation, which bit-exact parity with the reference requires.
"""

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, '_lib')
LIB = os.path.join(LIBDIR, 'liblt.so')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
HIPCC = os.path.join(ROCM, 'bin', 'hipcc')
ARCH = 'gfx950'

SOURCES = ['lt_decode.hip', 'lt_results.hip', 'lt_capi.cpp', 'lt_packer.cpp', 'lt_comm.cpp', 'lt_lookup.cpp']
HEADERS = ['lt_common.h', 'lt_internal.h', 'lt_error.h', 'lt_handles.h', 'lt_host.h', os.path.join('..', '..', 'include', 'lattice_decode.h'),
           os.path.join('..', '..', 'include', 'lattice_pack.h'),
           os.path.join('..', '..', 'include', 'lattice_lookup.h')]

PYOBJ_SRC = os.path.join(CSRC, 'lt_pyobj.c')
# named for the interpreter ABI it is built against (EXT_SUFFIX, e.g.
# .cpython-310-x86_64-linux-gnu.so): another CPython finds no stale build of
# the wrong ABI, it builds its own
PYOBJ = os.path.join(LIBDIR, '_ltpy' + (sysconfig.get_config_var('EXT_SUFFIX') or '.so'))

COMMON_FLAGS = ['-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', '-fno-fast-math',
                '-Wall', '-Wno-unused-result', '-I' + os.path.join(HERE, '..', 'include')]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(dp) > t for dp in deps)


def build_pyobj(force=False, verbose=True):
    """The CPython extension `_ltpy` (csrc/lt_pyobj.c: bulk Word / path
    construction for the returned Sequences), compiled with the host C
    compiler against this interpreter's headers."""
    os.makedirs(LIBDIR, exist_ok=True)
    if not force and not _stale(PYOBJ, [PYOBJ_SRC, __file__]):
        return PYOBJ
    tmp = PYOBJ + '.tmp'
    cmd = [os.environ.get('CC', 'gcc'), '-O2', '-Wall', '-shared', '-fPIC', '-fno-strict-aliasing',
           '-I' + sysconfig.get_paths()['include'], PYOBJ_SRC, '-o', tmp]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, PYOBJ)
    return PYOBJ


def build(force=False, verbose=True, defines=(), out=None):
    """Compile liblt.so if any source is newer than it.  Returns its path.
    ``defines``/``out``: an experiment build (e.g. ``('PK_WAVES=3',)``) to
    another file, selected at run time with LT_LIBRARY."""
    os.makedirs(LIBDIR, exist_ok=True)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [__file__]
    lib = out or LIB
    if out is None:
        build_pyobj(force, verbose)
    if not force and not _stale(lib, deps):
        return lib
    objs = []
    for src in SOURCES:
        # (objects named after the library too: experiment builds can run in parallel)
        obj = os.path.join(LIBDIR, os.path.splitext(os.path.basename(lib))[0] + '_' + os.path.splitext(src)[0] + '.o')
        extra = os.environ.get('LT_EXTRA_FLAGS', '').split() if out is not None else []   # experiment builds only
        cmd = [HIPCC, '--offload-arch=' + ARCH] + COMMON_FLAGS + extra + ['-D' + d for d in defines] + [
            '-c', os.path.join(CSRC, src), '-o', obj]
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + '.tmp'
    cmd = [HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', tmp] + objs + [
        '-Wl,-rpath,' + os.path.join(ROCM, 'lib'), '-ldl', '-Wl,--no-undefined']
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == '__main__':
    # python -m lattice_based_tagger_amd._build [--force] [-DNAME=V ... -o OUT]
    args = sys.argv[1:]
    defs = [a[2:] for a in args if a.startswith('-D')]
    out = args[args.index('-o') + 1] if '-o' in args else None
    build(force='--force' in args or bool(defs), defines=defs, out=out)
