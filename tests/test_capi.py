"""liblt.so builds, loads and exports every entry point include/lattice_decode.h
declares (no compute without a GPU)."""

import os
import re
import subprocess

import pytest

from lattice_based_tagger_amd import _build, _capi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      'include', 'lattice_decode.h')


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(lt_[a-z0-9_]+)\s*\(', text)))


def test_library_exports_every_declared_symbol():
    lib = _build.build(verbose=False)
    out = subprocess.run(['nm', '-D', '--defined-only', lib], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r'\bT (lt_\w+)', out))
    declared = declared_symbols()
    assert declared, 'no declarations parsed'
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(declared) == set(_capi.EXPORTED_SYMBOLS)


def test_library_loads_and_reports_abi():
    lib = _capi.load()
    assert lib.lt_abi_version() == _capi.ABI_VERSION == 6
    assert lib.lt_device_count() >= 0


def test_kernels_are_gfx950_code_objects():
    lib = _build.build(verbose=False)
    blob = open(lib, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob
    # the shipping kernels, and only those (the superseded lt_viterbi_k /
    # lt_beam_k of round 1 are gone)
    for name in (b'lt_viterbi_pk', b'lt_beam_hw', b'lt_beam_pk', b'lt_pack_write_k', b'lt_slab_to_host_k'):
        assert name in blob, name
    assert b'lt_viterbi_k' not in blob and b'lt_beam_k' not in blob


def test_context_without_gpu_fails_loudly():
    lib = _capi.load()
    if lib.lt_device_count() > 0:
        pytest.skip('GPU present')
    with pytest.raises(_capi.LTError):
        _capi.Context(0)


def test_kernel_name_without_gpu():
    """Host-only query: the kernel each beam width launches (profiling names)."""
    lib = _capi.load()
    assert lib.lt_kernel_name(1) == b'lt_viterbi_pk'
    assert lib.lt_kernel_name(2) == b'lt_beam_hw'
    assert lib.lt_kernel_name(5) == b'lt_beam_hw'
    assert lib.lt_kernel_name(16) == b'lt_beam_pk'
    assert lib.lt_kernel_name(32) == b'lt_beam_pk'
    assert lib.lt_kernel_name(33) == b'lt_beam_pk'
    assert lib.lt_kernel_name(256) == b'lt_beam_pk'
    assert lib.lt_kernel_name(257) == b'lt_beam_wide'      # the general kernel (also max_len > 8)
    assert lib.lt_kernel_name(0) is None or lib.lt_kernel_name(0) == b'lt_viterbi_pk'


@pytest.mark.parametrize('header', ['lattice_pack.h', 'lattice_lookup.h'])
def test_host_side_headers_are_exported(header):
    """The packer and lattice-builder entry points (include/lattice_pack.h,
    include/lattice_lookup.h) are exported and load through ctypes."""
    lib = _build.build(verbose=False)
    text = open(os.path.join(os.path.dirname(HEADER), header)).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    declared = sorted(set(re.findall(r'\b(lt_[a-z_0-9]+)\s*\(', text)))
    assert declared
    out = subprocess.run(['nm', '-D', '--defined-only', lib], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r'\bT (lt_\w+)', out))
    assert [s for s in declared if s not in exported] == []
    loaded = _capi.load()
    for s in declared:
        getattr(loaded, s)
