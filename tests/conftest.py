import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP decoder)')
    config.addinivalue_line('markers', 'slow: long CPU test')


@pytest.fixture(scope='session')
def gpu_decoder():
    """The device decoder; fails loudly when the HIP library or GPU is missing."""
    from lattice_based_tagger_amd import _capi
    from lattice_based_tagger_amd.beam import Decoder
    lib = _capi.load()
    assert lib.lt_device_count() > 0, 'no HIP device visible'
    return Decoder.get(0)
