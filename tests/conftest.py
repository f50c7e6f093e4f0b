import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "alphazero-multi-game_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(autouse=True)
def _az_poison(request):
    """AZ_TEST_POISON=<byte> (e.g. 255): every GPU test runs with az_diag_set_poison(byte), i.e. every
    activation / workspace buffer of a net is filled with that byte before each forward -- a kernel
    that reads memory its forward never wrote then fails the oracle / bitwise checks deterministically"""
    byte = os.environ.get("AZ_TEST_POISON")
    if byte is None or request.node.get_closest_marker("gpu") is None:
        yield
        return
    from az_amd import _lib
    _lib.lib().az_diag_set_poison(int(byte, 0))
    yield
    _lib.lib().az_diag_set_poison(-1)
