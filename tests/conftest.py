"""Shared test setup: markers, import helpers for the hyphenated package and the oracle."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def nexr_pkg():
    return importlib.import_module("nex-nccl_amd")


@pytest.fixture(scope="session")
def nexr():
    return nexr_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def golden_cases():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


class _ExtrasRing:
    """The ring module with RingComm / PeerRingComm defaulting to the opt-in extras library."""

    def __init__(self, mod):
        self._m = mod

    def __getattr__(self, k):
        return getattr(self._m, k)

    def RingComm(self, *a, **kw):  # noqa: N802 - mirrors the class name
        kw.setdefault("extras", True)
        return self._m.RingComm(*a, **kw)

    def PeerRingComm(self, *a, **kw):  # noqa: N802
        kw.setdefault("extras", True)
        return self._m.PeerRingComm(*a, **kw)


def extras_ring():
    """For the tests of include/nexr_extras.h (send/recv, the resident collectives): the ring module
    bound to libnexr_extras.so, or a skip when that opt-in library is not built."""
    r = importlib.import_module("nex-nccl_amd.ring")
    if not r.extras_available():
        pytest.skip("libnexr_extras.so not built (opt-in: make -C nex-nccl_amd/csrc EXTRAS=1)")
    return _ExtrasRing(r)
