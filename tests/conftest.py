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
