import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_sessionstart(session):
    # tuning only: DI_TEST_VARIANT=<path> runs the GPU tests against a kernel variant of the
    # library (tools/build_variants.py) before it is made the default build
    path = os.environ.get("DI_TEST_VARIANT")
    if path:
        from deepinteract_amd import _lib
        _lib.load_variant(path)
