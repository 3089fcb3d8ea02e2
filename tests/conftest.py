import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def pytest_sessionstart(session):
    # torch caches its device count on the first ask; asked only after a test
    # initialised HIP through the engine library (the JNI shim's tests do), it
    # answered "no GPU" and the tests that check torch skipped themselves
    _gpu_available()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine_factory():
    if not _gpu_available():
        pytest.skip("no GPU visible")
    from libjitsi_amd import SRTPEngine
    made = []

    def make(**kw):
        e = SRTPEngine(**kw)
        made.append(e)
        return e

    yield make
    for e in made:
        e.close()
