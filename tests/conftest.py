import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def engine():
    import torch
    from uflow_amd.batch import FrameCrcEngine
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X (torch.cuda.is_available() is False)")
    eng = FrameCrcEngine(0)
    yield eng
    eng.close()
