import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as o
    o.load()
    return o


@pytest.fixture(scope="session")
def ctx():
    import torch

    from ratis_amd import engine

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = engine.Context(0)
    yield c
    torch.cuda.synchronize()
    c.close()
