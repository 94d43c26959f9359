import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"

# torch's pageable copies (the tests' .cuda() / .cpu() of numpy arrays) go through the HIP runtime's
# own pinned staging buffers, never by page-locking the numpy memory in place (which the runtime does
# from ~1 MiB up: GPU_PINNED_MIN_XFER_SIZE, in MiB).  Both GPU faults of round 5 and the one of
# round 6 surfaced exactly at such an in-place-locked copy of a fresh numpy array; the
# library itself never hands caller memory to that path any more (rh::h2d / rh::d2h bounce buffers).
# Set before the runtime initialises (the first CUDA call); a value given by the caller wins.
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "4096")


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


_PROBE = []


def _install_fault_probe():
    """tests/fault_probe: prints the address, reason and mapping of a GPU memory fault when it
    happens (the HIP runtime only reports hipErrorIllegalAddress later).  Test infrastructure."""
    import ctypes

    import torch
    if _PROBE or not torch.cuda.is_available():
        return
    torch.cuda.init()   # the HSA runtime is up before the handler registers
    path = os.path.join(ROOT, "tests", "fault_probe", "_build", "libfault_probe.so")
    if os.path.exists(path):
        lib = ctypes.CDLL(path)
        lib.fault_probe_install()
        _PROBE.append(lib)


@pytest.fixture(autouse=True)
def _gpu_fault_attribution(request):
    """After every GPU test: the device drained, every live library context synchronised (its
    stream and an outstanding zero-copy stamp) and one small round trip on torch's stream -- so a
    fault of work a test left in flight fails THAT test's teardown instead of surfacing tests later
    at an unrelated copy (What's weak #1)."""
    if request.node.get_closest_marker("gpu") is not None:
        _install_fault_probe()
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch

    if not torch.cuda.is_initialized():
        return
    torch.cuda.synchronize()
    from ratis_amd import engine

    for c in engine.live_contexts():
        c.synchronize()
    x = torch.arange(8, device="cuda")
    assert int(x.sum().item()) == 28
    torch.cuda.synchronize()
