import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _poison_cached_gpu_memory(request):
    """DNN_POISON_CACHE=1 (diagnostic): before every GPU test, fill the caching allocator's free
    memory with 0xFF bytes (NaN as fp32 / bf16, -1 as int32), so a kernel that reads memory its
    test never wrote fails the same way every time instead of depending on what earlier tests
    left behind."""
    if os.environ.get("DNN_POISON_CACHE") != "1" or "gpu" not in request.node.keywords:
        yield
        return
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        junk = [torch.full((1 << 28,), 255, dtype=torch.uint8, device="cuda") for _ in range(4)]  # large pool
        junk += [torch.full((1 << 19,), 255, dtype=torch.uint8, device="cuda") for _ in range(256)]  # small pool
        torch.cuda.synchronize()
        del junk
    yield


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
