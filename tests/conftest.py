import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _have_gpu() -> bool:
    try:
        from deequ_amd import _lib
        return _lib.device_count() > 0
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _release_device_memory(request):
    """After each GPU test: collect unreachable tables and hand the cached device blocks (the
    library's pool, torch's allocator) back, so one test's memory does not crowd the next."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    gc.collect()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        from deequ_amd import _lib as L
        L.lib().dq_release_cached_memory(0)
    except Exception:  # noqa: BLE001 -- best effort
        pass


@pytest.fixture(scope="session")
def gpu():
    """Skips nothing: a test marked `gpu` that runs without a GPU must fail loudly."""
    if not _have_gpu():
        pytest.fail("no gfx950 device visible (the GPU tests must run on an MI355X)")
    import deequ_amd
    deequ_amd.set_device(0)
    return 0
