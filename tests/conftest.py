import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# PyTorch (device memory for the GPU tests) must bring its HIP runtime in
# before libbjxa.so.0 binds one.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP kernels)")
    config.addinivalue_line("markers", "routing: a GPU test that keeps the library's default "
                            "CPU/GPU routing of host-API calls")


@pytest.fixture(autouse=True)
def _gpu_route(request):
    """GPU tests drive the host API's calls to the kernels (offload threshold
    0) unless marked `routing`; CPU tests leave the routing alone (without a
    GPU every call runs on the CPU core anyway)."""
    if "gpu" in request.keywords and "routing" not in request.keywords:
        import bjxa_amd
        if os.path.exists(bjxa_amd.LIB_PATH):
            with bjxa_amd.offload(0):
                yield
            return
    yield


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_bytes(name):
    with gzip.open(os.path.join(GOLDEN, name + ".gz"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def golden():
    return golden_bytes


@pytest.fixture(scope="session")
def built():
    """libbjxa.so.0 and the oracle, built in-tree if missing."""
    import bjxa_amd
    import oracle
    if not os.path.exists(bjxa_amd.LIB_PATH):
        bjxa_amd.build()
    oracle.lib()
    return bjxa_amd
