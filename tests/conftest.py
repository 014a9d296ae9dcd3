import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU")
    config.addinivalue_line("markers", "slow: longer CPU test")
    config.addinivalue_line("markers", "perf: asserts wall-clock ratios (run alone on a quiet GPU; "
                                       "-m 'gpu and not perf' leaves them out)")


def pytest_collection_modifyitems(config, items):
    # wall-clock (perf) tests run after every parity test, so that under -x a
    # timing wobble on a shared host cannot hide the parity suite (stable
    # sort: both groups keep their collection order)
    items.sort(key=lambda item: "perf" in item.keywords)
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session", autouse=True)
def _native_library_is_this_tree(request):
    """Before any GPU test: the loaded liblfg_hip.so carries the source hash
    of this tree (a stale or foreign library fails the session loudly)."""
    if not any("gpu" in item.keywords for item in request.session.items):
        return
    try:
        import torch
        if not torch.cuda.is_available():
            return
    except Exception:
        return
    from lfit_python_amd import _native
    if os.environ.get("LFG_LIB") and os.environ.get("LFG_DIAGNOSTIC") == "1":
        return  # an explicitly loaded experiment build (tools/build_exp.sh)
    _native.verify()
