import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU-side oracle runs")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU gate: a gpu-marked test fails loudly if the HIP library or
    the device is missing (no silent fallback), or if the library was not
    built from the sources in this tree."""
    import torch  # noqa: F401  (device plumbing only; import checks ROCm runtime)
    from finitedifference_amd import _lib
    _lib.load()
    bid, sid = _lib.build_id(), _lib.source_id()
    assert bid == sid, (f"libburgers_hip.so build id {bid} != source id {sid} of this checkout: "
                        "rebuild (make -C finitedifference_amd/csrc)")
    # a knob build (race screen, A/B) only when asked for explicitly (BURG_LIB)
    assert _lib.is_default_build() or os.environ.get("BURG_LIB"), (
        f"the loaded library is a knob build ({_lib.build_flags()}), not the default one")
    return _lib


def pytest_terminal_summary(terminalreporter):
    """The library's build id next to the checkout's source id, at the end of
    every run (so a run's tail ties its results to the binary it loaded)."""
    try:
        from finitedifference_amd import _lib
        bid, sid = _lib.build_id(), _lib.source_id()
    except Exception as e:  # noqa: BLE001  (no library: say so, do not fail the summary)
        terminalreporter.write_line(f"libburgers_hip build id: unavailable ({e})")
        return
    terminalreporter.write_line(f"libburgers_hip build id {bid}, sources {sid}: "
                                f"{'match' if bid == sid else 'MISMATCH'}; flags: "
                                f"{_lib.build_flags()}")


@pytest.fixture(autouse=True)
def _gpu_device_sync_after(request):
    """After every gpu-marked test: synchronise the device, so an asynchronous
    GPU fault fails the test that caused it, not the next one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
