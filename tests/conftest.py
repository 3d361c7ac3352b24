import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

os.environ.setdefault("MXAR_LOGLEVEL", "ERROR")

# Several plane workers share this process (and the GPU) in the round-engine tests; their
# rounds run in one group kernel (csrc/hip/xgmi_plane.cc PlaneGroup), so the suite runs at the
# box's GPU_MAX_HW_QUEUES (4) - it does not raise it.


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run via gpurun")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")
    # a native crash prints its C++ frames before Python's faulthandler dump (no debugger on
    # the GPU boxes)
    try:
        import faulthandler

        faulthandler.enable()
        from akka_allreduce_1_amd._native import C as _C

        _C.install_native_backtrace()
    except Exception:  # noqa: BLE001 - a diagnostic only
        pass


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def C():
    from akka_allreduce_1_amd._native import C as _C

    return _C


@pytest.fixture(params=["host", pytest.param("device", marks=pytest.mark.gpu)])
def tk(request):
    """Deterministic TestKit; the `device` variant runs the same worker protocol with its
    DataBuffers and payloads in MI355X HBM (DevicePlane)."""
    from akka_allreduce_1_amd.testkit import TestKit

    plane = None
    if request.param == "device":
        from akka_allreduce_1_amd._native import C

        plane = C.hip.device_plane(0)
    kit = TestKit("MySpec", deterministic=True, plane=plane)
    yield kit
    kit.shutdown()
