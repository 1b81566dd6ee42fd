import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def progress(msg: str) -> None:
    """A progress line for long GPU tests: appended to gpurun_out/progress.log
    (the GPU box's watchdog sees files there change) and echoed to stderr."""
    import time
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "progress.log"), "a") as f:
        f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")
    print(msg, file=sys.stderr, flush=True)


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """GPU tests that ask torch for device properties (test_gpu_shape,
    test_gpu_replay_shape) need torch's HIP runtime initialised before the
    engine library's own first HIP calls in the process: torch's lazy init
    reported "No HIP GPUs are available" when it came second.  Initialise it
    up front whenever a GPU test is selected."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
