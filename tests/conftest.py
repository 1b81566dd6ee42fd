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

# No test asks torch.cuda anything: device facts come from the engine library
# (tbg_device_count / tbg_device_cu_count).  PyTorch's wheel bundles its own
# libamdhip64.so, which its libraries NEED by the unversioned name: loaded
# after the engine library (ROCm's libamdhip64.so.7) it maps as a SECOND HIP
# runtime, and whichever of the two initialises second finds no devices --
# the round-5 "No HIP GPUs are available" (DESIGN.md section 5).
