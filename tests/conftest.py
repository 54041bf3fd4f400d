import os
import sys

# The oracle uses OpenMP across envs (the bf16x3 oracle costs ~15 ms per
# N=1024 RHS, so its threads matter); default to this machine's CPU share, at
# most 8, unless the caller chose (the GPU box sets OMP_NUM_THREADS=16).
_ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
os.environ.setdefault("OMP_NUM_THREADS", str(max(1, min(8, _ncpu))))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libkura.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")
