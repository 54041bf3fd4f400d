import os
import sys

# The oracle uses OpenMP across envs; oversubscribing a small CPU share is
# slower than one thread, so default to 1 unless the caller chose.
os.environ.setdefault("OMP_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libkura.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")
