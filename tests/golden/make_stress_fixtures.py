#!/usr/bin/env python3
"""Records of BASELINE.json configs[4] (N=8192) in the BF16X3 coupling at
full size, computed once by the CPU oracle in the build container and
committed (tests/stress_scenarios.py says what a record holds):

    OMP_NUM_THREADS=8 python tests/golden/make_stress_fixtures.py [weak|strong ...]

writes tests/golden/stress_<scenario>.npz; tests/test_gpu_stress.py replays
each on the GPU through the production library and compares bit for bit."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import stress_scenarios as ss  # noqa: E402


def main(names):
    t0 = time.time()

    def progress(name, k):
        print(f"{name}: step {k} ({time.time() - t0:.0f} s)", flush=True)

    for name in names or list(ss.SCENARIOS):
        rec = ss.run_oracle(name, progress=progress)
        rec["coupling"] = np.array("bf16x3")
        path = os.path.join(HERE, f"stress_{name}.npz")
        np.savez_compressed(path, **rec)
        print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
