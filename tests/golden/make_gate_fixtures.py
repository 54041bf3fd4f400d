#!/usr/bin/env python3
"""Records of the N=1024 1000-step gates in the product arithmetic
(KURA_COUPLING_BF16X3), computed once by the CPU oracle in the build
container and committed (tests/gate_scenarios.py says what a record holds):

    OMP_NUM_THREADS=8 python tests/golden/make_gate_fixtures.py [scenario ...]

writes tests/golden/gate_<scenario>.npz for env0_r1, env1_r2 and env2_r1_vec
(~10 CPU-minutes each on 8 cores: 8 envs x 1000 steps x ~32 RHS at ~15 ms per
split-bf16 RHS).  tests/test_gpu_gates.py replays each scenario on the GPU
and compares bit for bit; tests/test_gate_fixtures.py re-runs a prefix of
each through the oracle on the CPU to check the records are the oracle's."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import gate_scenarios as gs  # noqa: E402


def main(names):
    t0 = time.time()

    def progress(name, k):
        print(f"{name}: step {k} ({time.time() - t0:.0f} s)", flush=True)

    for name in names or list(gs.SCENARIOS):
        rec = gs.run_oracle_env2(progress=progress) if name == "env2_r1_vec" else gs.run_oracle_env01(
            name, progress=progress)
        rec["coupling"] = np.array("bf16x3")
        path = os.path.join(HERE, f"gate_{name}.npz")
        np.savez_compressed(path, **rec)
        print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
