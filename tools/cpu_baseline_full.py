#!/usr/bin/env python3
"""The CPU baseline in SURVEY.md section 8(d)'s full protocol (VERDICT r05
weak #8): env0 default params (N=512), a single env, 1000 steps after
reset(), on the host's cores -- (i) one core, (ii) all cores with one env
per process -- through oracle/ref_numpy.py, the reference's step() op
sequence (fmod + direct N^2 sin coupling, env.py:252-256; Dopri5/PID/dense
output; R1).  The bench's default cpu_baseline is a bounded sample of the
same code (tens of seconds); this is the long form, run on the GPU box's
host without touching the GPU:

    python tools/cpu_baseline_full.py [--osc 512] [--steps 1000] [--procs P] > profiles/<name>.json

Test infrastructure (it imports oracle/), never the measured product."""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402

_ENV = None


def _child(steps):
    from oracle.ref_numpy import time_steps
    v, k, el = time_steps(_ENV, 1e9, np.random.default_rng(os.getpid()), max_steps=steps)
    return v, k, el


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--osc", type=int, default=512)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--procs", type=int, default=0, help="processes for leg (ii) (0 = the host's cores)")
    a = ap.parse_args(argv)
    global _ENV
    args = bench.parse(["--osc", str(a.osc), "--envs", "1", "--cpu-seconds", "0"])
    _ENV = bench._ref_env(args, a.osc)
    nproc = a.procs or bench._host_cores()
    from oracle.ref_numpy import time_steps
    v1, k1, el1 = time_steps(_ENV, 1e9, np.random.default_rng(0), max_steps=a.steps)
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(nproc) as pool:
        res = pool.map(_child, [a.steps] * nproc)
    el = time.perf_counter() - t0
    out = {
        "protocol": "SURVEY.md 8(d): env0 default params, one env, steps after reset(), (i) 1 core, (ii) all cores "
                    "one env per process (multiprocessing fork)",
        "code": "oracle/ref_numpy.py (reference op sequence: fmod + direct N^2 sin coupling, env.py:252-256; "
                "Dopri5/PID/dense output; R1), started from the reset() state (transient by the C oracle)",
        "n_osc": a.osc, "steps_per_env": a.steps,
        "single_core": {"value": v1, "unit": "env-steps/s", "steps": k1, "seconds": el1},
        "all_cores": {"value": float(sum(k for _, k, _ in res)) / el, "unit": "env-steps/s", "processes": nproc,
                      "steps": int(sum(k for _, k, _ in res)), "wall_seconds": el,
                      "per_process_min": float(min(v for v, _, _ in res)),
                      "per_process_max": float(max(v for v, _, _ in res))},
        "host": {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))},
        "published_reference": "16.96-19.77 steps/s JAX-CPU at N=512 (BASELINE.md section 1)",
    }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
