#!/usr/bin/env python3
"""The paper's evaluation protocol (aDBS_RL/evaluate_HF_DBS.py: 5 eval envs,
5 episodes of 1111 steps each, constant action 0 and 1, calc_psd_for_simple_eval
of the concatenated theta_mean) through the CPU oracle, per config:

    OMP_NUM_THREADS=8 python tests/golden/make_anchor_oracle.py [f32|bf16x3 ...]

writes tests/golden/anchor_oracle.json: per-env beta-band power for env0,
env1, env2 (encapsulation as shipped, env.py:509) and env2 with
encapsulation_mode="relative", plus the 1-episode env0 values the CPU test
re-runs, per coupling arithmetic (KuraConfig.coupling; runs of the couplings
not named are kept).  The GPU test reproduces these per-env values from the
HIP path (a bit-exact twin of the oracle) and both are held against the
paper's rows (tests/golden/paper_anchors.json).  The bf16x3 runs take ~20x
the f32 ones (the split oracle's cost): ~1.5 h on 8 cores."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from anchor_protocol import oracle_protocol  # noqa: E402

RUNS = [("env0", 5, {}), ("env1", 5, {}), ("env2", 5, {}), ("env2", 5, {"encapsulation_mode": "relative"}),
        ("env0", 1, {})]


def main(couplings):
    path = os.path.join(HERE, "anchor_oracle.json")
    out = {"protocol": "evaluate_HF_DBS.py: seed 228, 5 eval envs, n_eval_episodes episodes of 1111 steps, "
                       "actions 0 and 1, calc_psd_for_simple_eval(psd_dt=5e-4, 12.5-21 Hz) per env",
           "runs": []}
    if os.path.exists(path):
        old = json.load(open(path))
        out["runs"] = [r for r in old["runs"] if r.get("coupling", "f32") not in couplings]
    for coupling in couplings:
        for name, n_ep, ov in RUNS:
            if coupling != "f32" and n_ep == 1:
                continue   # the 1-episode run is the CPU test's (f32) re-run
            t0 = time.time()
            bb, sig = oracle_protocol(name, n_ep, coupling=coupling, **ov)
            out["runs"].append({"config": name, "episodes": n_ep, "overrides": ov, "coupling": coupling,
                                "bbpow_off": bb[0].tolist(), "bbpow_hf": bb[1].tolist(),
                                "signal_len": [len(s) for s in sig]})
            print(coupling, name, n_ep, ov, "off", bb[0].mean() * 1e3, "hf", bb[1].mean() * 1e3,
                  f"{time.time() - t0:.1f}s", flush=True)
            with open(path, "w") as f:   # after every run: a long job keeps what it has
                json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["f32", "bf16x3"])
