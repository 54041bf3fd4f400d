#!/usr/bin/env python3
"""Diagnostic: run GPU vs oracle for a few steps and report the first
difference (step, output, env, index).
Usage: [PART=256] parity_probe.py ENV N B STEPS ACT [LIB|-]"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import actions, ko, make_case  # noqa: E402


def main():
    name, N, B, steps, act = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    import torch
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B)
    cfg.part_osc = int(os.environ.get("PART", "0"))
    lib = sys.argv[6] if len(sys.argv) > 6 and sys.argv[6] != "-" else None
    sim = sim_mod.KuraSim(cfg, 0, lib_path=lib)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    o.reset(th0)
    g, r = sim.get_state(), o.state()
    print("reset y equal:", np.array_equal(g["y"], r["y"]))
    if not np.array_equal(g["y"], r["y"]):
        b = np.argwhere(g["y"] != r["y"])
        d = np.abs(g["y"].astype(np.float64) - r["y"])
        print("  reset diff envs", sorted(set(int(x[0]) for x in b)), "count", len(b), "max", d.max(),
              "ex", g["y"][tuple(b[0])], r["y"][tuple(b[0])], "t equal", np.array_equal(g["t"], r["t"]))
    for k in range(steps):
        a = actions(act, B, cfg.n_elec, k)
        sim.step(torch.from_numpy(a))
        ref = o.step(a)
        torch.cuda.synchronize()
        g, r = sim.get_state(), o.state()
        out = {"y": (g["y"], r["y"]), "obs": (sim.obs.cpu().numpy(), ref["obs"]),
               "lfp": (sim.lfp_true.cpu().numpy(), ref["lfp_true"]), "t": (g["t"], r["t"])}
        bad = {kk: np.argwhere(v[0] != v[1]) for kk, v in out.items()}
        if any(len(b) for b in bad.values()):
            for kk, b in bad.items():
                if len(b):
                    envs = sorted(set(int(x[0]) for x in b))
                    d = np.abs(out[kk][0].astype(np.float64) - out[kk][1])
                    print(f"step {k}: {kk} differs at {len(b)} places, envs {envs[:10]}, first {b[:3].tolist()}, "
                          f"max|d| {d.max():.3e}, gpu {out[kk][0][tuple(b[0])]!r} oracle {out[kk][1][tuple(b[0])]!r}")
            return
    print("all equal")


if __name__ == "__main__":
    main()
