"""Diagnostic: one step of the split build from a state set on both sides
(fp32 oracle reset, then kura_set_state) against the oracle's split mode."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import actions, make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")
lib = os.path.join(ROOT, "dbs-gym_amd", "csrc", os.environ.get("SPLIT_LIB", "libkura_split.so"))
for N in (256, 1024):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", N, 2, reward="bbpow_action")
    base = ko.Oracle(cfg, alpha)
    base.set_env_params(omega, gs, gr)
    base.set_spectral(ct, st)
    base.reset(th0)
    s0 = base.state()
    sim = sim_mod.KuraSim(cfg, 0, lib_path=lib)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    sim.set_state(s0)
    a = actions("off", 2, cfg.n_elec, 0)
    sim.step(torch.from_numpy(a))
    torch.cuda.synchronize()
    g = sim.get_state()
    sim.close()
    for split in (False, True):
        o = ko.Oracle(cfg, alpha)
        if split:
            o.set_split(True)
        o.set_env_params(omega, gs, gr)
        o.set_spectral(ct, st)
        o.reset(th0)
        o.set_state(s0)
        o.step(a)
        s = o.state()
        d = g["y"].astype(np.float64) - s["y"]
        print(f"N={N} one step from a common state: gpu-split vs oracle {'split' if split else 'fp32'}: "
              f"equal {np.array_equal(g['y'], s['y'])}, differing {int((g['y'] != s['y']).sum())}, "
              f"max|dy| {np.abs(d).max():.3e}, t equal {np.array_equal(g['t'], s['t'])}", flush=True)
