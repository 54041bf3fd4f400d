"""Diagnostic: split build reset vs oracle split reset over transient lengths."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")
lib = os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_split.so")
cfg0, *_ = make_case("env0", 256, 1, reward="bbpow_action")
wlen = cfg0.window * cfg0.dt
print("window", cfg0.window, "dt", cfg0.dt, "transient", cfg0.transient_len, flush=True)
for f in (1.05, 1.5, 3.0, None):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, 1, reward="bbpow_action")
    if f is not None:
        cfg.transient_len = wlen * f
    sim = sim_mod.KuraSim(cfg, 0, lib_path=lib)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    g = sim.get_state()
    sim.close()
    o = ko.Oracle(cfg, alpha)
    o.set_split(True)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    s = o.state()
    print(f"transient {cfg.transient_len:.4f}: y equal {np.array_equal(g['y'], s['y'])}, differing "
          f"{int((g['y'] != s['y']).sum())}, max|dy| {np.abs(g['y'].astype(np.float64) - s['y']).max():.3e}, "
          f"ring equal {np.array_equal(g['ring'], s['ring'])}", flush=True)
