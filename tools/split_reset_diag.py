"""Diagnostic: the split build's reset against the oracle in fp32 and in split
mode (which one it equals, and how far each is)."""
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
for name, N in (("env0", 256), ("env0", 1024)):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, 4, reward="bbpow_action")
    sim = sim_mod.KuraSim(cfg, 0, lib_path=os.path.join(ROOT, "dbs-gym_amd", "csrc", os.environ.get("SPLIT_LIB", "libkura_split.so")))
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    og = sim.reset(torch.from_numpy(th0)).cpu().numpy()
    yg = sim.get_state()["y"]
    for split in (False, True):
        o = ko.Oracle(cfg, alpha)
        if split:
            o.set_split(True)
        o.set_env_params(omega, gs, gr)
        o.set_spectral(ct, st)
        oo = o.reset(th0)
        yo = o.state()["y"]
        print(name, N, "oracle split" if split else "oracle fp32", "obs equal", np.array_equal(og, oo),
              "max|dobs| %.3e" % np.abs(og - oo).max(), "y equal", np.array_equal(yg, yo),
              "max|dy| %.3e" % np.abs(yg.astype(np.float64) - yo).max(), flush=True)
    sim.close()
