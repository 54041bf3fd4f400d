"""Diagnostic: determinism and env independence of the split build's reset."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")
for libname in ("libkura_split.so", "libkura.so"):
    lib = os.path.join(ROOT, "dbs-gym_amd", "csrc", libname)
    ys = []
    for B in (4, 4, 1):
        cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, B, reward="bbpow_action")
        sim = sim_mod.KuraSim(cfg, 0, lib_path=lib)
        sim.set_coupling(alpha)
        sim.set_env_params(omega, gs, gr)
        sim.set_spectral(ct, st)
        sim.reset(torch.from_numpy(th0))
        ys.append(sim.get_state()["y"].copy())
        sim.close()
    print(libname, "run-to-run equal", np.array_equal(ys[0], ys[1]), "max|d| %.3e" % np.abs(ys[0] - ys[1]).max(),
          "| env0 B=4 vs B=1 equal", np.array_equal(ys[0][0], ys[2][0]), flush=True)
