"""Shared test fixtures: build a small batch exactly as the env does."""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

kura = importlib.import_module("dbs-gym_amd")
from oracle import kura_oracle as ko  # noqa: E402


def make_case(name="env0", n_osc=512, n_envs=4, reward="bbpow_action", seed=0, split="train", coupling="auto",
              **overrides):
    """Returns (cfg, alpha_f32, omega, g_stim, g_rec, theta0, ctab, stab, hosts).
    coupling: KuraConfig.coupling ("auto" = the product default)."""
    from importlib import import_module
    sim = import_module("dbs-gym_amd.sim")
    if n_osc == 512:
        base = kura.reference_params(name, split, **overrides)
    else:
        base = kura.synthetic_params(name, n_osc, **overrides)
    plist = []
    for b in range(n_envs):
        p = dict(base)
        p["rand_seed"] = base["rand_seed"] + b
        plist.append(kura.fill_driver_arrays(p, w0_seed=seed * 1000 + b))
    hosts, shared = kura.build_batch(plist)
    omega, g_stim, g_rec, theta0 = kura.reset_arrays(hosts)
    cfg = sim.make_config(base, n_envs, reward_func=reward, coupling=coupling)
    bins = kura.spectral.beta_bins(cfg.window, base["verbose_dt"])
    ctab, stab = kura.spectral.twiddles(cfg.window, bins)
    return cfg, shared["alpha"].astype(np.float32), omega, g_stim, g_rec, theta0, ctab, stab, hosts


def actions(kind, n_envs, n_elec, step, seed=0):
    if kind == "off":
        return np.zeros((n_envs, n_elec), np.float32)
    if kind == "hf":
        return np.ones((n_envs, n_elec), np.float32)
    rng = np.random.default_rng(seed * 100003 + step)
    return rng.uniform(-1, 1, (n_envs, n_elec)).astype(np.float32)
