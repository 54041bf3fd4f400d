#!/usr/bin/env python3
"""Which envs of a batch part from the oracle after reset (+ steps), per
coupling arithmetic: prints, per (N, B, coupling), the envs whose state y
differs and the first differing sample of each obs row.
    python tools/coupling_env_probe.py"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import actions, make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402
import torch  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")


def probe(N, B, coupling, steps=0, name="env0"):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, coupling=coupling)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    o.reset(th0)
    for k in range(steps):
        a = actions("rand", B, 1, k)
        sim.step(torch.from_numpy(a))
        o.step(a)
    g = sim.get_state()
    bad = [b for b in range(B) if not np.array_equal(g["y"][b], o.y[b])]
    st_g = sim.stats()
    print(f"N={N} B={B} {coupling} steps={steps}: {len(bad)} envs differ {bad}; gpu stats {st_g[:5].tolist()} "
          f"oracle stats {o.stats.tolist()}", flush=True)
    sim.close()
    return bad


if __name__ == "__main__":
    cases = ((256, 4, "bf16x3", 0), (256, 16, "bf16x3", 0), (256, 16, "f32", 0), (512, 16, "bf16x3", 0),
             (1024, 16, "bf16x3", 0), (256, 16, "bf16x3", 2))
    if len(sys.argv) > 1 and sys.argv[1] == "quick":
        cases = ((512, 16, "bf16x3", 0), (1024, 16, "bf16x3", 0))
    print("library:", os.environ.get("KURA_LIB", "libkura.so"))
    for N, B, c, s in cases:
        probe(N, B, c, s)
