"""Time kura_envelope_stats on episode-length signals (eval-time metric, K5).

    python tools/envelope_bench.py [n_signals] [length]
"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import kura  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
L = int(sys.argv[2]) if len(sys.argv) > 2 else 105545
cfg = sim_mod.make_config(kura.reference_params("env0"), 4, reward_func="bbpow_action")
sim = sim_mod.KuraSim(cfg, 0)
rng = np.random.default_rng(0)
sig = [rng.standard_normal(L).astype(np.float32) for _ in range(n)]
sim.envelope_stats(sig[:1])
torch.cuda.synchronize()
t = time.perf_counter()
sim.envelope_stats(sig)
torch.cuda.synchronize()
dt = time.perf_counter() - t
# 2 passes x (L/2+1)*L complex-by-real/complex MACs: ~ 3 L^2 f64 FMA = 6 L^2 flop
fl = 6.0 * L * L * n
print(f'{{"signals": {n}, "len": {L}, "s": {dt:.4f}, "ms_per_signal": {1e3 * dt / n:.3f}, '
      f'"f64_tflops": {fl / dt / 1e12:.2f}}}')
sim.close()
