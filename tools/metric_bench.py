"""Time the episode metrics (kura_psd_bbpow, kura_envelope_stats: Bluestein
FFT pipeline, kura_fft.inc) on episode-length signals already on the device.

    python tools/metric_bench.py [n_signals] [length]

Default: 4096 signals of 105545 samples -- every env of the B=4096 bench
finishing a 5555-step training episode at once."""
import importlib
import json
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
abi = importlib.import_module("dbs-gym_amd.abi")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = int(sys.argv[2]) if len(sys.argv) > 2 else 105545
cfg = sim_mod.make_config(kura.reference_params("env0"), 4, reward_func="bbpow_action")
sim = sim_mod.KuraSim(cfg, 0)
dev = sim.device
g = torch.Generator(device=dev)
g.manual_seed(0)
sig = torch.randn((n, L), generator=g, device=dev, dtype=torch.float32)
lens = torch.full((n,), L, dtype=torch.int32, device=dev)
out_p = torch.empty(n, dtype=torch.float64, device=dev)
out_e = torch.empty((n, 3), dtype=torch.float64, device=dev)
st = sim._stream()


def psd():
    abi.check(sim.lib, sim.lib.kura_psd_bbpow(sim._h, abi.ptr(sig), abi.ptr(lens), L, n, 5e-4, 12.5, 21.0,
                                               abi.ptr(out_p), st), "psd")


def env():
    abi.check(sim.lib, sim.lib.kura_envelope_stats(sim._h, abi.ptr(sig), abi.ptr(lens), L, n, abi.ptr(out_e), st),
              "env")


res = {"signals": n, "len": L}
for name, fn in (("psd_bbpow", psd), ("envelope_stats", env)):
    fn()  # warm-up (scratch allocation)
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    res[name + "_s"] = dt
    res[name + "_ms_per_signal"] = 1e3 * dt / n
    assert torch.isfinite(out_p).all() and torch.isfinite(out_e).all()
print(json.dumps(res))
sim.close()
