"""BASELINE.json configs[4] (N=8192) in the BF16X3 coupling at full size,
shared by the record generator (tests/golden/make_stress_fixtures.py, the
CPU oracle in the build container) and the GPU replay
(tests/test_gpu_stress.py): each scenario is bench.py's shard of that
config, reset + STEPS steps, and a sample of envs spread over env groups,
the 16-env interleave and (weak form) both pairs a workgroup walks.  The
oracle runs the sampled envs only (envs are independent,
tests/test_oracle_props.py).  A record holds per-env SHA-1 digests of the
large state (y, ring, spec, obs) and the small arrays whole."""
import copy
import hashlib
import importlib
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 3
SCENARIOS = {
    "weak": (1024, [0, 5, 15, 16, 255, 256, 511, 512, 700, 1008, 1015, 1023]),   # 512 pairs on 256 WGs, parts of 1024
    "strong": (128, [0, 3, 15, 16, 47, 64, 100, 127]),                            # parts of 256
}
BIG = ("y", "ring", "spec")
SMALL = ("t", "step", "wpos")
OUT_BIG = ("obs",)
OUT_SMALL = ("reward", "done", "nsamp", "lfp_true", "lfp_rec")


def args_of(name):
    envs, _ = SCENARIOS[name]
    return types.SimpleNamespace(config="env0", osc=8192, envs=envs, seed=2024, random_k=False,
                                 reward="bbpow_action", part_osc=-1, coupling="bf16x3")


def shard(name):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    return bench.build_shard(args_of(name), 0)


def actions(name, k, n_elec):
    envs, _ = SCENARIOS[name]
    return np.random.default_rng(11 + k).uniform(-1, 1, (envs, n_elec)).astype(np.float32)


def digests(a):
    """Per-row SHA-1 of an array whose first axis is the env."""
    a = np.ascontiguousarray(a)
    return np.array([np.frombuffer(hashlib.sha1(a[i].tobytes()).digest(), np.uint8) for i in range(a.shape[0])])


def snapshot(state, outs=None, idx=None):
    """Record entries of a state dict (and step outputs) restricted to idx."""
    sel = (lambda a: np.asarray(a)) if idx is None else (lambda a: np.asarray(a)[idx])
    rec = {}
    for k in BIG:
        rec[k] = digests(sel(state[k]))
    for k in SMALL:
        rec[k] = sel(state[k]).copy()
    for k in OUT_BIG + OUT_SMALL:
        if outs is not None and k in outs:
            rec[k] = digests(sel(outs[k])) if k in OUT_BIG else sel(outs[k]).copy()
    return rec


def run_oracle(name, progress=None):
    from oracle import kura_oracle as ko
    cfg, alpha, omega, g_s, g_r, th0, ct, st, gain = shard(name)
    _, idx = SCENARIOS[name]
    idx = np.array(idx)
    c = copy.copy(cfg)
    c.n_envs = len(idx)
    o = ko.Oracle(c, alpha)
    o.set_env_params(omega[idx], g_s[idx], g_r[idx])
    o.set_gain(gain[idx])
    o.set_spectral(ct, st)
    obs = o.reset(th0[idx])
    out = {"idx": idx, "part_osc": np.array(cfg.part_osc)}
    for key, v in snapshot(o.state(), {"obs": obs}).items():
        out[f"reset_{key}"] = v
    if progress:
        progress(name, 0)
    for k in range(STEPS):
        ref = o.step(actions(name, k, cfg.n_elec)[idx])
        for key, v in snapshot(o.state(), ref).items():
            out[f"s{k + 1}_{key}"] = v
        if progress:
            progress(name, k + 1)
    o.close()
    return out
