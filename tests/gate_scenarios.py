"""The north_star 1000-step gates at N=1024 (BASELINE.json: phases within
1e-5 relative after 1000 steps) as replayable scenarios -- TEST
INFRASTRUCTURE shared by tests/golden/make_gate_fixtures.py (runs them through
the CPU oracle once, in this container, and commits the records) and
tests/test_gpu_gates.py (runs them through the HIP path on the GPU box and
compares against the committed records bit for bit).

The split-bf16 oracle costs ~15 ms per N=1024 RHS (38x the fp32 chain), so a
live 1000-step oracle run does not fit a GPU test; the committed records keep
the gates at full strength.  What a record holds per
scenario:
* at every checkpoint (steps 250/500/750/1000, and after every autoreset of
  the env2 scenario): the full state (y, t, step, wpos, spec) and the SHA-1 of
  the ring;
* per step: every env's reward (float64), and a running SHA-1 over all of a
  step's outputs (obs, reward, done, nsamp, lfp_true, lfp_rec), digested at
  each checkpoint -- so every output of every step is compared exactly;
* the final ring in full.
"""
from __future__ import annotations

import copy
import hashlib

import numpy as np

from helpers import actions, kura, ko, make_case

N, B, STEPS = 1024, 8, 1000
CHECK = (250, 500, 750, 1000)
ENV2_EPISODE = 300

# name -> (config, reward, action kind, envs); "env2" runs through KuraVectorEnv.
# The B=8 scenarios fill half of one 16-env workgroup; the *_b32 ones fill two
# whole workgroups (16 lockstep envs each, per-env accept/reject masks all
# active) -- VERDICT r05 weak #1.  Env b of a scenario draws the same inputs
# and actions at any batch size (make_case seeds per env, actions() draws
# (envs, n_elec) row-major), so the first 8 envs of a *_b32 record are the B=8
# record's envs (tests/test_gate_fixtures.py checks that).
SCENARIOS = {
    "env0_r1": ("env0", "bbpow_action", "rand", 8),
    "env1_r2": ("env1", "temp_const_action", "rand", 8),
    "env2_r1_vec": ("env2", "bbpow_action", "rand", 8),
    "env0_r1_b32": ("env0", "bbpow_action", "rand", 32),
    "env1_r2_b32": ("env1", "temp_const_action", "rand", 32),
}
STATE_KEYS = ("y", "t", "step", "wpos", "spec")


def sha1(*arrays) -> str:
    h = hashlib.sha1()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


class StepDigest:
    """Running SHA-1 over the outputs of every step, in step order."""

    def __init__(self):
        self.h = hashlib.sha1()

    def add(self, obs, reward, done, nsamp, lfp_true, lfp_rec):
        for a, dt in ((obs, np.float32), (reward, np.float64), (done, np.uint8), (nsamp, np.int32),
                      (lfp_true, np.float32), (lfp_rec, np.float64)):
            self.h.update(np.ascontiguousarray(np.asarray(a), dtype=dt).tobytes())

    def hexdigest(self) -> str:
        return self.h.copy().hexdigest()


def env01_case(name, reward, coupling="auto", envs=B):
    """The inputs of the env0/env1 scenarios (the same make_case as the live
    fp32 gates of tests/test_gpu_parity.py)."""
    return make_case(name, N, envs, reward=reward, coupling=coupling)


def env2_setup(coupling="auto"):
    """The env2 scenario: drift events and per-env K ~ U(0.3, 0.8) through
    KuraVectorEnv, 300-step episodes (3 autoresets per env in 1000 steps).
    Returns (plist, base) -- the env list and the shared driver arrays."""
    base = kura.fill_driver_arrays(kura.synthetic_params("env2", N), w0_seed=77)
    Ks = np.random.default_rng(19).uniform(0.3, 0.8, B)
    plist = []
    for b in range(B):
        p = copy.copy(base)
        p["K"] = float(Ks[b])
        p["rand_seed"] = 500 + b
        plist.append(p)
    return plist, base


def env2_actions(k, n_elec):
    return np.random.default_rng(5 + 1000003 * k).uniform(-1, 1, (B, n_elec)).astype(np.float32)


def _state_record(st, tag, rec):
    for k in STATE_KEYS:
        rec[f"{tag}_{k}"] = np.asarray(st[k]).copy()
    rec[f"{tag}_ring_sha1"] = np.frombuffer(bytes.fromhex(sha1(st["ring"])), np.uint8).copy()


def run_oracle_env01(scenario, coupling="auto", progress=None):
    """The env0/env1 scenario through the oracle: the committed record."""
    name, reward, act, envs = SCENARIOS[scenario]
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = env01_case(name, reward, coupling, envs)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    rec = {}
    obs0 = o.reset(th0)
    rec["reset_obs_sha1"] = np.frombuffer(bytes.fromhex(sha1(obs0)), np.uint8).copy()
    _state_record(o.state(), "reset", rec)
    dig = StepDigest()
    rewards = np.zeros((STEPS, envs), np.float64)
    for k in range(STEPS):
        a = actions(act, envs, cfg.n_elec, k)
        out = o.step(a)
        rewards[k] = out["reward"]
        dig.add(out["obs"], out["reward"], out["done"], out["nsamp"], out["lfp_true"], out["lfp_rec"])
        if k + 1 in CHECK:
            _state_record(o.state(), f"s{k + 1}", rec)
            rec[f"s{k + 1}_digest"] = np.frombuffer(bytes.fromhex(dig.hexdigest()), np.uint8).copy()
            if progress:
                progress(scenario, k + 1)
    rec["rewards"] = rewards
    rec["final_ring"] = o.state()["ring"]
    o.close()
    return rec


def run_oracle_env2(coupling="auto", progress=None):
    """The env2 scenario through the oracle with the reset draws of fresh
    EnvHosts (what KuraVectorEnv draws, in the reference's order)."""
    vec_cfg = _env2_config(coupling)
    plist, base = env2_setup(coupling)
    c = vec_cfg
    from importlib import import_module
    build_batch = import_module("dbs-gym_amd").build_batch
    _, shared = build_batch(plist)
    o = ko.Oracle(c, shared["alpha"].astype(np.float32))
    o.set_gain(np.array([np.float32(p["K"] / N) for p in plist], np.float32))
    bins = kura.spectral.beta_bins(c.window, base["verbose_dt"])
    o.set_spectral(*kura.spectral.twiddles(c.window, bins))
    hosts = [kura.EnvHost(copy.deepcopy(p)) for p in plist]

    def draw():
        w0, gs, gr, th = kura.reset_draws_batch(hosts)
        o.set_env_params(w0.astype(np.float32), gs, gr)
        return th.astype(np.float32)

    rec = {}
    obs0 = o.reset(draw())
    rec["reset_obs_sha1"] = np.frombuffer(bytes.fromhex(sha1(obs0)), np.uint8).copy()
    _state_record(o.state(), "reset", rec)
    dig = StepDigest()
    rewards = np.zeros((STEPS, B), np.float64)
    nres = 0
    for k in range(STEPS):
        a = env2_actions(k, c.n_elec)
        out = o.step(a)
        rewards[k] = out["reward"]
        dig.add(out["obs"], out["reward"], out["done"], out["nsamp"], out["lfp_true"], out["lfp_rec"])
        if (k + 1) % ENV2_EPISODE == 0:
            nres += 1
            obs_r = o.reset(draw())
            rec[f"r{nres}_obs_sha1"] = np.frombuffer(bytes.fromhex(sha1(obs_r)), np.uint8).copy()
            _state_record(o.state(), f"r{nres}", rec)
        if k + 1 in CHECK:
            _state_record(o.state(), f"s{k + 1}", rec)
            rec[f"s{k + 1}_digest"] = np.frombuffer(bytes.fromhex(dig.hexdigest()), np.uint8).copy()
            if progress:
                progress("env2_r1_vec", k + 1)
    rec["rewards"] = rewards
    rec["final_ring"] = o.state()["ring"]
    o.close()
    return rec


def _env2_config(coupling):
    sim = __import__("importlib").import_module("dbs-gym_amd.sim")
    plist, _ = env2_setup(coupling)
    return sim.make_config(plist[0], B, reward_func="bbpow_action", coupling=coupling)
