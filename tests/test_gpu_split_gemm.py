"""The split-bf16 coupling build (libkura_split.so, -DKURA_SPLIT_GEMM;
DESIGN.md section 9) is a twin of the oracle in its split mode
(Oracle.set_split: oracle_split_gemm_rows, the bf16 MFMA's exact
accumulation over three-way bf16 splits): its GEMM, its reset transients and
its steps bit-exact, as the shipped fp32 build is against the fmaf-chain
oracle (tests/test_gpu_parity.py).
Not the product path yet -- the experiment's parity gate (round 5 switches
the product once the long-horizon gates are re-planned around the split
oracle's cost)."""
import ctypes
import importlib
import os

import numpy as np
import pytest

from helpers import actions, make_case
from oracle import kura_oracle as ko

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPLIT_LIB = os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_split.so")


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(SPLIT_LIB):
        raise RuntimeError("libkura_split.so missing: run __graft_entry__.build()")
    return torch


def _cmp_state(g, o, where):
    for k in ("y", "t", "step", "ring", "wpos", "spec"):
        if not np.array_equal(g[k], o[k]):
            bad = np.argwhere(g[k] != o[k])
            raise AssertionError(f"{where}: state[{k}] differs at {len(bad)} places, first {bad[:3].tolist()}: "
                                 f"gpu={g[k][tuple(bad[0])]!r} oracle={o[k][tuple(bad[0])]!r}")


def _run_from_common_state(torch, name, N, B, reward, steps, act, **overrides):
    """Both sides start from the fp32 oracle's reset state (kura_set_state),
    then step with the split coupling: every step bit-exact."""
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, reward=reward, **overrides)
    base = ko.Oracle(cfg, alpha)
    base.set_env_params(omega, gs, gr)
    base.set_spectral(ct, st)
    base.reset(th0)
    s0 = base.state()
    sim = sim_mod.KuraSim(cfg, 0, lib_path=SPLIT_LIB)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    sim.set_state(s0)
    o = ko.Oracle(cfg, alpha)
    o.set_split(True)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    o.set_state(s0)
    for k in range(steps):
        a = actions(act, B, cfg.n_elec, k)
        sim.step(torch.from_numpy(a))
        ref = o.step(a)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(sim.obs.cpu().numpy(), ref["obs"])
        np.testing.assert_array_equal(sim.reward.cpu().numpy(), ref["reward"])
        np.testing.assert_array_equal(sim.done.cpu().numpy(), ref["done"])
        _cmp_state(sim.get_state(), o.state(), f"step {k}")
    sim.close()


def test_split_selftest_gemm_is_the_oracle_chain(torch_gpu):
    """kura_selftest_gemm of the split build == oracle_split_gemm_rows bit for
    bit (N = 1024, random operands), and within the fp32 chain's accuracy."""
    abi = importlib.import_module("dbs-gym_amd.abi")
    L = abi.load_library(SPLIT_LIB)
    L.kura_selftest_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    for N in (256, 512, 1024):
        rng = np.random.default_rng(N)
        X = rng.uniform(-1, 1, (32, N)).astype(np.float32)
        A = rng.uniform(-1, 1, (N, N)).astype(np.float32)
        Y = np.zeros((32, N), np.float32)
        assert L.kura_selftest_gemm(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N) == 0
        want = ko.split_gemm_rows(X, A)
        assert np.array_equal(Y.view(np.uint32), want.view(np.uint32)), N
        exact = X.astype(np.float64) @ A.astype(np.float64).T
        assert np.abs(Y - exact).max() <= 2.0 * np.abs(ko.gemm_chain(X, A) - exact).max() + 1e-6


@pytest.mark.parametrize("name,N,reward,act", [
    ("env0", 1024, "bbpow_action", "rand"),
    ("env1", 512, "bbpow_threth_action", "hf"),
    ("env0", 256, "bbpow_action", "off"),
])
def test_split_step_parity(torch_gpu, name, N, reward, act):
    _run_from_common_state(torch_gpu, name, N, 4, reward, 3, act)


def _run_pair(torch, name, N, B, reward, steps, act, **overrides):
    """reset (the transient: ~10^7 modelled MFMA outputs) and steps, both
    sides in split arithmetic from theta0: bit-exact throughout."""
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, reward=reward, **overrides)
    sim = sim_mod.KuraSim(cfg, 0, lib_path=SPLIT_LIB)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_split(True)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    np.testing.assert_array_equal(sim.reset(torch.from_numpy(th0)).cpu().numpy(), o.reset(th0))
    _cmp_state(sim.get_state(), o.state(), "reset")
    for k in range(steps):
        a = actions(act, B, cfg.n_elec, k)
        sim.step(torch.from_numpy(a))
        ref = o.step(a)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(sim.obs.cpu().numpy(), ref["obs"])
        np.testing.assert_array_equal(sim.reward.cpu().numpy(), ref["reward"])
        _cmp_state(sim.get_state(), o.state(), f"step {k}")
    sim.close()


@pytest.mark.parametrize("name,N,reward,act", [
    ("env0", 1024, "bbpow_action", "rand"),
    ("env1", 512, "bbpow_threth_action", "hf"),
    ("env0", 256, "bbpow_action", "off"),
])
def test_split_reset_and_step_parity(torch_gpu, name, N, reward, act):
    _run_pair(torch_gpu, name, N, 4, reward, 4, act)


def test_split_refuses_split_groups(torch_gpu):
    """n_osc > 1024 (the fp32 split-group path) is refused, not run wrong."""
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, *_ = make_case("env0", 2048, 2, reward="bbpow_action")
    with pytest.raises(Exception, match="1024"):
        sim_mod.KuraSim(cfg, 0, lib_path=SPLIT_LIB)
