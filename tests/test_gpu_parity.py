"""GPU parity: the HIP path vs the CPU oracle, bit for bit.

BASELINE.json's gate is 1e-5 relative on phases after 1000 steps; the HIP
kernels are built as a bit-exact twin of oracle/kura_oracle.c (DESIGN.md
"Numerics"), so every comparison here is exact equality, which implies the
1e-5 tolerance (asserted explicitly in test_phase_gate_1000_steps).
Both coupling arithmetics (kura.h KURA_COUPLING_*) are twins: the product
default (AUTO = BF16X3 at every N) and F32; the oracle follows the
config.  The 1000-step gates here run the F32 coupling against the live
oracle; the product arithmetic's gates replay committed oracle records
(tests/test_gpu_gates.py).
"""
from __future__ import annotations

import ctypes
import importlib

import numpy as np
import pytest

from helpers import actions, make_case, ko

pytestmark = pytest.mark.gpu
PHASE_RTOL = 1e-5  # BASELINE.json north_star


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def lib(torch_gpu):
    abi = importlib.import_module("dbs-gym_amd.abi")
    L = abi.load_library()
    L.kura_selftest_math.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    L.kura_selftest_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    L.kura_selftest_coupling.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 2
    return L


def test_detmath_bitwise(lib):
    rng = np.random.default_rng(1)
    n = 1 << 16
    x = np.concatenate([rng.uniform(0, 2 * np.pi, n // 4), rng.uniform(-50, 3000, n // 4),
                        rng.uniform(-1e4, 1e4, n // 4), rng.normal(0, 1, n // 4)]).astype(np.float32)
    y = np.concatenate([rng.uniform(1e-6, 10, n // 2), rng.uniform(-5, 5, n // 2)]).astype(np.float32)
    y[y == 0] = 1.0
    out = np.zeros((n, 10), np.float32)
    assert lib.kura_selftest_math(x.ctypes.data, y.ctypes.data, out.ctypes.data, n) == 0
    s, c = ko.sincos(x)
    np.testing.assert_array_equal(out[:, 0], s)
    np.testing.assert_array_equal(out[:, 1], c)
    np.testing.assert_array_equal(out[:, 2], ko.fmod2pi(x))
    np.testing.assert_array_equal(out[:, 3], ko.inv_fifth_root(np.abs(y)))
    np.testing.assert_array_equal(out[:, 4], np.sqrt(np.abs(x)))
    np.testing.assert_array_equal(out[:, 5], x / y)
    np.testing.assert_array_equal(out[:, 6], (x.astype(np.float64) / y.astype(np.float64)).astype(np.float32))
    np.testing.assert_array_equal(out[:, 7], np.ceil(x.astype(np.float64) / 0.05).astype(np.float32))
    sf, cf = ko.sincos_fmod2pi(x)
    np.testing.assert_array_equal(out[:, 8], sf)
    np.testing.assert_array_equal(out[:, 9], cf)


@pytest.mark.parametrize("N", [256, 512, 1024])
def test_mfma_gemm_is_fmaf_chain(lib, N):
    rng = np.random.default_rng(N)
    X = rng.uniform(-1, 1, (32, N)).astype(np.float32)
    A = rng.uniform(0.3, 1, (N, N)).astype(np.float32)
    Y = np.zeros((32, N), np.float32)
    assert lib.kura_selftest_gemm(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N) == 0
    np.testing.assert_array_equal(Y, ko.gemm_chain(X, A))


@pytest.mark.parametrize("N", [256, 512, 1024])
def test_bf16x3_gemm_is_the_oracle_chain(lib, N):
    """The product coupling GEMM (KURA_COUPLING_BF16X3, six bf16 MFMA part
    products per 16-deep k-block) == oracle_split_gemm_rows bit for bit on
    signed random operands, and as accurate as the fp32 chain (within 2x of
    its worst error against the exact sum)."""
    rng = np.random.default_rng(N + 1)
    X = rng.uniform(-1, 1, (32, N)).astype(np.float32)
    A = rng.uniform(-1, 1, (N, N)).astype(np.float32)
    Y = np.zeros((32, N), np.float32)
    assert lib.kura_selftest_coupling(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N, 2) == 0
    assert np.array_equal(Y.view(np.uint32), ko.split_gemm_rows(X, A).view(np.uint32))
    exact = X.astype(np.float64) @ A.astype(np.float64).T
    assert np.abs(Y - exact).max() <= 2.0 * np.abs(ko.gemm_chain(X, A) - exact).max() + 1e-6
    Yf = np.zeros((32, N), np.float32)   # KURA_COUPLING_F32 through the same entry point
    assert lib.kura_selftest_coupling(X.ctypes.data, A.ctypes.data, Yf.ctypes.data, N, 1) == 0
    np.testing.assert_array_equal(Yf, ko.gemm_chain(X, A))


def _run_pair(torch, name, N, B, reward, steps, act, check_every=1, gains=None, coupling="auto", **overrides):
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, reward=reward, coupling=coupling,
                                                          **overrides)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    if gains is not None:
        sim.set_env_gain(gains)
        o.set_gain(gains)
    obs_g = sim.reset(torch.from_numpy(th0)).cpu().numpy()
    obs_o = o.reset(th0)
    np.testing.assert_array_equal(obs_g, obs_o)
    _cmp_state(sim.get_state(), o.state(), "reset")
    for k in range(steps):
        a = actions(act, B, cfg.n_elec, k)
        sim.step(torch.from_numpy(a))
        ref = o.step(a)
        if (k + 1) % check_every == 0 or k == steps - 1:
            torch.cuda.synchronize()
            np.testing.assert_array_equal(sim.obs.cpu().numpy(), ref["obs"])
            np.testing.assert_array_equal(sim.reward.cpu().numpy(), ref["reward"])
            np.testing.assert_array_equal(sim.done.cpu().numpy(), ref["done"])
            np.testing.assert_array_equal(sim.nsamp.cpu().numpy(), ref["nsamp"])
            np.testing.assert_array_equal(sim.lfp_true.cpu().numpy(), ref["lfp_true"])
            np.testing.assert_array_equal(sim.lfp_rec.cpu().numpy(), ref["lfp_rec"])
            _cmp_state(sim.get_state(), o.state(), f"step {k}")
    st = sim.get_state()
    sim.close()
    return st, o.state()


def _cmp_state(g, o, where):
    for k in ("y", "t", "step", "ring", "wpos", "spec"):
        if not np.array_equal(g[k], o[k]):
            bad = np.argwhere(g[k] != o[k])
            raise AssertionError(f"{where}: state[{k}] differs at {len(bad)} places, first {bad[:3].tolist()}: "
                                 f"gpu={g[k][tuple(bad[0])]!r} oracle={o[k][tuple(bad[0])]!r}")


@pytest.mark.parametrize("name,N,reward,act,coupling", [
    ("env0", 512, "bbpow_action", "rand", "auto"),
    ("env1", 512, "bbpow_threth_action", "hf", "auto"),
    ("env1", 512, "temp_const_action", "rand", "auto"),
    ("env0", 256, "bbpow_action", "off", "auto"),
    ("env0", 1024, "bbpow_action", "rand", "auto"),
    ("env0", 512, "bbpow_action", "rand", "f32"),
    ("env1", 256, "temp_const_action", "hf", "f32"),
])
def test_step_parity_short(torch_gpu, name, N, reward, act, coupling):
    _run_pair(torch_gpu, name, N, 19, reward, 12, act, coupling=coupling)


def test_step_parity_random_gain(torch_gpu):
    """north_star 'random K': per-env coupling K ~ U(0.3, 0.8) (kura_set_env_gain)."""
    rng = np.random.default_rng(7)
    N, B = 512, 19
    gains = (rng.uniform(0.3, 0.8, B) / N).astype(np.float32)
    g, o = _run_pair(torch_gpu, "env0", N, B, "bbpow_action", 8, "rand", gains=gains)
    np.testing.assert_array_equal(g["y"], o["y"])


def test_step_parity_wavelet_directed(torch_gpu):
    """SURVEY 8(f) rank 4 options: wavelet coupling (signed alpha) + directional stimulation."""
    g, o = _run_pair(torch_gpu, "env0", 512, 19, "bbpow_action", 6, "hf", spatial_kernel="wavelet",
                     wavelet_amp=2.0, wavelet_steepness=0.5, directed_stimulation=True)
    np.testing.assert_array_equal(g["y"], o["y"])


def test_phase_gate_1000_steps(torch_gpu):
    """BASELINE.json gate: phases within 1e-5 relative after 1000 steps at
    N=1024, F32 coupling against the live oracle (the product arithmetic:
    tests/test_gpu_gates.py)."""
    g, o = _run_pair(torch_gpu, "env0", 1024, 8, "bbpow_action", 1000, "rand", check_every=250, coupling="f32")
    rel = np.abs(g["y"].astype(np.float64) - o["y"]) / np.maximum(np.abs(o["y"].astype(np.float64)), 1e-30)
    assert rel.max() <= PHASE_RTOL
    np.testing.assert_array_equal(g["y"], o["y"])


def test_phase_gate_1000_steps_env1_r2(torch_gpu):
    """The same gate on env1 (recorder-weighted f64 LFP, per-env contacts) with
    the R2 filter reward at N=1024 (TPW=4 gaussian save passes)."""
    g, o = _run_pair(torch_gpu, "env1", 1024, 8, "temp_const_action", 1000, "rand", check_every=250,
                     coupling="f32")
    rel = np.abs(g["y"].astype(np.float64) - o["y"]) / np.maximum(np.abs(o["y"].astype(np.float64)), 1e-30)
    assert rel.max() <= PHASE_RTOL
    np.testing.assert_array_equal(g["y"], o["y"])


def test_spectral_state_checkpoint(torch_gpu):
    """R1's spectral accumulators through get_state/set_state: restored
    exactly with 'spec' (kura_set_spec), re-formed from the ring without it
    (kura_spec_init_kernel) bit-exactly as the oracle re-forms them."""
    torch = torch_gpu
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    B = 19
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, B)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    o.reset(th0)
    for k in range(5):
        a = actions("rand", B, 1, k)
        sim.step(torch.from_numpy(a))
        o.step(a)
    g = sim.get_state()
    _cmp_state(g, o.state(), "after 5 steps")
    sim.set_state({k: v for k, v in g.items() if k != "spec"})
    o.set_state({k: v for k, v in o.state().items() if k != "spec"})
    _cmp_state(sim.get_state(), o.state(), "re-formed")
    sim.set_state(g)
    np.testing.assert_array_equal(sim.get_state()["spec"], g["spec"])
    o.set_state(g)
    for k in range(3):
        a = actions("rand", B, 1, 100 + k)
        sim.step(torch.from_numpy(a))
        ref = o.step(a)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(sim.reward.cpu().numpy(), ref["reward"])
    sim.close()
