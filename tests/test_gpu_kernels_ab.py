"""The A/B step/reset kernels for N <= 1024: K1t
(team-overlapped, KURA_KERNEL=k1t) and K1w (one wave per SIMD,
KURA_KERNEL=k1w) stay bit-exact against the oracle like the default K1, at
every tile count they instantiate (N = 256, 512, 1024), with a partial last
workgroup."""
import importlib

import numpy as np
import pytest

from helpers import actions, ko, make_case


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["k1t", "k1w"])
@pytest.mark.parametrize("name,n_osc,reward", [
    ("env0", 256, "bbpow_action"),
    ("env1", 512, "temp_const_action"),
    ("env1", 1024, "bbpow_threth_action"),
])
def test_ab_kernel_bit_exact(torch, monkeypatch, kernel, name, n_osc, reward):
    monkeypatch.setenv("KURA_KERNEL", kernel)
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    B = 24  # a partial last workgroup (16 + 8)
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, n_osc, B, reward=reward)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    o.reset(th0)
    for k in range(4):
        a = actions("rand", B, cfg.n_elec, k)
        obs, rew, done = sim.step(torch.from_numpy(a))
        torch.cuda.synchronize()
        ref = o.step(a)
        np.testing.assert_array_equal(obs.cpu().numpy(), ref["obs"], err_msg=f"obs step {k}")
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"], err_msg=f"reward step {k}")
    got, exp = sim.get_state(), o.state()
    for key in ("y", "t", "step", "ring", "wpos"):
        np.testing.assert_array_equal(got[key], exp[key], err_msg=key)
    sim.close()
