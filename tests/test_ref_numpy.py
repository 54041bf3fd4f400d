"""The reference-op-sequence CPU baseline (oracle/ref_numpy.py, BASELINE.md
section 3) agrees with the bit-exact oracle to rounding: one solve from the
same state, the RHS, and a reset + step on the LFP/reward level."""
import numpy as np
import pytest

from helpers import make_case
from oracle import kura_oracle as ko
from oracle.ref_numpy import RefOpEnv


@pytest.fixture(scope="module")
def case():
    cfg, alpha, omega, gs, gr, th0, ct, st, hosts = make_case("env0", 256, 1)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    env = RefOpEnv(alpha, omega[0], gs[0], K=hosts[0].p["K"], W=cfg.window, dbs_bounds=(cfg.dbs_lo, cfg.dbs_hi))
    yield cfg, alpha, omega, gs, th0, o, env
    o.close()


def test_rhs_matches_oracle(case):
    cfg, alpha, omega, gs, th0, o, env = case
    y = th0[0] * 3.0
    pulse = (gs[0, 0] * 2.5).astype(np.float32)
    env.pulse = pulse
    np.testing.assert_allclose(env.dynamics(y), o.rhs(y, omega[0], pulse), rtol=0, atol=5e-5)


def test_one_solve_matches_oracle(case):
    cfg, alpha, omega, gs, th0, o, env = case
    ts = np.arange(10.0, 10.75, 0.05)
    env.pulse = np.zeros(env.N, np.float32)
    got = env.forward(ts, th0[0])
    exp, _ = o.solve_rows(omega[0], np.zeros(env.N, np.float32), ts, th0[0])
    np.testing.assert_allclose(got, exp, rtol=0, atol=2e-4)


def test_reset_and_step_lfp_close(case):
    cfg, alpha, omega, gs, th0, o, env = case
    w_ref = env.reset(th0[0])
    w_or = o.reset(th0)[0]
    np.testing.assert_allclose(w_ref, w_or, rtol=0, atol=5e-3)
    obs, r = env.step(np.array([0.3]))
    exp = o.step(np.array([[0.3]], np.float32))
    np.testing.assert_allclose(obs[-19:], exp["obs"][0][-19:], rtol=0, atol=5e-3)
    assert np.isfinite(r) and abs(r - float(exp["reward"][0])) <= 0.05 * abs(float(exp["reward"][0])) + 1e-3
