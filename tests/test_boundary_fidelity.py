"""Boundary details callers read: sol_state_ keeps every
row of the step, sol_state after reset() the transient's rows (VERDICT r05
missing #4), get_attr('u') is the reference's rescale_action bit for bit."""
import importlib

import numpy as np
import pytest

from helpers import ko, kura


def _reference_rescale(a, x=-1, y=1, z=-5, k=5):
    """env.py:389-393 with float(a) (env.py:419): Python float arithmetic."""
    return z + ((k - z) * (float(a) - x)) / (y - x)


def test_u_formula_is_rescale_action():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(0)
    a = np.concatenate([rng.uniform(-1, 1, 20000), rng.uniform(-3, 3, 2000), [-1, 1, 0, -0.0, 0.5, 1e-8, -1e-30]]
                       ).astype(np.float32)
    # KuraVectorEnv.step: lo + ((hi - lo) * (a + 1.0)) / 2.0 in float64 -- the same IEEE operations
    got = (-5.0 + ((5.0 - -5.0) * (torch.from_numpy(a).double() + 1.0)) / 2.0).numpy()
    ref = np.array([_reference_rescale(v) for v in a])
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
def test_single_env_sol_state_rows():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.fill_driver_arrays(kura.reference_params("env1", "eval", 1), w0_seed=228)
    p["reward_func"] = "bbpow_action"
    env = vec.SpatialKuramoto(p)
    o = ko.Oracle(env._v.cfg, kura.model_setup.coupling_alpha(p["neur_coords"]).astype(np.float32))
    for k in range(5):
        env.step([0.4 * (k - 2)])
        rows = env.sol_state_
        S = len(env.theta_mean)
        assert rows.shape == (S + 1, env._v.N) and rows.dtype == np.float32
        # row S is the new state, the I/II boundary row is duplicated (env.py:440)
        np.testing.assert_array_equal(rows[S], env._v.sim.get_state()["y"][0])
        # every LFP sample is the oracle's LFP of the captured row (RM-order reduction, bit for bit)
        for s in range(S):
            n, r = o.lfp(rows[s], env._v._g_rec[0])
            assert n == env.theta_mean[s] and r == env.theta_records[s], (k, s)
    # the duplicate row: ys_II[0] == ys_I[-1]; find it as two equal consecutive rows
    assert any(np.array_equal(rows[i], rows[i + 1]) for i in range(2, 5))
    # sol_state (env.py:439) = ys_II: starts at the duplicated boundary row, ends at the state
    ys2 = env.sol_state
    assert np.array_equal(ys2[0], rows[len(rows) - len(ys2) - 1]) and np.array_equal(ys2[-1], rows[-1])
    assert len(ys2) in (15, 16)
    # init_state (env.py:594-598): the last reset's theta0 draws, float64
    th0 = env.init_state
    assert th0.dtype == np.float64 and th0.shape == (env._v.N,)
    env.reset()
    assert not np.array_equal(th0, env.init_state)
    # sol_state after reset() (env.py:610): the transient's rows, the oracle's
    # solve over arange(0, transient_state_len, verbose_dt) from init_state, bit
    # for bit; the last row is the state
    sol = env.sol_state
    ts = np.arange(0.0, p["transient_state_len"], p["verbose_dt"])
    assert sol.shape == (len(ts), env._v.N) and sol.dtype == np.float32
    rows_o, _st = o.solve_rows(env._v._omega[0], None, ts, env.init_state.astype(np.float32))
    np.testing.assert_array_equal(sol, rows_o)
    np.testing.assert_array_equal(sol[-1], env._v.sim.get_state()["y"][0])
    # theta_record_transient (env.py:611): the LFP of the 3999 transient rows,
    # whose last W are the observation the reset returned
    tr = env.theta_record_transient
    assert tr.shape == (3999,)
    np.testing.assert_array_equal(tr[-env._v.W:].astype(np.float32), env.theta_state.ravel())
    # ... and it is calc_lfp(sol_state[:-1]) (env.py:611), sampled rows
    for s in (0, 1, 1000, len(ts) - 2):
        _n, r = o.lfp(sol[s], env._v._g_rec[0])
        assert r == env._v.get_attr("theta_record_transient")[0][s], s
    # off: the reference attribute raises with the reason until the first step
    env._v.sim.capture_transient_rows(False)
    env.reset()
    with pytest.raises(AttributeError, match="transient"):
        env.sol_state
    env.close()


@pytest.mark.gpu
def test_transient_rows_beyond_32bit_offsets_are_rejected():
    """kura_set_transient_rows refuses a transient whose rows for one 16-env
    group exceed the save passes' 32-bit byte offsets (N=8192, 6000 rows:
    3.1 GB per group) instead of wrapping them."""
    import ctypes
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from helpers import make_case
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg = make_case("env0", 8192, 16)[0]
    cfg.transient_len = 300.0
    sim = sim_mod.KuraSim(cfg, 0)
    try:
        assert sim.lib.kura_transient_len(sim._h) == len(np.arange(0.0, 300.0, cfg.dt))
        rc = sim.lib.kura_set_transient_rows(sim._h, ctypes.c_void_p(256))   # rejected before any use
        assert rc != 0 and b"2 GiB" in sim.lib.kura_last_error()
        assert sim.lib.kura_set_transient_rows(sim._h, None) == 0
    finally:
        sim.close()
