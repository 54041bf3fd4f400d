"""Failure paths (VERDICT r1 missing #3 / weak #5): a solve that fails inside
the library is reported per env (kura.h KURA_F_*), identically to the oracle,
and the host raises like the reference's diffeqsolve (diffrax throw=True,
env.py:261-270) instead of continuing silently."""
from __future__ import annotations

import copy
import importlib

import numpy as np
import pytest

from helpers import actions, ko, make_case

pytestmark = pytest.mark.gpu
abi = importlib.import_module("dbs-gym_amd.abi")


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _pair(torch, cfg, alpha, omega, gs, gr, ct, st):
    sim = importlib.import_module("dbs-gym_amd.sim").KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    return sim, o


def _state_from_oracle(cfg, alpha, omega, gs, gr, ct, st, th0):
    """A valid post-reset state (computed with the default max_steps)."""
    c = copy.copy(cfg)
    c.max_steps = 4096
    o = ko.Oracle(c, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    return o.state()


def test_reset_max_steps_raises(torch_gpu):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 512, 5)
    cfg.max_steps = 2                      # the transient needs ~75 Dopri steps
    sim, o = _pair(torch_gpu, cfg, alpha, omega, gs, gr, ct, st)
    with pytest.raises(abi.KuraSolverError, match="maximum number of solver steps"):
        sim.reset(torch_gpu.from_numpy(th0), check_errors=True)
    o.reset(th0)
    np.testing.assert_array_equal(sim.flags.cpu().numpy(), o.flags)
    assert (o.flags == abi.KURA_F_MAX_STEPS).all()
    sim.close()


def test_step_max_steps_matches_oracle(torch_gpu):
    """max_steps = 2: the ON solve (2 Dopri steps) completes, the OFF solve
    (3) fails; the step is abandoned identically on both sides."""
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env1", 512, 7)
    state = _state_from_oracle(cfg, alpha, omega, gs, gr, ct, st, th0)
    cfg.max_steps = 2
    sim, o = _pair(torch_gpu, cfg, alpha, omega, gs, gr, ct, st)
    sim.set_state(state)
    o.set_state(state)
    a = actions("rand", 7, cfg.n_elec, 0)
    with pytest.raises(abi.KuraSolverError, match="maximum number of solver steps"):
        sim.step(torch_gpu.from_numpy(a), check_errors=True)
    ref = o.step(a)
    np.testing.assert_array_equal(sim.flags.cpu().numpy(), o.flags)
    assert (o.flags == abi.KURA_F_MAX_STEPS).all()
    for k in ("done", "reward", "nsamp"):
        np.testing.assert_array_equal(getattr(sim, k).cpu().numpy(), ref[k])
    g, r = sim.get_state(), o.state()
    for k in ("y", "t", "step", "ring", "wpos", "spec"):
        np.testing.assert_array_equal(g[k], r[k], err_msg=k)
    np.testing.assert_array_equal(g["t"], state["t"])          # time and window not advanced
    sim.close()


def test_nonfinite_state_flags_only_that_env(torch_gpu):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 512, 6)
    state = _state_from_oracle(cfg, alpha, omega, gs, gr, ct, st, th0)
    state["y"][2, 17] = np.nan
    state["y"][4, 3] = np.inf
    sim, o = _pair(torch_gpu, cfg, alpha, omega, gs, gr, ct, st)
    sim.set_state(state)
    o.set_state(state)
    a = actions("rand", 6, cfg.n_elec, 3)
    sim.step(torch_gpu.from_numpy(a))
    ref = o.step(a)
    fl = sim.flags.cpu().numpy()
    np.testing.assert_array_equal(fl, o.flags)
    assert fl[2] == abi.KURA_F_NONFINITE and fl[4] == abi.KURA_F_NONFINITE
    assert (fl[[0, 1, 3, 5]] == 0).all()
    ok = [0, 1, 3, 5]
    for k in ("obs", "reward", "done", "nsamp", "lfp_true"):
        g = getattr(sim, k).cpu().numpy()
        np.testing.assert_array_equal(g[ok], ref[k][ok], err_msg=k)
    np.testing.assert_array_equal(sim.done.cpu().numpy()[[2, 4]], [1, 1])
    g = sim.get_state()
    np.testing.assert_array_equal(g["y"][ok], o.state()["y"][ok])
    with pytest.raises(abi.KuraSolverError) as ei:
        sim.raise_on_failure()
    assert ei.value.envs == [2, 4]
    sim.close()


@pytest.mark.parametrize("check", ["eager", "deferred"])
def test_vector_env_policies(torch_gpu, check):
    """KuraVectorEnv: on_failure='raise' raises from reset/step; 'reset' reports
    the env truncated and autoresets it.  failure_check='eager' acts in the
    failing step; 'deferred' (default: no per-step synchronisation) acts at
    the start of the next step, before its launch (the failing step itself
    reports done = 1 from the kernel)."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    env = venv.KuraVectorEnv(p, num_envs=3, max_steps=2, failure_check=check)
    with pytest.raises(abi.KuraSolverError, match="kura_reset"):
        env.reset()
    env.close()
    env = venv.KuraVectorEnv(p, num_envs=3, on_failure="reset", failure_check=check)
    env.reset()
    st = env.sim.get_state()
    st["y"][1, 0] = np.nan
    env.sim.set_state(st)
    a = np.zeros((3, 1), np.float32)
    obs, rew, term, trunc, info = env.step(a)
    if check == "eager":
        assert list(info["failed_env_ids"]) == [1] and info["failure_flags"][0] == abi.KURA_F_NONFINITE
        assert bool(trunc[1]) and not bool(term[1]) and not bool(trunc[0])     # a truncation, not a termination
        assert list(info["terminal_env_ids"]) == [1] and env.steps[1] == 0 and env.steps[0] == 1
    else:
        # not known yet: not done (episode counters), not truncated
        assert "failed_env_ids" not in info and not bool(term[1]) and not bool(trunc[1])
        obs, rew, term, trunc, info = env.step(a)        # reported now; env 1 reset before this launch
        assert list(info["failed_env_ids"]) == [1] and info["failure_flags"][0] == abi.KURA_F_NONFINITE
        assert list(info["reset_before_step_ids"]) == [1] and bool(trunc[1]) and not bool(term[1])
        assert tuple(info["reset_before_step_observation"].shape) == (1, 1, env.W)
        assert env.steps[1] == 1 and env.steps[0] == 2 and np.isfinite(rew.cpu().numpy()).all()
    obs, rew, term, trunc, info = env.step(a)   # env 1 runs again after its reset
    assert "failed_env_ids" not in info and np.isfinite(rew.cpu().numpy()).all()
    obs, rew, term, trunc, info = env.step(a)
    assert "failed_env_ids" not in info
    env.close()
    # raise policy, deferred: the failure surfaces from the next call
    env = venv.KuraVectorEnv(p, num_envs=3, failure_check=check)
    env.reset()
    st = env.sim.get_state()
    st["y"][2, 5] = np.inf
    env.sim.set_state(st)
    if check == "eager":
        with pytest.raises(abi.KuraSolverError):
            env.step(a)
    else:
        env.step(a)
        with pytest.raises(abi.KuraSolverError, match="previous call"):
            env.step(a)
    env.close()


def test_vector_env_failed_resets_retry_then_raise(torch_gpu):
    """on_failure='reset': an autoreset whose transient fails is reported and
    retried; max_reset_failures consecutive failures of one env raise."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    env = venv.KuraVectorEnv(p, num_envs=2, max_steps=2, on_failure="reset", max_reset_failures=2)
    with pytest.raises(abi.KuraSolverError, match="repeated"):
        env.reset()
    assert (env._reset_fail_runs == 3).all()
    env.close()


def _nan_env(venv, p, n=3, **kw):
    env = venv.KuraVectorEnv(p, num_envs=n, **kw)
    env.reset()
    st = env.sim.get_state()
    st["y"][1, 0] = np.nan
    env.sim.set_state(st)
    return env


def test_deferred_failure_raises_from_reset_and_close(torch_gpu):
    """a failure of the last step before reset()/close() is not
    dropped with the deferred flags: on_failure='raise' raises there."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    a = np.zeros((3, 1), np.float32)
    env = _nan_env(venv, p)
    env.step(a)
    with pytest.raises(abi.KuraSolverError, match="previous call"):
        env.reset()
    env.close()
    env = _nan_env(venv, p)
    env.step(a)
    with pytest.raises(abi.KuraSolverError, match="before close"):
        env.close()
    env = _nan_env(venv, p, on_failure="reset")
    env.step(a)
    obs, info = env.reset()                                   # reset mode: reported, every env reset
    assert list(info["failed_env_ids"]) == [1]
    env.step(a)
    env.close()


def test_deferred_failure_closes_the_sb3_episode(torch_gpu):
    """with deferred checks an SB3 wrapper sees the failed episode
    end (terminal_observation, TimeLimit.truncated, Monitor summary of the
    steps before the failure) and the next one start."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    sb3 = importlib.import_module("dbs-gym_amd.sb3")
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    env = venv.KuraVectorEnv(p, num_envs=3, on_failure="reset")
    v = sb3.KuraSB3VecEnv(env)
    v.reset()
    a = np.zeros((3, 1), np.float32)
    v.step(a)
    v.step(a)
    st = env.sim.get_state()
    st["y"][1, 0] = np.nan
    env.sim.set_state(st)
    obs, rew, dones, infos = v.step(a)                        # fails on the device; not known yet
    assert not dones[1] and "terminal_observation" not in infos[1]
    obs, rew, dones, infos = v.step(a)                        # closed here, before this transition
    assert dones[1] and infos[1]["TimeLimit.truncated"] and infos[1]["terminal_observation"].shape == (1, env.W)
    assert infos[1]["episode"]["l"] == 3 and infos[1]["failure_flags"] == abi.KURA_F_NONFINITE
    assert not dones[0] and not dones[2]
    assert v._ep_len[1] == 1 and v._ep_len[0] == 4 and np.isfinite(rew).all()
    v.close()


def test_reset_failure_runs_count_consecutive_failures_only(torch_gpu, monkeypatch):
    """max_reset_failures counts failures in a row -- a confirmed
    reset clears the count, so fail, succeed, fail, succeed does not raise."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    p["total_episode_len"] = 2 * (p["electrode_width"] + p["electrode_pause"])   # 2-step episodes
    orig = venv.reset_draws_batch
    for check in ("eager", "deferred"):
        env = venv.KuraVectorEnv(p, num_envs=2, on_failure="reset", max_reset_failures=1, failure_check=check)
        host = env.hosts[0]
        calls = {"n": 0}
        poison = {1, 3}          # reset draws 1 and 3 of env 0 get a NaN phase (its transient fails)

        def draws(hosts):
            w0, gs, gr, th = orig(hosts)
            for k, h in enumerate(hosts):
                if h is host:
                    if calls["n"] in poison:
                        th[k, 0] = np.nan
                    calls["n"] += 1
            return w0, gs, gr, th
        monkeypatch.setattr(venv, "reset_draws_batch", draws)
        env.reset()                                            # draw 0: ok
        a = np.zeros((2, 1), np.float32)
        for _ in range(8):                                     # autoresets: draws 1 (fails), 2 (ok), 3 (fails), 4 ...
            env.step(a)
        assert calls["n"] >= 5
        assert env._reset_fail_runs[0] == 0
        env.close()


def _short_env(venv, kura, n, steps, **kw):
    p = kura.reference_params("env0", "eval", 0)
    p["reward_func"] = "bbpow_action"
    p["total_episode_len"] = steps * (p["electrode_width"] + p["electrode_pause"])
    return venv.KuraVectorEnv(p, num_envs=n, on_failure="reset", failure_check="deferred", **kw)


def _poison(env, b):
    st = env.sim.get_state()
    st["y"][b, 0] = np.nan
    env.sim.set_state(st)


def test_deferred_failure_on_terminal_step_same_step_resets_once(torch_gpu):
    """an env whose last step of the episode fails is autoreset in
    that call (same_step); the deferred check one call later reports the
    failure but must not reset it a second time (an extra draw from its RNG
    stream, and a bogus zero-length episode for an SB3 wrapper)."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    env = _short_env(venv, kura, 3, 2)
    env.reset()
    a = np.zeros((3, 1), np.float32)
    env.step(a)
    _poison(env, 1)
    obs, rew, term, trunc, info = env.step(a)                 # fails on the device; episode ends: autoreset
    assert list(info["terminal_env_ids"]) == [0, 1, 2]
    rc = [h.reset_count for h in env.hosts]
    obs, rew, term, trunc, info = env.step(a)
    assert list(info["failed_env_ids"]) == [1] and info["failure_flags"][0] == abi.KURA_F_NONFINITE
    assert "reset_before_step_ids" not in info and not bool(trunc[1])
    assert [h.reset_count for h in env.hosts] == rc           # no second reset
    assert env.steps[1] == 1 and np.isfinite(rew.cpu().numpy()).all()
    env.close()


def test_deferred_failure_next_step_mode_ends_the_episode_then_resets(torch_gpu):
    """ADVICE r04, gymnasium NEXT_STEP with deferred checks: the failure of
    call k is reported in call k+1 as the episode's end (truncated, the last
    observation, reward 0), and call k+2 resets the env (reset_env_ids) --
    not a reset before the launch of call k+1."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    env = _short_env(venv, kura, 3, 50, autoreset_mode="next_step")
    env.reset()
    a = np.zeros((3, 1), np.float32)
    env.step(a)
    _poison(env, 1)
    obs_k, rew, term, trunc, info = env.step(a)               # fails on the device (not known yet)
    assert "failed_env_ids" not in info and not bool(trunc[1])
    rc = [h.reset_count for h in env.hosts]
    obs, rew, term, trunc, info = env.step(a)                 # call k+1: the failed episode ends here
    assert list(info["failed_env_ids"]) == [1]
    assert bool(trunc[1]) and not bool(term[1]) and float(rew[1]) == 0.0
    assert not bool(trunc[0]) and not bool(trunc[2])
    np.testing.assert_array_equal(obs[1].cpu().numpy(), obs_k[1].cpu().numpy())   # its last observation
    assert [h.reset_count for h in env.hosts] == rc           # not reset yet
    obs, rew, term, trunc, info = env.step(a)                 # call k+2: reset
    assert list(info["reset_env_ids"]) == [1] and float(rew[1]) == 0.0 and not bool(trunc[1])
    assert "failed_env_ids" not in info                        # the discarded step's flags do not count
    assert [h.reset_count for h in env.hosts] == [rc[0], rc[1] + 1, rc[2]]
    obs, rew, term, trunc, info = env.step(a)
    assert "failed_env_ids" not in info and np.isfinite(rew.cpu().numpy()).all() and env.steps[1] == 1
    env.close()


def test_next_step_truncation_excludes_the_discarded_step(torch_gpu):
    """next_step mode with deferred checks, the failure of call k
    ends the episode in call k+1, whose step for that env is discarded: the
    episode length counts calls 1..k only, and the episode metrics are those
    of the episode buffer as call k left it."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    env = _short_env(venv, kura, 3, 50, autoreset_mode="next_step", episode_metrics=True)
    env.reset()
    a = np.zeros((3, 1), np.float32)
    env.step(a)
    env.step(a)
    _poison(env, 1)
    env.step(a)                                               # call k = 3 fails on the device
    m = torch_gpu.zeros(3, dtype=torch_gpu.uint8)
    m[1] = 1
    want_bb = env.sim.episode_bbpow(m, env.psd_dt, env.beta_band)[1].item()
    want_ev = env.sim.episode_envelope_stats(m)[1].cpu().numpy().copy()
    obs, rew, term, trunc, info = env.step(a)                 # call k+1: ends the episode, its step discarded
    assert list(info["failed_env_ids"]) == [1] and bool(trunc[1])
    ids = list(info["terminal_env_ids"])
    assert ids == [1]
    assert int(info["episode"]["l"][0]) == 3                 # calls 1..3, not the discarded 4th
    np.testing.assert_array_equal(info["episode"]["bbpow"][0], want_bb)   # (nan == nan: a 36-sample episode)
    np.testing.assert_array_equal(info["episode"]["envelope"][0], want_ev)
    env.close()


def test_deferred_failure_on_terminal_step_next_step_mode_resets_once(torch_gpu):
    """next_step mode, the failing step is the episode's last: the
    env is queued for its next_step reset; the deferred report must not reset
    it before that reset as well."""
    kura = importlib.import_module("dbs-gym_amd")
    venv = importlib.import_module("dbs-gym_amd.vec_env")
    env = _short_env(venv, kura, 3, 2, autoreset_mode="next_step")
    env.reset()
    a = np.zeros((3, 1), np.float32)
    env.step(a)
    _poison(env, 1)
    obs, rew, term, trunc, info = env.step(a)                 # fails; the episode ends (counters)
    assert bool(term[1])
    rc = [h.reset_count for h in env.hosts]
    obs, rew, term, trunc, info = env.step(a)                 # next_step resets + the deferred report
    assert list(info["failed_env_ids"]) == [1] and list(info["reset_env_ids"]) == [0, 1, 2]
    assert [h.reset_count for h in env.hosts] == [c + 1 for c in rc]
    env.close()
