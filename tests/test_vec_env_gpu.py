"""The gymnasium-shaped drop-in API on the GPU, checked against the oracle
driven through the same host draws (bit-exact)."""
import copy
import importlib

import numpy as np
import pytest

from helpers import kura, ko

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _mirror(venv):
    """An oracle + fresh EnvHosts replaying the same RNG streams."""
    o = ko.Oracle(venv.cfg, kura.model_setup.coupling_alpha(venv.params[0]["neur_coords"]).astype(np.float32))
    bins = kura.spectral.beta_bins(venv.cfg.window, 0.05)
    o.set_spectral(*kura.spectral.twiddles(venv.cfg.window, bins))
    hosts = [kura.EnvHost(p) for p in venv.params]
    o.set_gain(np.array([np.float32(p["K"] / p["num_oscillators"]) for p in venv.params], np.float32))
    return o, hosts


def _draw(o, hosts, idx, state):
    for b in idx:
        w0, gs, gr, th = hosts[b].reset_draws()
        state["w"][b], state["gs"][b], state["gr"][b], state["th"][b] = w0, gs, gr, th
    o.set_env_params(state["w"].astype(np.float32), state["gs"], state["gr"])


def test_vector_env_reset_step_autoreset(torch_gpu):
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env1", "eval", 2)
    B = 5
    env = vec.KuraVectorEnv(p, num_envs=B, reward_func="bbpow_action")
    env.episode_steps = 3  # short episodes to exercise autoreset
    o, hosts = _mirror(env)
    N = env.N
    st = dict(w=np.zeros((B, N)), gs=np.zeros((B, 1, N)), gr=np.zeros((B, 1, N)), th=np.zeros((B, N)))
    obs, info = env.reset()
    _draw(o, hosts, range(B), st)
    obs_o = o.reset(st["th"].astype(np.float32))
    assert obs.shape == (B, 1, env.W)
    np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), obs_o)
    rng = np.random.default_rng(4)
    for k in range(7):
        a = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
        obs, rew, term, trunc, info = env.step(a)
        ref = o.step(a)
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"])
        if (k + 1) % 3 == 0:
            assert "terminal_observation" in info and len(info["terminal_env_ids"]) == B
            np.testing.assert_array_equal(info["terminal_observation"][:, 0].cpu().numpy(), ref["obs"])
            _draw(o, hosts, range(B), st)
            obs_o = o.reset(st["th"].astype(np.float32))
            np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), obs_o)
        else:
            np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), ref["obs"])
    tm = env.get_attr("theta_mean")
    assert len(tm) == B and all(17 <= len(x) <= 19 for x in tm)
    assert env.get_attr("u")[0][0] == pytest.approx(5 * a[0, 0], rel=1e-6)
    env.close()


def test_single_env_dropin_and_reward_methods(torch_gpu):
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.fill_driver_arrays(kura.reference_params("env0", "eval", 0), w0_seed=228)
    p["reward_func"] = "bbpow_action"
    env = vec.SpatialKuramoto(p)
    assert env.observation_space.shape == (1, 2340) and env.action_space.shape == (1,)
    obs, r, d, tr, info = env.step([0.3])
    assert obs.shape == (1, 2340) and obs.dtype == np.float32 and isinstance(r, float) and d is False
    assert 17 <= len(env.theta_mean) <= 19
    x = np.asarray(obs[0], np.float64)
    cfg = copy.copy(env._v.cfg)
    o, _ = _mirror(env._v)
    for kind, fn in ((1, env.reward_bbpow_action), (2, env.reward_temp_const_lfp_betafilt_action),
                     (3, env.reward_bbpow_threth_action)):
        cfg.reward_kind = kind
        ref = ko.lib().oracle_reward(ko.ctypes.byref(cfg), x.ctypes.data, 1.5, o.ctab.ctypes.data, o.stab.ctypes.data)
        assert fn(x, [1.5]) == ref
    env.close()


def test_env2_drift_and_per_env_K(torch_gpu):
    """env2 (plasticity drift, electrode moves, encapsulation at every reset)
    with a different K per env, through two autoreset episodes."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    B = 4
    plist = []
    for b in range(B):
        p = kura.reference_params("env2", "train", b)
        p["K"] = [0.35, 0.52, 0.61, 0.78][b]
        plist.append(p)
    env = vec.KuraVectorEnv(plist, reward_func="temp_const_action")
    env.episode_steps = 2
    o, hosts = _mirror(env)
    N = env.N
    ne, nr = env.cfg.n_elec, max(env.cfg.n_rec, 1)
    st = dict(w=np.zeros((B, N)), gs=np.zeros((B, ne, N)), gr=np.zeros((B, nr, N)), th=np.zeros((B, N)))
    obs, _ = env.reset()
    _draw(o, hosts, range(B), st)
    np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), o.reset(st["th"].astype(np.float32)))
    rng = np.random.default_rng(11)
    for k in range(4):
        a = rng.uniform(-1, 1, (B, ne)).astype(np.float32)
        obs, rew, term, trunc, info = env.step(a)
        ref = o.step(a)
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"])
        if (k + 1) % 2 == 0:
            np.testing.assert_array_equal(info["terminal_observation"][:, 0].cpu().numpy(), ref["obs"])
            _draw(o, hosts, range(B), st)
            np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), o.reset(st["th"].astype(np.float32)))
        else:
            np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), ref["obs"])
    np.testing.assert_array_equal(env.sim.get_state()["y"], o.state()["y"])
    env.close()


def _run_modes(vec, p, mode, B, ncalls, offsets):
    """Per env and (episode, step): the observation and reward a KuraVectorEnv
    in the given autoreset mode returns; (b, e, 'reset'): the reset
    observation that opens episode e."""
    env = vec.KuraVectorEnv(p, num_envs=B, reward_func="bbpow_action", autoreset_mode=mode)
    env.episode_steps = 3
    env.reset()
    env.steps[:] = offsets              # envs finish in different calls
    pos = [[0, int(o)] for o in offsets]
    rec, pending = {}, set()

    def act(b, e, j):
        return np.random.default_rng(1000 * b + 10 * e + j).uniform(-1, 1)

    for _ in range(ncalls):
        a = np.array([[act(b, *pos[b])] for b in range(B)], np.float32)
        obs, rew, term, trunc, info = env.step(a)
        o_np, r_np, t_np = obs[:, 0].cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        assert not trunc.cpu().numpy().any()
        for b in range(B):
            e, j = pos[b]
            if b in pending:               # next_step: this call reset env b (its action ignored)
                assert r_np[b] == 0.0 and not t_np[b] and b in info["reset_env_ids"]
                rec[(b, e + 1, "reset")] = o_np[b]
                pending.discard(b)
                pos[b] = [e + 1, 0]
            elif j == 2:                   # the episode's last step
                assert t_np[b]
                if mode == "same_step":
                    k = list(info["terminal_env_ids"]).index(b)
                    rec[(b, e, j)] = (info["terminal_observation"][k, 0].cpu().numpy(), r_np[b])
                    rec[(b, e + 1, "reset")] = o_np[b]
                    pos[b] = [e + 1, 0]
                else:
                    assert "terminal_observation" not in info
                    rec[(b, e, j)] = (o_np[b], r_np[b])
                    pending.add(b)
                    pos[b] = [e, 3]
            else:
                assert not t_np[b]
                rec[(b, e, j)] = (o_np[b], r_np[b])
                pos[b] = [e, j + 1]
    env.close()
    return rec


def test_next_step_autoreset_mode_matches_same_step(torch_gpu):
    """gymnasium's NEXT_STEP autoreset: the finishing call returns the last
    observation, the next call resets the env (reward 0, not done) -- every
    env's episodes identical, step for step, to SB3's same-step mode (checked
    against the oracle above), with envs finishing in different calls."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 1)
    B, offsets = 4, [0, 1, 2, 2]
    same = _run_modes(vec, p, "same_step", B, 8, offsets)
    nxt = _run_modes(vec, p, "next_step", B, 11, offsets)
    common = set(same) & set(nxt)
    assert len(common) >= 4 * 7 and sum(1 for k in common if k[2] == "reset") >= 4 * 2
    for k in common:
        if k[2] == "reset":
            np.testing.assert_array_equal(nxt[k], same[k])
        else:
            np.testing.assert_array_equal(nxt[k][0], same[k][0])
            assert nxt[k][1] == same[k][1]


def test_state_dict_round_trip_keeps_the_coupling(torch_gpu):
    """a checkpoint records the arithmetic its trajectories were
    computed in; it restores bit for bit into an env of the same coupling and
    is refused by one of the other (the continuation would differ)."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    p = kura.reference_params("env0", "eval", 1)
    a = np.linspace(-1, 1, 3, dtype=np.float32).reshape(3, 1)
    env = vec.KuraVectorEnv(copy.deepcopy(p), num_envs=3, reward_func="bbpow_action")
    env.reset(seed=5)
    env.step(a)
    st = env.state_dict()
    assert st["coupling"] == "bf16x3"                         # AUTO
    _, r1, _, _, _ = env.step(a)
    env2 = vec.KuraVectorEnv(copy.deepcopy(p), num_envs=3, reward_func="bbpow_action")
    env2.reset(seed=9)
    env2.load_state_dict(st)
    _, r2, _, _, _ = env2.step(a)
    np.testing.assert_array_equal(r1.cpu().numpy(), r2.cpu().numpy())
    env3 = vec.KuraVectorEnv(copy.deepcopy(p), num_envs=3, reward_func="bbpow_action", coupling="f32")
    env3.reset(seed=5)
    with pytest.raises(ValueError, match="coupling"):
        env3.load_state_dict(st)
    for e in (env, env2, env3):
        e.close()
