"""BASELINE.json configs on the GPU against the oracle:
env1 at N=1024 (TPW=4 with the recorder-weighted f64 save passes, R1 and R2),
env2 at N=1024 through KuraVectorEnv (drift, per-env K, autoreset), and full
B=4096 grids (256 workgroups, every CU) for env0 and env1 with a sample of
envs from across the grid checked against the oracle (each env is
independent of the others, tests/test_oracle_props.py)."""
from __future__ import annotations

import importlib

import numpy as np
import pytest

from helpers import actions, kura, ko, make_case
from test_gpu_parity import _run_pair, _cmp_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("reward", ["bbpow_action", "temp_const_action"])
def test_env1_n1024_parity(torch_gpu, reward):
    """configs[2]: env1 spatial recorder LFP, N=1024 (TPW=4 gaussian save passes)."""
    _run_pair(torch_gpu, "env1", 1024, 19, reward, 8, "rand")


def test_env2_n1024_vector_env(torch_gpu):
    """configs[3] per GPU: env2 drift + per-env K at N=1024 through the
    VectorEnv (masked autoreset, parameter re-upload) vs the oracle."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    from test_vec_env_gpu import _draw, _mirror
    B = 6
    plist = []
    for b in range(B):
        p = kura.synthetic_params("env2", 1024)
        p["K"] = float(np.random.default_rng(b).uniform(0.3, 0.8))
        p["rand_seed"] = 100 + b
        plist.append(p)
    env = vec.KuraVectorEnv(plist, reward_func="bbpow_action")
    env.episode_steps = 2
    o, hosts = _mirror(env)
    N, ne, nr = env.N, env.cfg.n_elec, max(env.cfg.n_rec, 1)
    st = dict(w=np.zeros((B, N)), gs=np.zeros((B, ne, N)), gr=np.zeros((B, nr, N)), th=np.zeros((B, N)))
    obs, _ = env.reset()
    _draw(o, hosts, range(B), st)
    np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), o.reset(st["th"].astype(np.float32)))
    rng = np.random.default_rng(2)
    for k in range(6):
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


@pytest.mark.parametrize("name,reward,steps,coupling", [("env0", "bbpow_action", 24, "auto"),
                                                        ("env1", "temp_const_action", 24, "auto"),
                                                        ("env1", "bbpow_action", 16, "auto"),
                                                        ("env0", "bbpow_action", 50, "f32")])
def test_full_grid_b4096_sampled(torch_gpu, name, reward, steps, coupling):
    """configs[1]/[2] at full size: B=4096 (256 workgroups), reset + steps;
    envs sampled from first, middle and last workgroups and across the
    16-env interleave checked bit for bit against the oracle run on just them
    (the product arithmetic, and F32; the bf16x3 oracle costs ~0.5 s per
    N=1024 step of these 14 envs, hence fewer steps)."""
    torch = torch_gpu
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    B, N = 4096, 1024
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, reward=reward, coupling=coupling)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0), check_errors=True)
    idx = np.array([0, 1, 7, 15, 16, 31, 1000, 2047, 2048, 2051, 3333, 4080, 4094, 4095])
    import copy
    c = copy.copy(cfg)
    c.n_envs = len(idx)
    o = ko.Oracle(c, alpha)
    o.set_env_params(omega[idx], gs[idx], gr[idx])
    o.set_spectral(ct, st)
    o.reset(th0[idx])
    _cmp_state({k: v[idx] for k, v in sim.get_state().items()}, o.state(), "reset")
    for k in range(steps):
        a = actions("rand", B, cfg.n_elec, k)
        sim.step(torch.from_numpy(a), check_errors=True)
        ref = o.step(a[idx])
        for key in ("obs", "reward", "done", "nsamp", "lfp_true", "lfp_rec"):
            np.testing.assert_array_equal(getattr(sim, key).cpu().numpy()[idx], ref[key], err_msg=f"{key} step {k}")
        _cmp_state({kk: v[idx] for kk, v in sim.get_state().items()}, o.state(), f"step {k}")
    sim.close()


@pytest.mark.parametrize("name,N,elec,rec", [
    ("env1", 512, [[4, 3, 4], [2, 5, 3], [6, 2, 5]], [[1, 1, 1], [6, 6, 2]]),   # 3 contacts, 2 recorders
    ("env0", 1024, [[4, 3, 4], [3, 6, 2]], [[1, 1, 1]]),                        # 2 contacts, naive LFP
    ("env1", 1024, [[4, 3, 4], [2, 5, 3], [6, 2, 5], [5, 5, 5]],
     [[1, 1, 1], [6, 6, 2], [2, 6, 6], [5, 1, 3]]),                            # the 4 / 4 maximum
])
def test_multi_contact_parity(torch_gpu, name, N, elec, rec):
    """Several stimulating contacts (pulse = sum_e g_e u_e, env.py:419-424, one
    action per contact) and several recorders (sum over recorders of the
    weighted LFP, env.py:404-412), up to the ABI's 4 / 4."""
    g, o = _run_pair(torch_gpu, name, N, 19, "bbpow_action", 6, "rand", elec_coords=elec, rec_coords=rec,
                     electrode_amps=[1.0] * len(elec))
    np.testing.assert_array_equal(g["y"], o["y"])


def test_largest_window_parity(torch_gpu):
    """observe_wind_counts=142: W = 2556 samples, next to the kernel's 2560
    limit (WPL_MAX = 40 samples per lane), R1 and the window ring at its largest."""
    g, o = _run_pair(torch_gpu, "env0", 256, 19, "bbpow_action", 6, "rand", observe_wind_counts=142)
    np.testing.assert_array_equal(g["ring"], o["ring"])


def test_r3_n1024_parity(torch_gpu):
    """R3 (reward_bbpow_threth_action) at the headline N=1024."""
    g, o = _run_pair(torch_gpu, "env0", 1024, 19, "bbpow_threth_action", 8, "rand")
    np.testing.assert_array_equal(g["y"], o["y"])


def test_env2_b4096_vector_env_sampled(torch_gpu):
    """configs[3] per GPU at full size: env2 (drift,
    per-env K ~ U(0.3, 0.8)) at N=1024 x 4096 envs through KuraVectorEnv with
    masked autoreset across an episode boundary (episode of 3 steps, 5 steps
    run); 12 envs sampled across the grid checked bit for bit against the
    oracle run on just them, their reset draws replayed by fresh EnvHosts."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    import copy
    B, N = 4096, 1024
    base = kura.fill_driver_arrays(kura.synthetic_params("env2", N), w0_seed=31)
    Ks = np.random.default_rng(9).uniform(0.3, 0.8, B)
    plist = []
    for b in range(B):
        p = copy.copy(base)
        p["K"] = float(Ks[b])
        p["rand_seed"] = 1000 + b
        plist.append(p)
    env = vec.KuraVectorEnv(plist, reward_func="bbpow_action")
    env.episode_steps = 3
    idx = np.array([0, 5, 15, 16, 255, 1024, 2047, 2049, 3000, 4079, 4088, 4095])
    sub = [plist[i] for i in idx]
    c = copy.copy(env.cfg)
    c.n_envs = len(idx)
    o = ko.Oracle(c, env._alpha.astype(np.float32))
    o.set_gain(np.array([np.float32(p["K"] / N) for p in sub], np.float32))
    bins = kura.spectral.beta_bins(c.window, base["verbose_dt"])
    o.set_spectral(*kura.spectral.twiddles(c.window, bins))
    hosts = [kura.EnvHost(p) for p in sub]
    n = len(idx)
    ne, nr = c.n_elec, max(c.n_rec, 1)
    st = dict(w=np.zeros((n, N)), gs=np.zeros((n, ne, N)), gr=np.zeros((n, nr, N)), th=np.zeros((n, N)))

    def draw():
        for j in range(n):
            w0, gs, gr, th = hosts[j].reset_draws()
            st["w"][j], st["gs"][j], st["gr"][j], st["th"][j] = w0, gs, gr, th
        o.set_env_params(st["w"].astype(np.float32), st["gs"], st["gr"])

    obs, _ = env.reset()
    draw()
    np.testing.assert_array_equal(obs[idx, 0].cpu().numpy(), o.reset(st["th"].astype(np.float32)))
    rng = np.random.default_rng(3)
    for k in range(5):
        a = rng.uniform(-1, 1, (B, ne)).astype(np.float32)
        obs, rew, term, trunc, info = env.step(a)
        ref = o.step(a[idx])
        np.testing.assert_array_equal(rew.cpu().numpy()[idx], ref["reward"], err_msg=f"reward step {k}")
        np.testing.assert_array_equal(env.sim.lfp_true.cpu().numpy()[idx], ref["lfp_true"])
        if (k + 1) % 3 == 0:
            assert len(info["terminal_env_ids"]) == B
            np.testing.assert_array_equal(info["terminal_observation"][idx, 0].cpu().numpy(), ref["obs"])
            draw()
            np.testing.assert_array_equal(obs[idx, 0].cpu().numpy(), o.reset(st["th"].astype(np.float32)))
        else:
            np.testing.assert_array_equal(obs[idx, 0].cpu().numpy(), ref["obs"])
    np.testing.assert_array_equal(env.sim.get_state()["y"][idx], o.state()["y"])
    env.close()


def test_env2_phase_gate_1000_steps_vector_env(torch_gpu):
    """The north_star gate on env2: drift events and
    per-env K ~ U(0.3, 0.8) at N=1024 through KuraVectorEnv, 1000 steps with
    300-step episodes (3 autoresets per env, each with the reference's drift
    draws), rewards every step and phases at the end bit-exact against the
    oracle (hence within 1e-5 relative), the reset draws replayed by fresh
    EnvHosts.  F32 coupling against the live oracle; the product arithmetic's
    gate replays a committed oracle record (tests/test_gpu_gates.py)."""
    vec = importlib.import_module("dbs-gym_amd.vec_env")
    import copy
    B, N, L = 8, 1024, 300
    base = kura.fill_driver_arrays(kura.synthetic_params("env2", N), w0_seed=77)
    Ks = np.random.default_rng(19).uniform(0.3, 0.8, B)
    plist = []
    for b in range(B):
        p = copy.copy(base)
        p["K"] = float(Ks[b])
        p["rand_seed"] = 500 + b
        plist.append(p)
    env = vec.KuraVectorEnv(plist, reward_func="bbpow_action", coupling="f32")
    env.episode_steps = L
    c = copy.copy(env.cfg)
    o = ko.Oracle(c, env._alpha.astype(np.float32))
    o.set_gain(np.array([np.float32(p["K"] / N) for p in plist], np.float32))
    bins = kura.spectral.beta_bins(c.window, base["verbose_dt"])
    o.set_spectral(*kura.spectral.twiddles(c.window, bins))
    hosts = [kura.EnvHost(copy.deepcopy(p)) for p in plist]

    def draw():
        w0, gs, gr, th = kura.reset_draws_batch(hosts)
        o.set_env_params(w0.astype(np.float32), gs, gr)
        return th.astype(np.float32)

    obs, _ = env.reset()
    np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), o.reset(draw()))
    rng = np.random.default_rng(5)
    resets = 0
    for k in range(1000):
        a = rng.uniform(-1, 1, (B, c.n_elec)).astype(np.float32)
        obs, rew, term, trunc, info = env.step(a)
        ref = o.step(a)
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"], err_msg=f"reward step {k}")
        if (k + 1) % L == 0:
            resets += 1
            assert len(info["terminal_env_ids"]) == B
            np.testing.assert_array_equal(info["terminal_observation"][:, 0].cpu().numpy(), ref["obs"])
            np.testing.assert_array_equal(obs[:, 0].cpu().numpy(), o.reset(draw()))
            np.testing.assert_array_equal(env.sim.get_state()["y"], o.state()["y"])   # after the reset
    assert resets == 3
    g, r = env.sim.get_state(), o.state()
    for key in ("y", "t", "step", "ring", "wpos", "spec"):
        np.testing.assert_array_equal(g[key], r[key], err_msg=key)
    rel = np.abs(g["y"].astype(np.float64) - r["y"]) / np.maximum(np.abs(r["y"].astype(np.float64)), 1e-30)
    assert rel.max() <= 1e-5
    env.close()
