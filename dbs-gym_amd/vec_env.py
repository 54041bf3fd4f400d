"""Drop-in environments over libkura.

``KuraVectorEnv``  -- gymnasium-VectorEnv-shaped batch of B reference
                      environments on one GPU.
``SpatialKuramoto`` -- the single-env class of environment/env.py:274 with the
                      same constructor, reset/step signatures, spaces,
                      attributes and reward methods, backed by a B=1 batch.

Host code here only draws the reference's random numbers, builds conductances
and bookkeeps episode counters; every numeric of reset()/step() runs in the
HIP library.  Observations, rewards and LFP samples stay on the device as
torch tensors unless the caller asks for NumPy.
"""
from __future__ import annotations

import copy
import time

import numpy as np
import torch

from . import spectral
from .abi import KURA_S_MAX
from .batch import EnvHost, build_batch, fill_driver_arrays
from .abi import KuraSolverError
from .sim import KuraSim, make_config


class Box:
    """Minimal gymnasium.spaces.Box (gymnasium is not a dependency)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)


class KuraVectorEnv:
    """B SpatialKuramoto environments stepped together on one GPU.

    params:     one reference params dict for every env, or a list of B dicts
                (they must share N, the grid and the spatial kernel; K may
                differ per env).
                Driver-filled arrays (w0, neur_coords, ...) may be given; when
                absent they are drawn as train_aDBS_RL.py:95-112 does, from
                ``numpy.random.RandomState(w0_seed + b)``.
    rand_seeds: per-env ``rand_seed`` (env.py:291); default params' seed + b.
    autoreset:  SB3 DummyVecEnv semantics -- a finished env is reset inside the
                same step() and its last observation is returned in
                ``infos["terminal_observation"]``.
    profile:    time the phases of every autoreset (host draws, parameter
                upload, reset kernel, episode metrics; synchronising) into
                ``self.boundary_times`` -- bench.py --episode.
    on_failure: a solve that fails inside the library (kura.h KURA_F_*:
                max_steps, non-finite state, ...) -- "raise" (default) raises
                KuraSolverError from step()/reset(), as the reference's
                diffeqsolve does (diffrax throw=True, env.py:261-270);
                "reset" reports the env terminated + truncated with
                ``infos["failed_env_ids"]``/``infos["failure_flags"]`` and
                autoresets it.
    """

    metadata = {"render.modes": ["human"]}

    def __init__(self, params, num_envs: int | None = None, device=0, reward_func: str | None = None,
                 w0_seed: int = 228, rand_seeds=None, autoreset: bool = True, max_steps: int = 4096,
                 episode_metrics: bool = False, psd_dt: float = 5e-4, beta_band=(12.5, 21.0),
                 on_failure: str = "raise", profile: bool = False):
        if on_failure not in ("raise", "reset"):
            raise ValueError(f"on_failure={on_failure!r}: expected 'raise' or 'reset'")
        self.on_failure = on_failure
        self.profile = profile
        self.boundary_times: list[dict] = []
        if isinstance(params, dict):
            if num_envs is None:
                raise ValueError("num_envs is required with a single params dict")
            plist = [copy.deepcopy(params) for _ in range(num_envs)]
            if rand_seeds is None:
                rand_seeds = [params["rand_seed"] + b for b in range(num_envs)]
        else:
            plist = [copy.deepcopy(p) for p in params]
            num_envs = len(plist)
        if rand_seeds is not None:
            for p, s in zip(plist, rand_seeds):
                p["rand_seed"] = int(s)
        for b, p in enumerate(plist):
            if p.get("w0") is None or p.get("neur_grid") is None:
                plist[b] = fill_driver_arrays(p, w0_seed=w0_seed + b)
            if reward_func is not None:
                plist[b]["reward_func"] = reward_func
        self.params = plist
        self.num_envs = B = num_envs
        self.hosts, shared = build_batch(plist)
        ep_steps = int(plist[0]["total_episode_len"] / (plist[0]["electrode_width"] + plist[0]["electrode_pause"]))
        self.cfg = make_config(plist[0], B, reward_func=plist[0]["reward_func"], max_steps=max_steps,
                               episode_cap=(ep_steps + 1) * KURA_S_MAX if episode_metrics else 0)
        self.episode_metrics = episode_metrics
        self.psd_dt, self.beta_band = psd_dt, tuple(beta_band)
        self.sim = KuraSim(self.cfg, device)
        self.device = self.sim.device
        self.sim.set_coupling(shared["alpha"].astype(np.float32))
        self.sim.set_env_gain(shared["gain"])                      # per-env K (env.py:264)
        bins = spectral.beta_bins(self.cfg.window, plist[0]["verbose_dt"])
        self.sim.set_spectral(*spectral.twiddles(self.cfg.window, bins))
        self.W, self.N, self.n_elec = self.cfg.window, self.cfg.n_osc, self.cfg.n_elec
        # spaces (env.py:310-315)
        self.single_action_space = Box(-1.0, 1.0, (1,), np.float32)
        self.single_observation_space = Box(-1.5, 1.5, (1, self.W), np.float32)
        self.autoreset = autoreset
        self.steps = np.zeros(B, np.int64)
        self.episode_steps = self.cfg.episode_steps
        self.u = torch.zeros((B, self.n_elec), dtype=torch.float64, device=self.device)
        self._omega = np.zeros((B, self.N), np.float32)
        self._g_stim = np.zeros((B, self.n_elec, self.N))
        self._g_rec = np.zeros((B, max(self.cfg.n_rec, 1), self.N))
        self._was_reset = False

    # ---- gymnasium VectorEnv API --------------------------------------------
    def _draw(self, idx):
        """Host draws of reset() for the envs in idx; uploads only their
        parameters (one kura_set_env_params per contiguous run of envs)."""
        idx = sorted(int(b) for b in idx)
        t0 = time.perf_counter()
        th = np.zeros((self.num_envs, self.N), np.float32)
        for b in idx:
            w0, gs, gr, th0 = self.hosts[b].reset_draws()
            self._omega[b] = w0.astype(np.float32)
            self._g_stim[b] = gs
            self._g_rec[b] = gr
            th[b] = th0.astype(np.float32)
        self._t_draw = time.perf_counter() - t0
        k = 0
        while k < len(idx):
            j = k
            while j + 1 < len(idx) and idx[j + 1] == idx[j] + 1:
                j += 1
            a, b = idx[k], idx[j] + 1
            self.sim.set_env_params(self._omega[a:b], self._g_stim[a:b], self._g_rec[a:b], env0=a)
            k = j + 1
        out = torch.from_numpy(th).to(self.device)
        if self.profile:
            torch.cuda.synchronize(self.device)
        self._t_upload = time.perf_counter() - t0 - self._t_draw
        return out

    def reset(self, seed=None, options=None):
        """env.py:467-614 for every env.  ``seed`` (int or list) reseeds the
        per-env RNG streams before the draws, like np.random.seed."""
        if seed is not None:
            seeds = [seed + b for b in range(self.num_envs)] if np.isscalar(seed) else list(seed)
            for h, s in zip(self.hosts, seeds):
                h.rs.seed(int(s))
        th = self._draw(range(self.num_envs))
        obs = self.sim.reset(th)
        self._check_reset(None)
        self.steps[:] = 0
        self._was_reset = True
        return obs.view(self.num_envs, 1, self.W).clone(), {}

    def step(self, actions):
        """env.py:415-454 for every env; returns (obs (B,1,W), rewards (B,),
        terminated (B,), truncated (B,), infos)."""
        if not self._was_reset:
            raise RuntimeError("reset() must be called before step()")
        a = torch.as_tensor(np.asarray(actions, np.float32) if not torch.is_tensor(actions) else actions,
                            device=self.device, dtype=torch.float32).reshape(self.num_envs, self.n_elec)
        lo, hi = self.cfg.dbs_lo, self.cfg.dbs_hi
        self.u = lo + ((hi - lo) * (a.double() + 1.0)) / 2.0        # env.py:389-393 (for callers)
        obs, rew, done = self.sim.step(a)
        self.steps += 1
        infos: dict = {}
        term_host = self.steps >= self.episode_steps
        terminated = done.bool().clone()
        truncated = torch.zeros_like(terminated)
        failed, fflags = self.sim.failed_envs()          # synchronises: the step's outputs are ready
        if len(failed):
            if self.on_failure == "raise":
                raise KuraSolverError("kura_step", failed.tolist(), fflags.tolist())
            infos["failed_env_ids"] = failed
            infos["failure_flags"] = fflags
            truncated[torch.as_tensor(failed, device=self.device)] = True
            term_host = term_host.copy()
            term_host[failed] = True                     # autoreset keys on the same envs the flags name
        tb = {}
        if term_host.any():
            t0 = time.perf_counter()
            idx = np.nonzero(term_host)[0]
            infos["terminal_env_ids"] = idx
            infos["episode"] = {"l": self.steps[idx].copy()}
            if self.episode_metrics:  # calc_psd_for_simple_eval of the finished episodes (evaluate_HF_DBS.py:106)
                mask = torch.zeros(self.num_envs, dtype=torch.uint8)
                mask[idx] = 1
                bb = self.sim.episode_bbpow(mask, self.psd_dt, self.beta_band)
                infos["episode"]["bbpow"] = bb[torch.as_tensor(idx, device=self.device)].cpu().numpy()
                # per_episode/envelope/{mean,std,cum} of the training callback (custom_callbacks.py:146-148)
                ev = self.sim.episode_envelope_stats(mask)
                infos["episode"]["envelope"] = ev[torch.as_tensor(idx, device=self.device)].cpu().numpy()
            tb["metrics_s"] = time.perf_counter() - t0
        if self.autoreset and term_host.any():
            infos["terminal_observation"] = obs[torch.as_tensor(idx, device=self.device)].clone().view(-1, 1, self.W)
            mask = torch.zeros(self.num_envs, dtype=torch.uint8)
            mask[idx] = 1
            th = self._draw(idx)
            t1 = time.perf_counter()
            self.sim.reset(th, mask.to(self.device))
            self._check_reset(mask)
            if self.profile:
                torch.cuda.synchronize(self.device)
            self.steps[idx] = 0
            tb.update(n_reset=len(idx), host_draw_s=self._t_draw, upload_s=self._t_upload,
                      reset_kernel_s=time.perf_counter() - t1)
        if self.profile and tb:
            self.boundary_times.append(tb)
        return obs.view(self.num_envs, 1, self.W).clone(), rew.clone(), terminated, truncated, infos

    def _check_reset(self, mask):
        if self.on_failure == "raise":
            self.sim.raise_on_failure("kura_reset", None if mask is None else mask.to(self.device))

    # ---- attributes read by the reference's callers ----------------------------
    @property
    def theta_mean(self):
        """True LFP samples of the last step (env.py:444): (B, KURA_S_MAX) + counts."""
        return self.sim.lfp_true, self.sim.nsamp

    @property
    def theta_records(self):
        return self.sim.lfp_rec, self.sim.nsamp

    def get_attr(self, name: str, indices=None):
        """SB3 VecEnv.get_attr for the attributes the reference callers read
        (evaluate_HF_DBS.py:83, custom_callbacks.py:132-134,302)."""
        idx = range(self.num_envs) if indices is None else indices
        if name in ("theta_mean", "theta_records"):
            vals, n = (self.sim.lfp_true if name == "theta_mean" else self.sim.lfp_rec), self.sim.nsamp
            v, n = vals.cpu().numpy(), n.cpu().numpy()
            return [v[i, :n[i]] for i in idx]
        if name == "u":
            u = self.u.cpu().numpy()
            return [list(u[i]) for i in idx]
        if name == "params_dict":
            return [self.params[i] for i in idx]
        if name == "current_step":
            return [int(self.steps[i]) for i in idx]
        raise AttributeError(name)

    def reward_of(self, windows, u0, kind: int = 0):
        """reward_* (env.py:638-688) of given windows (n, W) and first amplitudes u0
        (kind: 1 bbpow_action, 2 temp_const_action, 3 bbpow_threth_action, 0 = config's)."""
        w = torch.as_tensor(np.asarray(windows, np.float64), device=self.device)
        u = torch.as_tensor(np.asarray(u0, np.float32), device=self.device)
        return self.sim.reward_of(w.reshape(-1, self.W), u.reshape(-1), kind)

    def state_dict(self):
        """Checkpointable env state (phases, times, counters, windows)."""
        st = self.sim.get_state()
        st["host_steps"] = self.steps.copy()
        st["rng"] = [h.rs.get_state() for h in self.hosts]
        st["reset_count"] = [h.reset_count for h in self.hosts]
        return st

    def load_state_dict(self, st):
        self.sim.set_state(st)
        self.steps[:] = st["host_steps"]
        for h, s, rc in zip(self.hosts, st["rng"], st["reset_count"]):
            h.rs.set_state(s)
            h.reset_count = rc
        self._was_reset = True

    def close(self):
        self.sim.close()


class SpatialKuramoto:
    """Single-env drop-in for environment/env.py:274 SpatialKuramoto."""

    metadata = {"render.modes": ["human"]}

    def __init__(self, params_dict, save_init=False, device=0):
        if save_init:
            raise NotImplementedError("save_init=True is not supported (the reference itself reads an "
                                      "undefined init_state on the first reset, env.py:594)")
        self.params_dict = params_dict
        self._v = KuraVectorEnv([params_dict], device=device, rand_seeds=[params_dict["rand_seed"]],
                                autoreset=False)
        self._v.sim.capture_rows(True)          # sol_state_: every row of the step (env.py:430,440)
        self.action_space = self._v.single_action_space
        self.observation_space = self._v.single_observation_space
        self.current_step = 0
        self.done = False
        self.reset()

    def reset(self, seed=None, options=None):
        if seed is not None:
            self._v.hosts[0].rs.seed(int(seed))
        obs, info = self._v.reset()
        self.current_step = 0
        self.done = False
        self.theta_state = obs[0].cpu().numpy()
        return self.theta_state.astype(np.float32), {}

    def step(self, action):
        obs, rew, term, trunc, info = self._v.step(np.asarray(action, np.float32).reshape(1, -1))
        self.current_step += 1
        self.done = bool(term[0].item())
        self.u = list(self._v.u[0].cpu().numpy())
        lf, n = self._v.sim.lfp_true[0].cpu().numpy(), int(self._v.sim.nsamp[0].item())
        self.theta_mean = lf[:n]
        self.theta_records = self._v.sim.lfp_rec[0].cpu().numpy()[:n]
        self.theta_state = obs[0].cpu().numpy()
        self.reward_ = float(rew[0].item())
        return self.theta_state.astype(np.float32), self.reward_, self.done, False, {}

    @property
    def sol_state_(self):
        """Every saved phase row of the last step, ys_I then ys_II (env.py:430,440): (nsamp + 1, N) float32."""
        n = int(self._v.sim.nsamp[0].item())
        return self._v.sim.rows[0, :n + 1].cpu().numpy()

    def _reward(self, kind, x_state, action_value):
        assert len(np.asarray(x_state).shape) == 1, "Incorrect dimension of theta_state"
        return float(self._v.reward_of(np.asarray(x_state)[None, :], [action_value[0]], kind)[0].item())

    def reward_bbpow_action(self, x_state, action_value, baseline=False):
        """env.py:638-650"""
        return self._reward(1, x_state, action_value)

    def reward_temp_const_lfp_betafilt_action(self, x_state, action_value, baseline=False):
        """env.py:653-666"""
        return self._reward(2, x_state, action_value)

    def reward_bbpow_threth_action(self, x_state, action_value, baseline=False):
        """env.py:669-688"""
        return self._reward(3, x_state, action_value)

    def render(self, mode="human", close=False):
        pass

    def close(self):
        self._v.close()


__all__ = ["KuraVectorEnv", "SpatialKuramoto", "Box", "EnvHost", "KURA_S_MAX"]
