"""Stable-Baselines3-shaped VecEnv over a KuraVectorEnv.

The reference's callers drive single ``SpatialKuramoto`` envs through SB3's
``DummyVecEnv`` (+ ``Monitor``): ``train_aDBS_RL.py:116-193``,
``aDBS_RL/evaluate_HF_DBS.py:33-119``, ``aDBS_RL/agents/custom_callbacks.py``.
``KuraSB3VecEnv`` gives those call shapes to a GPU batch without importing
stable-baselines3 (not installed here): it is duck-typed to SB3's ``VecEnv``

* ``reset() -> obs`` (NumPy, ``(n_envs, 1, W)`` float32);
* ``step(actions) -> (obs, rewards, dones, infos)`` with ``rewards`` float32
  (DummyVecEnv's ``buf_rews``), ``dones`` bool, ``infos`` a list of per-env
  dicts; a finished env is reset inside the same step and its last
  observation is ``info["terminal_observation"]``; ``info["TimeLimit.truncated"]``
  is set for ends that are not terminations;
* ``step_async``/``step_wait``, ``get_attr``/``set_attr``/``env_method``,
  ``env_is_wrapped``, ``seed``, ``close``;
* ``monitor=True`` adds SB3 ``Monitor``'s episode summary
  ``info["episode"] = {"r": round(sum of rewards, 6), "l": length, "t": seconds}``
  and makes ``env_is_wrapped(Monitor)`` report True, which switches
  ``evaluate_policy_`` (evaluate_HF_DBS.py:56,97-101) to the Monitor branch.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .vec_env import KuraVectorEnv

_REWARD_METHODS = ("reward_bbpow_action", "reward_temp_const_lfp_betafilt_action", "reward_bbpow_threth_action")


class KuraSB3VecEnv:
    def __init__(self, venv: KuraVectorEnv, monitor: bool = True, obs_buffers: int | None = None):
        if not venv.autoreset:
            raise ValueError("KuraSB3VecEnv needs a KuraVectorEnv with autoreset=True (DummyVecEnv semantics)")
        self.venv = venv
        self.num_envs = venv.num_envs
        self.observation_space = venv.single_observation_space
        self.action_space = venv.single_action_space
        self.render_mode = None
        self.monitor = monitor
        self._actions = None
        self._ep_rew = np.zeros(self.num_envs, np.float64)
        self._ep_len = np.zeros(self.num_envs, np.int64)
        self._t0 = np.full(self.num_envs, time.time())
        self._pin = None   # pinned host staging for the per-step device -> host copies
        # None (default): a fresh observation array every step, DummyVecEnv's
        # semantics (callers may keep references).  obs_buffers = k (opt-in):
        # a ring of k preallocated host arrays -- an array stays valid for
        # k - 1 further steps (SB3's rollout collection and evaluate_policy
        # copy or drop it after one) -- at ~half the host cost per step (no
        # page faults of a new (B, 1, W) array, tools/sb3_bench.py)
        self.obs_buffers = obs_buffers
        self._ring, self._ring_i = None, 0

    # ---- VecEnv core ----------------------------------------------------------
    def reset(self):
        obs, _ = self.venv.reset()
        self._ep_rew[:] = 0.0
        self._ep_len[:] = 0
        self._t0[:] = time.time()
        return obs.cpu().numpy()

    def step_async(self, actions) -> None:
        a = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, -1)
        self._actions = a

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        a, self._actions = self._actions, None
        obs, rew, term, trunc, info = self.venv.step(a)
        obs_h, rew64, term_h, trunc_h = self._to_host(obs, rew, term, trunc)
        dones = term_h | trunc_h
        infos = [{} for _ in range(self.num_envs)]
        # deferred failure checks: an env whose previous step failed was reset
        # before this launch -- its episode ended (truncated) before this
        # step's transition, which is the first of its new episode
        pre = info.get("reset_before_step_ids", np.zeros(0, np.int64))
        if len(pre):
            pobs = info["reset_before_step_observation"].cpu().numpy()
            now = time.time()
            for j, b in enumerate(pre):
                d = infos[b]
                d["terminal_observation"] = pobs[j]
                d["TimeLimit.truncated"] = True
                if self.monitor:
                    d["episode"] = {"r": round(float(self._ep_rew[b]), 6), "l": int(self._ep_len[b]),
                                    "t": round(now - self._t0[b], 6)}
                self._ep_rew[b] = 0.0
                self._ep_len[b] = 0
                self._t0[b] = now
        self._ep_rew += rew64
        self._ep_len += 1
        ended = info.get("terminal_env_ids", np.zeros(0, np.int64))
        if len(ended):
            tobs = info["terminal_observation"].cpu().numpy()
            now = time.time()
            for j, b in enumerate(ended):
                d = infos[b]
                d["terminal_observation"] = tobs[j]
                d["TimeLimit.truncated"] = bool(trunc_h[b] and not term_h[b])   # DummyVecEnv.step_wait
                if self.monitor:
                    d["episode"] = {"r": round(float(self._ep_rew[b]), 6), "l": int(self._ep_len[b]),
                                    "t": round(now - self._t0[b], 6)}
                for k in ("bbpow", "envelope"):
                    if k in info.get("episode", {}):
                        d.setdefault("episode_metrics", {})[k] = info["episode"][k][j]
                self._ep_rew[b] = 0.0
                self._ep_len[b] = 0
                self._t0[b] = now
        for k, key in (("failed_env_ids", "failure_flags"),):
            if k in info:
                for b, f in zip(info[k], info[key]):
                    infos[b]["failure_flags"] = int(f)
        return obs_h, rew64.astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _to_host(self, obs, rew, term, trunc):
        """All four step outputs to the host in one synchronisation: async
        copies into pinned staging buffers, then a fresh obs array per step
        (DummyVecEnv returns copies) made by a multithreaded torch copy --
        a pageable `.cpu()` of the (B, 1, W) float32 observation costs ~4x
        more at B=4096 (tools/sb3_bench.py)."""
        if self._pin is None or self._pin[0].shape != obs.shape:
            self._pin = (torch.empty(obs.shape, dtype=obs.dtype, pin_memory=True),
                         torch.empty(rew.shape, dtype=rew.dtype, pin_memory=True),
                         torch.empty(term.shape, dtype=torch.bool, pin_memory=True),
                         torch.empty(trunc.shape, dtype=torch.bool, pin_memory=True))
        po, pr, pt, pu = self._pin
        po.copy_(obs, non_blocking=True)
        pr.copy_(rew, non_blocking=True)
        pt.copy_(term, non_blocking=True)
        pu.copy_(trunc, non_blocking=True)
        torch.cuda.current_stream(obs.device).synchronize()
        if self.obs_buffers:
            if self._ring is None or self._ring[0].shape != po.shape:
                self._ring = [torch.zeros(po.shape, dtype=po.dtype) for _ in range(max(2, self.obs_buffers))]
            out = self._ring[self._ring_i]
            self._ring_i = (self._ring_i + 1) % len(self._ring)
            out.copy_(po)
        else:
            out = po.clone()
        return out.numpy(), pr.numpy().copy(), pt.numpy().copy(), pu.numpy().copy()

    def close(self) -> None:
        self.venv.close()

    def seed(self, seed=None):
        """SB3 VecEnv.seed: env i is reset with seed + i at the next reset, which
        seeds only its gymnasium np_random (env.py:471); the reference's draws
        come from the global NumPy RNG and continue their streams."""
        if seed is None:
            return [None] * self.num_envs
        self.venv.np_random = [np.random.default_rng(int(seed) + i) for i in range(self.num_envs)]
        return [int(seed) + i for i in range(self.num_envs)]

    # ---- attribute / method access ------------------------------------------------
    def _idx(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    def get_attr(self, attr_name: str, indices=None):
        return self.venv.get_attr(attr_name, self._idx(indices))

    def set_attr(self, attr_name: str, value, indices=None) -> None:
        """SB3 VecEnv.set_attr: takes effect (KuraVectorEnv.set_attr) or raises."""
        self.venv.set_attr(attr_name, value, self._idx(indices))

    def env_method(self, method_name: str, *args, indices=None, **kwargs):
        """The reference env methods callers invoke through a VecEnv: the three
        reward functions (env.py:638-688, aDBS_RL/agents/simple_dbs.py:83-90)."""
        if method_name not in _REWARD_METHODS:
            raise AttributeError(f"env_method({method_name!r}) is not supported on the batched env")
        kind = 1 + _REWARD_METHODS.index(method_name)
        x_state, action_value = args[0], args[1]
        idx = self._idx(indices)
        w = np.repeat(np.asarray(x_state, np.float64)[None, :], len(idx), axis=0)
        u = np.full(len(idx), float(action_value[0]), np.float32)
        return [float(v) for v in self.venv.reward_of(w, u, kind).cpu().numpy()]

    def env_is_wrapped(self, wrapper_class, indices=None):
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        return [self.monitor and name == "Monitor"] * len(self._idx(indices))

    def get_images(self):
        return [None] * self.num_envs

    def render(self, mode=None):
        return None

    @property
    def unwrapped(self):
        return self

    def __len__(self):
        return self.num_envs


__all__ = ["KuraSB3VecEnv"]
