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
import os
import time
from types import SimpleNamespace

import numpy as np
import torch

from . import spectral
from . import abi
from .abi import KURA_S_MAX
from .batch import EnvHost, build_batch, fill_driver_arrays, fill_driver_arrays_batch, log_temporal_events, reset_draws_batch
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
    autoreset:  reset finished envs automatically.
    autoreset_mode: "same_step" (default; SB3 DummyVecEnv semantics) -- a
                finished env is reset inside the same step() and its last
                observation is returned in ``infos["terminal_observation"]``;
                "next_step" (gymnasium 1.x vector envs' default,
                AutoresetMode.NEXT_STEP) -- the finishing step() returns the
                env's last observation, and the next step() resets it instead
                of stepping it (its action is ignored): reset observation,
                reward 0, terminated/truncated False, ``infos["reset_env_ids"]``.
                Either way each env's reset draws come from its own stream in
                the reference's order, so an env's episodes are the same.
    profile:    time the phases of every autoreset (host draws, parameter
                upload, reset kernel, episode metrics; synchronising) into
                ``self.boundary_times`` -- bench.py --episode.
    on_failure: a solve that fails inside the library (kura.h KURA_F_*:
                max_steps, non-finite state, ...) -- "raise" (default) raises
                KuraSolverError from step()/reset(), as the reference's
                diffeqsolve does (diffrax throw=True, env.py:261-270);
                "reset" reports the env terminated + truncated with
                ``infos["failed_env_ids"]``/``infos["failure_flags"]`` and
                autoresets it; an autoreset whose transient fails is reported
                in ``infos["failed_reset_ids"]`` and retried, up to
                ``max_reset_failures`` times in a row per env, then raises.
    failure_check: "deferred" (default) -- the library's per-env failure
                flags of a launch travel to the host by an asynchronous copy
                into pinned memory and are acted on at the start of the next
                step() / reset() / close() (before its launch), so a step never
                blocks on the device.  A failed env is reported one call late:
                "raise" raises there; "reset" resets it before that call's
                launch and reports the failed episode as truncated in that
                call -- ``infos["reset_before_step_ids"]`` and
                ``infos["reset_before_step_observation"]`` (its last
                observation), ``failed_env_ids``/``failure_flags`` -- so an
                SB3 wrapper closes the episode before counting that call's
                transition (which belongs to the new episode).  In the failing
                call itself the env is not reported done (terminated comes
                from the episode counters, not the kernel's done = 1).
                "eager": every step() synchronises and acts at once (the
                failed env is truncated and autoreset in the same call).
                Either way a solver failure ends the episode as truncated, not
                terminated.
    coupling:   arithmetic of the O(N^2) coupling sums (kura.h
                KURA_COUPLING_*, ``make_config``): "auto" (default; "bf16x3"
                at every N), "bf16x3" or "f32".
    """

    metadata = {"render.modes": ["human"]}

    def __init__(self, params, num_envs: int | None = None, device=0, reward_func: str | None = None,
                 w0_seed: int = 228, rand_seeds=None, autoreset: bool = True, max_steps: int = 4096,
                 episode_metrics: bool = False, psd_dt: float = 5e-4, beta_band=(12.5, 21.0),
                 on_failure: str = "raise", profile: bool = False, failure_check: str = "deferred",
                 max_reset_failures: int = 3, autoreset_mode: str = "same_step", coupling: str = "auto"):
        if autoreset_mode not in ("same_step", "next_step"):
            raise ValueError(f"autoreset_mode={autoreset_mode!r}: expected 'same_step' or 'next_step'")
        self.autoreset_mode = autoreset_mode
        self._next_reset = None     # next_step mode: envs that finished in the last step() (reset in the next)
        if on_failure not in ("raise", "reset"):
            raise ValueError(f"on_failure={on_failure!r}: expected 'raise' or 'reset'")
        if failure_check not in ("deferred", "eager"):
            raise ValueError(f"failure_check={failure_check!r}: expected 'deferred' or 'eager'")
        self.on_failure = on_failure
        self.failure_check = failure_check
        self.max_reset_failures = int(max_reset_failures)
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
        todo = [b for b, p in enumerate(plist) if p.get("w0") is None or p.get("neur_grid") is None]
        if todo:   # train_aDBS_RL.py:95-112, from RandomState(w0_seed + b) per env
            for b, q in zip(todo, fill_driver_arrays_batch([plist[b] for b in todo], [w0_seed + b for b in todo])):
                plist[b] = q
        if reward_func is not None:
            for p in plist:
                p["reward_func"] = reward_func
        self.params = plist
        self.num_envs = B = num_envs
        self.hosts, shared = build_batch(plist)
        ep_steps = int(plist[0]["total_episode_len"] / (plist[0]["electrode_width"] + plist[0]["electrode_pause"]))
        self.cfg = make_config(plist[0], B, reward_func=plist[0]["reward_func"], max_steps=max_steps,
                               episode_cap=(ep_steps + 1) * KURA_S_MAX if episode_metrics else 0,
                               coupling=coupling)
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
        self._alpha = shared["alpha"]                                # float64, env.py:219-229 (kuramoto.alpha)
        self._gain = shared["gain"]
        # gymnasium Env.reset(seed) only seeds the env's own np_random, which
        # SpatialKuramoto never draws from (env.py:471): kept for callers
        self.np_random = [None] * B
        # deferred failure flags: pinned host copies of the last step's and the
        # last autoreset's per-env flags, and the events that complete them
        self._pend = None          # (flags_pinned, event, reset_mask or None, reset_flags_pinned)
        self._pend_ignore = None   # envs whose step flags of the pending launch do not count (bool mask):
                                   # next_step resets (step discarded) and envs reported truncated
        self._trunc_next = None    # next_step + deferred: (env ids, last obs) to report truncated after the launch
        self._reset_fail_runs = np.zeros(B, np.int64)   # consecutive failed resets per env
        self._pending_gain = {}    # env -> float32(K/N) of a set_attr'd params_dict, applied at its next reset
        self._omega = np.zeros((B, self.N), np.float32)
        self._g_stim = np.zeros((B, self.n_elec, self.N))
        self._g_rec = np.zeros((B, max(self.cfg.n_rec, 1), self.N))
        self._theta0 = np.zeros((B, self.N))      # init_state of each env's last reset (env.py:594-598)
        self._was_reset = False

    # ---- gymnasium VectorEnv API --------------------------------------------
    def _draw(self, idx):
        """Host draws of reset() for the envs in idx; uploads only their
        parameters (one kura_set_env_params per contiguous run of envs)."""
        idx = sorted(int(b) for b in idx)
        t0 = time.perf_counter()
        for b in idx:   # K of a set_attr'd params_dict: the reset builds KuramotoJAX with it (env.py:570-572)
            if b in self._pending_gain:
                self._gain[b] = self._pending_gain.pop(b)
                self.sim.set_env_gain(self._gain[b:b + 1], env0=b)
        th = np.zeros((self.num_envs, self.N), np.float32)
        if idx:
            w0, gs, gr, th0 = reset_draws_batch([self.hosts[b] for b in idx])
            for b in idx:
                self._log_events(b)
            self._omega[idx] = w0.astype(np.float32)
            self._g_stim[idx] = gs
            self._g_rec[idx] = gr
            self._theta0[idx] = th0
            th[idx] = th0.astype(np.float32)
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

    def _log_events(self, b):
        log_temporal_events(self.params[b], self.hosts[b])           # env.py:559-562

    def reset(self, seed=None, options=None):
        """env.py:467-614 for every env.  ``seed`` (int or list) seeds each
        env's gymnasium ``np_random`` only (env.py:471 super().reset(seed)); the
        reference's draws come from the global NumPy RNG, which reset(seed)
        does not touch, so they continue their streams."""
        if seed is not None:
            seeds = [seed + b for b in range(self.num_envs)] if np.isscalar(seed) else list(seed)
            self.np_random = [np.random.default_rng(int(x)) for x in seeds]
        infos: dict = {}
        # deferred flags of the last step() (a failure there raises here in
        # "raise" mode, as the reference's failing diffeqsolve would have)
        pre_failed, pre_flags, pre_rfail, _ = self._take_pending()
        if self.on_failure == "raise" and (len(pre_failed) or len(pre_rfail)):
            self._act_on_failures(pre_failed, pre_flags, pre_rfail, {}, "kura_step (previous call)")
        if len(pre_failed):
            infos["failed_env_ids"], infos["failure_flags"] = pre_failed, pre_flags
        th = self._draw(range(self.num_envs))
        obs = self.sim.reset(th)
        self._check_reset(None, infos)
        self.steps[:] = 0
        self._next_reset = None
        self._trunc_next = None
        self._was_reset = True
        return obs.view(self.num_envs, 1, self.W).clone(), infos

    def _failures_now(self):
        """Flags of the last launch, synchronously."""
        return self.sim.failed_envs()

    def _take_pending(self):
        """The deferred flags of the previous step (and of its autoreset):
        (failed env ids, flags, failed reset ids, ended), ``ended[i]``: the
        episode of failed env i already ended in that call -- same_step mode:
        it was autoreset there; next_step mode: it finished there and is reset
        in this call -- so it needs its failure reported, not a reset
        (ADVICE r04).  Waits only for the copies, which the previous launches
        completed long ago in a stepping loop."""
        if self._pend is None:
            self._pend_ignore = None
            return np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, bool)
        fl, ev, rmask, rfl = self._pend
        self._pend = None
        ev.synchronize()
        f = fl.numpy().copy()
        if self._pend_ignore is not None:
            f[self._pend_ignore] = 0      # steps discarded in that launch (reset instead, or already reported)
        self._pend_ignore = None
        idx = np.nonzero(f)[0]
        ended = np.zeros(len(idx), bool)
        if rmask is not None and self.autoreset_mode == "same_step":
            ended |= rmask[idx]
        if self._next_reset is not None:
            ended |= self._next_reset[idx]
        ridx = np.zeros(0, np.int64)
        if rmask is not None:
            rf = np.where(rmask, rfl.numpy(), 0)
            ridx = np.nonzero(rf)[0]
            self._reset_fail_runs[rmask & (rf == 0)] = 0      # those resets succeeded
        return idx, f[idx], ridx, ended

    def _ignore_flags(self, envs):
        """The pending launch's step flags of these envs do not count."""
        m = np.zeros(self.num_envs, bool)
        m[np.asarray(envs, np.int64)] = True
        self._pend_ignore = m if self._pend_ignore is None else (self._pend_ignore | m)

    def _stash_flags(self, reset_mask=None):
        """Start the asynchronous copy of the last launch's flags (step, or the
        autoreset that followed it) into pinned memory."""
        if self._pend is None or reset_mask is None:
            fl = torch.empty(self.num_envs, dtype=torch.int32, pin_memory=True)
            fl.copy_(self.sim.flags, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._pend = (fl, ev, None, None)
        else:
            fl, _, _, _ = self._pend
            rfl = torch.empty(self.num_envs, dtype=torch.int32, pin_memory=True)
            rfl.copy_(self.sim.flags, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._pend = (fl, ev, reset_mask, rfl)

    def step(self, actions):
        """env.py:415-454 for every env; returns (obs (B,1,W), rewards (B,),
        terminated (B,), truncated (B,), infos)."""
        if not self._was_reset:
            raise RuntimeError("reset() must be called before step()")
        a = torch.as_tensor(np.asarray(actions, np.float32) if not torch.is_tensor(actions) else actions,
                            device=self.device, dtype=torch.float32).reshape(self.num_envs, self.n_elec)
        infos: dict = {}
        # the previous step's deferred failures (and its autoreset's), before this launch
        pre_failed, pre_flags, pre_rfail, pre_ended = self._take_pending()
        if len(pre_failed) or len(pre_rfail):
            self._act_on_failures(pre_failed, pre_flags, pre_rfail, infos, "kura_step (previous call)", pre_ended)
        trunc = self._trunc_next   # next_step mode: failed episodes to end in this call's outputs
        self._trunc_next = None
        lo, hi = self.cfg.dbs_lo, self.cfg.dbs_hi
        x, y = self.cfg.act_lo, self.cfg.act_hi
        self.u = lo + ((hi - lo) * (a.double() - x)) / (y - x)      # env.py:389-393 (for callers)
        pre_metrics = None
        if trunc is not None and self.episode_metrics:
            # the truncated episodes ended with the failed call: their metrics
            # come from the episode buffer as it stands before this launch (whose
            # step for them is discarded) may append to it
            m = torch.zeros(self.num_envs, dtype=torch.uint8)
            m[trunc[0]] = 1
            pre_metrics = (self.sim.episode_bbpow(m, self.psd_dt, self.beta_band).clone(),
                           self.sim.episode_envelope_stats(m).clone())
        obs, rew, done = self.sim.step(a)
        self.steps += 1
        if trunc is not None:
            self.steps[trunc[0]] -= 1      # the discarded step is not part of the truncated episode
        # next_step mode: the envs that finished in the previous call are reset
        # in this one -- their step above is discarded (the reset below
        # overwrites its state and outputs)
        nxt = None
        if self._next_reset is not None and self._next_reset.any():
            nxt = np.nonzero(self._next_reset)[0]
            self.steps[nxt] = 0
        self._next_reset = None
        term_host = self.steps >= self.episode_steps
        # episode ends from the counters (== the kernel's done for every env whose
        # step succeeded; the kernel also sets done = 1 for a failed env, which is
        # reported as a truncation instead, below or one call later)
        terminated = torch.from_numpy(term_host).to(self.device, non_blocking=True)
        truncated = torch.zeros_like(terminated)
        if "reset_before_step_ids" in infos:
            truncated[torch.as_tensor(infos["reset_before_step_ids"], device=self.device)] = True
        if trunc is not None:
            # next_step mode (gymnasium NEXT_STEP): the failed episode ends in this
            # call with its last observation, truncated, reward 0; its step in this
            # launch (from an undefined state) is discarded and the next call
            # resets it, as for an episode that ends on its own
            tids, last_obs = trunc
            d = torch.as_tensor(tids, device=self.device)
            obs[d] = last_obs
            rew[d] = 0.0
            truncated[d] = True
            terminated[d] = False
            term_host = term_host.copy()
            term_host[tids] = True
            if self.failure_check != "eager":
                self._ignore_flags(tids)
        if self.failure_check == "eager":
            failed, fflags = self._failures_now()         # synchronises: the step's outputs are ready
            if nxt is not None:                           # discarded steps do not fail an episode
                keep = ~np.isin(failed, nxt)
                failed, fflags = failed[keep], fflags[keep]
            if len(failed):
                if self.on_failure == "raise":
                    raise KuraSolverError("kura_step", failed.tolist(), fflags.tolist())
                infos["failed_env_ids"] = failed
                infos["failure_flags"] = fflags
                truncated[torch.as_tensor(failed, device=self.device)] = True
                term_host = term_host.copy()
                term_host[failed] = True                 # autoreset keys on the same envs the flags name
        else:
            self._stash_flags()
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
                # per_episode/envelope/{mean,std,cum} of the training callback (custom_callbacks.py:146-148)
                ev = self.sim.episode_envelope_stats(mask)
                if pre_metrics is not None:
                    td = torch.as_tensor(trunc[0], device=self.device)
                    bb, ev = bb.clone(), ev.clone()
                    bb[td], ev[td] = pre_metrics[0][td], pre_metrics[1][td]
                infos["episode"]["bbpow"] = bb[torch.as_tensor(idx, device=self.device)].cpu().numpy()
                infos["episode"]["envelope"] = ev[torch.as_tensor(idx, device=self.device)].cpu().numpy()
            tb["metrics_s"] = time.perf_counter() - t0
        if nxt is not None:   # next_step mode: reset observation, reward 0, not done
            infos["reset_env_ids"] = nxt
            mask = torch.zeros(self.num_envs, dtype=torch.uint8)
            mask[nxt] = 1
            th = self._draw(nxt)
            t1 = time.perf_counter()
            self.sim.reset(th, mask.to(self.device))
            nxt_dev = torch.as_tensor(nxt, device=self.device)
            rew[nxt_dev] = 0.0
            terminated[nxt_dev] = False
            truncated[nxt_dev] = False
            if self.failure_check == "eager":
                self._check_reset(mask)
            else:
                self._stash_flags(reset_mask=mask.numpy().astype(bool))
                self._ignore_flags(nxt)
            if self.profile:
                torch.cuda.synchronize(self.device)
            tb.update(n_reset=len(nxt), host_draw_s=self._t_draw, upload_s=self._t_upload,
                      reset_kernel_s=time.perf_counter() - t1)
        if self.autoreset and self.autoreset_mode == "next_step" and term_host.any():
            self._next_reset = term_host.copy()
        if self.autoreset and self.autoreset_mode == "same_step" and term_host.any():
            infos["terminal_observation"] = obs[torch.as_tensor(idx, device=self.device)].clone().view(-1, 1, self.W)
            mask = torch.zeros(self.num_envs, dtype=torch.uint8)
            mask[idx] = 1
            th = self._draw(idx)
            t1 = time.perf_counter()
            self.sim.reset(th, mask.to(self.device))
            if self.failure_check == "eager":
                self._check_reset(mask)
            else:
                self._stash_flags(reset_mask=mask.numpy().astype(bool))
            if self.profile:
                torch.cuda.synchronize(self.device)
            self.steps[idx] = 0
            tb.update(n_reset=len(idx), host_draw_s=self._t_draw, upload_s=self._t_upload,
                      reset_kernel_s=time.perf_counter() - t1)
        if self.profile and tb:
            self.boundary_times.append(tb)
        return obs.view(self.num_envs, 1, self.W).clone(), rew.clone(), terminated, truncated, infos

    def _check_reset(self, mask, infos=None):
        """Synchronous check of a reset launch: raise, or (on_failure='reset')
        report the failed envs and reset them again."""
        if self.on_failure == "raise":
            self.sim.raise_on_failure("kura_reset", None if mask is None else mask.to(self.device))
            return
        ridx, _ = self.sim.failed_envs(None if mask is None else mask.to(self.device))
        ok = np.ones(self.num_envs, bool) if mask is None else mask.cpu().numpy().astype(bool)
        ok[ridx] = False
        self._reset_fail_runs[ok] = 0                    # a confirmed reset ends a run of failures
        if len(ridx):
            self._retry_resets(ridx, infos if infos is not None else {})

    def _retry_resets(self, ridx, infos):
        self._reset_fail_runs[ridx] += 1
        over = ridx[self._reset_fail_runs[ridx] > self.max_reset_failures]
        if len(over):
            raise KuraSolverError("kura_reset (repeated)", over.tolist(), [0] * len(over))
        infos["failed_reset_ids"] = np.asarray(ridx)
        mask = torch.zeros(self.num_envs, dtype=torch.uint8)
        mask[ridx] = 1
        th = self._draw(ridx)
        self.sim.reset(th, mask.to(self.device))
        self.steps[ridx] = 0
        self._check_reset(mask, infos)

    def _act_on_failures(self, failed, fflags, rfailed, infos, what, ended=None):
        """Deferred failures of the previous call: raise, or report them and
        end those episodes.  same_step mode: reset the envs now (before this
        step's launch), their last observation in
        ``infos["reset_before_step_observation"]``; next_step mode: this
        call reports them truncated with their last observation and the next
        call resets them (``_trunc_next``).  Envs whose episode already ended
        in the previous call (``ended``: autoreset there, or queued for this
        call's next_step reset) are only reported -- resetting them again
        would take an extra draw from their RNG stream."""
        if self.on_failure == "raise":
            if len(failed):
                raise KuraSolverError(what, failed.tolist(), fflags.tolist())
            raise KuraSolverError("kura_reset (autoreset of the previous call)", rfailed.tolist(),
                                  [0] * len(rfailed))
        live = np.zeros(0, np.int64)
        if len(failed):
            infos["failed_env_ids"] = failed
            infos["failure_flags"] = fflags
            live = failed if ended is None else failed[~np.asarray(ended, bool)]
        if len(live) and self.autoreset_mode == "next_step":
            # the last observation, before this call's launch overwrites the buffer
            self._trunc_next = (live, self.sim.obs[torch.as_tensor(live, device=self.device)].clone())
            live = np.zeros(0, np.int64)
        elif len(live):
            # the failed episodes end here (truncated): their last observation,
            # before the reset below overwrites the buffer
            infos["reset_before_step_ids"] = live
            infos["reset_before_step_observation"] = \
                self.sim.obs[torch.as_tensor(live, device=self.device)].clone().view(-1, 1, self.W)
        redo = np.union1d(live, rfailed).astype(np.int64)
        if len(rfailed):
            self._reset_fail_runs[rfailed] += 1
            over = rfailed[self._reset_fail_runs[rfailed] > self.max_reset_failures]
            if len(over):
                raise KuraSolverError("kura_reset (repeated)", over.tolist(), [0] * len(over))
            infos["failed_reset_ids"] = rfailed
        if len(redo):
            mask = torch.zeros(self.num_envs, dtype=torch.uint8)
            mask[redo] = 1
            th = self._draw(redo)
            self.sim.reset(th, mask.to(self.device))
            self.steps[redo] = 0
            self._check_reset(mask, infos)

    # ---- attributes read by the reference's callers ----------------------------
    @property
    def theta_mean(self):
        """True LFP samples of the last step (env.py:444): (B, KURA_S_MAX) + counts."""
        return self.sim.lfp_true, self.sim.nsamp

    @property
    def theta_records(self):
        return self.sim.lfp_rec, self.sim.nsamp

    def kuramoto_view(self, b):
        """The attributes of env b's KuramotoJAX / SimpleDBS (env.py:191-249,
        :61-156) that callers read, e.g. ``env.kuramoto.dbs.conductances``
        (explore_kuramoto_dynamics.ipynb cell 13): the last reset's values."""
        p, h = self.params[b], self.hosts[b]
        gs, gr = h._conductances() if hasattr(h, "_conductances") else (None, None)
        dbs = SimpleNamespace(conductances=None if gs is None else [np.array(g) for g in gs],
                              rec_conductances=None if gr is None else [np.array(g) for g in gr],
                              elec_coords=getattr(h, "elec_coords", p["elec_coords"]),
                              rec_coords=getattr(h, "rec_coords", p["rec_coords"]))
        return SimpleNamespace(K=p["K"], n_neurons=p["num_oscillators"], w0=getattr(h, "w0", None),
                               grid_size=p["grid_size"], neur_coords=p["neur_coords"], neur_grid=p["neur_grid"],
                               spatial_kernel=p["spatial_kernel"], alpha=self._alpha, dbs=dbs,
                               pulse=np.zeros(p["num_oscillators"]))

    # attributes of SpatialKuramoto (env.py:277-614) served by get_attr
    _HOST_ATTRS = ("reset_count", "temporal_events", "spatial_events", "elec_coords", "rec_coords",
                   "encapsulation_coeff", "w0_without_locus")

    def get_attr(self, name: str, indices=None):
        """SB3 VecEnv.get_attr for the attributes of the reference env that its
        callers read (evaluate_HF_DBS.py:83, custom_callbacks.py:107-134,302,
        the notebooks' env.kuramoto.dbs.conductances) and the bookkeeping
        reset() sets (env.py:473-476, :600-603)."""
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
        if name == "current_time":
            t = self.sim.times()
            return [float(t[i]) for i in idx]
        if name == "theta_state":
            o = self.sim.obs.cpu().numpy()
            return [o[i][None, :].astype(np.float32) for i in idx]
        if name == "done":
            return [bool(self.steps[i] >= self.episode_steps) for i in idx]
        if name == "kuramoto":
            return [self.kuramoto_view(i) for i in idx]
        if name == "kw0":                                           # env.py:601
            return [self.hosts[i].w0 for i in idx]
        if name == "kneur_grid":                                    # env.py:602
            return [self.params[i]["neur_grid"] for i in idx]
        if name == "kgrid_size":                                    # env.py:603
            return [self.params[i]["grid_size"] for i in idx]
        if name in self._HOST_ATTRS:
            return [getattr(self.hosts[i], name) for i in idx]
        if name == "np_random":
            return [self.np_random[i] for i in idx]
        if name == "init_state":                                    # env.py:594-598 (float64 draws)
            return [self._theta0[i].copy() for i in idx]
        if name == "theta_record_transient":                        # env.py:611
            tr = getattr(self.sim, "lfp_transient", None)
            if tr is None:
                raise AttributeError(_UNSERVED[name])
            v = tr.cpu().numpy()
            naive = self.sim.cfg.rec_kernel == 0
            return [v[i].astype(np.float32) if naive else v[i].copy() for i in idx]
        if name in _UNSERVED:
            raise AttributeError(_UNSERVED[name])
        raise AttributeError(name)

    # params the batch is built around: they cannot change on a running handle
    _FIXED_KEYS = ("num_oscillators", "grid_size", "neur_coords", "neur_grid", "spatial_kernel", "wavelet_amp",
                   "wavelet_steepness", "electrode_width", "electrode_pause", "verbose_dt", "observe_wind_counts",
                   "total_episode_len", "transient_state_len", "reward_func", "recording_kernel",
                   "dbs_action_bounds")

    def set_attr(self, name: str, value, indices=None) -> None:
        """SB3 VecEnv.set_attr.  ``params_dict`` takes effect from the next
        reset of those envs, which is where the reference reads it: reset()
        rebuilds KuramotoJAX(K=params_dict['K'], ...) (env.py:570-572) and
        forward() then uses that fixed self.K (env.py:264).  Per-reset draws,
        drift/spatial settings, conductances and K follow the new dict from
        that reset on; keys the batch's shared setup is built on (N, grid,
        window, timing, reward, kernels) must stay equal or ValueError is
        raised.  Other names raise AttributeError."""
        idx = list(range(self.num_envs)) if indices is None else list(indices)
        if name != "params_dict":
            raise AttributeError(f"set_attr({name!r}) is not supported on the batched env")
        for i in idx:
            old = self.params[i]
            for k in self._FIXED_KEYS:
                a, b = old.get(k), value.get(k)
                same = np.array_equal(np.asarray(a), np.asarray(b)) if isinstance(a, (list, tuple, np.ndarray)) \
                    else a == b
                if not same:
                    raise ValueError(f"set_attr('params_dict'): {k!r} cannot change on a running batch "
                                     "(build a new env)")
            newp = copy.deepcopy(value)
            for k in ("w0", "w0_without_locus", "locus_without_w0", "locus_mask"):
                if newp.get(k) is None:
                    newp[k] = old.get(k)
            self.params[i] = newp
            self.hosts[i].p = newp
            kn = np.float32(newp["K"] / newp["num_oscillators"])
            if kn != self._gain[i]:
                self._pending_gain[i] = kn          # applied by _draw at env i's next reset
            else:
                self._pending_gain.pop(i, None)

    def reward_of(self, windows, u0, kind: int = 0):
        """reward_* (env.py:638-688) of given 1-D windows (n, L) of any length L
        and first amplitudes u0 (kind: 1 bbpow_action, 2 temp_const_action,
        3 bbpow_threth_action, 0 = config's).  The beta bins follow len(x)
        as in the reference (utils.py:21-27)."""
        w = torch.as_tensor(np.asarray(windows, np.float64), device=self.device)
        w = w.reshape(1, -1) if w.ndim == 1 else w.reshape(w.shape[0], -1)
        # the action as the caller gives it, in float64 (the step kernels take
        # the float32 actions of the action space, env.py:310-312)
        u = torch.as_tensor(np.asarray(u0, np.float64), device=self.device).reshape(-1)
        L = int(w.shape[1])
        kind = kind or self.cfg.reward_kind
        bins = spectral.beta_bins(L, self.params[0]["verbose_dt"])
        ct, st = spectral.twiddles(L, bins) if len(bins) else (np.zeros((0, L)), np.zeros((0, L)))
        if kind == 2 and L <= self.cfg.padlen:
            raise ValueError(f"The length of the input vector x must be greater than padlen, which is "
                             f"{self.cfg.padlen}.")
        return self.sim.reward_n(w, u, kind, ct, st)

    def state_dict(self):
        """Checkpointable env state (phases, times, counters, windows)."""
        st = self.sim.get_state()
        # the arithmetic the trajectories were computed in: a run continues
        # bit for bit only in the same one (kura.h KURA_COUPLING_*)
        st["coupling"] = abi.coupling_of(self.sim.cfg)
        st["host_steps"] = self.steps.copy()
        st["rng"] = [h.rs.get_state() for h in self.hosts]
        st["reset_count"] = [h.reset_count for h in self.hosts]
        return st

    def load_state_dict(self, st):
        have = abi.coupling_of(self.sim.cfg)
        if st.get("coupling", have) != have:
            raise ValueError(f"state_dict was saved with coupling={st['coupling']!r}; this env runs {have!r} "
                             "(pass coupling= to KuraVectorEnv)")
        self.sim.set_state(st)
        self.steps[:] = st["host_steps"]
        for h, s, rc in zip(self.hosts, st["rng"], st["reset_count"]):
            h.rs.set_state(s)
            h.reset_count = rc
        self._was_reset = True

    def close(self):
        """Releases the handle; in "raise" mode a failure of the last step()
        that was not yet read (deferred flags) is raised after the release."""
        pre_failed, pre_flags, pre_rfail, _ = self._take_pending() if self._pend is not None else ([], [], [], [])
        self.sim.close()
        if self.on_failure == "raise" and (len(pre_failed) or len(pre_rfail)):
            self._act_on_failures(np.asarray(pre_failed), np.asarray(pre_flags), np.asarray(pre_rfail), {},
                                  "kura_step (last call before close)")


_SOL_STATE_AFTER_RESET = ("sol_state after reset() is the transient's rows (env.py:610), kept only on request: "
                          "call venv.sim.capture_transient_rows(True) before reset() (SpatialKuramoto does); "
                          "or read the state (its last row) with get_state()['y']")

# reference attributes the GPU path does not keep (no caller in the reference
# reads them: aDBS_RL/, the notebooks); asking for them raises with the reason
_UNSERVED = {
    "theta_record_transient": "theta_record_transient (env.py:611: the LFP of all 3999 transient rows) is kept only "
                              "on request: call venv.sim.capture_transient(True) before reset() (SpatialKuramoto "
                              "does); otherwise the reset kernel forms only the last W samples, the observation "
                              "window (DESIGN.md section 5, K2)",
}


class SpatialKuramoto:
    """Single-env drop-in for environment/env.py:274 SpatialKuramoto."""

    metadata = {"render.modes": ["human"]}

    def __init__(self, params_dict, save_init=False, device=0):
        if save_init:
            raise NotImplementedError("save_init=True is not supported (the reference itself reads an "
                                      "undefined init_state on the first reset, env.py:594)")
        self.params_dict = params_dict
        self._v = KuraVectorEnv([params_dict], device=device, rand_seeds=[params_dict["rand_seed"]],
                                autoreset=False, failure_check="eager")
        self._v.sim.capture_rows(True)          # sol_state_: every row of the step (env.py:430,440)
        self._v.sim.capture_transient(True)     # theta_record_transient (env.py:611)
        self._v.sim.capture_transient_rows(True)  # sol_state after reset() (env.py:610)
        self.action_space = self._v.single_action_space
        self.observation_space = self._v.single_observation_space
        self.current_step = 0
        self.done = False
        self.reset()

    def reset(self, seed=None, options=None):
        """env.py:467-614.  ``seed`` seeds gymnasium's np_random only
        (env.py:471): the draws continue the env's global-RNG stream."""
        obs, info = self._v.reset(seed=None if seed is None else [int(seed)])
        self._n_on = None
        self.current_step = 0
        self.done = False
        self.theta_state = obs[0].cpu().numpy()
        return self.theta_state.astype(np.float32), {}

    def step(self, action):
        t0 = self._v.sim.times()[0]           # current_time before the step: the ON grid's length
        p = self.params_dict
        self._n_on = len(np.arange(t0, t0 + p["electrode_width"], p["verbose_dt"]))   # env.py:426-428
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

    # reference attributes set by __init__/reset()/step() (env.py:289, :473-476,
    # :600-603) and the model objects (env.py:570-593): served by the batch
    @property
    def reset_count(self):
        return self._v.hosts[0].reset_count

    @property
    def current_time(self):
        return self._v.get_attr("current_time")[0]

    @property
    def kuramoto(self):
        return self._v.kuramoto_view(0)

    @property
    def np_random(self):
        return self._v.np_random[0]

    def __getattr__(self, name):
        # only reached for names not set on the instance / class
        if name.startswith("_"):
            raise AttributeError(name)
        if name in ("kw0", "kneur_grid", "kgrid_size") + KuraVectorEnv._HOST_ATTRS:
            return self._v.get_attr(name)[0]
        # (a property that raises AttributeError lands here: keep its reason)
        if name == "sol_state":
            raise AttributeError(_SOL_STATE_AFTER_RESET)
        if name in _UNSERVED:
            raise AttributeError(_UNSERVED[name])
        raise AttributeError(f"'SpatialKuramoto' object has no attribute {name!r}")

    @property
    def sol_state_(self):
        """Every saved phase row of the last step, ys_I then ys_II (env.py:430,440): (nsamp + 1, N) float32."""
        n = int(self._v.sim.nsamp[0].item())
        return self._v.sim.rows[0, :n + 1].cpu().numpy()

    @property
    def sol_state(self):
        """The last solve's rows (env.py:429,439, :610): after step(), the
        stim-OFF solve's ys_II (sol_state_ from the duplicated I/II boundary
        row on); after reset(), the transient's rows (T, N), T =
        len(arange(0, transient_state_len, verbose_dt)), the last being the
        state (kura_set_transient_rows)."""
        if getattr(self, "_n_on", None) is None:
            rt = getattr(self._v.sim, "rows_transient", None)
            if rt is None:
                raise AttributeError(_SOL_STATE_AFTER_RESET)
            return rt[0].cpu().numpy()
        return self.sol_state_[self._n_on:]

    @property
    def init_state(self):
        """theta0 of the last reset (env.py:594-598), float64."""
        return self._v.get_attr("init_state")[0]

    @property
    def theta_record_transient(self):
        """calc_lfp(sol_state[:-1]) of the last reset's transient (env.py:611): (T-1,)"""
        return self._v.get_attr("theta_record_transient")[0]

    def _reward(self, kind, x_state, action_value):
        """Any 1-D length (the bins follow len(x_state), utils.py:21-27)."""
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
