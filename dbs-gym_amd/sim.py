"""KuraSim: thin owner of one libkura handle (one GPU, B environments).

This is the seam the reference's ``KuramotoJAX.forward`` + ``SpatialKuramoto``
step/reset occupy (env.py:260-271, :415-454, :467-614).  All numerics run in
the HIP library; this class only allocates PyTorch-ROCm tensors (storage),
passes raw device pointers through the C ABI and maps error codes to the
reference's exception types.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import abi
from . import spectral
from .abi import KURA_S_MAX, KuraConfig, KuraSolverError, check, ptr


def auto_part_osc(n_osc: int, n_envs: int, n_cu: int = 256) -> int:
    """Split-group part width (N > 1024) for a handle of n_envs envs: the
    largest of 1024 / 512 / 256 oscillators per workgroup that still gives
    every compute unit of the GPU (MI355X: 256) a workgroup, 256 otherwise;
    0 (not split) for N <= 1024."""
    if n_osc <= 1024:
        return 0
    groups = -(-n_envs // 16)
    for part in (1024, 512, 256):
        if n_osc % part == 0 and groups * (n_osc // part) >= n_cu:
            return part
    return 256 if n_osc % 256 == 0 else 1024


def make_config(params: dict, n_envs: int, reward_func: str | None = None, max_steps: int = 4096,
                episode_cap: int = 0, part_osc: int = 0, coupling: str = "auto") -> KuraConfig:
    """Build the C config from a reference params dict (env.py:277-338).
    part_osc: split-group part width for N > 1024 (0 = 1024; auto_part_osc
    picks one that fills the GPU).  coupling: the arithmetic of the O(N^2)
    coupling sums (kura.h KURA_COUPLING_*): "bf16x3" (three-way bf16 splits on
    the bf16 MFMA, fp32 accumulation), "f32" (fmaf chain on the fp32 MFMA) or
    "auto" (bf16x3 at every N); results depend on it bit for bit."""
    p = params
    step_len = p["electrode_width"] + p["electrode_pause"]                      # env.py:294
    wind_len = step_len * p["observe_wind_counts"]                               # env.py:296
    W = int(wind_len / p["verbose_dt"])                                          # env.py:297
    if p["transient_state_len"] < wind_len:                                      # env.py:303-304
        raise ValueError("Transient state should be longer than RL agent observation window!")
    rf = reward_func if reward_func is not None else p.get("reward_func")
    if rf not in abi.REWARD_KINDS:                                               # env.py:323-330
        raise ValueError("Wrong reward function!")
    if p["recording_kernel"] not in abi.REC_KERNELS:                            # env.py:333-338
        raise ValueError("Wrong recording kernel function!")
    if len(p["electrode_amps"]) != len(p["elec_coords"]):                        # env.py:91
        raise AssertionError("Number of amplitudes is not equal to number of electrode coordinates!")
    c = KuraConfig()
    c.abi_version = abi.KURA_ABI_VERSION
    c.n_osc = int(p["num_oscillators"])
    c.n_envs = int(n_envs)
    c.window = W
    c.n_elec = len(p["elec_coords"])
    c.n_rec = len(p["rec_coords"])
    c.rec_kernel = abi.REC_KERNELS[p["recording_kernel"]]
    c.reward_kind = abi.REWARD_KINDS[rf]
    c.episode_steps = int(p["total_episode_len"] / step_len)                     # env.py:300
    c.max_steps = int(max_steps)
    bins = spectral.beta_bins(W, p["verbose_dt"])
    if len(bins) > abi.KURA_MAX_BINS:
        raise ValueError("too many beta-band bins")
    c.n_bins = len(bins)
    for i, b in enumerate(bins):
        c.bins[i] = int(b)
    b, a, zi = spectral.butter_bandpass(p["verbose_dt"])
    c.padlen = 3 * max(len(a), len(b))                                           # scipy filtfilt default
    for i in range(5):
        c.bw_b[i] = float(b[i])
        c.bw_a[i] = float(a[i])
    for i in range(4):
        c.bw_zi[i] = float(zi[i])
    c.dt = float(p["verbose_dt"])
    c.width = float(p["electrode_width"])
    c.pause = float(p["electrode_pause"])
    c.transient_len = float(p["transient_state_len"])
    c.act_lo, c.act_hi = -1.0, 1.0                                               # env.py:309
    c.dbs_lo, c.dbs_hi = float(p["dbs_action_bounds"][0]), float(p["dbs_action_bounds"][1])
    c.rtol = c.atol = np.float32(1e-5)                                           # env.py:249
    c.kn = np.float32(p["K"] / p["num_oscillators"])                            # env.py:264
    c.dt0 = np.float32(0.05)                                                     # env.py:267
    c.episode_cap = int(episode_cap)
    if part_osc and (part_osc not in (256, 512, 1024) or c.n_osc % part_osc):
        raise ValueError(f"part_osc={part_osc}: expected 256, 512 or 1024 dividing num_oscillators={c.n_osc}")
    c.part_osc = int(part_osc)
    if coupling not in abi.COUPLINGS:
        raise ValueError(f"coupling={coupling!r}: expected one of {sorted(abi.COUPLINGS)}")
    c.coupling = abi.COUPLINGS[coupling]
    if W < KURA_S_MAX:   # kura_create: a step's samples never wrap the ring twice
        raise ValueError(f"observation window of {W} samples: libkura needs at least {KURA_S_MAX} "
                         "(observe_wind_counts * (electrode_width + electrode_pause) / verbose_dt)")
    return c


class KuraSim:
    """B environments on one GPU behind libkura."""

    def __init__(self, cfg: KuraConfig, device: torch.device | str | int = 0, lib_path: str | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("KuraSim needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "there is no CPU implementation of the step path")
        self.lib = abi.load_library(lib_path)
        self.cfg = cfg
        self.device = torch.device("cuda", torch.device(device).index if not isinstance(device, int) else device)
        if self.device.index is None:
            self.device = torch.device("cuda", 0)
        self.B, self.N, self.W = cfg.n_envs, cfg.n_osc, cfg.window
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)), "kura_create")
        self._h = h
        dev = self.device
        B = self.B
        self.obs = torch.zeros((B, self.W), dtype=torch.float32, device=dev)
        self.reward = torch.zeros(B, dtype=torch.float64, device=dev)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.lfp_true = torch.zeros((B, KURA_S_MAX), dtype=torch.float32, device=dev)
        self.lfp_rec = torch.zeros((B, KURA_S_MAX), dtype=torch.float64, device=dev)
        self.nsamp = torch.zeros(B, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(B, dtype=torch.int32, device=dev)   # KURA_F_* of the last launch

    # ---- setup --------------------------------------------------------------
    def set_coupling(self, alpha: np.ndarray) -> None:
        a = np.ascontiguousarray(alpha, dtype=np.float32)
        if a.shape != (self.N, self.N):
            raise ValueError(f"alpha shape {a.shape} != ({self.N}, {self.N})")
        check(self.lib, self.lib.kura_set_coupling(self._h, a.ctypes.data), "kura_set_coupling")

    def set_env_params(self, omega, g_stim, g_rec=None, env0: int = 0) -> None:
        w = np.ascontiguousarray(omega, dtype=np.float32)
        n = w.shape[0]
        gs = np.ascontiguousarray(g_stim, dtype=np.float64)
        gr = None if g_rec is None else np.ascontiguousarray(g_rec, dtype=np.float64)
        check(self.lib, self.lib.kura_set_env_params(self._h, env0, n, w.ctypes.data, gs.ctypes.data,
                                                     None if gr is None else gr.ctypes.data),
              "kura_set_env_params")

    def set_env_gain(self, kn, env0: int = 0) -> None:
        """Per-env coupling gain float32(K_b / N) (env.py:264)."""
        k = np.ascontiguousarray(kn, dtype=np.float32).reshape(-1)
        check(self.lib, self.lib.kura_set_env_gain(self._h, env0, len(k), k.ctypes.data), "kura_set_env_gain")

    def set_spectral(self, cos_tab, sin_tab) -> None:
        c = np.ascontiguousarray(cos_tab, dtype=np.float64)
        s = np.ascontiguousarray(sin_tab, dtype=np.float64)
        check(self.lib, self.lib.kura_set_spectral(self._h, c.ctypes.data, s.ctypes.data), "kura_set_spectral")

    # ---- hot path -------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, theta0: torch.Tensor, mask: torch.Tensor | None = None, check_errors: bool = False):
        """check_errors: synchronise and raise KuraSolverError if a masked
        env's transient failed (otherwise see ``flags`` / ``raise_on_failure``)."""
        th = theta0.to(self.device, torch.float32).contiguous()
        if th.shape != (self.B, self.N):
            raise ValueError("theta0 must be (B, N)")
        m = None if mask is None else mask.to(self.device, torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_reset(self._h, ptr(m), ptr(th), ptr(self.obs), self._stream()),
                  "kura_reset")
            check(self.lib, self.lib.kura_get_env_flags(self._h, ptr(self.flags), self._stream()),
                  "kura_get_env_flags")
        self._keep = (th, m)  # keep inputs alive until the stream consumes them
        if check_errors:
            self.raise_on_failure("kura_reset", m)
        return self.obs

    def step(self, action: torch.Tensor, check_errors: bool = False):
        """One reference step() for every env.  Failed solves never throw in
        the library (kura.h KURA_F_*): the env reports done = 1 and its bits
        land in ``flags``; check_errors=True synchronises and raises
        KuraSolverError as the reference's diffeqsolve would."""
        a = action.to(self.device, torch.float32).contiguous()
        if a.numel() != self.B * self.cfg.n_elec:
            raise ValueError("action must have B * n_elec elements")
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_step(self._h, ptr(a), ptr(self.obs), ptr(self.reward), ptr(self.done),
                                               ptr(self.lfp_true), ptr(self.lfp_rec), ptr(self.nsamp),
                                               self._stream()), "kura_step")
            check(self.lib, self.lib.kura_get_env_flags(self._h, ptr(self.flags), self._stream()),
                  "kura_get_env_flags")
        self._keep = (a,)
        if check_errors:
            self.raise_on_failure("kura_step")
        return self.obs, self.reward, self.done

    def capture_rows(self, on: bool = True) -> None:
        """Keep every saved phase row of each step in ``self.rows`` (B, KURA_S_MAX+1, N):
        rows 0..nsamp of env b are the reference's sol_state_ (env.py:430,440)."""
        if on:
            self.rows = torch.zeros((self.B, KURA_S_MAX + 1, self.N), dtype=torch.float32, device=self.device)
            check(self.lib, self.lib.kura_set_row_capture(self._h, ptr(self.rows)), "kura_set_row_capture")
        else:
            check(self.lib, self.lib.kura_set_row_capture(self._h, None), "kura_set_row_capture")
            self.rows = None

    def capture_transient(self, on: bool = True) -> None:
        """Keep theta_record_transient (env.py:611) of every reset in
        ``self.lfp_transient`` (B, T-1) float64: the LFP of each transient row
        but the last, T = len(np.arange(0, transient_state_len, verbose_dt));
        its last W columns are the reset's observation window.  Costs the LFP
        of T-1-W more rows per reset (kura_set_transient_capture)."""
        if on:
            T = len(np.arange(0.0, self.cfg.transient_len, self.cfg.dt))
            self.lfp_transient = torch.zeros((self.B, T - 1), dtype=torch.float64, device=self.device)
            check(self.lib, self.lib.kura_set_transient_capture(self._h, ptr(self.lfp_transient)),
                  "kura_set_transient_capture")
        else:
            check(self.lib, self.lib.kura_set_transient_capture(self._h, None), "kura_set_transient_capture")
            self.lfp_transient = None

    def capture_transient_rows(self, on: bool = True) -> None:
        """Keep the transient's rows of every reset in ``self.rows_transient``
        (B, T, N) float32 -- the reference's sol_state after reset()
        (env.py:610), row T-1 being the new state; T*N*4 bytes per env (16 MB
        at N=1024), so meant for a few envs (kura_set_transient_rows)."""
        if on:
            T = self.lib.kura_transient_len(self._h)
            if T <= 0:
                check(self.lib, T if T < 0 else -1, "kura_transient_len")
            self.rows_transient = torch.zeros((self.B, T, self.N), dtype=torch.float32, device=self.device)
            check(self.lib, self.lib.kura_set_transient_rows(self._h, ptr(self.rows_transient)),
                  "kura_set_transient_rows")
        else:
            check(self.lib, self.lib.kura_set_transient_rows(self._h, None), "kura_set_transient_rows")
            self.rows_transient = None

    def failed_envs(self, mask: torch.Tensor | None = None):
        """(env indices, KURA_F_* bits) of the envs whose last launch failed (synchronises)."""
        f = self.flags.cpu().numpy()
        if mask is not None:
            f = np.where(mask.cpu().numpy().astype(bool), f, 0)
        idx = np.nonzero(f)[0]
        return idx, f[idx]

    def raise_on_failure(self, what: str = "kura_step", mask: torch.Tensor | None = None) -> None:
        idx, fl = self.failed_envs(mask)
        if len(idx):
            raise KuraSolverError(what, idx.tolist(), fl.tolist())

    def reward_of(self, window: torch.Tensor, u0: torch.Tensor, kind: int = 0) -> torch.Tensor:
        w = window.to(self.device, torch.float64).contiguous()
        u = u0.to(self.device, torch.float32).contiguous()
        n = w.shape[0]
        out = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_reward(self._h, int(kind), ptr(w), ptr(u), ptr(out), n, self._stream()),
                  "kura_reward")
        return out

    # ---- episode evaluation metric (aDBS_RL/evaluate_HF_DBS.py:122-135) ---------
    def psd_bbpow(self, signals, psd_dt: float = 5e-4, beta=(12.5, 21.0)) -> np.ndarray:
        """calc_psd_for_simple_eval of arbitrary float32 signals (list of 1-D arrays)."""
        n = len(signals)
        ld = max(2, max(len(x) for x in signals))
        buf = np.zeros((n, ld), np.float32)
        for j, x in enumerate(signals):
            buf[j, :len(x)] = x
        lens = torch.tensor([len(x) for x in signals], dtype=torch.int32, device=self.device)
        sig = torch.from_numpy(buf).to(self.device)
        out = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_psd_bbpow(self._h, ptr(sig), ptr(lens), ld, n, float(psd_dt),
                                                    float(beta[0]), float(beta[1]), ptr(out), self._stream()),
                  "kura_psd_bbpow")
        return out.cpu().numpy()

    def envelope_stats(self, signals) -> np.ndarray:
        """[n, 3] mean, std(ddof=1), sum of |hilbert(x)| per float32 signal
        (custom_callbacks.py:146-148, utils.py:835-836)."""
        n = len(signals)
        ld = max(1, max((len(x) for x in signals), default=1))
        buf = np.zeros((n, ld), np.float32)
        for j, x in enumerate(signals):
            buf[j, :len(x)] = x
        lens = torch.tensor([len(x) for x in signals], dtype=torch.int32, device=self.device)
        sig = torch.from_numpy(buf).to(self.device)
        out = torch.empty((n, 3), dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_envelope_stats(self._h, ptr(sig), ptr(lens), ld, n, ptr(out),
                                                         self._stream()), "kura_envelope_stats")
        return out.cpu().numpy()

    def episode_envelope_stats(self, mask: torch.Tensor | None = None) -> torch.Tensor:
        """The same statistics of each env's running episode (config.episode_cap > 0): [B, 3]."""
        out = torch.empty((self.B, 3), dtype=torch.float64, device=self.device)
        m = None if mask is None else mask.to(self.device, torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_episode_envelope_stats(self._h, ptr(m), ptr(out), self._stream()),
                  "kura_episode_envelope_stats")
        return out

    def episode_bbpow(self, mask: torch.Tensor | None = None, psd_dt: float = 5e-4,
                      beta=(12.5, 21.0)) -> torch.Tensor:
        """The same metric of each env's running episode (config.episode_cap > 0)."""
        out = torch.empty(self.B, dtype=torch.float64, device=self.device)
        m = None if mask is None else mask.to(self.device, torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_episode_bbpow(self._h, ptr(m), float(psd_dt), float(beta[0]),
                                                        float(beta[1]), ptr(out), self._stream()),
                  "kura_episode_bbpow")
        self._keep_mask = m
        return out

    # ---- state ------------------------------------------------------------------
    def get_state(self) -> dict:
        B, N, W = self.B, self.N, self.W
        st = dict(y=np.empty((B, N), np.float32), t=np.empty(B, np.float64), step=np.empty(B, np.int32),
                  ring=np.empty((B, W), np.float64), wpos=np.empty(B, np.int32))
        check(self.lib, self.lib.kura_get_state(self._h, st["y"].ctypes.data, st["t"].ctypes.data,
                                                st["step"].ctypes.data, st["ring"].ctypes.data,
                                                st["wpos"].ctypes.data), "kura_get_state")
        st["spec"] = np.empty((B, 2 * self.cfg.n_bins), np.float64)   # R1/R3 spectral accumulators
        check(self.lib, self.lib.kura_get_spec(self._h, st["spec"].ctypes.data), "kura_get_spec")
        return st

    def times(self) -> np.ndarray:
        """current_time of every env (env.py:431,441,609), float64 (syncs)."""
        t = np.empty(self.B, np.float64)
        check(self.lib, self.lib.kura_get_state(self._h, None, t.ctypes.data, None, None, None), "kura_get_state")
        return t

    def reward_n(self, x: torch.Tensor, u0: torch.Tensor, kind: int, cos_tab, sin_tab) -> torch.Tensor:
        """reward_* of n windows of any length L (x: (n, L)); twiddles (n_bins, L)
        for that length (kura_reward_n)."""
        w = x.to(self.device, torch.float64).contiguous()
        u = u0.to(self.device, torch.float64).contiguous()
        n, L = w.shape
        ct = torch.as_tensor(np.ascontiguousarray(cos_tab, np.float64), device=self.device)
        st = torch.as_tensor(np.ascontiguousarray(sin_tab, np.float64), device=self.device)
        nb = int(ct.shape[0]) if ct.ndim == 2 else 0
        out = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.kura_reward_n(self._h, int(kind), ptr(w), L, L, n, ptr(ct) if nb else None,
                                                   ptr(st) if nb else None, nb, ptr(u), ptr(out), self._stream()),
                  "kura_reward_n")
        self._keep_rw = (w, u, ct, st)
        return out

    def set_state(self, st: dict) -> None:
        arrs = [np.ascontiguousarray(st["y"], np.float32), np.ascontiguousarray(st["t"], np.float64),
                np.ascontiguousarray(st["step"], np.int32), np.ascontiguousarray(st["ring"], np.float64),
                np.ascontiguousarray(st["wpos"], np.int32)]
        check(self.lib, self.lib.kura_set_state(self._h, *[a.ctypes.data for a in arrs]), "kura_set_state")
        if "spec" in st:   # exact accumulators of a checkpoint (else re-formed from the ring)
            sp = np.ascontiguousarray(st["spec"], np.float64)
            if sp.shape != (self.B, 2 * self.cfg.n_bins):
                raise ValueError(f"spec shape {sp.shape} != ({self.B}, {2 * self.cfg.n_bins})")
            check(self.lib, self.lib.kura_set_spec(self._h, sp.ctypes.data), "kura_set_spec")

    def stats(self) -> np.ndarray:
        out = np.zeros(abi.KURA_NSTATS, np.int64)
        check(self.lib, self.lib.kura_get_stats(self._h, out.ctypes.data, len(out)), "kura_get_stats")
        return out

    def stamps(self) -> np.ndarray:
        out = np.zeros((8, 24), np.uint64)   # [wave][KURA_NSTAMP]
        check(self.lib, self.lib.kura_get_stamps(self._h, out.ctypes.data), "kura_get_stamps")
        return out

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.kura_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
