"""ctypes wrapper of the CPU oracle (oracle/libkura_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import c_double, c_int, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libkura_oracle.so")
S_MAX = 32


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "kura_oracle.c")):
        subprocess.run(["make", "-C", HERE, "-B" if force else "all"], check=True, capture_output=True)
    return LIB


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        # KURA_ORACLE_LIB: an alternative build of the same source, e.g. the
        # ASan+UBSan one of `make -C oracle asan` (run with its runtime preloaded)
        alt = os.environ.get("KURA_ORACLE_LIB")
        if not alt:
            build()
        L = ctypes.CDLL(alt or LIB)
        L.oracle_create.restype = c_void_p
        L.oracle_create.argtypes = [c_void_p, c_void_p]
        L.oracle_destroy.argtypes = [c_void_p]
        L.oracle_reset.restype = c_int
        L.oracle_reset.argtypes = [c_void_p, c_int] + [c_void_p] * 14
        L.oracle_reset_ex.restype = c_int
        L.oracle_reset_ex.argtypes = [c_void_p, c_int] + [c_void_p] * 15
        L.oracle_step.restype = c_int
        L.oracle_step.argtypes = [c_void_p, c_int] + [c_void_p] * 20
        L.oracle_spec_init.argtypes = [c_void_p, c_int] + [c_void_p] * 4
        L.oracle_solve_rows.restype = c_int
        L.oracle_solve_rows.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]
        L.oracle_rhs.argtypes = [c_void_p] * 5
        L.oracle_reward.restype = c_double
        L.oracle_reward.argtypes = [c_void_p, c_void_p, c_double, c_void_p, c_void_p]
        L.oracle_r64_f32.restype = ctypes.c_float
        L.oracle_r64_f32.argtypes = [c_void_p, c_int]
        L.oracle_r64_f64.restype = c_double
        L.oracle_r64_f64.argtypes = [c_void_p, c_int]
        L.oracle_arange.restype = c_int
        L.oracle_arange.argtypes = [c_double, c_double, c_double, c_void_p, c_int]
        for n in ("oracle_sincos", "oracle_sincos_fmod2pi"):
            getattr(L, n).argtypes = [c_void_p, c_void_p, c_void_p, c_int]
        for n in ("oracle_fmod2pi", "oracle_inv_fifth_root"):
            getattr(L, n).argtypes = [c_void_p, c_void_p, c_int]
        L.oracle_gemm_chain.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int]
        L.oracle_lfp.argtypes = [c_void_p] * 5
        L.oracle_set_gain.restype = c_int
        L.oracle_set_gain.argtypes = [c_void_p, c_int, c_void_p]
        L.oracle_set_split.restype = c_int
        L.oracle_set_split.argtypes = [c_void_p, c_int]
        L.oracle_split_prepare.restype = c_void_p
        L.oracle_split_prepare.argtypes = [c_void_p, c_int, c_int]
        L.oracle_split_gemm_rows.argtypes = [c_void_p, c_void_p, c_int, c_void_p]
        L.oracle_split_free.argtypes = [c_void_p]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class Oracle:
    """Mirror of KuraSim on the CPU (same state layout, host arrays)."""

    def __init__(self, cfg, alpha: np.ndarray):
        self.cfg = cfg
        self.N, self.B, self.W = cfg.n_osc, cfg.n_envs, cfg.window
        self._alpha = np.ascontiguousarray(alpha, np.float32)
        self._ctx = lib().oracle_create(ctypes.byref(cfg), self._alpha.ctypes.data)
        if not self._ctx:
            raise ValueError(f"oracle_create refused the config (coupling={cfg.coupling}, n_osc={cfg.n_osc})")
        B, N, W = self.B, self.N, self.W
        self.y = np.zeros((B, N), np.float32)
        self.t = np.zeros(B, np.float64)
        self.step_count = np.zeros(B, np.int32)
        self.ring = np.zeros((B, W), np.float64)
        self.wpos = np.zeros(B, np.int32)
        self.spec = np.zeros((B, 2 * cfg.n_bins), np.float64)   # R1/R3 spectral accumulators
        self.stats = np.zeros(4, np.int64)
        self.flags = np.zeros(B, np.int32)   # KURA_F_* of the last reset/step per env

    def set_env_params(self, omega, g_stim, g_rec=None):
        self.omega = np.ascontiguousarray(omega, np.float32)
        self.g_stim = np.ascontiguousarray(g_stim, np.float64)
        nr = max(self.cfg.n_rec, 1)
        self.g_rec = (np.ascontiguousarray(g_rec, np.float64) if g_rec is not None
                      else np.zeros((self.B, nr, self.N), np.float64))

    def set_split(self, on=True):
        """Override the config's coupling arithmetic (kura.h KURA_COUPLING_*):
        on = KURA_COUPLING_BF16X3 (three-way bf16 splits on the bf16 MFMA's
        exact accumulation), off = KURA_COUPLING_F32 (the fp32 fmaf chain).
        The constructor already follows cfg.coupling (kura_coupling_of)."""
        rc = lib().oracle_set_split(self._ctx, int(bool(on)))
        if rc != 0:
            raise ValueError(f"oracle_set_split: rc={rc} (N <= 1024, N % 16 == 0)")

    def set_gain(self, kn):
        self._kn = np.ascontiguousarray(kn, np.float32).reshape(-1)
        assert lib().oracle_set_gain(self._ctx, len(self._kn), self._kn.ctypes.data) == 0

    def set_spectral(self, ctab, stab):
        self.ctab = np.ascontiguousarray(ctab, np.float64)
        self.stab = np.ascontiguousarray(stab, np.float64)

    def reset(self, theta0, transient=False):
        """oracle_reset; transient=True also returns theta_record_transient
        (B, T-1) float64, the LFP of every transient row but the last
        (env.py:611, oracle_reset_ex)."""
        th = np.ascontiguousarray(theta0, np.float32)
        obs = np.zeros((self.B, self.W), np.float32)
        T = len(arange(0.0, self.cfg.transient_len, self.cfg.dt))
        tr = np.zeros((self.B, T - 1), np.float64) if transient else None
        rc = lib().oracle_reset_ex(self._ctx, self.B, _p(self.omega), _p(self.g_rec), _p(th), _p(self.y), _p(self.t),
                                   _p(self.step_count), _p(self.ring), _p(self.wpos), _p(obs), _p(self.stats),
                                   _p(self.flags), _p(getattr(self, "ctab", None)), _p(getattr(self, "stab", None)),
                                   _p(self.spec) if hasattr(self, "ctab") else None, _p(tr))
        assert rc == 0
        return (obs, tr) if transient else obs

    def step(self, action):
        a = np.ascontiguousarray(action, np.float32)
        B = self.B
        out = dict(obs=np.zeros((B, self.W), np.float32), reward=np.zeros(B, np.float64),
                   done=np.zeros(B, np.uint8), lfp_true=np.zeros((B, S_MAX), np.float32),
                   lfp_rec=np.zeros((B, S_MAX), np.float64), nsamp=np.zeros(B, np.int32))
        rc = lib().oracle_step(self._ctx, B, _p(self.omega), _p(self.g_stim), _p(self.g_rec), _p(self.ctab),
                               _p(self.stab), _p(a), _p(self.y), _p(self.t), _p(self.step_count), _p(self.ring),
                               _p(self.wpos), _p(out["obs"]), _p(out["reward"]), _p(out["done"]),
                               _p(out["lfp_true"]), _p(out["lfp_rec"]), _p(out["nsamp"]), _p(self.stats),
                               _p(self.flags), _p(self.spec))
        assert rc == 0
        return out

    def state(self):
        return dict(y=self.y.copy(), t=self.t.copy(), step=self.step_count.copy(), ring=self.ring.copy(),
                    wpos=self.wpos.copy(), spec=self.spec.copy())

    def set_state(self, st):
        """kura_set_state (+ kura_set_spec when st has 'spec'; else the
        accumulators are re-formed from the ring, as the library does)."""
        self.y[...] = st["y"]
        self.t[...] = st["t"]
        self.step_count[...] = st["step"]
        self.ring[...] = st["ring"]
        self.wpos[...] = st["wpos"]
        if "spec" in st:
            self.spec[...] = st["spec"]
        elif self.cfg.reward_kind != 2 and self.cfg.n_bins:
            lib().oracle_spec_init(ctypes.byref(self.cfg), self.B, _p(self.ring), _p(self.ctab), _p(self.stab),
                                   _p(self.spec))

    def solve_rows(self, omega, pulse, ts, y0):
        N = self.N
        ts = np.ascontiguousarray(ts, np.float64)
        rows = np.zeros((len(ts), N), np.float32)
        st = np.zeros(4, np.int64)
        rc = lib().oracle_solve_rows(self._ctx, _p(np.ascontiguousarray(omega, np.float32)),
                                     _p(None if pulse is None else np.ascontiguousarray(pulse, np.float32)),
                                     _p(ts), len(ts), _p(np.ascontiguousarray(y0, np.float32)), _p(rows), _p(st))
        assert rc == 0
        return rows, st

    def rhs(self, y, omega, pulse):
        f = np.zeros(self.N, np.float32)
        lib().oracle_rhs(self._ctx, _p(np.ascontiguousarray(y, np.float32)), _p(np.ascontiguousarray(omega, np.float32)),
                         _p(np.ascontiguousarray(pulse, np.float32)), _p(f))
        return f

    def lfp(self, row, g_rec=None):
        """(naive fp32 LFP, records) of one saved row (env.py:396-412)."""
        n = ctypes.c_float()
        r = ctypes.c_double()
        gr = (np.zeros((max(self.cfg.n_rec, 1), self.N)) if g_rec is None
              else np.ascontiguousarray(g_rec, np.float64))
        lib().oracle_lfp(self._ctx, _p(np.ascontiguousarray(row, np.float32)), _p(gr), ctypes.byref(n),
                         ctypes.byref(r))
        return n.value, r.value

    def reward(self, window, u0):
        return lib().oracle_reward(ctypes.byref(self.cfg), _p(np.ascontiguousarray(window, np.float64)), float(u0),
                                   _p(self.ctab), _p(self.stab))

    def close(self):
        if self._ctx:
            lib().oracle_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sincos(x):
    x = np.ascontiguousarray(x, np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().oracle_sincos(_p(x), _p(s), _p(c), x.size)
    return s, c


def mfma_bf16_dot16(x_bf16, y_bf16, c):
    """oracle_mfma_bf16_dot16 for each row of x, y (uint16 bf16 bit patterns,
    (n, 16)) and c (n,): the gfx950 bf16 MFMA's accumulation model."""
    L = lib()
    f = L.oracle_mfma_bf16_dot16
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float]
    x = np.ascontiguousarray(x_bf16, np.uint16)
    y = np.ascontiguousarray(y_bf16, np.uint16)
    return np.array([f(x[t].ctypes.data, y[t].ctypes.data, float(c[t])) for t in range(len(c))], np.float32)


def mfma_bf16_dot16_i64(x_bf16, y_bf16, c):
    """oracle_mfma_bf16_dot16_i64: the same model in int64 arithmetic."""
    L = lib()
    f = L.oracle_mfma_bf16_dot16_i64
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float]
    x = np.ascontiguousarray(x_bf16, np.uint16)
    y = np.ascontiguousarray(y_bf16, np.uint16)
    return np.array([f(x[t].ctypes.data, y[t].ctypes.data, float(c[t])) for t in range(len(c))], np.float32)


def split_bf16_chain(xp, ap, i64=False):
    """oracle_split_bf16_chain (or its int64 form) for each row: xp, ap
    (n, 3, K) bf16 bit patterns of the split operands -> (n,) float32 (the
    split GEMM's accumulation)."""
    L = lib()
    f = L.oracle_split_bf16_chain_i64 if i64 else L.oracle_split_bf16_chain
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    xp = np.ascontiguousarray(xp, np.uint16)
    ap = np.ascontiguousarray(ap, np.uint16)
    K = xp.shape[2]
    return np.array([f(xp[t].ctypes.data, ap[t].ctypes.data, K) for t in range(len(xp))], np.float32)


def split_gemm_rows(X, A):
    """oracle_split_gemm_rows: Y[r][i] = split-bf16 chain of X[r] and A[i] in
    the K1 k order (per 16-deep block the even k form the first MFMA
    product group, the odd k the second), vectorised across outputs."""
    L = lib()
    X = np.ascontiguousarray(X, np.float32)
    A = np.ascontiguousarray(A, np.float32)
    (R, K), N = X.shape, A.shape[0]
    prep = L.oracle_split_prepare(A.ctypes.data, N, K)
    if not prep:
        raise ValueError("split_gemm_rows: N % 8 and K % 16 must be 0")
    Y = np.empty((R, N), np.float32)
    L.oracle_split_gemm_rows(prep, X.ctypes.data, R, Y.ctypes.data)
    L.oracle_split_free(prep)
    return Y


def sincos_fmod2pi(x):
    """sin, cos of fmod(x, 2pi_f) as the RHS takes them (kdm_sincos_fmod2pi)"""
    x = np.ascontiguousarray(x, np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().oracle_sincos_fmod2pi(_p(x), _p(s), _p(c), x.size)
    return s, c


def fmod2pi(x):
    x = np.ascontiguousarray(x, np.float32)
    r = np.empty_like(x)
    lib().oracle_fmod2pi(_p(x), _p(r), x.size)
    return r


def inv_fifth_root(x):
    x = np.ascontiguousarray(x, np.float32)
    r = np.empty_like(x)
    lib().oracle_inv_fifth_root(_p(x), _p(r), x.size)
    return r


def gemm_chain(X, A):
    X = np.ascontiguousarray(X, np.float32)
    A = np.ascontiguousarray(A, np.float32)
    M, K = X.shape
    N = A.shape[0]
    Y = np.empty((M, N), np.float32)
    lib().oracle_gemm_chain(_p(X), _p(A), _p(Y), M, N, K)
    return Y


def r64_f32(x):
    x = np.ascontiguousarray(x, np.float32)
    return lib().oracle_r64_f32(_p(x), x.size)


def r64_f64(x):
    x = np.ascontiguousarray(x, np.float64)
    return lib().oracle_r64_f64(_p(x), x.size)


def arange(start, stop, step, cap=100000):
    out = np.empty(cap, np.float64)
    n = lib().oracle_arange(start, stop, step, _p(out), cap)
    return out[:n]
