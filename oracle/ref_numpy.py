"""NumPy restatement of the reference's step()/reset() *op sequence* -- the
CPU baseline of BASELINE.md section 3.  TEST INFRASTRUCTURE: only bench.py's
cpu_baseline leg and tests/ use it; the product path never imports oracle/.

Unlike oracle/kura_oracle.c (the bit-exact twin of the HIP kernels, with the
factorised coupling), this module evaluates the right-hand side exactly as
KuramotoJAX.dynamics writes it (environment/env.py:252-256, jnp read as
NumPy, fp32):

    theta  = fmod(y, 2*pi)
    dtheta = w0 + K/N * sum(alpha * sin(theta - tile(theta, (N, 1)).T), axis=1) + pulse

i.e. N^2 sines per evaluation, which is what the reference pays per RHS on a
CPU.  The solver is the same diffrax 0.7.0 Dopri5 / PID / dense-output
algorithm the C oracle restates (kura_oracle.c solve(), env.py:247-271),
vectorised over the N oscillators; the step is env.py:415-454 (arange grids
:426-436, naive LFP :396-401, window :447-448, R1 reward :638-650 with
utils.py:21-27 calc_beta_band_power).  Results agree with the C oracle to
rounding (different summation order), not bit for bit.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
# Dormand-Prince tableau (diffrax _dopri5_tableau) cast to fp32 as jnp does
_A = [[], [1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9],
      [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
      [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
      [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]]
A = [[F32(a) for a in row] for row in _A]
E = [F32(35 / 384 - 1951 / 21600), F32(0.0), F32(500 / 1113 - 22642 / 50085), F32(125 / 192 - 451 / 720),
     F32(-2187 / 6784 + 12231 / 42400), F32(11 / 84 - 649 / 6300), F32(-1 / 60)]
M = [F32(6025192743 / 30085553152 / 2), F32(0.0), F32(51252292925 / 65400821598 / 2),
     F32(-2691868925 / 45128329728 / 2), F32(187940372067 / 1594534317056 / 2),
     F32(-1776094331 / 19743644256 / 2), F32(11237099 / 235043384 / 2)]
TWO_PI = F32(2 * np.pi)


class RefOpEnv:
    """One env of env.py's SpatialKuramoto with the reference RHS op sequence.

    alpha (N, N) f32, omega (N,) f32, g_stim (n_elec, N) f64, K, and the
    step/window parameters of the config (verbose_dt, electrode width/pause,
    observation window W, transient length, action bounds)."""

    def __init__(self, alpha, omega, g_stim, K, W=2340, dt=0.05, width=0.15, pause=0.75, transient=200.0,
                 dbs_bounds=(-5.0, 5.0), rtol=1e-5, atol=1e-5, max_steps=4096):
        self.alpha = np.asarray(alpha, F32)
        self.w0 = np.asarray(omega, F32)
        self.g_stim = np.atleast_2d(np.asarray(g_stim, np.float64))
        self.N = self.w0.shape[0]
        self.kn = F32(K / self.N)
        self.W, self.dt, self.width, self.pause, self.transient = W, dt, width, pause, transient
        self.dbs_lo, self.dbs_hi = dbs_bounds
        self.rtol, self.atol, self.max_steps = F32(rtol), F32(atol), max_steps
        self.pulse = np.zeros(self.N, F32)
        self.rhs_count = 0

    def dynamics(self, y):
        """env.py:252-256 (args = (w0, K/N, N, alpha, pulse))."""
        self.rhs_count += 1
        theta = np.fmod(y, TWO_PI)
        return self.w0 + self.kn * np.sum(self.alpha * np.sin(theta - np.tile(theta, (self.N, 1)).T), axis=1) \
            + self.pulse

    def forward(self, ts, y0):
        """diffeqsolve(Dopri5, PIDController(rtol, atol), dt0=0.05, SaveAt(ts)) -> ys (len(ts), N)."""
        ts = np.asarray(ts, np.float64)
        n = ts.shape[0]
        ys = np.empty((n, self.N), F32)
        y0 = np.asarray(y0, F32).copy()
        if n == 1:
            ys[0] = y0
            return ys
        t0, t1 = F32(ts[0]), F32(ts[-1])
        tprev, tnext = t0, min(F32(t0 + F32(0.05)), t1)
        f = [None] * 7
        f[0] = self.dynamics(y0)
        si, nsteps = 0, 0
        while tprev < t1:
            if nsteps >= self.max_steps:
                raise RuntimeError("max_steps reached (diffrax throw=True, env.py:261-270)")
            nsteps += 1
            h = F32(tnext - tprev)
            k = [None] * 7
            k[0] = h * f[0]
            for s in range(1, 7):
                acc = A[s][0] * k[0]
                for j in range(1, s):
                    if A[s][j] != 0:
                        acc = acc + A[s][j] * k[j]
                ys_s = y0 + acc
                if s == 6:
                    y1 = ys_s
                f[s] = self.dynamics(ys_s)
                k[s] = h * f[s]
            err = E[0] * k[0]
            for j in (2, 3, 4, 5, 6):
                err = err + E[j] * k[j]
            den = self.atol + np.maximum(np.abs(y0), np.abs(y1)) * self.rtol
            rms = F32(np.sqrt(np.mean((err / den) ** 2, dtype=F32)))
            keep = rms < 1
            fac = F32(0.9) * (rms ** F32(-0.2) if rms > 0 else F32(np.inf))
            fac = min(max(fac, F32(1.0) if keep else F32(0.2)), F32(10.0))
            dtn = F32(h * fac)
            if keep:
                acc = M[0] * k[0]
                for j in (2, 3, 4, 5, 6):
                    acc = acc + M[j] * k[j]
                ym = y0 + acc
                ca = 2 * (k[6] - k[0]) - 8 * (y1 + y0) + 16 * ym
                cb = 5 * k[0] - 3 * k[6] + 18 * y0 + 14 * y1 - 32 * ym
                cc = k[6] - 4 * k[0] - 11 * y0 - 5 * y1 + 16 * ym
                while si < n and F32(ts[si]) <= tnext:
                    x = F32((F32(ts[si]) - tprev) / (tnext - tprev))
                    ys[si] = (((ca * x + cb) * x + cc) * x + k[0]) * x + y0
                    si += 1
                y0, f[0], tprev = y1, f[6], tnext
            tn = F32(tprev + dtn)
            tprev = min(tprev, t1)
            if tn > t1 - F32(1e-6):
                tn = t1 if keep else F32(tprev + F32(0.5) * (t1 - tprev))
            tnext = tn
        return ys

    def reset(self, theta0):
        """env.py:594-614: transient over arange(0, transient, dt), window = last W LFP samples."""
        ts = np.arange(0.0, self.transient, self.dt)
        self.t = ts[-1]
        self.pulse = np.zeros(self.N, F32)
        self.sol = self.forward(ts, theta0)
        self.window = np.mean(np.cos(self.sol[:-1]), axis=1)[-self.W:]
        return self.window.astype(F32)

    def step(self, action):
        """env.py:415-454 with the R1 reward (env.py:638-650)."""
        a = np.atleast_1d(np.asarray(action, np.float64))
        u = self.dbs_lo + ((self.dbs_hi - self.dbs_lo) * (a + 1.0)) / 2.0
        self.pulse = np.sum(self.g_stim * u[:, None], axis=0).astype(F32)
        ts1 = np.arange(self.t, self.t + self.width, self.dt)
        s1 = self.forward(ts1, self.sol[-1])
        self.t = ts1[-1]
        self.pulse = np.zeros(self.N, F32)
        ts2 = np.arange(self.t, self.t + self.pause, self.dt)
        s2 = self.forward(ts2, s1[-1])
        self.t = ts2[-1]
        self.sol = s2
        rows = np.concatenate([s1, s2])[:-1]
        lfp = np.mean(np.cos(rows), axis=1)
        self.window = np.append(self.window, lfp)[-self.W:]
        sig = self.window
        n = sig.shape[0]
        ft = np.abs(np.fft.rfft(sig) / n) ** 2 * 2
        freq = np.fft.rfftfreq(n, self.dt / 100.0)
        r = -1e4 * np.sum(ft[(freq > 12.5) & (freq < 21)]) - 1e-2 * abs(u[0])
        return self.window.astype(F32), float(r)


def time_steps(env, seconds, rng=None, max_steps=1000):
    """Steps/s of env.step with U(-1, 1) actions for about `seconds` (after reset)."""
    import time
    rng = rng or np.random.default_rng(0)
    t0 = time.perf_counter()
    k = 0
    while k < max_steps:
        env.step(rng.uniform(-1, 1, 1))
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return k / el, k, el
