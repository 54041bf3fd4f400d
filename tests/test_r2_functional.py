"""R2's filter term as a linear functional, and the R1/R3 spectral
accumulators (CPU only).

* reward_temp_const_lfp_betafilt_action (env.py:653-666) uses d = f[-1] -
  mean(f) of f = scipy filtfilt(b, a, x) (utils.py:794-816) -- linear in x, so
  d = c . x with c from dbs-gym_amd/csrc/kura_r2.h.  Pinned here against
  scipy itself and against an extended-precision filtfilt, and the host
  compilers of libkura (clang, via hipcc) and of the oracle (gcc) must build
  the same c bit for bit (GPU and oracle then take the same dot product).
* R1/R3 in step() come from running accumulators over ring positions; they
  must track the direct DFT of the window (oracle_reward) to float64 rounding
  over long runs, and re-forming them from the ring (kura_set_state) must
  agree with the running values.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest
from scipy import signal

from helpers import ROOT, actions, ko, make_case

HDR = os.path.join(ROOT, "dbs-gym_amd", "csrc", "kura_r2.h")
SRC = r'''
#include "%s"
int r2c(const double* b, const double* a, const double* zi, int W, int P, double* c) {
    return kura_r2_functional(b, a, zi, W, P, c);
}
''' % HDR


def _build(cc, tmp):
    src = os.path.join(tmp, "r2c.c")
    open(src, "w").write(SRC)
    so = os.path.join(tmp, f"r2c_{os.path.basename(cc)}.so")
    subprocess.run([cc, "-O3", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC", "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    lib.r2c.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 2 + [ctypes.c_void_p]
    return lib


def _coeffs():
    b, a = signal.butter(2, [12 / 1000, 30 / 1000], "band")     # utils.py:812, fs = 2000 Hz
    return b, a, signal.lfilter_zi(b, a)


def _c(lib, W, P=15):
    b, a, zi = _coeffs()
    c = np.zeros(W)
    assert lib.r2c(b.ctypes.data, a.ctypes.data, zi.ctypes.data, W, P, c.ctypes.data) == 0
    return c


def _filtfilt_ld(x, P=15):
    """scipy's filtfilt (odd padding, lfilter_zi * first input, DF2T) in long double"""
    b, a, zi = (v.astype(np.longdouble) for v in _coeffs())

    def lf(u):
        z = zi * u[0]
        y = np.empty(len(u), np.longdouble)
        for k, xn in enumerate(u):
            yn = z[0] + b[0] * xn
            z[0] = (z[1] + xn * b[1]) - yn * a[1]
            z[1] = (z[2] + xn * b[2]) - yn * a[2]
            z[2] = (z[3] + xn * b[3]) - yn * a[3]
            z[3] = xn * b[4] - yn * a[4]
            y[k] = yn
        return y
    x = x.astype(np.longdouble)
    W = len(x)
    ext = np.concatenate([2 * x[0] - x[P:0:-1], x, 2 * x[-1] - x[-2:-P - 2:-1]])
    f = lf(lf(ext)[::-1])[::-1][P:P + W]
    return f[-1] - f.mean()


@pytest.fixture(scope="module")
def libs(tmp_path_factory):
    tmp = str(tmp_path_factory.mktemp("r2"))
    clang = "/opt/rocm/llvm/bin/clang"
    return _build("gcc", tmp), (_build(clang, tmp) if os.path.exists(clang) else None)


@pytest.mark.parametrize("W", [2340, 2556, 4680, 100, 16])
def test_functional_matches_scipy_filtfilt(libs, W):
    c = _c(libs[0], W)
    rng = np.random.default_rng(W)
    for k in range(4):
        x = rng.standard_normal(W) * 0.3 + (0.5 if k % 2 else -0.2)
        f = signal.filtfilt(*_coeffs()[:2], x)
        d = f[-1] - f.mean()
        assert abs(c @ x - d) <= 1e-10 * abs(d) + 1e-16, (W, c @ x, d)


@pytest.mark.parametrize("W", [2340, 100])
def test_functional_is_closer_to_exact_than_scipy(libs, W):
    """against an extended-precision filtfilt: c . x within float64 rounding
    of its terms (scipy's own float64 filtfilt is ~1e-12 relative off here)"""
    c = _c(libs[0], W)
    rng = np.random.default_rng(7)
    for _ in range(2):
        x = rng.standard_normal(W) * 0.3 + 0.5
        dl = _filtfilt_ld(x)
        assert abs(float(c @ x - dl)) <= 1e-14 * float(np.abs(c * x).sum())


def test_host_compilers_build_the_same_functional(libs):
    gcc, clang = libs
    if clang is None:
        pytest.skip("no clang")
    for W in (2340, 2556, 9360, 16):
        assert _c(gcc, W).tobytes() == _c(clang, W).tobytes(), W


def test_step_reward_tracks_the_direct_dft():
    """R1 / R3 from the spectral accumulators vs the direct float64 DFT of the
    observed window (oracle_reward) over 300 steps: float64 rounding only.
    (The accumulators do not depend on the coupling arithmetic: f32 keeps the
    oracle cheap.)"""
    for reward in ("bbpow_action", "bbpow_threth_action"):
        cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, 3, reward=reward, coupling="f32")
        o = ko.Oracle(cfg, alpha)
        o.set_env_params(omega, gs, gr)
        o.set_spectral(ct, st)
        o.reset(th0)
        worst = 0.0
        for k in range(300):
            a = actions("rand", 3, cfg.n_elec, k)
            out = o.step(a)
            for b in range(3):
                x = out["obs"][b].astype(np.float64)
                win = np.roll(o.ring[b], -o.wpos[b])            # the un-cast window (oldest first)
                np.testing.assert_array_equal(win.astype(np.float32), out["obs"][b])
                u = 5.0 * float(a[b, 0])
                r = o.reward(win, u)
                if reward == "bbpow_action":
                    worst = max(worst, abs(out["reward"][b] - r) / abs(r))
                else:
                    assert out["reward"][b] == r
            del x
        assert worst < 1e-12, worst


def test_accumulators_hold_over_a_whole_episode():
    """a whole 5555-step training episode (~1e5 updates
    of every accumulator: 17-19 new samples per step, each folded into every
    bin) -- at every 100th step the band power from the running accumulators
    against the direct float64 DFT of the window (utils.py:21-27; the
    accumulators Y_k themselves against numpy's float64 DFT of the ring):
    relative error <= 1e-12.  (Measured drift: DESIGN.md section 2.)"""
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, 1, reward="bbpow_action", coupling="f32")
    assert cfg.episode_steps == 5555
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    W = cfg.window
    bins = np.array(cfg.bins[:cfg.n_bins])
    ph = 2.0 * np.pi * np.outer(bins, np.arange(W)) / W
    np.testing.assert_allclose(ct, np.cos(ph), rtol=0, atol=5e-14)   # the twiddles (numpy: argument rounding)
    np.testing.assert_allclose(np.abs(st), np.abs(np.sin(ph)), rtol=0, atol=5e-14)
    worst_bb, worst_y = 0.0, 0.0
    for k in range(cfg.episode_steps):
        a = actions("rand", 1, cfg.n_elec, k)
        out = o.step(a)
        if (k + 1) % 100 and k + 1 != cfg.episode_steps:
            continue
        u = abs(5.0 * float(a[0, 0]))
        bb_acc = -(out["reward"][0] + 1e-2 * u) / 1e4
        win = np.roll(o.ring[0], -o.wpos[0])
        bb_dir = -(o.reward(win, 5.0 * float(a[0, 0])) + 1e-2 * u) / 1e4
        worst_bb = max(worst_bb, abs(bb_acc - bb_dir) / abs(bb_dir))
        ring = o.ring[0]
        Y = np.stack([ct @ ring, st @ ring], axis=1).reshape(-1)   # (re, im) per bin: the twiddle rows . ring
        scale = np.abs(ring).sum()
        worst_y = max(worst_y, float(np.abs(o.spec[0] - Y).max() / scale))
    assert o.step_count[0] == cfg.episode_steps
    assert worst_bb <= 1e-12, worst_bb
    assert worst_y <= 1e-12, worst_y
    print(f"accumulator drift over 5555 steps: band power {worst_bb:.2e} rel, Y_k {worst_y:.2e} of sum|x|")


def test_reformed_accumulators_equal_running_ones():
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", 256, 2)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    for k in range(60):
        o.step(actions("rand", 2, cfg.n_elec, k))
    run = o.state()
    s2 = dict(run)
    del s2["spec"]
    o.set_state(s2)                                   # re-formed from the ring
    np.testing.assert_allclose(o.spec, run["spec"], rtol=1e-12, atol=1e-12)
    o.set_state(run)                                  # exact
    np.testing.assert_array_equal(o.spec, run["spec"])
