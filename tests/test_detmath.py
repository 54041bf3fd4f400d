"""kura_detmath.h (compiled into the oracle) against libm / numpy in float64.

The same header is compiled into the HIP kernels; tests/test_gpu_parity.py
checks the device results are bit-identical to these."""
import numpy as np

from helpers import ko


def _ulp_err(got, ref):
    got = got.astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(got - ref) / ulp


def test_sincos_accuracy():
    rng = np.random.default_rng(0)
    for lo, hi in ((0, 2 * np.pi), (-10, 10), (0, 3000), (-1e4, 1e4)):
        x = rng.uniform(lo, hi, 200_000).astype(np.float32)
        s, c = ko.sincos(x)
        xd = x.astype(np.float64)
        # absolute error relative to 1 ulp of 1.0 is the meaningful bound for
        # cos/sin values near zero; relative ulps elsewhere
        for got, ref in ((s, np.sin(xd)), (c, np.cos(xd))):
            big = np.abs(ref) > 1e-3
            assert _ulp_err(got[big], ref[big]).max() <= 3.0, (lo, hi)
            assert np.abs(got - ref).max() <= 2e-7 * max(1.0, hi / 1e3)


def test_sincos_special_points():
    s, c = ko.sincos(np.array([0.0, -0.0], np.float32))
    assert s[0] == 0.0 and c[0] == 1.0 and c[1] == 1.0


def test_fmod_is_exact():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-2e4, 2e4, 400_000), rng.uniform(0, 20, 100_000),
                        np.arange(-50, 50) * np.float64(np.float32(2 * np.pi)),
                        [0.0, 6.2831855, 6.283185, 5e6, 3e7]]).astype(np.float32)
    got = ko.fmod2pi(x)
    ref = np.fmod(x, np.float32(2 * np.pi))  # C fmodf semantics, exact
    np.testing.assert_array_equal(got, ref)


def test_inv_fifth_root():
    rng = np.random.default_rng(2)
    x = np.concatenate([10.0 ** rng.uniform(-30, 30, 200_000), [1.0, 32.0, 1e-40, 3e38]]).astype(np.float32)
    got = ko.inv_fifth_root(x)
    ref = x.astype(np.float64) ** -0.2
    assert _ulp_err(got, ref).max() <= 1.0
    sp = ko.inv_fifth_root(np.array([0.0, np.inf, np.nan], np.float32))
    assert np.isinf(sp[0]) and sp[1] == 0.0 and np.isnan(sp[2])


def test_r64_order():
    rng = np.random.default_rng(3)
    for n in (1, 63, 64, 100, 512, 1024, 2340):
        x = rng.standard_normal(n).astype(np.float32)
        p = np.zeros(64, np.float32)
        for l in range(64):
            a = np.float32(0)
            for i in range(l, n, 64):
                a = np.float32(a + x[i])
            p[l] = a
        for o in (32, 16, 8, 4, 2, 1):
            p = (p + p[np.arange(64) ^ o]).astype(np.float32)
        assert ko.r64_f32(x) == p[0]
        xd = x.astype(np.float64)
        assert abs(ko.r64_f64(xd) - xd.sum()) <= 1e-12 * max(1, np.abs(xd).sum())


def test_folded_fmod_sincos_matches_sin_of_fmod():
    """kdm_sincos_fmod2pi (the RHS: sin/cos of theta = fmod(y, 2pi_f) with the
    fmod folded into the Cody-Waite reduction) against libm's sin/cos of the
    exact float32 fmod in float64: within the unfolded form's accuracy, plus
    2pi - 2pi_f = 1.7e-7 rad where the folded quotient differs from fmod's
    (|y| near a multiple of 2pi_f)."""
    rng = np.random.default_rng(4)
    two_pi_f = np.float32(2 * np.pi)
    x = np.concatenate([rng.uniform(0, 2 * np.pi, 200_000), rng.uniform(0, 6000, 400_000),
                        rng.uniform(-50, 50, 100_000), np.arange(-40, 40) * np.float64(two_pi_f),
                        np.arange(1, 4000) * np.float64(two_pi_f) + 1e-4]).astype(np.float32)
    s, c = ko.sincos_fmod2pi(x)
    th = np.fmod(x, two_pi_f).astype(np.float64)     # the reference's theta (exact)
    for got, ref in ((s, np.sin(th)), (c, np.cos(th))):
        assert np.abs(got - ref).max() <= 4e-7
    # away from the 2pi_f boundaries it is the unfolded result's accuracy (<= 3 ulp)
    far = (np.abs(th) > 2e-3) & (np.abs(np.abs(th) - float(two_pi_f)) > 2e-3)
    for got, ref in ((s, np.sin(th)), (c, np.cos(th))):
        big = far & (np.abs(ref) > 1e-3)
        assert _ulp_err(got[big], ref[big]).max() <= 3.0
    # beyond 2^22 the exact fmod path is taken
    xs = np.array([5e6, -3e7, 2.0 ** 23 + 1], np.float32)
    s2, c2 = ko.sincos_fmod2pi(xs)
    s3, c3 = ko.sincos(ko.fmod2pi(xs))
    np.testing.assert_array_equal(s2, s3)
    np.testing.assert_array_equal(c2, c3)
