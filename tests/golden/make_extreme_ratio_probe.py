"""Inputs of the extreme-ratio MFMA probe (tests/golden/mfma_bf16_extreme_ratio_probe.npz):

    python tests/golden/make_extreme_ratio_probe.py gen        # -> trace_in/cases.bin
    ./tools/mfma_case_probe trace_in/cases.bin gpurun_out/cases_out.bin   (MI355X)
    python tests/golden/make_extreme_ratio_probe.py keep       # -> the fixture

60 000 single MFMAs: eight group-0 products (group 1 zero), the accumulator's
leading one 2^16-2^30 above them, its low bits chosen so that acc + sum sits
near a half-ulp boundary in most cases.  Kept: every case the model misses
and 2000 random others."""
import os
import sys
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gen(n_target=60000):
    rng = np.random.default_rng(77)
    bf = lambda s, e, m: (s << 15) | ((e + 127) << 7) | m
    X, Y, C = [], [], []
    while len(C) < n_target:
        msb = int(rng.integers(-2, 7))
        ratio = int(rng.integers(16, 30))
        emax = msb - ratio
        ex = rng.integers(-4, 2, 8)
        ey = emax - ex - rng.integers(0, 6, 8)
        mode = rng.integers(0, 3)
        sx = np.zeros(8, int) if mode == 0 else rng.integers(0, 2, 8)
        sy = sx.copy() if mode == 2 else np.zeros(8, int)
        mx, my = rng.integers(0, 128, 8), rng.integers(0, 128, 8)
        x = [bf(int(sx[i]), int(ex[i]), int(mx[i])) for i in range(8)] + [0] * 8
        y = [bf(int(sy[i]), int(ey[i]), int(my[i])) for i in range(8)] + [0] * 8
        if any(((v >> 7) & 0xFF) in (0, 255) for v in x[:8] + y[:8]):
            continue
        P = sum(Fraction((-1) ** ((x[i] >> 15) ^ (y[i] >> 15))) * (128 | (x[i] & 0x7F)) * (128 | (y[i] & 0x7F))
                * Fraction(2) ** ((((x[i] >> 7) & 0xFF) - 127) + (((y[i] >> 7) & 0xFF) - 127) - 14) for i in range(8))
        ulp = Fraction(2) ** (msb - 23)
        acc = (1 if rng.random() < 0.5 else -1) * Fraction(int(rng.integers(2 ** 23, 2 ** 24))) * ulp
        r = (acc + P) / ulp
        frac = r - (r.numerator // r.denominator)
        if not (abs(frac - Fraction(1, 2)) < Fraction(1, 16) or frac < Fraction(1, 64) or frac > Fraction(63, 64)) \
                and rng.random() < 0.8:
            continue
        X.append(x)
        Y.append(y)
        C.append(float(acc))
    os.makedirs(os.path.join(ROOT, "trace_in"), exist_ok=True)
    with open(os.path.join(ROOT, "trace_in", "cases.bin"), "wb") as fh:
        np.array([len(C)], np.int32).tofile(fh)
        np.array(X, np.uint16).tofile(fh)
        np.array(Y, np.uint16).tofile(fh)
        np.array(C, np.float32).tofile(fh)


def keep():
    sys.path.insert(0, ROOT)
    from oracle import kura_oracle as ko
    raw = open(os.path.join(ROOT, "trace_in", "cases.bin"), "rb").read()
    n = int(np.frombuffer(raw, np.int32, 1)[0])
    x = np.frombuffer(raw, np.uint16, n * 16, 4).reshape(n, 16)
    y = np.frombuffer(raw, np.uint16, n * 16, 4 + n * 32).reshape(n, 16)
    c = np.frombuffer(raw, np.float32, n, 4 + n * 64)
    hw = np.fromfile(os.path.join(ROOT, "gpurun_out", "cases_out.bin"), np.float32)
    m = ko.mfma_bf16_dot16(x, y, c)
    bad = np.flatnonzero(m.view(np.uint32) != hw.view(np.uint32))
    sel = np.union1d(bad, np.random.default_rng(1).choice(n, 2000, replace=False))
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "mfma_bf16_extreme_ratio_probe.npz"),
                        x_bf16=x[sel], y_bf16=y[sel], c=c[sel], gpu=hw[sel], model_misses=bad.astype(np.int64),
                        n_probed=np.int64(n), index=sel.astype(np.int64))


if __name__ == "__main__":
    gen() if sys.argv[1] == "gen" else keep()
