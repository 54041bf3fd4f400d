"""Bit sweeps around the ratio-28 misses of the regime probe
(tests/golden/mfma_bf16_regime_probe.npz, r28): for each missed MFMA, the
accumulator's 6 low mantissa bits swept (64 variants), and the y mantissa of
its largest and of its smallest product swept (2 x 128 variants).
    python tests/golden/make_mfma_r28_sweep.py gen    # -> trace_in/cases_sweep.bin
    ./tools/mfma_case_probe trace_in/cases_sweep.bin gpurun_out/cases_sweep_out.bin   (MI355X)
    python tests/golden/make_mfma_r28_sweep.py keep   # -> tests/golden/mfma_bf16_r28_sweep.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gen():
    d = np.load(os.path.join(ROOT, "tests", "golden", "mfma_bf16_regime_probe.npz"))
    miss = np.isin(d["r28_index"], d["r28_model_misses"])
    X, Y, C, B = [], [], [], []
    for b, i in enumerate(np.flatnonzero(miss)):
        x, y, c = d["r28_x_bf16"][i].copy(), d["r28_y_bf16"][i].copy(), np.float32(d["r28_c"][i])
        cu = np.array([c], np.float32).view(np.uint32)[0]
        for j in range(64):
            X.append(x); Y.append(y); C.append(np.array([(cu & ~np.uint32(63)) | np.uint32(j)], np.uint32).view(np.float32)[0]); B.append(b)
        e = [((int(x[k]) >> 7) & 0xFF) + ((int(y[k]) >> 7) & 0xFF) + np.log2((128 | (int(x[k]) & 0x7F)) * (128 | (int(y[k]) & 0x7F))) for k in range(8)]
        for k in (int(np.argmax(e)), int(np.argmin(e))):
            for m in range(128):
                yy = y.copy()
                yy[k] = (int(y[k]) & 0xFF80) | m
                X.append(x); Y.append(yy); C.append(c); B.append(b)
    os.makedirs(os.path.join(ROOT, "trace_in"), exist_ok=True)
    with open(os.path.join(ROOT, "trace_in", "cases_sweep.bin"), "wb") as fh:
        np.array([len(C)], np.int32).tofile(fh)
        np.array(X, np.uint16).tofile(fh)
        np.array(Y, np.uint16).tofile(fh)
        np.array(C, np.float32).tofile(fh)
    np.save(os.path.join(ROOT, "trace_in", "cases_sweep_base.npy"), np.array(B, np.int32))


def keep():
    raw = open(os.path.join(ROOT, "trace_in", "cases_sweep.bin"), "rb").read()
    n = int(np.frombuffer(raw, np.int32, 1)[0])
    x = np.frombuffer(raw, np.uint16, n * 16, 4).reshape(n, 16)
    y = np.frombuffer(raw, np.uint16, n * 16, 4 + n * 32).reshape(n, 16)
    c = np.frombuffer(raw, np.float32, n, 4 + n * 64)
    hw = np.fromfile(os.path.join(ROOT, "gpurun_out", "cases_sweep_out.bin"), np.float32)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "mfma_bf16_r28_sweep.npz"), x_bf16=x, y_bf16=y, c=c,
                        gpu=hw, base=np.load(os.path.join(ROOT, "trace_in", "cases_sweep_base.npy")))


if __name__ == "__main__":
    gen() if sys.argv[1] == "gen" else keep()
