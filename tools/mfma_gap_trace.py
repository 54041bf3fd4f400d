#!/usr/bin/env python3
"""Per-MFMA traces of the outputs where the in-solver bf16x3 GEMM and the
oracle's MFMA model part (operands from tools/coupling_dump_probe.py dumps):
for each mismatching (row, col) the split chain runs through
tools/mfma_chain_trace (the accumulator after every MFMA), saved with its
operands to gpurun_out/gap_traces.npz for the model analysis on the CPU.
    python tools/mfma_gap_trace.py probe_in/dump_*.npz"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402
import split_gemm_check as sk  # noqa: E402

TRACE = os.path.join(ROOT, "tools", "mfma_chain_trace")
out = {"xp": [], "ap": [], "acc": [], "want": [], "model": [], "src": []}
for f in sys.argv[1:]:
    d = np.load(f)
    X, Y, W = d["X"], d["Y"], d["W"]
    N = X.shape[1]
    _, alpha, *_ = make_case("env0", N, 16, coupling="bf16x3")
    perm = (np.arange(N).reshape(-1, 16)[:, np.r_[0:16:2, 1:16:2]]).ravel()
    for r, c in np.argwhere(Y.view(np.uint32) != W.view(np.uint32)):
        xp, ap = sk.split3(X[r, perm]), sk.split3(alpha[c, perm])
        with tempfile.TemporaryDirectory() as t:
            fi, fo = os.path.join(t, "in.bin"), os.path.join(t, "out.bin")
            with open(fi, "wb") as fh:
                np.array([N], np.int32).tofile(fh)
                xp.astype(np.uint16).tofile(fh)
                ap.astype(np.uint16).tofile(fh)
            subprocess.run([TRACE, fi, fo], check=True, capture_output=True)
            acc = np.fromfile(fo, np.float32)
        out["xp"].append(xp)
        out["ap"].append(ap)
        out["acc"].append(acc)
        out["want"].append(Y[r, c])
        out["model"].append(W[r, c])
        out["src"].append(f"{os.path.basename(f)}:{r},{c}")
        print(f"{os.path.basename(f)} ({r},{c}): trace end {acc[-1]!r} in-solver {Y[r, c]!r} model {W[r, c]!r}",
              flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "gap_traces.npz"), **{k: np.array(v) for k, v in out.items()})
