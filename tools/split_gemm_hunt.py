"""Hunt for outputs where the split build's GEMM and the oracle's bf16 MFMA
model disagree: many random (X, A) at N = 1024 with sin/cos-like rows and
cos-of-distance-like or signed A; writes every mismatching chain (K1 k
order) as a trace input for tools/mfma_chain_trace.
    python tools/split_gemm_hunt.py OUTDIR [n_gemms]"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import kura_oracle as ko  # noqa: E402
import split_gemm_check as sk  # noqa: E402

abi = importlib.import_module("dbs-gym_amd.abi")
L = abi.load_library()   # the bf16x3 GEMM through kura_selftest_coupling (KURA_COUPLING_BF16X3 = 2)
out, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
os.makedirs(out, exist_ok=True)
N = 1024
perm = (np.arange(N).reshape(-1, 16)[:, np.r_[0:16:2, 1:16:2]]).ravel()
tot = bad_n = 0
for seed in range(n):
    rng = np.random.default_rng(int(os.environ.get("HUNT_BASE", "1000")) + seed)
    th = rng.uniform(0, 2 * np.pi, (16, N)).astype(np.float32)
    X = np.concatenate([np.sin(th), np.cos(th)]).astype(np.float32)
    kind = seed % 3
    if kind == 0:
        A = rng.uniform(-1, 1, (N, N)).astype(np.float32)
    elif kind == 1:
        A = np.cos(rng.uniform(0, 2.2, (N, N))).astype(np.float32)
    else:
        A = (rng.uniform(0.3, 1, (N, N)) * np.where(rng.random((N, N)) < 0.1, -1, 1)).astype(np.float32)
    Y = np.zeros((32, N), np.float32)
    assert L.kura_selftest_coupling(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N, 2) == 0
    W = ko.split_gemm_rows(X, A)
    bad = np.argwhere(Y.view(np.uint32) != W.view(np.uint32))
    tot += Y.size
    bad_n += len(bad)
    for r, c in bad[:4]:
        xp, ap = sk.split3(X[r, perm]), sk.split3(A[c, perm])
        with open(os.path.join(out, f"s{seed}_r{r}_c{c}.bin"), "wb") as fh:
            np.array([N], np.int32).tofile(fh)
            xp.astype(np.uint16).tofile(fh)
            ap.astype(np.uint16).tofile(fh)
    print(f"seed {seed} kind {kind}: {len(bad)} mismatches", flush=True)
print(f"total {bad_n} of {tot} outputs", flush=True)
