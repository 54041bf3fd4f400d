"""Dump the bf16x3 coupling GEMM (kura_selftest_coupling) for offline model checks:
    python tools/split_gemm_dump.py out.npz [N] [lo]   (A ~ U(lo, 1), X ~ U(-1, 1))"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
abi = importlib.import_module("dbs-gym_amd.abi")
L = abi.load_library()   # the bf16x3 GEMM through kura_selftest_coupling (KURA_COUPLING_BF16X3 = 2)
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
lo = float(sys.argv[3]) if len(sys.argv) > 3 else -1.0
rng = np.random.default_rng(N)
X = rng.uniform(-1, 1, (32, N)).astype(np.float32)
A = rng.uniform(lo, 1, (N, N)).astype(np.float32)
Y = np.zeros((32, N), np.float32)
assert L.kura_selftest_coupling(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N, 2) == 0
np.savez(sys.argv[1], X=X, A=A, Y=Y)
print("ok", N, lo)
