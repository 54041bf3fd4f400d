"""Dump kura_selftest_gemm of the split build for offline model checks:
    python tools/split_gemm_dump.py out.npz [N] [lo]   (A ~ U(lo, 1), X ~ U(-1, 1))"""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
abi = importlib.import_module("dbs-gym_amd.abi")
L = abi.load_library(os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_split.so"))
L.kura_selftest_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
lo = float(sys.argv[3]) if len(sys.argv) > 3 else -1.0
rng = np.random.default_rng(N)
X = rng.uniform(-1, 1, (32, N)).astype(np.float32)
A = rng.uniform(lo, 1, (N, N)).astype(np.float32)
Y = np.zeros((32, N), np.float32)
assert L.kura_selftest_gemm(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N) == 0
np.savez(sys.argv[1], X=X, A=A, Y=Y)
print("ok", N, lo)
