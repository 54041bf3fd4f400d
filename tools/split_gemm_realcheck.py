"""kura_selftest_gemm of libkura_split.so on the real coupling (env0, N=1024)
and sin/cos operand rows vs oracle_split_gemm_rows (diagnostic)."""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402

abi = importlib.import_module("dbs-gym_amd.abi")
L = abi.load_library(os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_split.so"))
L.kura_selftest_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
for name, N in (("env0", 1024), ("env1", 512), ("env0", 256)):
    cfg, alpha, *_ = make_case(name, N, 2, reward="bbpow_action")
    A = np.ascontiguousarray(alpha, np.float32)
    rng = np.random.default_rng(1)
    th = rng.uniform(0, 2 * np.pi, (16, N)).astype(np.float32)
    X = np.concatenate([np.sin(th), np.cos(th)]).astype(np.float32)
    X[3, :50] = 0.0
    Y = np.zeros((32, N), np.float32)
    assert L.kura_selftest_gemm(X.ctypes.data, A.ctypes.data, Y.ctypes.data, N) == 0
    W = ko.split_gemm_rows(X, A)
    bad = np.argwhere(Y.view(np.uint32) != W.view(np.uint32))
    print(name, N, "mismatches", len(bad), "of", Y.size, bad[:4].tolist(), flush=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"realcheck_{name}_{N}.npz"), X=X, A=A, Y=Y)
