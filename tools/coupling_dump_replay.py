#!/usr/bin/env python3
"""Replays the operands captured by tools/coupling_dump_probe.py through the
stand-alone GEMM (kura_selftest_coupling): equal to the in-solver sums (the
oracle's model misses the hardware), or to the oracle (the solver context
differs)?
    python tools/coupling_dump_replay.py gpurun_out/dump_512_*.npz"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402

abi = importlib.import_module("dbs-gym_amd.abi")

L = abi.load_library()
for f in sys.argv[1:]:
    d = np.load(f)
    X, Y, W = d["X"], d["Y"], d["W"]
    N = X.shape[1]
    _, alpha, *_ = make_case("env0", N, 16, coupling="bf16x3")
    Z = np.zeros((32, N), np.float32)
    assert L.kura_selftest_coupling(X.ctypes.data, alpha.ctypes.data, Z.ctypes.data, N, 2) == 0
    u = lambda a: a.view(np.uint32)
    print(f"{os.path.basename(f)}: selftest vs in-solver {int((u(Z) != u(Y)).sum())} differ, selftest vs oracle "
          f"{int((u(Z) != u(W)).sum())} differ, in-solver vs oracle {int((u(Y) != u(W)).sum())}", flush=True)
