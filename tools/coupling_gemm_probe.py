#!/usr/bin/env python3
"""The bf16x3 coupling GEMM (kura_selftest_coupling) on solver-like operands:
X = [sin theta; cos theta] of 16 envs' phase states from oracle trajectories
(rows 0-15 sin, 16-31 cos, as the step kernel lays them out) against
oracle_split_gemm_rows; counts mismatching outputs per row, and repeats with
the rows rotated (is it the row position or the data?).
    python tools/coupling_gemm_probe.py [N] [n_states]"""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import actions, make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402

abi = importlib.import_module("dbs-gym_amd.abi")


def main(N=256, n_states=24):
    L = abi.load_library()
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", N, 16, coupling="f32")
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    states = [o.y.copy()]
    for k in range(n_states - 1):
        o.step(actions("rand", 16, 1, k))
        states.append(o.y.copy())
    bad_rows = np.zeros(32, np.int64)
    bad_rot = np.zeros(32, np.int64)
    total = 0
    for y in states:
        s, c = ko.sincos_fmod2pi(y.reshape(-1))
        X = np.concatenate([s.reshape(16, N), c.reshape(16, N)]).astype(np.float32)
        for rot, acc in ((0, bad_rows), (4, bad_rot)):
            Xr = np.roll(X, rot, axis=0)
            Y = np.zeros((32, N), np.float32)
            assert L.kura_selftest_coupling(Xr.ctypes.data, alpha.ctypes.data, Y.ctypes.data, N, 2) == 0
            W = ko.split_gemm_rows(Xr, alpha)
            diff = (Y.view(np.uint32) != W.view(np.uint32)).sum(axis=1)
            acc += np.roll(diff, -rot)      # indexed by the data's own row
        total += 32 * N
    print(f"N={N}: {len(states)} operands, {total} outputs; mismatches per data row {bad_rows.tolist()}; "
          f"rows rotated by 4: {bad_rot.tolist()}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256, int(sys.argv[2]) if len(sys.argv) > 2 else 24)
