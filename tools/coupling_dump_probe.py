#!/usr/bin/env python3
"""The coupling GEMM inside the solver, sweep by sweep (libkura_debug.so,
kura_debug_gemm_dump): workgroup 0's sin/cos operand and P/Q of the first
sweeps of a reset, against the oracle's GEMM of that same operand
(oracle_split_gemm_rows / the fmaf chain).  Prints the first sweeps and rows
where they part.
    python tools/coupling_dump_probe.py [N] [sweeps] [coupling]"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402
from oracle import kura_oracle as ko  # noqa: E402
import torch  # noqa: E402

sim_mod = importlib.import_module("dbs-gym_amd.sim")
DEBUG_LIB = os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_debug.so")


def main(N=512, n=120, coupling="bf16x3"):
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case("env0", N, 16, coupling=coupling)
    sim = sim_mod.KuraSim(cfg, 0, lib_path=DEBUG_LIB)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    buf = torch.zeros((n, 2, 32, N), dtype=torch.float32, device="cuda")
    assert sim.lib.kura_debug_gemm_dump(sim._h, buf.data_ptr(), n) == 0
    sim.reset(torch.from_numpy(th0))
    torch.cuda.synchronize()
    d = buf.cpu().numpy()
    nbad = 0
    for k in range(n):
        X, Y = d[k, 0], d[k, 1]
        W = ko.split_gemm_rows(X, alpha) if coupling == "bf16x3" else ko.gemm_chain(X, alpha)
        bad = np.argwhere(Y.view(np.uint32) != W.view(np.uint32))
        if len(bad):
            nbad += 1
            rows = sorted(set(bad[:, 0].tolist()))
            r, c = bad[0]
            if nbad <= 6:
                print(f"sweep {k}: {len(bad)} outputs differ, rows {rows}; first ({r},{c}): gpu {Y[r, c]!r} "
                      f"oracle {W[r, c]!r} diff {float(Y[r, c]) - float(W[r, c]):.3e}", flush=True)
                np.savez(os.path.join(ROOT, "gpurun_out", f"dump_{N}_{k}.npz"), X=X, Y=Y, W=W)
    print(f"N={N} {coupling}: {nbad} of {n} sweeps with differing outputs", flush=True)
    sim.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(int(a[0]) if a else 512, int(a[1]) if len(a) > 1 else 120, a[2] if len(a) > 2 else "bf16x3")
