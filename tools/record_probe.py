#!/usr/bin/env python3
"""Diagnostic (round 3): localise where two kernel generations part ways.

Runs the reset of a seeded batch with max_steps = 1, 2, ... (the solve stops
after that many Dopri steps: flag MAX_STEPS) through K1 (KURA_KERNEL=k1) and
K1w, copies each one's solver workspace (kura_debug_read_workspace) and
prints, for the first max_steps where they differ, every record slot that
differs with its (env, column) positions.  Slots Y0/F0 are skipped (K1
applies FSAL inside post_step, K1w only before the next attempt).  Since the
FSAL renaming (Slot::par) K1's physical slots Y0<->Y1 and F0<->F6 are swapped
after an odd number of all-accepted steps: compare at max_steps = 1 or read
the swapped pairs accordingly.
Usage: [LIB=libkura_x.so] record_probe.py ENV N B [KMAX]"""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_case  # noqa: E402

SLOTS = ["Y0", "F0", "F1", "F2", "F3", "F4", "F5", "F6", "Y1", "CA", "CB", "CC", "W", "P"]


def unswizzle(R, B, N):
    """[Bp/16][slot][N][16] with the lane-contiguous tile layout -> [slot][env][col]."""
    Bp = (B + 15) // 16 * 16
    R = R.reshape(Bp // 16, 14, N // 32, 2, 64, 4)    # group, slot, tile, half, lane, q&3
    out = np.zeros((14, Bp, N), np.float32)
    lane = np.arange(64)
    col = (lane & 31)
    for h in range(2):
        for q3 in range(4):
            env_in = q3 + 8 * h + 4 * (lane >> 5)       # mfma_env(q = q3 + 4h, lane)
            for g in range(Bp // 16):
                for t in range(N // 32):
                    out[:, g * 16 + env_in, 32 * t + col] = R[g, :, t, h, :, q3]
    return out


def run(kernel, name, N, B, k):
    import torch
    os.environ["KURA_KERNEL"] = kernel
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B)
    cfg.max_steps = k
    lib = os.environ.get("LIB")
    sim = sim_mod.KuraSim(cfg, 0, lib_path=os.path.join(ROOT, "dbs-gym_amd", "csrc", lib) if lib else None)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    torch.cuda.synchronize()
    Bp = (B + 15) // 16 * 16
    R = np.zeros(Bp * 14 * N, np.float32)
    rc = sim.lib.kura_debug_read_workspace(sim._h, R.ctypes.data, R.size)
    assert rc == 0
    y = sim.get_state()["y"]
    sim.close()
    return unswizzle(R, B, N), y


def main():
    name, N, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    kmax = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    for k in range(1, kmax + 1):
        a, ya = run("k1", name, N, B, k)
        b, yb = run("k1w", name, N, B, k)
        bad = []
        for s in range(2, 12):
            d = np.argwhere(a[s, :B] != b[s, :B])
            if len(d):
                bad.append((SLOTS[s], d))
        print(f"max_steps={k}: differing slots {[x[0] for x in bad]}", flush=True)
        for sname, d in bad:
            envs = sorted(set(d[:, 0].tolist()))
            cols = sorted(set(d[:, 1].tolist()))
            print(f"  {sname}: {len(d)} elements, envs {envs}, {len(cols)} columns, first cols {cols[:16]}")
        if bad:
            s0 = [SLOTS.index(x[0]) for x in bad][0]
            d = bad[0][1][:5]
            for e, c in d:
                print(f"   {SLOTS[s0]}[{e},{c}] k1={a[s0, e, c]!r} k1w={b[s0, e, c]!r}")
            break


if __name__ == "__main__":
    main()
