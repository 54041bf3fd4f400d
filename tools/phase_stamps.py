#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the step kernel (KURA_STAMPS build;
slot 19 = 1 + SIMD id).

Builds dbs-gym_amd/csrc/libkura_stamps.so with -DKURA_STAMPS and runs a few
bench-shaped steps, printing the share of wave cycles in each phase."""
import importlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

SI = os.environ.get("SI") == "1"  # stage-input sub-phases (KURA_STAMPS_SI build, no record prefetch)
COUPLING = os.environ.get("COUPLING", "auto")  # auto | f32 | bf16x3 (KuraConfig.coupling, a run-time choice)
LIB = os.path.join(ge.CSRC, "libkura_stamps_si.so" if SI else "libkura_stamps.so")
PHASES = ["stage_input", "barrier1", "gemm", "epilogue", "barrier2", "post_err", "flag_sync", "post_decide",
          "post_saves", "post_fsal", "post_time", "save_setup", "save_loadwait", "save_compute", "save_publish",
          "save_totals", "si_load", "si_compute", "si_lds", "si_misc", "tail_window", "tail_reward", "tail_other",
          "simd_id"]


def main():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(ge.CSRC, "kura_kernels.hip")):
        subprocess.run([ge.HIPCC, *ge.HIP_FLAGS, "-DKURA_STAMPS", *(["-DKURA_STAMPS_SI"] if SI else []),
                        "-o", LIB,
                        os.path.join(ge.CSRC, "kura_kernels.hip")], check=True)
    import numpy as np
    import torch
    import bench
    sim_mod = importlib.import_module("dbs-gym_amd.sim")

    class A:
        config = os.environ.get("CFG", "env0")
        osc = int(os.environ.get("OSC", "1024"))
        envs = int(os.environ.get("ENVS", "4096"))
        reward = os.environ.get("REWARD", "bbpow_action")
        seed = 7
        random_k = False
        coupling = COUPLING
    cfg, alpha, omega, gs, gr, th0, ct, st, gain = bench.build_shard(A, 0)
    sim = sim_mod.KuraSim(cfg, 0, lib_path=LIB)
    sim.set_coupling(alpha)
    sim.set_env_gain(gain)
    sim.set_env_params(omega, gs, gr)
    sim.set_spectral(ct, st)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sim.stamps()
    ev0.record()
    sim.reset(torch.from_numpy(th0))
    ev1.record()
    torch.cuda.synchronize()
    s_reset = sim.stamps().astype(np.float64)
    ms_reset = ev0.elapsed_time(ev1)
    a = torch.zeros((cfg.n_envs, cfg.n_elec), device="cuda")
    nsteps = 5
    ev0.record()
    for _ in range(nsteps):
        sim.step(a)
    ev1.record()
    torch.cuda.synchronize()
    s = sim.stamps().astype(np.float64)
    if os.environ.get("MODE") == "reset":  # the reset transient's breakdown instead (one launch)
        s, nsteps = s_reset, 1
        ev_ms = ms_reset
    else:
        ev_ms = ev0.elapsed_time(ev1) / nsteps
    names = PHASES
    nwaves = 8
    s = s[:nwaves]
    tot = s.sum(axis=1, keepdims=True)
    share = (s / np.maximum(tot, 1)).mean(axis=0)
    nwg = (cfg.n_envs + 15) // 16
    cyc_per_step_wave = s.sum(axis=0) / (nwaves * nwg * nsteps)
    out = {"mode": os.environ.get("MODE", "step"), "ms_per_launch": ev_ms,
           "kernel": "K1", "share": dict(zip(names, [round(float(x), 4) for x in share])),
           "cycles_per_step_per_wave": dict(zip(names, [round(float(x)) for x in cyc_per_step_wave])),
           # per wave (rows), cycles per step of the phases that differ between waves
           "per_wave": {names[k]: [round(float(v)) for v in s[:, k] / (nwg * nsteps)]
                        for k in range(len(PHASES)) if s[:, k].sum() > 0}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
