#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the reference itself.

Run in the build container only (the reference tree is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference

The reference cannot be imported as shipped: jax, diffrax, gymnasium, seaborn
and imageio are absent.  This script writes minimal
stand-ins into a temporary directory (never into the reference tree):

* ``jax.numpy`` = NumPy (the reference RHS uses only fmod/sin/tile/sum/pi/array);
* ``gymnasium`` with ``Env`` and ``spaces.Box``; empty ``seaborn``/``imageio``;
* ``diffrax``: ``diffeqsolve`` delegates to THIS build's CPU solver
  (oracle/kura_oracle.c ``oracle_solve_rows``) after casting the arguments to
  float32 the way jax does with x64 disabled.

So the fixtures pin everything around the ODE solver (setup RNG streams, grid,
coupling, conductances, arange grids, pulse, LFP, window, rewards, reset and
step plumbing) to the reference's own code; the solver arithmetic itself is
the build's restatement of diffrax 0.7.0 (unpinned: diffrax is not available).
Only data is written: inputs and the reference's outputs, as .npz files.
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def _write_stubs(d: str, solve) -> None:
    os.makedirs(os.path.join(d, "jax"), exist_ok=True)
    os.makedirs(os.path.join(d, "gymnasium"), exist_ok=True)
    for m in ("seaborn", "imageio"):
        os.makedirs(os.path.join(d, m), exist_ok=True)
        open(os.path.join(d, m, "__init__.py"), "w").close()
    open(os.path.join(d, "jax", "__init__.py"), "w").write("from . import numpy\n")
    open(os.path.join(d, "jax", "numpy.py"), "w").write("from numpy import *\n")
    open(os.path.join(d, "gymnasium", "__init__.py"), "w").write(
        "class Env:\n"
        "    def reset(self, seed=None, options=None):\n"
        "        pass\n"
        "from . import spaces\n")
    open(os.path.join(d, "gymnasium", "spaces.py"), "w").write(
        "import numpy as np\n"
        "class Box:\n"
        "    def __init__(self, low, high, shape=None, dtype=np.float32):\n"
        "        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype\n")
    # diffrax is provided as an in-memory module so the solver hook is ours
    dfx = types.ModuleType("diffrax")

    class ODETerm:
        def __init__(self, f):
            self.vector_field = f

    class Dopri5:
        pass

    class PIDController:
        def __init__(self, rtol, atol, **kw):
            self.rtol, self.atol = rtol, atol

    class SaveAt:
        def __init__(self, ts):
            self.ts = ts

    class _Sol:
        def __init__(self, ys):
            self.ys = ys

    def diffeqsolve(term, solver, args, t0, t1, dt0, y0, saveat, stepsize_controller):
        return _Sol(solve(term.vector_field, args, t0, t1, dt0, y0, saveat.ts, stepsize_controller))

    dfx.ODETerm, dfx.Dopri5, dfx.PIDController, dfx.SaveAt, dfx.diffeqsolve = (
        ODETerm, Dopri5, PIDController, SaveAt, diffeqsolve)
    sys.modules["diffrax"] = dfx


class OracleSolve:
    """diffrax.diffeqsolve stand-in: float32 casts (jax x64 off) + oracle_solve_rows."""

    def __init__(self, coupling: str = "f32"):
        from oracle import kura_oracle as ko
        self.ko = ko
        self.ctx = {}
        self.calls = 0
        self.enabled = True
        self.coupling = coupling   # KuraConfig.coupling of the solver (reference_golden.npz: "f32")

    def __call__(self, f, args, t0, t1, dt0, y0, ts, ctrl):
        w0, kn, n, alpha, pulse = args
        ts = np.asarray(ts, np.float64)
        if not self.enabled:  # plumbing-only runs: cheap constant solution
            return np.repeat(np.asarray(y0, np.float32)[None, :], len(ts), axis=0)
        a32 = np.asarray(alpha, np.float32)
        key = (int(n), float(np.float32(kn)), hashlib.sha1(a32.tobytes()).hexdigest(), self.coupling)
        if key not in self.ctx:
            import importlib
            sim = importlib.import_module("dbs-gym_amd.sim")
            kura = importlib.import_module("dbs-gym_amd")
            prm = kura.reference_params("env0")
            prm["num_oscillators"] = int(n)
            cfg = sim.make_config(prm, 1, reward_func="bbpow_action", coupling=self.coupling)
            cfg.kn = np.float32(kn)
            cfg.rtol, cfg.atol = np.float32(ctrl.rtol), np.float32(ctrl.atol)
            cfg.dt0 = np.float32(dt0)
            self.ctx[key] = self.ko.Oracle(cfg, a32)
        o = self.ctx[key]
        self.calls += 1
        rows, _ = o.solve_rows(np.asarray(w0, np.float32), np.asarray(pulse, np.float32), ts,
                               np.asarray(y0, np.float32))
        return rows


def main(ref_root: str) -> None:
    solver = OracleSolve()
    tmp = tempfile.mkdtemp(prefix="kura_stubs_")
    _write_stubs(tmp, solver)
    sys.path.insert(0, tmp)
    sys.path.insert(0, HERE)
    sys.path.insert(0, ref_root)
    import contextlib
    import io
    import environment.utils as U   # noqa: E402
    import environment.env as E     # noqa: E402
    from environment.env_configs import env0 as C0, env1 as C1  # noqa: E402

    out = {}
    quiet = contextlib.redirect_stdout(io.StringIO())

    # 1. driver-side setup RNG streams (utils.py:909-942)
    for tag, cfg in (("env0", C0.params_dict_train), ("env1e0", C1.eval_envs_list[0])):
        np.random.seed(228)
        r = U.generate_w0_with_locus(512, [8, 8, 8], 0.1, locus_center=cfg["locus_center"],
                                     locus_size=cfg["locus_size"], wmuL=cfg["wmuL"], wsdL=cfg["wsdL"], show=False)
        for k, v in zip(("w0", "coords", "grid", "w0_wo", "w_locus", "lmask"), r):
            out[f"setup_{tag}_{k}"] = np.asarray(v)

    # 2. coupling + conductances through KuramotoJAX/SimpleDBS (env.py:191-244)
    coords, grid = out["setup_env0_coords"], out["setup_env0_grid"]
    for tag, ec, rc, cm in (("a", [[4, 3, 4]], [[1, 1, 1]], 0.1), ("b", [[5, 2, 3]], [[3, 5, 1]], 0.1),
                            ("c", [[4, 3, 4]], [[1, 1, 1]], 0.15), ("d", [[4, 3, 4]], [[1, 1, 1]], 2.1)):
        with quiet:
            kj = E.KuramotoJAX(512, 0.52, [8, 8, 8], out["setup_env0_w0"].copy(), coords, grid, ec, rc, cm,
                               spatial_kernel="cos", electrode_amps=[0.0], electrode_prc_type="dummy")
        out[f"cond_{tag}_gstim"] = np.asarray(kj.dbs.conductances[0])
        out[f"cond_{tag}_grec"] = np.asarray(kj.dbs.rec_conductances[0])
        if tag == "a":
            a32 = np.asarray(kj.alpha, np.float32)
            out["alpha_rows_idx"] = np.array([0, 73, 284, 511])
            out["alpha_rows"] = a32[[0, 73, 284, 511]]
            out["alpha_sha1"] = np.frombuffer(hashlib.sha1(a32.tobytes()).digest(), np.uint8)
            out["dist_rows"] = np.asarray(kj.distance_matrix)[[0, 73, 284, 511]]
            # 3. reference RHS on random float32 states with float32 args (jax x64 off)
            rng = np.random.default_rng(5)
            ys = rng.uniform(0, 2000, (4, 512)).astype(np.float32)
            pulse = (np.asarray(kj.dbs.conductances[0]) * 3.7).astype(np.float32)
            args = (np.asarray(kj.w0, np.float32), np.float32(0.52 / 512), 512, a32, pulse)
            out["rhs_y"] = ys
            out["rhs_pulse"] = pulse
            out["rhs_w0"] = args[0]
            out["rhs_f"] = np.stack([np.asarray(kj.dynamics(0.0, y, args), np.float32) for y in ys])

    # 4./5. LFP and rewards on fixed signals (env.py:396-412, :638-688)
    rng = np.random.default_rng(11)
    sig = rng.uniform(0, 3000, (19, 512)).astype(np.float32)
    out["lfp_sig"] = sig
    with quiet:
        env = _make_env(E, C1.eval_envs_list[0], out, "bbpow_action")
    out["lfp_naive"] = np.asarray(env.calc_naive_lfp(sig))
    out["lfp_dist"] = np.asarray(env.calc_distance_lfp(sig))
    out["lfp_grec"] = np.asarray(env.kuramoto.dbs.rec_conductances[0])
    t = np.arange(2340) * 5e-4
    wins = [rng.uniform(-0.3, 0.3, 2340), 0.2 * np.sin(2 * np.pi * 17.0 * t) + 0.05 * rng.standard_normal(2340),
            0.01 * np.sin(2 * np.pi * 15.0 * t)]
    W = np.stack(wins)
    out["rew_win64"] = W
    out["rew_u"] = np.array([0.0, 2.5, -5.0])
    out["rew_r1_f64"] = np.array([env.reward_bbpow_action(w, [u]) for w, u in zip(W, out["rew_u"])])
    out["rew_r1_f32"] = np.array([env.reward_bbpow_action(w.astype(np.float32), [u]) for w, u in zip(W, out["rew_u"])])
    out["rew_r2_f64"] = np.array([env.reward_temp_const_lfp_betafilt_action(w, [u]) for w, u in zip(W, out["rew_u"])])
    out["rew_r3_f64"] = np.array([env.reward_bbpow_threth_action(w, [u]) for w, u in zip(W, out["rew_u"])])

    # 6. arange time grid over a full training episode (plumbing-only solve)
    solver.enabled = False
    with quiet:
        env = _make_env(E, C0.params_dict_train, out, "bbpow_action")
        nI, nII, tcur = [], [], []
        for _ in range(5555):
            env.step([0.0])
            nI.append(len(env.t_eval_step_I))
            nII.append(len(env.t_eval_step_II))
            tcur.append(env.current_time)
    out["grid_nI"] = np.array(nI, np.int32)
    out["grid_nII"] = np.array(nII, np.int32)
    out["grid_t"] = np.array(tcur, np.float64)
    out["grid_done_last"] = np.array([env.done])
    solver.enabled = True

    # 7./9. seeded construction + reset + 60 steps through the reference env with
    # the build's solver plugged in (env.py:277-614)
    for tag, cfg_d, rew in (("env0", C0.eval_envs_list[0], "bbpow_action"),
                            ("env1", C1.eval_envs_list[0], "temp_const_action")):
        with quiet:
            env = _make_env(E, cfg_d, out, rew)
        out[f"traj_{tag}_theta0"] = np.asarray(env.init_state, np.float64)
        out[f"traj_{tag}_w0"] = np.asarray(env.kuramoto.w0, np.float64)
        out[f"traj_{tag}_gstim"] = np.asarray(env.kuramoto.dbs.conductances, np.float64)
        out[f"traj_{tag}_grec"] = np.asarray(env.kuramoto.dbs.rec_conductances, np.float64)
        out[f"traj_{tag}_obs0"] = np.asarray(env.theta_state, np.float32)
        out[f"traj_{tag}_y0"] = np.asarray(env.sol_state[-1], np.float32)
        out[f"traj_{tag}_t0"] = np.array([env.current_time])
        arng = np.random.default_rng(3)
        acts = arng.uniform(-1, 1, 60).astype(np.float32)
        obs, rews, tm, ys, ts = [], [], [], [], []
        with quiet:
            for a in acts:
                o, r, d, tr, info = env.step([a])
                obs.append(o[0])
                rews.append(r)
                tm.append(np.pad(np.asarray(env.theta_mean, np.float32), (0, 32 - len(env.theta_mean))))
                ys.append(np.asarray(env.sol_state_[-1], np.float32))
                ts.append(env.current_time)
        out[f"traj_{tag}_actions"] = acts
        out[f"traj_{tag}_obs"] = np.stack(obs)
        out[f"traj_{tag}_rew"] = np.array(rews, np.float64)
        out[f"traj_{tag}_theta_mean"] = np.stack(tm)
        out[f"traj_{tag}_y"] = np.stack(ys)
        out[f"traj_{tag}_t"] = np.array(ts)

    # 8. env2 plasticity random walk (env.py:21-57)
    np.random.seed(77)
    out["perturb_init"] = out["setup_env0_w0_wo"]
    out["perturb_walk"] = E.generate_perturbations(out["setup_env0_w0_wo"], M=20, step_scale=0.02)

    path = os.path.join(HERE, "reference_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(out)} arrays, {solver.calls} oracle solves)")


def _make_env(E, cfg_d, out, reward):
    d = dict(cfg_d)
    tag = "env1e0" if list(d["locus_center"]) == [1, 2, 3] else "env0"
    d["w0"] = out[f"setup_{tag}_w0"].copy()
    d["w0_without_locus"] = out[f"setup_{tag}_w0_wo"].copy()
    d["locus_without_w0"] = out[f"setup_{tag}_w_locus"].copy()
    d["locus_mask"] = out[f"setup_{tag}_lmask"].copy()
    d["neur_coords"] = out[f"setup_{tag}_coords"].copy()
    d["neur_grid"] = out[f"setup_{tag}_grid"].copy()
    d["reward_func"] = reward
    return E.SpatialKuramoto(params_dict=d)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
