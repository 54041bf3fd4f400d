#!/usr/bin/env python3
"""Golden fixtures of the product coupling arithmetic (KURA_COUPLING_BF16X3,
kura.h) from the reference itself.  Run in the build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r05.py /root/reference

Same stand-ins as make_golden.py (jax.numpy = NumPy, a gymnasium/seaborn/
imageio stub, a diffrax whose diffeqsolve runs this build's CPU solver), with
the solver in the bf16x3 coupling.  Writes tests/golden/reference_r05.npz:

* ``rhs_<case>_*``: the reference's own ``KuramotoJAX.dynamics``
  (env.py:252-256: fmod, the direct N^2 sin(theta_j - theta_i) sum) on float32
  states with float32 arguments (jax x64 off) for the cases the bf16x3 pin
  must hold on: env0 (cos kernel) with |y| up to 6e3,
  env1's eval env (its locus and electrode), the wavelet kernel (signed alpha,
  utils.py:469-475) and N = 1024 on the 16x8x8 grid of the BASELINE configs;
* ``traj_<tag>_*``: reset + 60 steps of the reference ``SpatialKuramoto``
  (its own step()/reset() plumbing, env.py:415-614) with the bf16x3 solver,
  for env0 (R1) and env1 (R2): the plumbing pin of the product arithmetic.

Only data is written (inputs and the reference's outputs)."""
from __future__ import annotations

import contextlib
import io
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def _rhs_case(E, kj, ys, pulse_scale, n):
    """The reference RHS of kj on the states ys (float32 args, jax x64 off)."""
    a32 = np.asarray(kj.alpha, np.float32)
    pulse = (np.asarray(kj.dbs.conductances[0]) * pulse_scale).astype(np.float32)
    args = (np.asarray(kj.w0, np.float32), np.float32(0.52 / n), n, a32, pulse)
    f = np.stack([np.asarray(kj.dynamics(0.0, y, args), np.float32) for y in ys])
    return dict(y=ys, pulse=pulse, w0=args[0], alpha=a32, f=f)


def main(ref_root: str) -> None:
    solver = mg.OracleSolve()
    solver.coupling = "bf16x3"
    tmp = tempfile.mkdtemp(prefix="kura_stubs_")
    mg._write_stubs(tmp, solver)
    sys.path.insert(0, tmp)
    sys.path.insert(0, ref_root)
    import environment.utils as U   # noqa: E402
    import environment.env as E     # noqa: E402
    from environment.env_configs import env0 as C0, env1 as C1  # noqa: E402

    G = np.load(os.path.join(HERE, "reference_golden.npz"))
    out = {k: G[k] for k in G.files if k.startswith("setup_")}   # the setup arrays _make_env reads
    quiet = contextlib.redirect_stdout(io.StringIO())
    res = {}
    rng = np.random.default_rng(505)
    with quiet:
        # env0: the cos kernel on the reference grid, phases up to 6e3 rad
        kj = E.KuramotoJAX(512, 0.52, [8, 8, 8], out["setup_env0_w0"].copy(), out["setup_env0_coords"],
                           out["setup_env0_grid"], [[4, 3, 4]], [[1, 1, 1]], 0.1, spatial_kernel="cos",
                           electrode_amps=[0.0], electrode_prc_type="dummy")
        ys = np.concatenate([rng.uniform(0, 6000, (3, 512)), rng.uniform(5000, 6000, (1, 512)),
                             rng.uniform(0, 2 * np.pi, (1, 512))]).astype(np.float32)
        res["env0"] = _rhs_case(E, kj, ys, 3.7, 512)
        # env1's first eval env: its locus draws and electrode / recorder
        c1 = C1.eval_envs_list[0]
        kj = E.KuramotoJAX(512, 0.52, [8, 8, 8], out["setup_env1e0_w0"].copy(), out["setup_env1e0_coords"],
                           out["setup_env1e0_grid"], c1["elec_coords"], c1["rec_coords"], 0.1,
                           spatial_kernel="cos", electrode_amps=[0.0] * len(c1["elec_coords"]),
                           electrode_prc_type="dummy")
        ys = rng.uniform(0, 3000, (4, 512)).astype(np.float32)
        res["env1"] = _rhs_case(E, kj, ys, -2.1, 512)
        # the wavelet kernel: signed alpha (utils.py:469-475)
        kj = E.KuramotoJAX(512, 0.52, [8, 8, 8], out["setup_env0_w0"].copy(), out["setup_env0_coords"],
                           out["setup_env0_grid"], [[4, 3, 4]], [[1, 1, 1]], 0.1, spatial_kernel="wavelet",
                           wavelet_amp=2.0, wavelet_steepness=0.5, electrode_amps=[0.0],
                           electrode_prc_type="dummy")
        ys = rng.uniform(0, 4000, (4, 512)).astype(np.float32)
        res["wavelet"] = _rhs_case(E, kj, ys, 5.0, 512)
        # N = 1024 on the 16x8x8 grid (BASELINE configs[1]-[3])
        np.random.seed(228)
        r = U.generate_w0_with_locus(1024, [16, 8, 8], 0.1, locus_center=[4, 4, 4], locus_size=0.55, wmuL=17,
                                     wsdL=1, show=False)
        kj = E.KuramotoJAX(1024, 0.52, [16, 8, 8], np.asarray(r[0]).copy(), np.asarray(r[1]), np.asarray(r[2]),
                           [[4, 3, 4]], [[1, 1, 1]], 0.1, spatial_kernel="cos", electrode_amps=[0.0],
                           electrode_prc_type="dummy")
        ys = np.concatenate([rng.uniform(0, 6000, (3, 1024)), rng.uniform(0, 2 * np.pi, (1, 1024))]).astype(np.float32)
        res["n1024"] = _rhs_case(E, kj, ys, 3.7, 1024)
    fx = {}
    for case, d in res.items():
        for k, v in d.items():
            fx[f"rhs_{case}_{k}"] = v

    # reset + 60 steps through the reference env, bf16x3 solver plugged in
    for tag, cfg_d, rew in (("env0", C0.eval_envs_list[0], "bbpow_action"),
                            ("env1", C1.eval_envs_list[0], "temp_const_action")):
        with quiet:
            env = mg._make_env(E, cfg_d, out, rew)
        fx[f"traj_{tag}_theta0"] = np.asarray(env.init_state, np.float64)
        fx[f"traj_{tag}_w0"] = np.asarray(env.kuramoto.w0, np.float64)
        fx[f"traj_{tag}_gstim"] = np.asarray(env.kuramoto.dbs.conductances, np.float64)
        fx[f"traj_{tag}_grec"] = np.asarray(env.kuramoto.dbs.rec_conductances, np.float64)
        fx[f"traj_{tag}_obs0"] = np.asarray(env.theta_state, np.float32)
        fx[f"traj_{tag}_y0"] = np.asarray(env.sol_state[-1], np.float32)
        fx[f"traj_{tag}_t0"] = np.array([env.current_time])
        acts = np.random.default_rng(3).uniform(-1, 1, 60).astype(np.float32)
        obs, rews, tm, ys, ts = [], [], [], [], []
        with quiet:
            for a in acts:
                o, r, d, tr, info = env.step([a])
                obs.append(o[0])
                rews.append(r)
                tm.append(np.pad(np.asarray(env.theta_mean, np.float32), (0, 32 - len(env.theta_mean))))
                ys.append(np.asarray(env.sol_state_[-1], np.float32))
                ts.append(env.current_time)
        fx[f"traj_{tag}_actions"] = acts
        fx[f"traj_{tag}_obs"] = np.stack(obs)
        fx[f"traj_{tag}_rew"] = np.array(rews, np.float64)
        fx[f"traj_{tag}_theta_mean"] = np.stack(tm)
        fx[f"traj_{tag}_y"] = np.stack(ys)
        fx[f"traj_{tag}_t"] = np.array(ts)

    path = os.path.join(HERE, "reference_r05.npz")
    np.savez_compressed(path, **fx)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(fx)} arrays, {solver.calls} oracle solves)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
