#!/usr/bin/env python3
"""Pin the per-reset host decisions of SpatialKuramoto.reset()
(environment/env.py:467-598: env2 electrode drift, encapsulation and
plasticity events, env1/env2 spatial resampling, natural frequencies,
conductances and initial phases) against the reference itself.  Build
container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_resets.py /root/reference

Uses the stub harness of make_golden.py with the plumbing-only solve (the
transient's values do not feed any later draw).  Two reference bugs must be
stepped around to run env2 at all, in the harness
only -- the reference tree is never modified:
  * env.py:368 asserts plasticity_drift_freq >= 2, which every shipped env2
    config violates: the env is constructed with 2 and plasticity_episode /
    params_dict['plasticity_drift_freq'] are set to the config's 1 right
    after (the first drift decision happens at reset 1, after construction);
  * env.py:520 calls the undefined calc_next_temp_event: aliased to
    calc_next_event (the name the paper-era bytecode used).
Writes tests/golden/reference_resets.npz: per reset the electrode/recorder
coordinates, the encapsulation coefficient and SHA-1 digests of w0 and theta0
(float64 bytes) and the conductances (deduplicated arrays), for
  * env1 train (spatial variation every 10 resets) and env2 train, 40 resets
    of one env each;
  * the evaluate_HF_DBS.py protocol (seed 228; for each of the five eval
    configs in turn generate_w0_with_locus then the constructor, all on the
    global RNG; then 1 + 5 resets per env, env by env) for env0, env1 and
    env2."""
from __future__ import annotations

import contextlib
import copy
import hashlib
import io
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import OracleSolve, _write_stubs  # noqa: E402


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(np.asarray(a, np.float64)).tobytes()).hexdigest()


def record(env):
    k = env.kuramoto
    return {"elec": np.asarray(env.elec_coords, np.int64).reshape(-1, 3),
            "rec": np.asarray(env.rec_coords, np.int64).reshape(-1, 3),
            "encaps": float(env.encapsulation_coeff),
            "w0": sha(k.w0), "gstim": np.asarray(k.dbs.conductances, np.float64),
            "grec": np.asarray(k.dbs.rec_conductances, np.float64),
            "theta0": sha(env.init_state)}


def make_env(E, U, d, rs_seed_global=None):
    d = copy.deepcopy(d)
    env2 = d.get("temporal_drift") and d.get("plasticity_drift_freq", 2) < 2
    freq = d.get("plasticity_drift_freq")
    if env2:
        d["plasticity_drift_freq"] = 2
    env = E.SpatialKuramoto(params_dict=d)
    if env2:
        env.plasticity_episode = freq
        env.params_dict["plasticity_drift_freq"] = freq
    return env


def fill(U, d):
    r = U.generate_w0_with_locus(d["num_oscillators"], d["grid_size"], d["coord_modif"],
                                 locus_center=d["locus_center"], locus_size=d["locus_size"],
                                 wmuL=d["wmuL"], wsdL=d["wsdL"], show=False)
    for k, v in zip(("w0", "neur_coords", "neur_grid", "w0_without_locus", "locus_without_w0", "locus_mask"), r):
        d[k] = v
    return d


def main(ref_root: str) -> None:
    solver = OracleSolve()
    solver.enabled = False   # plumbing only: the transient's values feed no later draw
    tmp = tempfile.mkdtemp(prefix="kura_stubs_")
    _write_stubs(tmp, solver)
    sys.path.insert(0, tmp)
    sys.path.insert(0, ref_root)
    import environment.utils as U   # noqa: E402
    import environment.env as E     # noqa: E402
    from environment.env_configs import env0 as C0, env1 as C1, env2 as C2  # noqa: E402
    E.SpatialKuramoto.calc_next_temp_event = E.SpatialKuramoto.calc_next_event
    quiet = contextlib.redirect_stdout(io.StringIO())
    out = {}

    def put(tag, recs):
        out[f"{tag}_elec"] = np.stack([r["elec"][0] for r in recs])
        out[f"{tag}_rec"] = np.stack([r["rec"][0] for r in recs])
        out[f"{tag}_encaps"] = np.array([r["encaps"] for r in recs])
        for k in ("w0", "theta0"):
            out[f"{tag}_{k}"] = np.array([r[k] for r in recs])
        # conductances as arrays (deduplicated): the reference's distances go
        # through BLAS (np.linalg.norm), which may fuse, so they are compared
        # to 1 ulp, not by digest
        for k in ("gstim", "grec"):
            tab, idx = [], []
            for r in recs:
                for j, t in enumerate(tab):
                    if np.array_equal(t, r[k]):
                        idx.append(j)
                        break
                else:
                    idx.append(len(tab))
                    tab.append(r[k])
            out[f"{tag}_{k}_tab"] = np.stack(tab)
            out[f"{tag}_{k}_idx"] = np.array(idx)

    # (a) one training env, 40 resets (the constructor's reset is reset 0)
    for tag, C, wseed in (("env1train", C1, 228), ("env2train", C2, 228)):
        d = copy.deepcopy(C.params_dict_train)
        np.random.seed(wseed)
        d = fill(U, d)
        d["reward_func"] = "bbpow_action"
        out[f"{tag}_w0seed"] = np.array([wseed])
        with quiet:
            env = make_env(E, U, d)
            recs = [record(env)]
            for _ in range(39):
                env.reset()
                recs.append(record(env))
        put(tag, recs)
        print(tag, "encaps", out[f"{tag}_encaps"][:12], "elec moves", len(set(map(tuple, out[f"{tag}_elec"]))))

    # (b) the evaluate_HF_DBS.py protocol: seed 228 (:20); for each of the 5 eval
    # configs in turn generate_w0_with_locus then make_env (:195-218) -- the
    # constructor reseeds the global RNG, so env k+1's frequencies follow env k's
    # construction -- then 1 + 5 resets per env (evaluate_policy_)
    for tag, C in (("proto_env0", C0), ("proto_env1", C1), ("proto_env2", C2)):
        np.random.seed(228)
        recs = []
        with quiet:
            envs = []
            for k in range(5):
                d = copy.deepcopy(C.eval_envs_list[k])
                d = fill(U, d)
                d["reward_func"] = "bbpow_action"
                d["dbs_action_bounds"] = [-5, 5]
                envs.append(make_env(E, U, d))
                recs.append(record(envs[-1]))
            for env in envs:
                for _ in range(6):
                    env.reset()
                    recs.append(record(env))
        put(tag, recs)   # order: 5 constructor resets, then env 0's six resets, env 1's, ...
        print(tag, len(recs), "resets")
    path = os.path.join(HERE, "reference_resets.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
