#!/usr/bin/env python3
"""Round-3 boundary fixtures from the reference itself (build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r03.py /root/reference

Uses the stub harness of make_golden.py (plumbing-only solve: none of these
values depends on the solver arithmetic) with gymnasium's Env.reset(seed)
semantics (it seeds only the env's own ``np_random``, gymnasium 1.1
``Env.reset``).  Writes tests/golden/reference_boundary.npz:

* ``seed_*``   -- reset(seed=s) does not touch the draws: the global NumPy
  RNG state after construction + reset() + reset(seed=123) + reset(seed=7)
  equals the unseeded sequence's (digests of the MT19937 key and position,
  and of the initial phases drawn by each reset);
* ``rw_*``     -- reward_bbpow_action / reward_temp_const_lfp_betafilt_action /
  reward_bbpow_threth_action (env.py:638-688) on seeded 1-D windows of
  several lengths (2 * 2340 as PIDController.predict's observation.ravel()
  of a 2-env VecEnv, 1000, 4681, 100, 16), action 0.3;
* ``attr_*``   -- side attributes after construction and 5 resets of an env2
  train env with save_events and a log_path: reset_count, current_time,
  kw0 digest, the files np.save wrote (env.py:559-562) and the keys/lengths
  of temporal_events;
* ``cond_*``   -- env.kuramoto.dbs.conductances of the env1 explore setup.
Only data is written (inputs, outputs, digests)."""
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
from make_golden_resets import fill, make_env  # noqa: E402

LENGTHS = (4680, 1000, 4681, 100, 16)


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(np.asarray(a, np.float64)).tobytes()).hexdigest()


def rng_digest():
    st = np.random.get_state()
    return hashlib.sha1(st[1].tobytes() + np.int64(st[2]).tobytes()).hexdigest()


def main(ref_root: str) -> None:
    solver = OracleSolve()
    solver.enabled = False
    tmp = tempfile.mkdtemp(prefix="kura_stubs_")
    _write_stubs(tmp, solver)
    # gymnasium 1.1 Env.reset(seed): seeds self.np_random only
    open(os.path.join(tmp, "gymnasium", "__init__.py"), "w").write(
        "import numpy as _np\n"
        "class Env:\n"
        "    def reset(self, seed=None, options=None):\n"
        "        if seed is not None:\n"
        "            self._np_random = _np.random.default_rng(seed)\n"
        "from . import spaces\n")
    sys.path.insert(0, tmp)
    sys.path.insert(0, ref_root)
    import environment.env as E     # noqa: E402
    import environment.utils as U   # noqa: E402
    from environment.env_configs import env1 as C1, env2 as C2  # noqa: E402
    E.SpatialKuramoto.calc_next_temp_event = E.SpatialKuramoto.calc_next_event
    quiet = contextlib.redirect_stdout(io.StringIO())
    out = {}

    # (1) reset(seed) leaves the draw streams alone
    runs = {}
    for tag, seeds in (("plain", (None, None, None)), ("seeded", (None, 123, 7))):
        d = copy.deepcopy(C1.params_dict_train)
        np.random.seed(228)
        d = fill(U, d)
        d["reward_func"] = "bbpow_action"
        with quiet:
            env = make_env(E, U, d)
            th, rs = [sha(env.init_state)], [rng_digest()]
            for s in seeds:
                env.reset(seed=s)
                th.append(sha(env.init_state))
                rs.append(rng_digest())
        runs[tag] = (th, rs)
        out[f"seed_{tag}_theta0"] = np.array(th)
        out[f"seed_{tag}_rng"] = np.array(rs)
    out["seed_w0seed"] = np.array([228])
    assert runs["plain"] == runs["seeded"], "reference reset(seed) changed the draws"

    # (2) rewards on arbitrary lengths
    d = copy.deepcopy(C1.params_dict_train)
    np.random.seed(11)
    d = fill(U, d)
    d["reward_func"] = "bbpow_action"
    with quiet:
        env = make_env(E, U, d)
    rng = np.random.default_rng(2024)
    for L in LENGTHS:
        x = (0.08 * np.sin(2 * np.pi * 16.0 * np.arange(L) * 5e-4) + 0.02 * rng.standard_normal(L)).astype(np.float64)
        out[f"rw_x_{L}"] = x
        out[f"rw_r1_{L}"] = np.array([env.reward_bbpow_action(x, [0.3])])
        out[f"rw_r3_{L}"] = np.array([env.reward_bbpow_threth_action(x, [0.3])])
        try:
            r2 = env.reward_temp_const_lfp_betafilt_action(x, [0.3])
        except ValueError:
            r2 = np.nan
        out[f"rw_r2_{L}"] = np.array([r2])
    try:
        env.reward_temp_const_lfp_betafilt_action(np.zeros(15), [0.3])
        out["rw_r2_15_raises"] = np.array([0])
    except ValueError:
        out["rw_r2_15_raises"] = np.array([1])
    out["rw_lengths"] = np.array(LENGTHS)
    out["rw_verbose_dt"] = np.array([d["verbose_dt"]])

    # (3) side attributes and event logging of an env2 train env
    logdir = tempfile.mkdtemp(prefix="kura_events_")
    d = copy.deepcopy(C2.params_dict_train)
    np.random.seed(5)
    d = fill(U, d)
    d["reward_func"] = "bbpow_action"
    d["save_events"] = True
    d["log_path"] = logdir
    with quiet:
        env = make_env(E, U, d)
        rc, ct, kw = [env.reset_count], [env.current_time], [sha(env.kw0)]
        for _ in range(5):
            env.reset()
            rc.append(env.reset_count)
            ct.append(env.current_time)
            kw.append(sha(env.kw0))
    out["attr_reset_count"] = np.array(rc)
    out["attr_current_time"] = np.array(ct)
    out["attr_kw0"] = np.array(kw)
    out["attr_files"] = np.array(sorted(os.listdir(logdir)))
    ev = env.temporal_events
    out["attr_event_keys"] = np.array(sorted(ev.keys()))
    out["attr_event_lens"] = np.array([len(ev[k]) for k in sorted(ev.keys())])
    out["attr_kgrid_size"] = np.array(env.kgrid_size)

    # (4) kuramoto.dbs.conductances of the explore notebook's env1 setup (cell 13)
    d = copy.deepcopy(C1.params_dict_train)
    np.random.seed(10)
    d = fill(U, d)
    d["reward_func"] = "bbpow_action"
    with quiet:
        env = make_env(E, U, d)
    out["cond_stim"] = np.asarray(env.kuramoto.dbs.conductances, np.float64)
    out["cond_rec"] = np.asarray(env.kuramoto.dbs.rec_conductances, np.float64)
    out["cond_w0seed"] = np.array([10])

    path = os.path.join(HERE, "reference_boundary.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)")
    for k in sorted(out):
        if k.startswith(("rw_r", "attr_", "seed_")):
            print(k, out[k] if out[k].size < 12 else out[k].shape)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
