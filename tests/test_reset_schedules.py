"""Row a18: the host decisions of reset() -- env2 electrode drift,
encapsulation and plasticity events, env1/env2 spatial resampling, and the
natural frequencies / conductances / initial phases they produce -- bit for
bit against the reference's own reset() (environment/env.py:483-598), and the
evaluate_HF_DBS.py protocol's draw order (dbs-gym_amd/evaluation.py).
Fixtures: tests/golden/make_golden_resets.py (stub-imported reference,
plumbing-only solve)."""
import hashlib
import importlib
import os

import numpy as np
import pytest

kura = importlib.import_module("dbs-gym_amd")
ev = importlib.import_module("dbs-gym_amd.evaluation")

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_resets.npz"))


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(np.asarray(a, np.float64)).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["env1", "env2"])
def test_training_env_reset_schedule(name):
    tag = f"{name}train"
    p = kura.fill_driver_arrays(kura.reference_params(name), w0_seed=int(G[f"{tag}_w0seed"][0]))
    p["reward_func"] = "bbpow_action"
    h = kura.EnvHost(p)
    n = len(G[f"{tag}_encaps"])
    for r in range(n):
        w0, gs, gr, th0 = h.reset_draws()
        assert h.elec_coords[0] == G[f"{tag}_elec"][r].tolist(), (r, h.elec_coords)
        assert h.rec_coords[0] == G[f"{tag}_rec"][r].tolist(), (r, h.rec_coords)
        assert h.encapsulation_coeff == G[f"{tag}_encaps"][r], r
        assert sha(w0) == G[f"{tag}_w0"][r], f"w0 differs at reset {r}"
        _cond(tag, r, gs, gr)
        assert sha(th0) == G[f"{tag}_theta0"][r], f"theta0 differs at reset {r}"


def _cond(tag, r, gs, gr):
    # the reference's distances go through BLAS (np.linalg.norm) and may fuse:
    # conductances agree to 1 ulp (as in test_golden_reference.test_conductances)
    for k, v in (("gstim", gs), ("grec", gr)):
        ref = G[f"{tag}_{k}_tab"][G[f"{tag}_{k}_idx"][r]]
        np.testing.assert_allclose(v, ref, rtol=0, atol=4.5e-16, err_msg=f"{k} at reset {r}")


def test_schedules_exercise_every_event():
    # the fixtures cover spatial resampling (env1) and all three env2 drifts
    assert len({tuple(x) for x in G["env1train_elec"]}) >= 3
    assert len({tuple(x) for x in G["env2train_elec"]}) >= 5
    assert G["env2train_encaps"].max() > G["env2train_encaps"][0]
    assert len(set(G["env2train_w0"])) > 10            # plasticity walk + its periodic restart


@pytest.mark.parametrize("name", ["env0", "env1", "env2"])
def test_eval_protocol_draw_order(name):
    tag = f"proto_{name}"
    plist, draws = ev.protocol_draws(name, n_episodes=5)
    order = [d[0] for d in draws] + [x for d in draws for x in d[1:]]   # constructors, then env by env
    assert len(order) == len(G[f"{tag}_theta0"])
    for r, (w0, gs, gr, th0) in enumerate(order):
        assert sha(w0) == G[f"{tag}_w0"][r], f"w0 differs at protocol reset {r}"
        _cond(tag, r, gs, gr)
        assert sha(th0) == G[f"{tag}_theta0"][r], f"theta0 differs at protocol reset {r}"
