"""BASELINE.json configs[4] at full size on the production library (VERDICT
r04 next #3): N=8192 all-to-all coupling, built exactly as bench.py builds
its shard (bench.build_shard), checked against the oracle on a sample of envs.

* weak form, 1024 envs per GPU: 64 env groups x 8 parts of 1024 = 512
  (group, part) pairs on a persistent grid of 256 workgroups (each loops over
  two pairs);
* strong form at 8 GPUs, 128 envs per GPU: auto part width 256, 8 groups x 32
  parts = 256 workgroups.

Reset + 3 steps; envs sampled across groups, across the 16-env interleave and
from both pairs a workgroup walks, each checked bit for bit against the oracle
run on just them (envs are independent, tests/test_oracle_props.py)."""
import copy
import importlib
import os
import sys
import types

import numpy as np
import pytest

from helpers import ko

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _bench():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def _cmp(g, o, idx, where):
    for k in ("y", "t", "step", "ring", "wpos", "spec"):
        a, b = np.asarray(g[k])[idx], o[k]
        if not np.array_equal(a, b):
            bad = np.argwhere(a != b)
            raise AssertionError(f"{where}: state[{k}] differs at {len(bad)} places, first {bad[:3].tolist()}")


@pytest.mark.parametrize("envs,idx", [
    (1024, [0, 5, 15, 16, 255, 256, 511, 512, 700, 1008, 1015, 1023]),   # weak form: pairs 0..511 on 256 WGs
    (128, [0, 3, 15, 16, 47, 64, 100, 127]),                              # strong form: parts of 256
])
def test_stress_n8192_full_size_sampled(torch_gpu, envs, idx):
    torch = torch_gpu
    bench = _bench()
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    args = types.SimpleNamespace(config="env0", osc=8192, envs=envs, seed=2024, random_k=False,
                                 reward="bbpow_action", part_osc=-1, coupling="f32")   # BF16X3 (AUTO): records below
    cfg, alpha, omega, g_s, g_r, th0, ct, st, gain = bench.build_shard(args, 0)
    assert cfg.part_osc == (1024 if envs == 1024 else 256)   # sim.auto_part_osc
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, g_s, g_r)
    sim.set_env_gain(gain)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0), check_errors=True)
    assert not (sim.stats()[3] & 16), "group barrier timed out"
    idx = np.array(idx)
    c = copy.copy(cfg)
    c.n_envs = len(idx)
    o = ko.Oracle(c, alpha)
    o.set_env_params(omega[idx], g_s[idx], g_r[idx])
    o.set_gain(gain[idx])
    o.set_spectral(ct, st)
    o.reset(th0[idx])
    _cmp(sim.get_state(), o.state(), idx, "reset")
    rng = np.random.default_rng(11)
    for k in range(3):
        a = rng.uniform(-1, 1, (envs, cfg.n_elec)).astype(np.float32)
        sim.step(torch.from_numpy(a), check_errors=True)
        ref = o.step(a[idx])
        for key in ("obs", "reward", "done", "nsamp", "lfp_true", "lfp_rec"):
            np.testing.assert_array_equal(getattr(sim, key).cpu().numpy()[idx], ref[key], err_msg=f"{key} step {k}")
        _cmp(sim.get_state(), o.state(), idx, f"step {k}")
    assert not (sim.stats()[3] & 16)
    o.close()
    sim.close()


@pytest.mark.parametrize("name", ["weak", "strong"])
def test_stress_n8192_bf16x3_against_records(torch_gpu, name):
    """The same two forms in the BF16X3 coupling (the split-group bf16x3
    GEMMs: per-k-block split at parts of 1024, staged split with alpha split
    in registers at parts of 256), replayed against the CPU oracle's records
    committed by tests/golden/make_stress_fixtures.py (the split oracle at
    N=8192 takes ~15 CPU-minutes per form, too long for the GPU box)."""
    import stress_scenarios as ss
    path = os.path.join(ROOT, "tests", "golden", f"stress_{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    R = np.load(path)
    assert str(R["coupling"]) == "bf16x3"
    torch = torch_gpu
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, g_s, g_r, th0, ct, st, gain = ss.shard(name)
    assert cfg.part_osc == int(R["part_osc"])
    idx = R["idx"]
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, g_s, g_r)
    sim.set_env_gain(gain)
    sim.set_spectral(ct, st)
    obs = sim.reset(torch.from_numpy(th0), check_errors=True).cpu().numpy()
    assert not (sim.stats()[3] & 16), "group barrier timed out"

    def check(tag, rec):
        for k, v in rec.items():
            assert np.array_equal(v, R[f"{tag}_{k}"]), f"{tag}: {k} differs for envs {idx}"

    check("reset", ss.snapshot(sim.get_state(), {"obs": obs}, idx))
    for k in range(ss.STEPS):
        sim.step(torch.from_numpy(ss.actions(name, k, cfg.n_elec)), check_errors=True)
        outs = {key: getattr(sim, key).cpu().numpy() for key in ss.OUT_BIG + ss.OUT_SMALL}
        check(f"s{k + 1}", ss.snapshot(sim.get_state(), outs, idx))
    assert not (sim.stats()[3] & 16)
    sim.close()
