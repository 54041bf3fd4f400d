"""The committed records of the product-arithmetic 1000-step gates
(tests/golden/gate_*.npz, tests/golden/make_gate_fixtures.py) are the
oracle's: a prefix of each scenario re-run live through the split-bf16 oracle
on the CPU reproduces the record's reset state, reset observation and
rewards bit for bit.  (The GPU side replays the whole record,
tests/test_gpu_gates.py.)"""
import os

import numpy as np
import pytest

import gate_scenarios as gs

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("scenario,steps", [("env0_r1", 2), ("env1_r2", 1), ("env2_r1_vec", 1)])
def test_record_prefix_is_the_oracle(scenario, steps, monkeypatch):
    R = np.load(os.path.join(GOLDEN, f"gate_{scenario}.npz"))
    assert str(R["coupling"]) == "bf16x3"
    monkeypatch.setattr(gs, "STEPS", steps)
    monkeypatch.setattr(gs, "CHECK", ())
    rec = gs.run_oracle_env2() if scenario == "env2_r1_vec" else gs.run_oracle_env01(scenario)
    assert rec["reset_obs_sha1"].tobytes() == R["reset_obs_sha1"].tobytes()
    for k in gs.STATE_KEYS:
        np.testing.assert_array_equal(rec[f"reset_{k}"], R[f"reset_{k}"], err_msg=k)
    assert rec["reset_ring_sha1"].tobytes() == R["reset_ring_sha1"].tobytes()
    np.testing.assert_array_equal(rec["rewards"], R["rewards"][:steps])


def test_records_hold_the_gate():
    """Each record reaches step 1000 with a finite state, the env2 one through
    three autoresets (reset step counters back at 0 at steps 300/600/900)."""
    for name, (_, _, _, envs) in gs.SCENARIOS.items():
        R = np.load(os.path.join(GOLDEN, f"gate_{name}.npz"))
        assert R["rewards"].shape == (gs.STEPS, envs)
        assert np.all(np.isfinite(R["rewards"])) and np.all(np.isfinite(R["s1000_y"]))
        if name == "env2_r1_vec":
            assert R["s1000_t"].min() > 200.0 + 80.0   # the transient + 100 steps since the third reset
            for r in (1, 2, 3):
                assert np.all(R[f"r{r}_step"] == 0)
            np.testing.assert_array_equal(R["s1000_step"], 100)
        else:
            assert R["s1000_t"].min() > 200.0 + 800.0   # the transient + 1000 steps of 0.80-0.90 units
            np.testing.assert_array_equal(R["s1000_step"], 1000)


def test_stress_records_hold_three_steps():
    """The N=8192 BF16X3 records (tests/golden/make_stress_fixtures.py):
    reset + 3 steps of the sampled envs, clocks advancing, every env's step
    counter at 3 and finite rewards (the GPU replay is
    tests/test_gpu_stress.py)."""
    import stress_scenarios as ss
    for name, (envs, idx) in ss.SCENARIOS.items():
        R = np.load(os.path.join(GOLDEN, f"stress_{name}.npz"))
        assert str(R["coupling"]) == "bf16x3"
        np.testing.assert_array_equal(R["idx"], idx)
        assert int(R["part_osc"]) == (1024 if envs == 1024 else 256)
        assert R["reset_y"].shape == (len(idx), 20)
        np.testing.assert_array_equal(R[f"s{ss.STEPS}_step"], ss.STEPS)
        assert np.all(R[f"s{ss.STEPS}_t"] > R["reset_t"])
        assert all(np.all(np.isfinite(R[f"s{k}_reward"])) for k in range(1, ss.STEPS + 1))


@pytest.mark.parametrize("name", ["env0_r1", "env1_r2"])
def test_b32_records_extend_the_b8_records(name):
    """Env b draws the same inputs and actions at any batch size, and the
    oracle steps every env on its own, so the first 8 envs of the B=32 record
    (two full workgroups on the GPU) are the B=8 record: rewards of every step
    and the checkpoint states."""
    R8 = np.load(os.path.join(GOLDEN, f"gate_{name}.npz"))
    R32 = np.load(os.path.join(GOLDEN, f"gate_{name}_b32.npz"))
    np.testing.assert_array_equal(R32["rewards"][:, :8], R8["rewards"])
    for tag in ("reset",) + tuple(f"s{c}" for c in gs.CHECK):
        for k in gs.STATE_KEYS:
            np.testing.assert_array_equal(R32[f"{tag}_{k}"][:8], R8[f"{tag}_{k}"], err_msg=f"{tag}_{k}")
    np.testing.assert_array_equal(R32["final_ring"][:8], R8["final_ring"])
