"""theta_record_transient (env.py:611): with kura_set_transient_capture the
reset kernel evaluates the LFP of every transient row but the last and writes
it beside the ring; bit-identical to the oracle's oracle_reset_ex, the ring
and state unchanged by the capture, both LFP kinds, both couplings, and the
split-group kernels."""
import importlib

import numpy as np
import pytest
import torch

from helpers import ko, make_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("name,N,B,part,coupling", [("env0", 512, 19, 0, "auto"), ("env1", 1024, 6, 0, "f32"),
                                                    ("env1", 2048, 5, 512, "bf16x3")])
def test_transient_record_matches_oracle(torch_gpu, name, N, B, part, coupling):
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    reward = "temp_const_action" if name == "env1" else "bbpow_action"
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B, reward=reward, coupling=coupling)
    cfg.part_osc = part
    sims = []
    for cap in (True, False):
        sim = sim_mod.KuraSim(cfg, 0)
        sim.set_coupling(alpha)
        sim.set_env_params(omega, gs, gr)
        sim.set_spectral(ct, st)
        if cap:
            sim.capture_transient(True)
        sim.reset(torch.from_numpy(th0), check_errors=True)
        sims.append(sim)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    obs, tr = o.reset(th0, transient=True)
    g = sims[0].lfp_transient.cpu().numpy()
    assert g.shape == tr.shape == (B, 3999)
    np.testing.assert_array_equal(g, tr)
    np.testing.assert_array_equal(sims[0].obs.cpu().numpy(), obs)
    a, b = sims[0].get_state(), sims[1].get_state()
    for k in ("y", "t", "ring", "spec"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(tr[:, -cfg.window:], a["ring"])
    for s in sims:
        s.close()
    o.close()
