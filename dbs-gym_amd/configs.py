"""Environment configurations (restated from environment/env_configs/env{0,1,2}.py).

``reference_params(name, split, idx)`` returns the same ``params_dict`` the
reference builds (keys identical to env_configs/*.py), without the
driver-filled arrays (w0, neur_coords, ...), which ``vec_env`` fills the way
aDBS_RL/train_aDBS_RL.py:95-112 does.
"""
from __future__ import annotations

import copy

import numpy as np

# env_configs/env1.py:4-20 -- (stim, record, locus) triples used by the
# spatial-variation feature (env.py:544-557) and the env1/env2 eval configs.
STIM_REC_LOCUS = [
    [[5, 2, 3], [3, 5, 1], [1, 2, 3]],
    [[4, 3, 1], [2, 5, 4], [2, 1, 4]],
    [[4, 3, 6], [2, 6, 4], [4, 3, 2]],
    [[5, 2, 1], [3, 5, 3], [5, 2, 5]],
    [[1, 3, 2], [4, 1, 4], [4, 5, 4]],
    [[6, 6, 4], [4, 4, 3], [3, 6, 5]],
    [[6, 5, 3], [1, 6, 4], [3, 2, 6]],
    [[6, 3, 5], [4, 1, 1], [5, 6, 1]],
    [[6, 5, 4], [1, 6, 3], [3, 2, 1]],
    [[4, 5, 3], [3, 3, 1], [6, 4, 1]],
    [[2, 3, 2], [4, 5, 3], [1, 5, 4]],
    [[5, 3, 2], [5, 5, 4], [5, 2, 5]],
    [[1, 6, 2], [6, 5, 1], [3, 2, 4]],
    [[2, 3, 3], [3, 3, 6], [1, 1, 5]],
    [[3, 5, 2], [1, 6, 4], [1, 3, 3]],
]

N_NEURONS = 512
GRID_SIZE = [8, 8, 8]
COORD_MODIF = 0.1
LOCUS_CENTER = [4, 4, 4]
LOCUS_SIZE = 0.55

# Common keys (env_configs/env0.py:10-79).
_BASE = {
    "logger_name": "k", "log_path": None, "rand_seed": 10, "verbose": 1,
    "model_type": "2dspatial", "K": 0.52, "num_oscillators": N_NEURONS, "grid_size": GRID_SIZE,
    "w0": None, "wmuL": 17, "wsdL": 1, "neur_coords": None, "neur_grid": None, "coord_modif": COORD_MODIF,
    "spatial_kernel": "cos", "wavelet_amp": 1.0, "wavelet_steepness": 0.6,
    "elec_coords": [[4, 3, 4]], "rec_coords": [[1, 1, 1]], "directed_stimulation": False,
    "conduct_modifier": 0.1, "recording_kernel": "naive", "locus_size": LOCUS_SIZE,
    "locus_center": LOCUS_CENTER,
    "transient_state_len": 200.0, "electrode_width": 0.15, "electrode_pause": 0.75,
    "electrode_amps": [0.0], "dbs_action_bounds": [-5, 5],
    "electrode_prc_scaling": 1.0, "electrode_prc_type": "dummy", "naive_dbs": False,
    "verbose_dt": 0.05, "total_episode_len": 5000, "reward_func": None, "observe_wind_counts": 130,
    "init_state_type": "normal", "init_state_mean": np.pi, "init_state_sd": 0.6,
    "temporal_drift": False, "random_freq_update": True, "save_events": False,
    "electrode_drift_freq": 0, "plasticity_drift_freq": 0, "plasticity_percent": 0,
    "reset_plasticity_episode": 0, "encapsulation_drift_freq": 0, "encapsulation_percent": 0,
    "mov_modulation_drift_freq": 0, "spatial_feature": False, "spatial_var_freq": -1,
}

# Per-config train overrides (env0.py:10-79, env1.py:29-99, env2.py:29-101).
_TRAIN = {
    "env0": {},
    "env1": {"recording_kernel": "gaussian", "spatial_feature": True, "spatial_var_freq": 10},
    "env2": {"recording_kernel": "gaussian", "temporal_drift": True, "electrode_drift_freq": 5,
             "plasticity_drift_freq": 1, "plasticity_percent": 2, "reset_plasticity_episode": 10,
             "encapsulation_drift_freq": 7, "encapsulation_percent": 2, "mov_modulation_drift_freq": 3,
             "spatial_feature": True, "spatial_var_freq": 10},
}

# Eval overrides (env*.py eval0..eval4, eval_envs_list at env0.py:442 etc.).
_EVAL = {
    "env0": [{"rand_seed": s, "total_episode_len": 1000} for s in (11, 10, 20, 30, 40)],
    "env1": [{"elec_coords": [STIM_REC_LOCUS[i][0]], "rec_coords": [STIM_REC_LOCUS[i][1]],
              "locus_center": STIM_REC_LOCUS[i][2], "total_episode_len": 1000,
              "spatial_feature": False, "spatial_var_freq": 0} for i in range(5)],
    "env2": [{"elec_coords": [e], "rec_coords": [r], "locus_center": lc, "total_episode_len": 1000,
              "random_freq_update": False, "save_events": True, "electrode_drift_freq": 2,
              "reset_plasticity_episode": 7, "encapsulation_drift_freq": 2, "spatial_feature": False,
              "spatial_var_freq": -1}
             for e, r, lc in ([[4, 3, 6], [2, 1, 5], [5, 1, 4]], [[2, 4, 6], [6, 6, 4], [2, 5, 1]],
                              [[1, 6, 1], [6, 6, 2], [3, 2, 3]], [[5, 5, 1], [3, 4, 3], [4, 2, 1]],
                              [[3, 2, 4], [6, 2, 3], [4, 4, 2]])],
}


def reference_params(name: str = "env0", split: str = "train", idx: int = 0, **overrides) -> dict:
    """The reference's params dict for env0/env1/env2 (train or eval[idx])."""
    if name not in _TRAIN:
        raise ValueError(f"unknown config {name!r}")
    d = copy.deepcopy(_BASE)
    d.update(copy.deepcopy(_TRAIN[name]))
    if split == "eval":
        d.update(copy.deepcopy(_EVAL[name][idx]))
    elif split != "train":
        raise ValueError(split)
    d.update(overrides)
    return d


def synthetic_params(name: str = "env0", n_osc: int = 1024, **overrides) -> dict:
    """BASELINE.json synthetic configs: the reference config scaled to N
    oscillators on a regular grid with spacing 0.1: 16x8x8 for N=1024 and
    32x16x16 for the N=8192 stress config,
    16x16x8 / 16x16x16 for 2048 / 4096, 8x8x(N/64) below, so the reference-indexed
    electrode [4,3,4], recorder [1,1,1] and locus [4,4,4] stay on the grid."""
    if n_osc % 64 or n_osc < 256:
        raise ValueError("synthetic grids need n_osc >= 256 and a multiple of 64")
    d = reference_params(name, "train", **overrides)
    d["num_oscillators"] = n_osc
    big = {2048: [16, 16, 8], 4096: [16, 16, 16], 8192: [32, 16, 16]}   # 8192: SURVEY 8(d) stress grid
    if n_osc in big:
        d["grid_size"] = big[n_osc]
    else:
        d["grid_size"] = [n_osc // 64, 8, 8] if n_osc >= 512 else [8, 8, n_osc // 64]
    d.update(overrides)
    return d
