"""Host-side per-environment bookkeeping for a batch of reference envs.

``EnvHost`` reproduces, for one environment, everything
``SpatialKuramoto.__init__``/``reset`` (env.py:277-386, :467-614) decide on
the host before the transient solve: RNG draws, temporal drift (env2),
spatial variation (env1/env2), natural frequencies, conductances and initial
phases.  ``build_batch`` stacks B of them into the arrays libkura consumes.
"""
from __future__ import annotations

import os
from copy import deepcopy

import numpy as np

from . import model_setup as ms
from .configs import STIM_REC_LOCUS


class EnvHost:
    """``rs``: the RandomState standing in for the reference's process-global
    NumPy RNG.  By default each env owns one; pass a shared one to replay a
    driver that constructs several envs in one process (it is reseeded here
    with this env's rand_seed, as SpatialKuramoto.__init__ does, env.py:291)."""

    def __init__(self, params: dict, rs: np.random.RandomState | None = None):
        p = params
        self.p = p
        if rs is None:
            rs = np.random.RandomState()
        rs.seed(p["rand_seed"])                                                # env.py:291
        self.rs = rs
        self.reset_count = -1
        self.N = int(p["num_oscillators"])
        self.grid = np.asarray(p["neur_grid"])
        self.w0_without_locus = np.array(p["w0_without_locus"], dtype=np.float64)
        self.w0_without_locus_ = deepcopy(self.w0_without_locus)
        self.elec_coords = deepcopy(p["elec_coords"])
        self.rec_coords = deepcopy(p["rec_coords"])
        self.encapsulation_coeff = p["conduct_modifier"]                      # env.py:349
        # env.py:356-359 (logged when save_events; kept here always)
        self.temporal_events = {"electrode_drift": [], "encapsulation_drift": [], "plasticity_drift": [],
                                "mov_modulation_drift": []}
        self.w0 = None                 # kuramoto.w0 of the last reset (env.py:213, :601 kw0)
        if p["temporal_drift"]:                                                # env.py:352-377
            self.random_freq_update = p["random_freq_update"]
            self.elec_drift_episode = p["electrode_drift_freq"]
            self.elec_encaps_episode = p["encapsulation_drift_freq"]
            self.encaps_precent = p["encapsulation_percent"]
            # env.py:509 adds encapsulation_percent to the conduct modifier as
            # is (+2 on 0.1: SURVEY.md Appendix C3).  "relative" reads the
            # config's "[%]" unit literally: each event adds that percentage of
            # the initial modifier -- the reading the paper's env2 HF-DBS row
            # agrees with (statistical anchors).
            mode = p.get("encapsulation_mode", "raw")
            if mode == "relative":
                self.encaps_precent = p["encapsulation_percent"] * 0.01 * p["conduct_modifier"]
            elif mode != "raw":
                raise ValueError(f"encapsulation_mode {mode!r}: expected 'raw' or 'relative'")
            # env.py:368 asserts plasticity_drift_freq >= 2, which makes every shipped
            # env2 config unconstructible; the paper-era code had no such assert
            # (SURVEY.md Appendix C1), so it is not enforced here.
            self.plasticity_episode = p["plasticity_drift_freq"]
            self.plasticity_percent = p["plasticity_percent"]
            self.reset_plasticity_episode = p["reset_plasticity_episode"]
            self.plasticity_process_count = 0
            self.w0_process = ms.generate_perturbations(self.rs, self.w0_without_locus,
                                                        M=self.reset_plasticity_episode * 2,
                                                        step_scale=self.plasticity_percent * 0.01)
        self.spatial_events = []
        self.spatial_var_freq = p["spatial_var_freq"]                          # env.py:382-384
        self.spatial_var_episode = self.spatial_var_freq

    def _next_event(self, f, deltas):
        """env.py:457-464 calc_next_event (also used where the reference calls the
        undefined calc_next_temp_event, env.py:520)."""
        if self.random_freq_update:
            return self.rs.choice([f + d for d in deltas])
        return f

    def reset_draws(self):
        """env.py:473-598 up to the transient: returns (w0 f64[N], g_stim f64[ne,N],
        g_rec f64[nr,N], theta0 f64[N])."""
        p = self.p
        self.reset_count += 1
        if p["temporal_drift"]:
            if self.elec_drift_episode == self.reset_count:                    # env.py:485-498
                self.elec_drift_episode += self._next_event(p["electrode_drift_freq"], [-1, 0, 1])
                new = [[10000, 0, 0]]
                b1, b2 = 1, min(p["grid_size"]) - 2
                while any(c < b1 or c > b2 for c in new[0]):
                    d = np.empty(3)
                    for i in range(3):
                        d[i] = self.rs.choice([-1, 1]) * self.rs.choice([0, 1])
                    new = np.asarray(self.elec_coords + d).astype(int).tolist()
                self.elec_coords = new
                self.temporal_events["electrode_drift"].append([self.reset_count, self.elec_coords])
            if self.elec_encaps_episode == self.reset_count:                   # env.py:506-513
                self.elec_encaps_episode += self._next_event(p["encapsulation_drift_freq"], [-2, -1, 0, 1, 2])
                self.encapsulation_coeff += self.encaps_precent
                self.temporal_events["encapsulation_drift"].append([self.reset_count, self.encaps_precent])
            if self.plasticity_episode == self.reset_count:                    # env.py:519-527
                self.plasticity_episode += self._next_event(p["plasticity_drift_freq"], [0, 1])
                self.w0_without_locus = self.w0_process[self.plasticity_process_count]
                self.plasticity_process_count += 1
                self.temporal_events["plasticity_drift"].append([self.reset_count, deepcopy(self.w0_without_locus)])
            if self.reset_count % self.reset_plasticity_episode == 0:           # env.py:532-541
                self.plasticity_process_count = 0
                self.w0_without_locus = deepcopy(self.w0_without_locus_)
                self.w0_process = ms.generate_perturbations(self.rs, self.w0_without_locus,
                                                            M=self.reset_plasticity_episode * 2,
                                                            step_scale=self.plasticity_percent * 0.01)
        if p["spatial_feature"]:                                               # env.py:544-557
            if self.spatial_var_episode == self.reset_count and self.reset_count > 2:
                index = self.rs.choice(len(STIM_REC_LOCUS))
                self.elec_coords = [STIM_REC_LOCUS[index][0]]
                self.rec_coords = [STIM_REC_LOCUS[index][1]]
                self.spatial_var_episode += self.spatial_var_freq
                self.spatial_events.append([self.reset_count, STIM_REC_LOCUS[index]])
        w0 = ms.apply_locus_mask(self.w0_without_locus, p["locus_without_w0"], p["locus_mask"])  # env.py:566
        w0 = ms.remove_negative_w0(self.rs, w0)                                # KuramotoJAX.__init__ env.py:213
        if np.min(w0) < 0:
            raise AssertionError("Natural frequencies w0 must be positive!")   # env.py:214
        g_stim, g_rec = self._conductances()
        theta0 = ms.initial_phases(self.rs, self.N, p["init_state_mean"], p["init_state_sd"])  # env.py:595-598
        self.w0 = w0
        return w0, g_stim, g_rec, theta0


    def _conductances(self):
        """SimpleDBS conductances of the current contacts (env.py:106-156).  They
        depend only on the contacts, the encapsulation modifier and the
        naive_dbs / directed_stimulation / grid_size settings (the reference
        rebuilds SimpleDBS from params_dict at every reset, env.py:584-592),
        which change only at drift / spatial-variation events or a set_attr,
        so the last result is reused until one of them changes (returned
        read-only)."""
        p = self.p
        key = (repr(self.elec_coords), repr(self.rec_coords), float(self.encapsulation_coeff),
               repr(list(p["grid_size"])), bool(p["naive_dbs"]), bool(p.get("directed_stimulation")))
        if getattr(self, "_g_key", None) != key:
            p = self.p
            gs, naive = p["grid_size"], p["naive_dbs"]
            g_stim = ms.conductances(self.grid, gs, self.elec_coords, self.encapsulation_coeff, naive)
            g_rec = ms.conductances(self.grid, gs, self.rec_coords, self.encapsulation_coeff, naive)
            if p.get("directed_stimulation"):                                  # env.py:125-140
                g_stim = ms.directed_conductances(self.grid, gs, self.elec_coords, g_stim)
            g_stim.setflags(write=False)
            g_rec.setflags(write=False)
            self._g_key, self._g = key, (g_stim, g_rec)
        return self._g


def log_temporal_events(params: dict, host: EnvHost) -> str | None:
    """env.py:559-562, after a reset's drift/spatial updates: with save_events
    and a log_path, every reset after the second np.save-s the env's temporal
    events to log_path/temp_<reset_count>.npy (a pickled dict, as the reference
    writes it).  The reference keeps temporal_events only for temporal-drift
    configs (env.py:355-359), so save_events without one raises AttributeError
    there; so does this.  Returns the written path (or None)."""
    if params.get("save_events") and params.get("log_path") is not None and host.reset_count > 1:
        if not params.get("temporal_drift"):
            raise AttributeError("'SpatialKuramoto' object has no attribute 'temporal_events'")
        path = os.path.join(params["log_path"], f"temp_{host.reset_count}.npy")
        np.save(path, host.temporal_events, allow_pickle=True)
        return path
    return None


def fill_driver_arrays(params: dict, w0_seed: int | None = None, rs: np.random.RandomState | None = None) -> dict:
    """What the driver does before constructing the env (train_aDBS_RL.py:95-112):
    generate_w0_with_locus from the driver RNG, then store the arrays."""
    p = deepcopy(params)
    if rs is None:
        rs = np.random.RandomState(w0_seed)
    w0, coords, grid, w0_wo, wl, lm = ms.generate_w0_with_locus(
        rs, p["num_oscillators"], p["grid_size"], p["coord_modif"], p["locus_center"], p["locus_size"],
        p["wmuL"], p["wsdL"])
    p.update(w0=w0, w0_without_locus=w0_wo, locus_without_w0=wl, locus_mask=lm, neur_coords=coords, neur_grid=grid)
    return p


def build_batch(params_list: list[dict]) -> tuple[list[EnvHost], dict]:
    """Host setup for B envs sharing N, the grid and the spatial kernel: returns
    the EnvHost list and the shared coupling alpha (float64, env.py:219-229).
    K may differ per env (its float32(K/N) gain goes to kura_set_env_gain)."""
    hosts = [EnvHost(p) for p in params_list]
    p0 = params_list[0]
    for p in params_list[1:]:
        if p["num_oscillators"] != p0["num_oscillators"] or list(p["grid_size"]) != list(p0["grid_size"]):
            raise ValueError("all envs of a batch must share N and the grid")
        if p["spatial_kernel"] != p0["spatial_kernel"]:
            raise ValueError("all envs of a batch must share the spatial coupling kernel")
    alpha = ms.coupling_alpha(p0["neur_coords"], p0["spatial_kernel"], p0["wavelet_amp"], p0["wavelet_steepness"])
    gains = np.array([np.float32(p["K"] / p["num_oscillators"]) for p in params_list], np.float32)  # env.py:264
    return hosts, {"alpha": alpha, "gain": gains}


def reset_arrays(hosts: list[EnvHost], idx=None):
    """Run reset_draws for the given envs and stack: omega f32, g_stim f64, g_rec f64, theta0 f32."""
    idx = range(len(hosts)) if idx is None else idx
    ws, gss, grs, ths = [], [], [], []
    for i in idx:
        w, gs, gr, th = hosts[i].reset_draws()
        ws.append(w)
        gss.append(gs)
        grs.append(gr)
        ths.append(th)
    return (np.stack(ws).astype(np.float32), np.stack(gss), np.stack(grs), np.stack(ths).astype(np.float32))
