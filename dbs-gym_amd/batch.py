"""Host-side per-environment bookkeeping for a batch of reference envs.

``EnvHost`` reproduces, for one environment, everything
``SpatialKuramoto.__init__``/``reset`` (env.py:277-386, :467-614) decide on
the host before the transient solve: RNG draws, temporal drift (env2),
spatial variation (env1/env2), natural frequencies, conductances and initial
phases.  ``build_batch`` stacks B of them into the arrays libkura consumes.
"""
from __future__ import annotations

import functools
import gc
import os
from copy import deepcopy

import numpy as np

from . import hostrng
from . import model_setup as ms
from .configs import STIM_REC_LOCUS


def _without_gc(fn):
    """Batch setup allocates ~10 container objects per env and none of them
    form cycles: the cyclic collector's passes over the growing heap were
    ~0.2 s of a 4096-env setup, so it is paused for the call."""
    @functools.wraps(fn)
    def run(*a, **k):
        on = gc.isenabled()
        gc.disable()
        try:
            return fn(*a, **k)
        finally:
            if on:
                gc.enable()
    return run


def _own_stream(seed):
    """The env's own RNG stream: a native MT19937 stream (hostrng.Stream, bit
    for bit RandomState(seed)) for an integer seed in [0, 2**32), otherwise
    numpy's RandomState itself (which accepts array seeds too)."""
    if isinstance(seed, (int, np.integer)) and 0 <= int(seed) <= 0xFFFFFFFF:
        return hostrng.StreamBank([int(seed)]).stream(0)
    return np.random.RandomState(seed)


def _copy_coords(c):
    """deepcopy of a contact list ([[x, y, z], ...]) without copy.deepcopy's
    per-object overhead."""
    if isinstance(c, list) and all(isinstance(r, list) and all(isinstance(v, (int, float)) for v in r) for r in c):
        return [list(r) for r in c]
    return deepcopy(c)


class EnvHost:
    """``rs``: the RNG standing in for the reference's process-global NumPy
    RNG.  By default each env owns a stream (``stream``: a row of a batch's
    hostrng.StreamBank, already seeded with rand_seed; otherwise one is made);
    pass a shared numpy RandomState as ``rs`` to replay a driver that
    constructs several envs in one process (it is reseeded here with this
    env's rand_seed, as SpatialKuramoto.__init__ does, env.py:291)."""

    def __init__(self, params: dict, rs=None, stream=None, defer_perturbations: bool = False):
        p = params
        self.p = p
        if rs is not None:
            rs.seed(p["rand_seed"])
        elif stream is not None:      # a row of a hostrng.StreamBank, seeded with rand_seed by the caller
            rs = stream
        else:
            rs = _own_stream(p["rand_seed"])                                   # env.py:291
        self.rs = rs
        self.reset_count = -1
        self.N = int(p["num_oscillators"])
        self.grid = np.asarray(p["neur_grid"])
        self.w0_without_locus = np.array(p["w0_without_locus"], dtype=np.float64)
        self.w0_without_locus_ = self.w0_without_locus.copy()
        self.elec_coords = _copy_coords(p["elec_coords"])
        self.rec_coords = _copy_coords(p["rec_coords"])
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
            self.w0_process = None
            if not defer_perturbations:     # else the caller draws it (perturb_batch), first on this stream
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
        w0, gs, gr, th = reset_draws_batch([self])
        return w0[0], gs[0], gr[0], th[0]

    def _advance_events(self):
        """env.py:473-557: the reset counter and the drift / spatial-variation
        events of this reset (their draws, in the reference's order)."""
        if self._advance_drift():
            perturb_batch([self])
        self._advance_spatial()

    def _advance_drift(self) -> bool:
        """env.py:473-531 and the first half of :532-541: the reset counter and
        the temporal-drift events; returns whether this reset regenerates the
        plasticity random walk (env.py:535-541), which the caller then draws
        (perturb_batch) before _advance_spatial."""
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
                return True
        return False

    def _advance_spatial(self):
        """env.py:544-557: the spatial-variation event of this reset."""
        p = self.p
        if p["spatial_feature"]:                                               # env.py:544-557
            if self.spatial_var_episode == self.reset_count and self.reset_count > 2:
                index = self.rs.choice(len(STIM_REC_LOCUS))
                self.elec_coords = [STIM_REC_LOCUS[index][0]]
                self.rec_coords = [STIM_REC_LOCUS[index][1]]
                self.spatial_var_episode += self.spatial_var_freq
                self.spatial_events.append([self.reset_count, STIM_REC_LOCUS[index]])


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
            # shared by the envs of a process that sit on the same grid with the same contacts
            ck = (_grid_key(self.grid),) + key
            hit = _COND_CACHE.get(ck)
            if hit is None:
                gs, naive = p["grid_size"], p["naive_dbs"]
                g_stim = ms.conductances(self.grid, gs, self.elec_coords, self.encapsulation_coeff, naive)
                g_rec = ms.conductances(self.grid, gs, self.rec_coords, self.encapsulation_coeff, naive)
                if p.get("directed_stimulation"):                              # env.py:125-140
                    g_stim = ms.directed_conductances(self.grid, gs, self.elec_coords, g_stim)
                g_stim.setflags(write=False)
                g_rec.setflags(write=False)
                hit = (g_stim, g_rec)
                if len(_COND_CACHE) >= 256:
                    _COND_CACHE.pop(next(iter(_COND_CACHE)))
                _COND_CACHE[ck] = hit
            self._g_key, self._g = key, hit
        return self._g


_COND_CACHE: dict = {}   # (grid bytes, contacts, modifier, settings) -> read-only (g_stim, g_rec)
_GRID_KEYS: dict = {}    # id(read-only grid) -> (grid, its bytes): one bytes object (hashed once) per grid


def _grid_key(grid: np.ndarray) -> bytes:
    """grid.tobytes(), shared by every env on the same read-only grid array
    (fill_driver_arrays_batch hands all envs of a geometry the same one), so
    the 24 KB key is built and hashed once, not once per env."""
    if grid.flags.writeable:
        return grid.tobytes()
    e = _GRID_KEYS.get(id(grid))
    if e is None or e[0] is not grid:
        if len(_GRID_KEYS) >= 64:
            _GRID_KEYS.clear()
        e = (grid, grid.tobytes())
        _GRID_KEYS[id(grid)] = e
    return e[1]


def perturb_batch(hosts: list[EnvHost]) -> None:
    """host.w0_process = generate_perturbations(host.rs, host.w0_without_locus,
    M=2*reset_plasticity_episode, step_scale=plasticity_percent/100)
    (env.py:21-57, :377, :537-541) for each host: one native call per stream
    bank and (M, step) for hosts on native streams, numpy otherwise (in list
    order, for a shared RandomState)."""
    groups: dict = {}
    for h in hosts:
        M, step = h.reset_plasticity_episode * 2, h.plasticity_percent * 0.01
        if isinstance(h.rs, hostrng.Stream):
            groups.setdefault((id(h.rs.bank), M, step), (h.rs.bank, []))[1].append(h)
        else:
            h.w0_process = ms.generate_perturbations(h.rs, h.w0_without_locus, M=M, step_scale=step)
    for (_b, M, step), (bank, hs) in groups.items():
        out = bank.perturbations([h.rs.row for h in hs], np.stack([h.w0_without_locus for h in hs]), M, step)
        for h, o in zip(hs, out):
            h.w0_process = o


def _check_w0(w0: np.ndarray) -> None:
    if np.min(w0) < 0:
        raise AssertionError("Natural frequencies w0 must be positive!")       # env.py:214


@_without_gc
def reset_draws_batch(hosts: list[EnvHost]):
    """EnvHost.reset_draws of several envs, bit-identical to one call per env
    (each env draws from its own stream, in the reference's order):
      env.py:473-557  drift / spatial-variation events (per env);
      env.py:566      w0 = apply_locus_mask(...)   (elementwise, all envs at once);
      env.py:213      remove_negative_w0(w0): draws randn(k) only for the k <= 0
                      entries -- none for a positive w0, so only envs with
                      such entries take that call;
      env.py:214      the positivity assertion;
      env.py:595-598  theta0 = normal(mean, sd, N) per env, then
                      remove_negative_w0(theta0) (again only when needed).
    Returns (w0 (n, N), g_stim (n, ne, N), g_rec (n, nr, N), theta0 (n, N)),
    float64; each host keeps its w0 (a row of the returned array).
    Hosts that are not EnvHosts (evaluation.ReplayHost: pre-drawn resets)
    answer their own reset_draws()."""
    if not all(isinstance(h, EnvHost) for h in hosts):
        d = [h.reset_draws() for h in hosts]
        return tuple(np.stack([np.asarray(r[k], np.float64) for r in d]) for k in range(4))
    regen = [h for h in hosts if h._advance_drift()]   # each env's draws stay in the reference's order:
    perturb_batch(regen)                                 # drift events, the plasticity walk, spatial events
    for h in hosts:
        h._advance_spatial()
    w0wo = np.stack([h.w0_without_locus for h in hosts])
    wl = np.stack([np.asarray(h.p["locus_without_w0"], np.float64) for h in hosts])
    lm0 = hosts[0].p["locus_mask"] if hosts else None
    if all(h.p["locus_mask"] is lm0 for h in hosts):
        lm = np.asarray(lm0, np.float64)[None, :]            # one geometry (broadcast: same elementwise ops)
    else:
        lm = np.stack([np.asarray(h.p["locus_mask"], np.float64) for h in hosts])
    w0 = ms.apply_locus_mask(w0wo, wl, lm)                                      # env.py:566
    th = np.empty_like(w0)
    gss, grs = [], []
    banks: dict = {}     # id(bank) -> (bank, batch indices, bank rows)
    for k, h in enumerate(hosts):
        g_stim, g_rec = h._conductances()
        gss.append(g_stim)
        grs.append(g_rec)
        if isinstance(h.rs, hostrng.Stream):
            b = banks.setdefault(id(h.rs.bank), (h.rs.bank, [], []))
            b[1].append(k)
            b[2].append(h.rs.row)
        else:    # a (possibly shared) numpy RandomState: the reference's order, env by env
            if (w0[k] <= 0.).any():
                w0[k] = ms.remove_negative_w0(h.rs, w0[k])                      # env.py:213
            _check_w0(w0[k])
            t = h.rs.normal(loc=h.p["init_state_mean"], scale=h.p["init_state_sd"], size=h.N)   # env.py:595-597
            if (t <= 0.).any():
                t = ms.remove_negative_w0(h.rs, t)                              # env.py:598
            th[k] = t
    # the same draws for envs on their own native streams, each stream in the
    # order above, one call per bank and draw (remove_negative_w0 draws only
    # for rows with entries <= 0)
    for bank, ks, rows in banks.values():
        ks = np.asarray(ks)
        wk = np.ascontiguousarray(w0[ks])
        bank.remove_nonpositive(rows, wk)                                       # env.py:213
        for r in wk:
            _check_w0(r)
        w0[ks] = wk
        t = bank.normal(rows, [hosts[k].p["init_state_mean"] for k in ks],
                        [hosts[k].p["init_state_sd"] for k in ks], th.shape[1])   # env.py:595-597
        bank.remove_nonpositive(rows, t)                                        # env.py:598
        th[ks] = t
    for k, h in enumerate(hosts):
        h.w0 = w0[k]
    return w0, np.stack(gss), np.stack(grs), th


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


@_without_gc
def fill_driver_arrays_batch(params_list: list[dict], w0_seeds) -> list[dict]:
    """fill_driver_arrays for many envs at once, bit-identical to calling it
    per env (tests/test_host.py): the grid, coordinates and locus mask are
    built once per distinct geometry and shared (read-only) by every env's
    dict; each env's two driver draws (rand(N) then uniform(N),
    utils.py:868,927) come from its own MT19937 stream seeded w0_seeds[b];
    the inverse-CDF transform and the locus blend run on the stacked (B, N)
    draws.  The env dicts are shallow copies of the given ones plus the new
    arrays.  (A per-env loop took ~1.1 s of bench.py's 1.64 s host setup at
    4096 envs, BENCH_r03 extra.host_setup_s.)"""
    B = len(params_list)
    if B == 0:
        return []
    geo = {}
    N = int(params_list[0]["num_oscillators"])
    keys = []
    for p in params_list:
        if int(p["num_oscillators"]) != N:
            raise ValueError("fill_driver_arrays_batch: every env must have the same num_oscillators")
        key = (tuple(p["grid_size"]), float(p["coord_modif"]), tuple(p["locus_center"]), float(p["locus_size"]))
        if key not in geo:
            coords, grid = ms.neuron_grid_3d(*p["grid_size"], N, coord_modif=p["coord_modif"])
            lm = ms.locus_mask(grid, p["grid_size"], p["locus_center"], p["locus_size"])
            for a_ in (coords, grid, lm):
                a_.setflags(write=False)
            geo[key] = (coords, grid, lm)
        keys.append(key)
    # each env's driver stream RandomState(w0_seeds[b]): rand(N) (sample_w0,
    # utils.py:868) then uniform(N) (utils.py:927), all envs in two native calls
    bank = hostrng.StreamBank(w0_seeds)
    rows = np.arange(B)
    rands = bank.random_sample(rows, N)
    wls = bank.uniform(rows, [p["wmuL"] - p["wsdL"] for p in params_list],
                       [p["wmuL"] + p["wsdL"] for p in params_list], N)
    w0_deg = ms.w0_from_uniform(rands)
    # apply_locus_mask (utils.py:902-906) per geometry on the stacked rows
    w = np.empty_like(w0_deg)
    groups: dict = {}
    for b, k in enumerate(keys):
        groups.setdefault(k, []).append(b)
    for k, bs in groups.items():
        idx = np.asarray(bs)
        w[idx] = ms.apply_locus_mask(w0_deg[idx], wls[idx], geo[k][2][None, :])
    w *= 0.065
    w0_deg *= 0.065
    wls *= 0.065
    out = []
    for b, p in enumerate(params_list):
        coords, grid, lm = geo[keys[b]]
        q = dict(p)
        q.update(w0=w[b], w0_without_locus=w0_deg[b], locus_without_w0=wls[b],
                 locus_mask=lm, neur_coords=coords, neur_grid=grid)
        out.append(q)
    return out


@_without_gc
def build_batch(params_list: list[dict]) -> tuple[list[EnvHost], dict]:
    """Host setup for B envs sharing N, the grid and the spatial kernel: returns
    the EnvHost list and the shared coupling alpha (float64, env.py:219-229).
    K may differ per env (its float32(K/N) gain goes to kura_set_env_gain)."""
    # the envs' own streams (env.py:291 RandomState(rand_seed)) in one bank
    ok = [isinstance(p["rand_seed"], (int, np.integer)) and 0 <= int(p["rand_seed"]) <= 0xFFFFFFFF
          for p in params_list]
    rows = np.cumsum(ok) - 1
    bank = hostrng.StreamBank([int(p["rand_seed"]) for p, o in zip(params_list, ok) if o])
    hosts = [EnvHost(p, stream=bank.stream(int(r)) if o else None, defer_perturbations=bool(o))
             for p, o, r in zip(params_list, ok, rows)]
    perturb_batch([h for h in hosts if getattr(h, "w0_process", 0) is None])   # env.py:377, on each env's own stream
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
    """Run the reset draws of the given envs (reset_draws_batch) and stack:
    omega f32, g_stim f64, g_rec f64, theta0 f32."""
    idx = range(len(hosts)) if idx is None else idx
    w, gs, gr, th = reset_draws_batch([hosts[i] for i in idx])
    return w.astype(np.float32), gs, gr, th.astype(np.float32)

