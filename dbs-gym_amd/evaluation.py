"""The reference's evaluation protocol, replayed over a batch.

``aDBS_RL/evaluate_HF_DBS.py`` (the script behind the paper's DBS-OFF / HF-DBS
table, ``data/kur-table-metrics.xlsx``) runs, in ONE process with the global
NumPy RNG:

1. ``np.random.seed(228)`` (:20);
2. for each of the five eval configs in turn (:195-218): ``generate_w0_with_locus``
   from the global RNG (:198-205), then ``make_env`` = ``SpatialKuramoto(params)``
   (:23-30, :218), whose constructor reseeds the global RNG with the config's
   ``rand_seed`` (env.py:291), draws env2's plasticity walk (env.py:375-377)
   and runs ``reset()`` once (env.py:386) -- so env k+1's frequencies come
   from the RNG state env k's constructor left behind;
3. ``evaluate_policy_`` env by env (:138-151): ``DummyVecEnv.reset()`` and one
   autoreset after every finished episode, the last one included, each
   ``reset()`` drawing from the same global RNG (env.py:483-598);
4. per env, the ``theta_mean`` of every step of every episode concatenated
   (:82-83, :112-114) and reduced by ``calc_psd_for_simple_eval`` (:122-135);
   the table reports mean (sd) over the five envs.

Resets draw nothing that depends on the simulated trajectory, so every
draw of the protocol can be made up front in the reference's order
(``protocol_draws``) and the episodes then run as one batch on the GPU
(``run_protocol``): per env and per action arm the same initial conditions
the reference script would have used.
"""
from __future__ import annotations

import numpy as np

from .batch import EnvHost, fill_driver_arrays
from .configs import reference_params


class ReplayHost:
    """Stands in for an EnvHost in a KuraVectorEnv: returns pre-drawn resets in order."""

    def __init__(self, draws):
        self.draws = list(draws)
        self.reset_count = -1

    def reset_draws(self):
        self.reset_count += 1
        if self.reset_count >= len(self.draws):
            raise RuntimeError("ReplayHost: more resets than were drawn")
        return self.draws[self.reset_count]


def protocol_draws(name: str, n_episodes: int, n_envs: int = 5, seed: int = 228,
                   rs: np.random.RandomState | None = None, reward_func: str = "bbpow_action", **overrides):
    """Steps 1-3: returns (params list, per-env list of reset draws) where
    draws[k][0] is the constructor's reset (its transient is discarded by the
    script) and draws[k][1:] the n_episodes + 1 resets of evaluate_policy_
    (the DummyVecEnv reset, then one autoreset per finished episode);
    ``overrides`` update every params dict (e.g. encapsulation_mode="relative")."""
    rs = rs if rs is not None else np.random.RandomState()
    rs.seed(seed)                                                               # :20
    plist, hosts, draws = [], [], []
    for k in range(n_envs):              # generate_w0_with_locus, then make_env, config by config
        p = reference_params(name, "eval", k, **overrides)
        p["reward_func"] = reward_func                                        # :207
        p["dbs_action_bounds"] = [-5, 5]                                      # :216
        p = fill_driver_arrays(p, rs=rs)                                      # :198-214
        h = EnvHost(p, rs=rs)                                                 # :218 -> env.py:291
        draws.append([h.reset_draws()])                                       # env.py:386
        plist.append(p)
        hosts.append(h)
    for h, d in zip(hosts, draws):       # evaluate_policy_ env by env
        for _ in range(n_episodes + 1):
            d.append(h.reset_draws())
    return plist, draws


def run_protocol(name: str, actions=(0.0, 1.0), n_episodes: int = 5, n_envs: int = 5, seed: int = 228,
                 device=0, psd_dt: float = 5e-4, beta=(12.5, 21.0), coupling: str = "auto", **overrides):
    """Runs the protocol on the GPU for every (action, env) pair as one batch
    and returns {"bbpow": [n_actions, n_envs], "reward": [n_actions, n_envs, n_episodes],
    "lfp": list of per-env concatenated theta_mean signals}.  coupling: the
    coupling arithmetic (KuraVectorEnv / make_config)."""
    import torch

    from .vec_env import KuraVectorEnv

    plist, draws = protocol_draws(name, n_episodes, n_envs, seed, **overrides)
    A = len(actions)
    batch_params = [p for _ in actions for p in plist]
    env = KuraVectorEnv(batch_params, device=device, rand_seeds=[p["rand_seed"] for p in batch_params],
                        autoreset=True, coupling=coupling)
    # the reference's draws, in the reference's order; both action arms replay
    # the same ones (each arm is a separate run of the script)
    env.hosts = [ReplayHost(draws[k][1:]) for _ in actions for k in range(n_envs)]
    B = env.num_envs
    env.reset()
    act = torch.tensor([a for a in actions for _ in range(n_envs)], dtype=torch.float32,
                       device=env.device).reshape(B, 1)
    steps = n_episodes * env.episode_steps
    cap = steps * 32 + 32
    lfp = torch.zeros((B, cap), dtype=torch.float32, device=env.device)
    lens = torch.zeros(B, dtype=torch.int64, device=env.device)
    ar = torch.arange(32, device=env.device)
    rew = np.zeros((B, n_episodes))
    ep = np.zeros(B, np.int64)
    cur = torch.zeros(B, dtype=torch.float64, device=env.device)
    for _ in range(steps):
        _, r, term, _, info = env.step(act)
        cur += r
        # append this step's theta_mean (evaluate_HF_DBS.py:83); the zero
        # padding past nsamp is overwritten by the next step's samples
        lfp.scatter_(1, lens[:, None] + ar[None, :], env.sim.lfp_true)
        lens += env.sim.nsamp.to(torch.int64)
        if "terminal_env_ids" in info:
            idx = info["terminal_env_ids"]
            c = cur.cpu().numpy()
            for b in idx:
                if ep[b] < n_episodes:
                    rew[b, ep[b]] = c[b]
                ep[b] += 1
            cur[torch.as_tensor(idx, device=env.device)] = 0.0
    lens_h = lens.cpu().numpy()
    sig = lfp.cpu().numpy()
    signals = [sig[b, :lens_h[b]] for b in range(B)]
    bb = env.sim.psd_bbpow(signals, psd_dt, beta)
    env.close()
    return {"bbpow": bb.reshape(A, n_envs), "reward": rew.reshape(A, n_envs, n_episodes), "lfp": signals,
            "actions": list(actions)}


__all__ = ["ReplayHost", "protocol_draws", "run_protocol"]
