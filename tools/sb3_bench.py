"""Per-step cost of the SB3-shaped boundary (NumPy obs/rewards/dones/infos on
the host) against the device-resident KuraVectorEnv, at the bench config.

    python tools/sb3_bench.py [envs] [steps]
"""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
kura = importlib.import_module("dbs-gym_amd")
vec = importlib.import_module("dbs-gym_amd.vec_env")
sb3 = importlib.import_module("dbs-gym_amd.sb3")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p = kura.synthetic_params("env0", 1024)
venv = vec.KuraVectorEnv(p, num_envs=B, reward_func="bbpow_action")
rng = np.random.default_rng(0)
acts = [rng.uniform(-1, 1, (B, 1)).astype(np.float32) for _ in range(K + 3)]
res = {"envs": B, "steps": K}
venv.reset(seed=1)
dacts = [torch.from_numpy(a).to(venv.device) for a in acts]
for k in range(3):
    venv.step(dacts[k])
torch.cuda.synchronize()
t = time.perf_counter()
for k in range(K):
    venv.step(dacts[3 + k])
torch.cuda.synchronize()
res["vector_env_ms_per_step"] = 1e3 * (time.perf_counter() - t) / K
env = sb3.KuraSB3VecEnv(venv)
env.reset()
for k in range(3):
    env.step(acts[k])
t = time.perf_counter()
for k in range(K):
    obs, rew, dones, infos = env.step(acts[3 + k])
res["sb3_ms_per_step"] = 1e3 * (time.perf_counter() - t) / K
res["sb3_overhead"] = res["sb3_ms_per_step"] / res["vector_env_ms_per_step"] - 1.0
print(json.dumps(res))
env.close()

# breakdown of one SB3 step: the device step, the host staging, the rest
if os.environ.get("BREAKDOWN"):
    env = sb3.KuraSB3VecEnv(vec.KuraVectorEnv(p, num_envs=B, reward_func="bbpow_action"))
    env.reset()
    orig = env._to_host
    acc = {"to_host": 0.0, "venv_step": 0.0}
    ostep = env.venv.step

    def th(*a):
        t0 = time.perf_counter(); r = orig(*a); acc["to_host"] += time.perf_counter() - t0; return r

    def vs(*a):
        t0 = time.perf_counter(); r = ostep(*a); torch.cuda.synchronize(); acc["venv_step"] += time.perf_counter() - t0
        return r
    env._to_host = th
    env.venv.step = vs
    t = time.perf_counter()
    for k in range(K):
        env.step(acts[3 + k])
    tot = time.perf_counter() - t
    pin = torch.empty((B, 1, 2340), pin_memory=True)
    t0 = time.perf_counter()
    for _ in range(5):
        pin.clone()
    clone_ms = 1e3 * (time.perf_counter() - t0) / 5
    print(json.dumps({"ms_per_step": 1e3 * tot / K, "venv_step_ms": 1e3 * acc["venv_step"] / K,
                      "to_host_ms": 1e3 * acc["to_host"] / K, "pinned_clone_ms": clone_ms,
                      "torch_threads": torch.get_num_threads()}))
