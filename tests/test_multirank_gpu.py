"""Multi-process sharding on the GPU (world_size 2, both ranks on cuda:0 of a
one-GPU box): each rank builds its contiguous env shard exactly as bench.py
does (global env id = rank*B + b seeds the env and its K) and steps it
through the HIP path; the gathered GPU shards equal the CPU oracle run of the
whole batch in one process, bit for bit.  gloo carries only the result
gather and the max-over-ranks timing reduction (bench.py uses RCCL for the
same two calls; RCCL cannot put two ranks on one device, gloo can), so this
is the N>1 data path on real hardware -- no collective on it."""
import os
import socket
import sys

import numpy as np
import pytest

from helpers import ROOT, actions, ko

pytestmark = pytest.mark.gpu

B = 24        # envs per rank: one full workgroup of 16 plus a padded one
STEPS = 3


class Args:
    config = "env1"
    osc = 512
    envs = B
    reward = "bbpow_action"
    seed = 7
    random_k = True
    part_osc = -1


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import importlib
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    sim_mod = importlib.import_module("dbs-gym_amd.sim")
    cfg, alpha, omega, gs, gr, th0, ct, st, gain = bench.build_shard(Args(), rank)
    sim = sim_mod.KuraSim(cfg, 0)
    sim.set_coupling(alpha)
    sim.set_env_params(omega, gs, gr)
    sim.set_env_gain(gain)
    sim.set_spectral(ct, st)
    sim.reset(torch.from_numpy(th0))
    rews = []
    for k in range(STEPS):
        _, rew, _ = sim.step(torch.from_numpy(actions("rand", B, 1, k + 1000 * rank)))
        rews.append(rew.cpu().numpy())
    torch.cuda.synchronize()
    y = torch.from_numpy(np.ascontiguousarray(sim.get_state()["y"]))
    r = torch.from_numpy(np.stack(rews, 1))
    ys = [torch.empty_like(y) for _ in range(world)]
    rs = [torch.empty_like(r) for _ in range(world)]
    dist.all_gather(ys, y)
    dist.all_gather(rs, r)
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((torch.cat(ys).numpy(), torch.cat(rs).numpy(), float(el.item())))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_gpu_ranks_shards_equal_single_process_oracle():
    import torch.multiprocessing as mp
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        y_gpu, r_gpu, el = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert el == 2.0
    sys.path.insert(0, ROOT)
    import bench
    a = Args()
    a.envs = world * B
    cfg, alpha, omega, gs, gr, th0, ct, st, gain = bench.build_shard(a, 0)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_gain(gain)
    o.set_spectral(ct, st)
    o.reset(th0)
    rews = []
    for k in range(STEPS):
        act = np.concatenate([actions("rand", B, 1, k + 1000 * r) for r in range(world)])
        rews.append(o.step(act)["reward"])
    np.testing.assert_array_equal(y_gpu, o.y)
    np.testing.assert_array_equal(r_gpu, np.stack(rews, 1))
