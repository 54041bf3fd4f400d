"""Multi-process sharding (world_size 2, gloo on CPU): each rank builds and
steps its own contiguous shard of envs (global env id = rank*B + b seeds the
env, as bench.py does on GPUs); the gathered shards equal a single-process run
of the whole batch bit for bit.  No data-path collective exists; gloo is used
here only to gather results for the check."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class Args:
    config = "env0"
    osc = 256
    envs = 3
    reward = "bbpow_action"
    seed = 99
    random_k = True  # per-env K derived from the global env id, like the seeds


def _run_shard(rank, B):
    import sys
    from helpers import ROOT, ko, actions
    sys.path.insert(0, ROOT)
    import bench
    a = Args()
    a.envs = B
    cfg, alpha, omega, gs, gr, th0, ct, st, gain = bench.build_shard(a, rank)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_gain(gain)
    o.set_spectral(ct, st)
    o.reset(th0)
    rews = []
    for k in range(2):
        act = actions("rand", B, 1, k + 1000 * rank)
        rews.append(o.step(act)["reward"])
    return o.y.copy(), np.stack(rews, 1)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y, _ = _run_shard(rank, Args.envs)
    t = torch.from_numpy(y)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)   # bench.py's max-over-ranks timing
    if rank == 0:
        q.put((torch.cat(parts).numpy(), float(el.item())))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_equal_single_process():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, el = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert el == 2.0
    # single process over the union: rank r's envs are global ids r*B .. r*B+B-1
    import sys
    from helpers import ROOT, ko
    sys.path.insert(0, ROOT)
    import bench
    a = Args()
    a.envs = world * Args.envs
    cfg, alpha, omega, gs, gr, th0, ct, st, gain = bench.build_shard(a, 0)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_gain(gain)
    o.set_spectral(ct, st)
    o.reset(th0)
    from helpers import actions
    for k in range(2):
        act = np.concatenate([actions("rand", Args.envs, 1, k + 1000 * r) for r in range(world)])
        o.step(act)
    np.testing.assert_array_equal(gathered, o.y)

