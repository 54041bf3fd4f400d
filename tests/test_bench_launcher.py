"""bench.py --gpus N without torchrun: the parent
starts N rank processes itself, relays rank 0's line and fails loudly on a
GPU-count mismatch or a failing rank.  CPU only: --launcher-selftest ranks
join a gloo process group and report who joined (no GPU is touched)."""
import json
import os
import subprocess
import sys

from helpers import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env)


def test_launcher_starts_n_ranks():
    r = _run(["--gpus", "3", "--share-device", "--dist-backend", "gloo", "--launcher-selftest"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["dist_world_size"] == 3
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2]
    assert len({x["pid"] for x in d["ranks"]}) == 3 and os.getpid() not in {x["pid"] for x in d["ranks"]}
    assert all(x["local_rank"] == 0 for x in d["ranks"])       # --share-device


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--launcher-selftest"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_failing_rank_fails_the_job():
    r = _run(["--gpus", "2", "--share-device", "--launcher-selftest"], {"KURA_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "rank 1" in r.stderr


def test_launcher_refuses_more_gpus_than_visible():
    # no GPU in the CPU container: a real (non-selftest) 2-GPU launch must refuse before any rank starts
    import torch
    if torch.cuda.device_count() >= 2:
        return
    r = _run(["--gpus", "2", "--cpu-seconds", "0"])
    assert r.returncode != 0 and "visible" in r.stderr
