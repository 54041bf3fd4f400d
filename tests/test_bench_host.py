"""Host-side pieces of the strong-scaling / split-group configuration (no GPU):
the automatic part width, the kernel naming the bench reports, and that the
part width reaches the C config (and so the oracle's RM order)."""
import importlib
import os
import sys

import pytest

from helpers import ROOT, kura

sys.path.insert(0, ROOT)


def test_auto_part_osc_fills_the_cus():
    sim = importlib.import_module("dbs-gym_amd.sim")
    assert sim.auto_part_osc(1024, 4096) == 0            # not split
    assert sim.auto_part_osc(8192, 1024) == 1024         # 64 groups x 8 parts = 512 >= 256
    assert sim.auto_part_osc(8192, 256) == 512           # 16 groups x 16 parts = 256
    assert sim.auto_part_osc(8192, 128) == 256           # strong form at 8 GPUs: 8 x 32 = 256
    assert sim.auto_part_osc(2048, 16) == 256            # too few envs for any width: smallest
    for n, b in ((2048, 19), (4096, 300), (8192, 4096)):
        part = sim.auto_part_osc(n, b)
        assert part in (256, 512, 1024) and n % part == 0


def test_part_width_reaches_the_config():
    sim = importlib.import_module("dbs-gym_amd.sim")
    p = kura.synthetic_params("env0", 2048)
    assert sim.make_config(p, 32, reward_func="bbpow_action").part_osc == 0
    assert sim.make_config(p, 32, reward_func="bbpow_action", part_osc=256).part_osc == 256
    for bad in (128, 768, 2048):
        with pytest.raises(ValueError):
            sim.make_config(p, 32, reward_func="bbpow_action", part_osc=bad)


def test_bench_kernel_name():
    """The names bench.py looks up in the rocprof summaries are the kernel
    instantiations libkura.so carries (demangled symbols)."""
    bench = importlib.import_module("bench")
    assert bench.kernel_name(1024, 0, "bf16x3") == "kura_step_kernel<4, false, true>"
    assert bench.kernel_name(1024) == "kura_step_kernel<4, false, false>"
    assert bench.kernel_name(512, 0, "bf16x3") == "kura_step_kernel<2, false, true>"
    assert bench.kernel_name(8192) == "kura_step_kernel<4, true, false>"
    assert bench.kernel_name(8192, 256) == "kura_step_kernel<1, true, false>"
    assert bench.kernel_name(8192, 512) == "kura_step_kernel<2, true, false>"
    lib = os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura.so")
    if not os.path.exists(lib):
        pytest.skip("libkura.so not built")
    import subprocess
    # the kernels live in the gfx950 code object: their host-side stubs carry the same names
    syms = subprocess.run(["nm", "-C", lib], capture_output=True, text=True, check=True).stdout
    for n, part, c in ((1024, 0, "bf16x3"), (1024, 0, "f32"), (512, 0, "bf16x3"), (8192, 0, "f32"),
                       (8192, 256, "f32")):
        k = bench.kernel_name(n, part, c)
        assert f"void {k}(" in syms or f"{k}(" in syms, k


@pytest.mark.parametrize("flag", ["--episode", "--global-envs", "--part-osc", "--episode-metrics"])
def test_bench_modes_are_documented(flag):
    src = open(f"{ROOT}/bench.py").read()
    assert f'"{flag}"' in src


def test_rocprof_summary_backs_the_bench_roofline():
    """The bench line's roofline.traffic comes from the committed rocprofv3
    summary of the same workload, and that summary's traced kernel average
    agrees with the HIP-event average measured in the traced run."""
    import json
    bench = importlib.import_module("bench")
    d = json.load(open(f"{ROOT}/profiles/latest_rocprof.json"))
    import glob
    paths = sorted(glob.glob(f"{ROOT}/profiles/latest_rocprof*.json"))
    assert f"{ROOT}/profiles/latest_rocprof.json" in paths
    for path in paths:     # the headline and each N=8192 form: one summary per workload
        d = json.load(open(path))
        wl = d["bench_under_trace"]["config"]["workload"]
        n = int(wl.split("N=")[1].split()[0])
        part = d["bench_under_trace"]["config"].get("part_osc", 0)
        kname = bench.kernel_name(n, part, "bf16x3")                 # the product arithmetic (AUTO)
        k = d["kernels"][kname]
        traffic, src, clock = bench.pmc_traffic(wl, kname)
        assert traffic == k["traffic_bytes_per_dispatch"] > 0, path
        assert d["source"] in src and os.path.basename(path) in src and 1.3 < clock < 2.6
        hip_ms = d["bench_under_trace"]["avg_kernel_ms_hip_events"]
        assert k["min_ms"] <= hip_ms * 1.001 and abs(k["avg_ms"] - hip_ms) / hip_ms < 0.05, path
    assert bench.pmc_traffic("no such workload", kname) == (None, None, None)
