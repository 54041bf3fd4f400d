#!/usr/bin/env python3
"""Summarise a tools/rocprof_run.sh output directory into one JSON for profiles/.

    python tools/summarize_rocprof.py gpurun_out/prof5 profiles/r01_rocprof_summary.json

Per kernel: calls and average duration from the kernel-trace stats, FETCH_SIZE
and WRITE_SIZE per dispatch from the two --pmc passes.  rocprofv3 reports both
in KiB; FETCH_SIZE is doubled (gfx950 tallies 128-B requests of 16 B/lane
streaming reads at 64 B, MI355X_MICROARCH.md "HBM").  Both count L2 misses to
the fabric, Infinity-Cache hits included, so they bound HBM traffic from above.
"""
import csv
import json
import os
import sys


def _kname(n):
    return n.split("(")[0].replace("void ", "").strip()


def main(src, dst):
    out = {"source": os.path.basename(os.path.normpath(src)), "kernels": {}}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            k = _kname(r["Name"])
            if not k.startswith("kura_"):
                continue
            out["kernels"][k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                 "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    for pas, counter, scale in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        vals = {}
        with open(os.path.join(src, pas, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                vals.setdefault(_kname(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            if k.startswith("kura_"):
                d = out["kernels"].setdefault(k, {})
                d[counter.lower() + "_bytes_per_dispatch"] = scale * 1024.0 * sum(v) / len(v)
                d[counter.lower() + "_dispatches"] = len(v)
    # effective shader clock: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / dispatch time
    clk = os.path.join(src, "clock", "run_counter_collection.csv")
    if os.path.exists(clk):
        per = {}
        with open(clk) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                    continue
                ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                if ns > 0:
                    per.setdefault(_kname(r["Kernel_Name"]), []).append(float(r["Counter_Value"]) / 8.0 / ns)
        for k, v in per.items():
            if k.startswith("kura_"):
                out["kernels"].setdefault(k, {})["effective_clock_ghz"] = sum(v) / len(v)
    for k, d in out["kernels"].items():
        if "fetch_size_bytes_per_dispatch" in d and "write_size_bytes_per_dispatch" in d:
            d["traffic_bytes_per_dispatch"] = d["fetch_size_bytes_per_dispatch"] + d["write_size_bytes_per_dispatch"]
            if "avg_ms" in d:
                d["traffic_gbs"] = d["traffic_bytes_per_dispatch"] / (d["avg_ms"] * 1e-3) / 1e9
    for name in ("bench_trace.json",):
        p = os.path.join(src, name)
        if os.path.exists(p):
            with open(p) as f:
                b = json.loads(f.read().strip().splitlines()[-1])
            out["bench_under_trace"] = {"value": b["value"], "avg_kernel_ms_hip_events": b["roofline"]["avg_kernel_ms"],
                                        "config": b["config"]}
            if "xl_launch" in b.get("extra", {}):   # split groups: cooperative or plain (KURA_XL_LAUNCH) launch
                out["bench_under_trace"]["xl_launch"] = b["extra"]["xl_launch"]
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
