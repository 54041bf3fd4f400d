#!/usr/bin/env python3
"""Summarise tools/power_probe.sh output: per amd-smi sample the socket power,
the mean of the per-XCD gfx clocks and the hotspot temperature, plus the
board's power limit.   python tools/summarize_power.py gpurun_out/<dir> [...]"""
import json
import os
import sys


def objects(path):
    text, dec, i = open(path).read(), json.JSONDecoder(), 0
    while True:
        while i < len(text) and text[i] in " \r\n\t":
            i += 1
        if i >= len(text):
            return
        obj, i = dec.raw_decode(text, i)
        yield obj


def val(x):
    return x["value"] if isinstance(x, dict) and "value" in x else None


def summarise(d):
    lim = None
    if os.path.exists(os.path.join(d, "limits.json")):
        for o in objects(os.path.join(d, "limits.json")):
            lim = val(o["gpu_data"][0]["limit"]["ppt0"]["socket_power_limit"])
    rows = []
    for o in objects(os.path.join(d, "samples.jsonl")):
        g = o["gpu_data"][0]
        clks = [val(v["clk"]) for k, v in g["clock"].items() if k.startswith("gfx_") and val(v.get("clk"))]
        temp = g.get("temperature", {})
        rows.append({"socket_w": val(g["power"]["socket_power"]),
                     "gfx_mhz_mean": sum(clks) / len(clks) if clks else None,
                     "hotspot_c": val(temp.get("hotspot")) if isinstance(temp, dict) else None})
    bench = None
    bf = os.path.join(d, "bench.json")
    if os.path.exists(bf):
        lines = [l for l in open(bf) if l.startswith("{")]
        if lines:
            b = json.loads(lines[-1])
            bench = {"value": b["value"], "ms_per_step": b["ms_per_step"], "coupling": b["config"].get("coupling"),
                     "dtype": b.get("dtype")}
    w = [r["socket_w"] for r in rows if r["socket_w"]]
    c = [r["gfx_mhz_mean"] for r in rows if r["gfx_mhz_mean"]]
    return {"dir": d, "socket_power_limit_w": lim, "samples": len(rows),
            "socket_w_median": sorted(w)[len(w) // 2] if w else None, "socket_w_max": max(w) if w else None,
            "gfx_mhz_median": sorted(c)[len(c) // 2] if c else None, "bench": bench, "rows": rows}


if __name__ == "__main__":
    print(json.dumps([summarise(d) for d in sys.argv[1:]], indent=1))
