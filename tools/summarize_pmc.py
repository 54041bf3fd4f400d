#!/usr/bin/env python3
"""Per-dispatch averages of the counters of tools/pmc_pass.sh runs for the
kura_* kernels:  python tools/summarize_pmc.py gpurun_out/r03l_k1t [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(src, dst=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
        per = defaultdict(float)  # (dispatch, kernel, counter) -> summed over dims
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if not k.startswith("kura_"):
                continue
            per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, k, c), v in per.items():
            acc[k][c].append(v)
    out = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in acc.items()}
    for k, cs in out.items():
        print(k)
        for c, v in cs.items():
            print(f"   {c:34s} {v:16.4g}")
    if dst:
        json.dump({"source": os.path.basename(os.path.normpath(src)), "per_dispatch_mean": out}, open(dst, "w"),
                  indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
