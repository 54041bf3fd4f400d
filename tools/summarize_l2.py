#!/usr/bin/env python3
"""L2 hit/miss per kura_* kernel from a `rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum`
pass (tools/diag_r02a.sh):  python tools/summarize_l2.py <dir>/l2 out.json"""
import collections
import csv
import json
import sys


def main(src, dst):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(f"{src}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if k.startswith("kura_"):
                d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in d.items():
        hit = sum(v["TCC_HIT_sum"]) / len(v["TCC_HIT_sum"])
        miss = sum(v["TCC_MISS_sum"]) / len(v["TCC_MISS_sum"])
        out[k] = {"dispatches": len(v["TCC_HIT_sum"]), "tcc_hit_per_dispatch": hit, "tcc_miss_per_dispatch": miss,
                  "hit_rate": hit / (hit + miss), "miss_bytes_128B_per_dispatch": miss * 128}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
