#!/usr/bin/env python3
"""Per-kernel resource usage of libkura: compiles
kura_kernels.hip with -Rpass-analysis=kernel-resource-usage (same flags as the
production build) and prints one row per step/reset instantiation:
VGPR / AGPR / SGPR / scratch bytes per lane / VGPR spills / LDS / occupancy.
    python tools/resource_table.py > profiles/r03_resource_usage.txt
(KURA_RES_FLAGS="-DKURA_SAVE_SCALAR ..." adds defines: the table of an A/B variant)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def main():
    src = os.path.join(ge.CSRC, "kura_kernels.hip")
    flags = [f for f in ge.HIP_FLAGS if f not in ("-shared",)] + os.environ.get("KURA_RES_FLAGS", "").split()
    cmd = [ge.HIPCC, *flags, "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/tmp/_kura_res.o", src]
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=ge.CSRC).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +(.*?) \[-Rpass-analysis", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    demangled = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                               text=True).stdout.splitlines()
    print("# libkura kernels, hipcc " + " ".join(flags) + " (ROCm 7.2, gfx950)")
    print("# kernel | VGPRs | AGPRs | SGPRs | scratch B/lane | VGPR spill | LDS B (static) | waves/SIMD")
    for r, d in zip(rows, demangled):
        d = d.split("(")[0].replace("void ", "")
        if not re.match(r"kura_(step|reset)", d):
            continue
        print(f"{d:34s} | {r.get('VGPRs', '?'):>4} | {r.get('AGPRs', '?'):>4} | {r.get('TotalSGPRs', '?'):>4} | "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>5} | {r.get('VGPRs Spill', '?'):>4} | "
              f"{r.get('LDS Size [bytes/block]', '?'):>6} | {r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
