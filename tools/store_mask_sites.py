#!/usr/bin/env python3
"""Map the spilled-exec-mask store sites of the shipped libkura.so to source
(the census is tools/check_store_hazards.py's
find_spilled_store_masks).

The shipped library has no line tables, so the same source is built again
with -gline-tables-only (line tables do not change code generation; the tool
checks the census of both builds lists the same functions and store counts
in the same order).  For every site it prints the guarded
stores and the source line each one comes from.

    python tools/store_mask_sites.py [--debug] [--out FILE]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import check_store_hazards as csh  # noqa: E402

_LINE = re.compile(r"^; (/\S+?):(\d+)")


def build_with_lines(out: str, extra=()) -> None:
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    src = os.path.join(g.CSRC, "kura_kernels.hip")
    subprocess.run([g.HIPCC, *g.HIP_FLAGS, *extra, "-gline-tables-only", "-o", out, src], check=True)


def parse_with_lines(text: str):
    """csh.parse() plus, per function, the source location of each instruction."""
    funcs, locs, cur, start, loc = [], [], None, 0, None
    for line in text.splitlines():
        m = csh._FUNC.match(line)
        if m:
            start = int(m.group(1), 16)
            cur = (m.group(2), [])
            funcs.append(cur)
            locs.append([])
            continue
        lm = _LINE.match(line)
        if lm:
            loc = (lm.group(1), int(lm.group(2)))
            continue
        if cur is None:
            continue
        m = csh._INSN.match(line)
        if not m:
            continue
        mnem, rest, addr, tfun, toff = m.groups()
        tgt = None
        if tfun is not None and (mnem.startswith("s_cbranch") or mnem == "s_branch"):
            tgt = start + int(toff, 16) if tfun == cur[0] else None
        cur[1].append((int(addr, 16), mnem, csh._operands(rest), tgt))
        locs[-1].append(loc)
    return funcs, locs


def census(lib: str, lines: bool):
    with tempfile.TemporaryDirectory() as d:
        co = csh.code_object(lib, d)
        args = [f"{csh.LLVM}/llvm-objdump", "-d", "--mcpu=gfx950"] + (["-l"] if lines else []) + [co]
        text = subprocess.run(args, check=True, capture_output=True, text=True).stdout
    if lines:
        funcs, locs = parse_with_lines(text)
    else:
        funcs, locs = csh.parse(text), None
    return funcs, locs, csh.find_spilled_store_masks(funcs)


def main(argv):
    out = None
    debug = "--debug" in argv   # libkura_debug.so (-DKURA_DEBUG) instead of libkura.so
    argv = [a for a in argv if a != "--debug"]
    if argv[:1] == ["--out"]:
        out = argv[1]
    shipped = os.path.join(ROOT, "dbs-gym_amd", "csrc", "libkura_debug.so" if debug else "libkura.so")
    _, _, sites = census(shipped, False)
    with tempfile.TemporaryDirectory() as d:
        glib = os.path.join(d, "libkura_lines.so")
        build_with_lines(glib, ["-DKURA_DEBUG"] if debug else [])
        gfuncs, glocs, gsites = census(glib, True)
    # the same sites (function, guarded stores) in the same order; instruction
    # indices may shift by a few where the line tables move a scheduling boundary
    same = [(n, k) for n, _i, _v, k in sites] == [(n, k) for n, _i, _v, k in gsites]
    shift = max((abs(a[1] - b[1]) for a, b in zip(sites, gsites)), default=0)
    lines = [f"shipped {os.path.basename(shipped)}: {len(sites)} sites, {sum(k for *_r, k in sites)} stores under a spilled exec mask",
             f"line-table build: {len(gsites)} sites -- same functions and store counts as the shipped build: {same} "
             f"(largest instruction-index shift {shift})", ""]
    fidx = {name: j for j, (name, _ins) in enumerate(gfuncs)}
    srcs = {}
    for name, i, v, k in gsites:
        j = fidx[name]
        ins, loc = gfuncs[j][1], glocs[j]
        lines.append(f"{name} @ instruction {i} (s_and_saveexec_b64 of a pair read back from {v}):")
        n = 0
        for t in range(i + 1, min(i + 40, len(ins))):
            a, m, o, _tg = ins[t]
            if m == "s_or_b64" and o[:1] == ["exec"]:
                break
            if csh._MASKED_STORE.match(m):
                f, ln = loc[t] if loc[t] else ("?", 0)
                if f not in srcs and os.path.exists(f):
                    srcs[f] = open(f).read().splitlines()
                text = srcs[f][ln - 1].strip() if f in srcs and 0 < ln <= len(srcs[f]) else ""
                lines.append(f"    {m} {' '.join(o)}   <- {os.path.basename(f)}:{ln}  {text}")
                n += 1
        lines.append("")
    report = "\n".join(lines)
    print(report)
    if out:
        with open(out, "w") as f:
            f.write(report + "\n")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
