#!/usr/bin/env python3
"""Build gate for the gfx950 store-data hazard ("The
round-2 miscompiles, root-caused").

A VMEM store of more than 8 bytes (buffer/global/flat/scratch ..._dwordx3/x4,
_b96/_b128) reads its data VGPRs after issue; a VALU instruction that writes
one of those VGPRs within the next 2 wait states can land first, and the store
then writes the NEW value.  (The hazard -- and LLVM's guard for it,
GCNHazardRecognizer::createsVALUHazard -- is for data wider than 64 bits: the
compiler places VALU writes right behind 8-byte stores, e.g. ~430 scratch
dwordx2 spills in libkura.so, which is correct code; the tool counts them.)  LLVM inserts the wait states after
global/flat/scratch stores but exempts MUBUF stores whose soffset is an SGPR,
which is how the round-2 builds miscompiled.  The kernels now keep every
record store's offset in the VGPR (store_rec_b128), and this tool proves that
no hazard is left in the shipped machine code:

  * extracts the gfx950 code object of each library (objcopy .hip_fatbin +
    clang-offload-bundler) and disassembles it (llvm-objdump);
  * for every wide VMEM store, walks every control-flow path from it
    (fall-through, s_branch and s_cbranch_* targets) until 2 wait states have
    elapsed (one per instruction, k+1 for s_nop k) and flags a v_* instruction
    on the way that writes one of the store's data VGPRs;
  * calls/returns (s_swappc/s_setpc) end a path: each function's own entry
    sequence is checked on its own (LLVM's recognizer is not
    inter-procedural either).

    python tools/check_store_hazards.py [lib.so ...]      # exit 1 on a hazard

__graft_entry__.build() runs it on libkura.so and libkura_debug.so, and
tests/test_store_hazards.py runs it on the shipped libraries and on a build
with the old SGPR-soffset store form (which it must flag).
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
WAIT_STATES = 2

_WIDE_STORE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx[34]|b96|b128)\b")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_INSN = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-F]+):[^<]*(?:<(.+)\+0x([0-9a-f]+)>)?\s*$")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def _vregs(tok: str) -> set[int]:
    m = _VREG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def _operands(rest: str) -> list[str]:
    return [t.strip() for t in rest.split(",")] if rest.strip() else []


def code_object(lib: str, out_dir: str) -> str:
    """gfx950 device code object of a HIP shared library (path)."""
    fat = os.path.join(out_dir, os.path.basename(lib) + ".fatbin")
    co = os.path.join(out_dir, os.path.basename(lib) + ".gfx950.o")
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(out_dir, "_discard.so")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={fat}", f"--output={co}",
                    f"--targets={TARGET}"], check=True, capture_output=True)
    return co


def disassemble(obj: str) -> str:
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", obj], check=True, capture_output=True,
                          text=True).stdout


def parse(text: str):
    """-> list of functions: (name, [(addr, mnemonic, operands, branch_target_addr|None)])."""
    funcs, cur, start = [], None, 0
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            start = int(m.group(1), 16)
            cur = (m.group(2), [])
            funcs.append(cur)
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        mnem, rest, addr, tfun, toff = m.groups()
        tgt = None
        if tfun is not None and (mnem.startswith("s_cbranch") or mnem == "s_branch"):
            tgt = start + int(toff, 16) if tfun == cur[0] else None
        cur[1].append((int(addr, 16), mnem, _operands(rest), tgt))
    return funcs


def _writes(mnem: str, ops: list[str]) -> set[int]:
    """VGPRs a VALU instruction writes (empty for non-VALU / SGPR destinations)."""
    if not mnem.startswith("v_") or not ops:
        return set()
    if mnem.startswith(("v_readlane", "v_readfirstlane", "v_cmp_", "v_cmpx_")) and not mnem.startswith("v_cmpx_"):
        return set()
    w = _vregs(ops[0])
    if mnem.startswith("v_swap"):
        w |= _vregs(ops[1]) if len(ops) > 1 else set()
    return w


def _wait_states(mnem: str, ops: list[str]) -> int:
    if mnem == "s_nop" and ops:
        try:
            return int(ops[0], 0) + 1
        except ValueError:
            return 1
    return 1


def find_hazards(funcs):
    """Every (function, store, offending instruction, path length) within WAIT_STATES of a wide store."""
    out = []
    for name, insns in funcs:
        index = {a: i for i, (a, *_r) in enumerate(insns)}
        for i, (addr, mnem, ops, _t) in enumerate(insns):
            if not _WIDE_STORE.match(mnem) or not ops:
                continue
            # MUBUF: vdata, vaddr, srsrc, soffset;  global/flat/scratch: vaddr, vdata[, saddr]
            data = _vregs(ops[0] if mnem.startswith("buffer_") else (ops[1] if len(ops) > 1 else ""))
            if not data:
                continue
            # DFS over successors with the wait states elapsed so far
            stack, seen = [(i, 0)], set()
            while stack:
                j, ws = stack.pop()
                succ = []
                _a, m, o, t = insns[j]
                if j != i:
                    if _writes(m, o) & data:
                        out.append((name, addr, mnem, " ".join(ops), insns[j][0], m, ws))
                        continue
                    ws += _wait_states(m, o)
                if ws >= WAIT_STATES and j != i:
                    continue
                if m in ("s_endpgm", "s_setpc_b64", "s_swappc_b64", "s_trap"):
                    continue
                if m == "s_branch":
                    if t is not None and t in index:
                        succ.append(index[t])
                else:
                    if m.startswith("s_cbranch") and t is not None and t in index:
                        succ.append(index[t])
                    if j + 1 < len(insns):
                        succ.append(j + 1)
                for k in succ:
                    key = (k, ws)
                    if key not in seen:
                        seen.add(key)
                        stack.append((k, ws))
    return out


_SREG = re.compile(r"^s(\d+)$|^s\[(\d+):(\d+)\]$")
_MASKED_STORE = re.compile(r"^(buffer|global|flat)_store_")


def _sregs(tok: str) -> set[int]:
    m = _SREG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def parse_asm(text: str):
    """-> the parse() form from compiler assembly (hipcc -S) instead of a
    disassembly: the round-4 failing build survives only as such a listing."""
    funcs, cur = [], None
    for line in text.splitlines():
        if re.match(r"^[A-Za-z_][\w.$]*:", line) and not line.startswith(".L"):
            cur = (line.split(":")[0], [])
            funcs.append(cur)
            continue
        if cur is None or not line.startswith("\t") or line.strip().startswith((".", ";")):
            continue
        body = line.split(";")[0].strip()
        if not body:
            continue
        mnem, _, rest = body.partition(" ")
        cur[1].append((len(cur[1]), mnem, _operands(rest), None))
    return funcs


def find_spilled_store_masks(funcs):
    """Census (not a gate) of the round-4 lost-store shape: a VMEM
    store (buffer/global/flat) under an exec mask that s_and_saveexec_b64 took
    from an SGPR pair restored by v_readlane_b32 from a spill lane.  Returns
    (function, index of the s_and_saveexec, lane register, stores guarded).
    Straight-line scan: a restored pair stays 'from a lane' until an
    instruction whose first operand writes one of its registers."""
    out = []
    for name, insns in funcs:
        lane = {}                       # sgpr -> spill VGPR it was read from
        for i, (_a, mnem, ops, _t) in enumerate(insns):
            if not ops:
                continue
            if mnem == "v_readlane_b32":
                for r in _sregs(ops[0]):
                    lane[r] = ops[1]
                continue
            if mnem == "s_and_saveexec_b64" and len(ops) > 1:
                src = _sregs(ops[1])
                if src and all(r in lane for r in src):
                    dst, n = ops[0], 0
                    for _b, m2, o2, _t2 in insns[i + 1:i + 40]:
                        if m2 == "s_or_b64" and o2[:1] == ["exec"] and o2[-1] == dst:
                            break
                        n += bool(_MASKED_STORE.match(m2))
                    if n:
                        out.append((name, i, lane[min(src)], n))
            for r in _sregs(ops[0]):
                lane.pop(r, None)
    return out


def check_library(lib: str):
    """(number of wide VMEM stores, hazards) of a built HIP library."""
    with tempfile.TemporaryDirectory() as d:
        text = disassemble(code_object(lib, d))
    funcs = parse(text)
    nstores = sum(1 for _n, ins in funcs for (_a, m, _o, _t) in ins if _WIDE_STORE.match(m))
    return nstores, find_hazards(funcs), find_spilled_store_masks(funcs)


BASELINE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "store_mask_baseline.json")


def census_key(sm):
    """{function: stores under a spilled exec mask} of a census."""
    out = {}
    for name, _i, _v, k in sm:
        out[name] = out.get(name, 0) + k
    return out


def over_baseline(lib, sm, baseline):
    """Functions whose spilled-mask stores exceed the committed baseline
    (tools/store_mask_baseline.json): a new site needs an explicit review --
    map it (tools/store_mask_sites.py), name the GPU test that executes it,
    then raise the baseline."""
    base = baseline.get(os.path.basename(lib), {})
    return sorted((f, k, base.get(f, 0)) for f, k in census_key(sm).items() if k > base.get(f, 0))


def main(argv):
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gate = "--baseline" in argv
    argv = [a for a in argv if a != "--baseline"]
    libs = argv or [os.path.join(root, "dbs-gym_amd", "csrc", n) for n in ("libkura.so", "libkura_debug.so")]
    baseline = json.load(open(BASELINE))["stores_per_function"] if gate else {}
    bad = 0
    for lib in libs:
        if not os.path.exists(lib):
            print(f"{lib}: missing")
            bad += 1
            continue
        n, hz, sm = check_library(lib)
        print(f"{os.path.basename(lib)}: {n} wide VMEM stores, {len(hz)} store-data hazards, "
              f"{len(sm)} sites / {sum(k for *_r, k in sm)} stores under a spilled exec mask")
        for name, a, m, o, b, bm, ws in hz[:20]:
            print(f"  {name}: {m} {o} @0x{a:x} <- {bm} @0x{b:x} after {ws} wait state(s)")
        for name, i, v, k in sm[:40]:
            print(f"  {name}: {k} store(s) under a mask read back from {v} (instruction {i})")
        bad += bool(hz)
        if gate:   # the spilled-mask census may not grow past its reviewed baseline
            over = over_baseline(lib, sm, baseline)
            for f, k, b in over:
                print(f"  OVER BASELINE: {f}: {k} stores under a spilled exec mask (baseline {b})")
            bad += bool(over)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
