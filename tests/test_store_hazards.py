"""The store-data hazard as a build gate (DESIGN.md
section 5): tools/check_store_hazards.py walks every control-flow path after
each >8-byte VMEM store of the shipped machine code and flags a VALU write of
the store's data VGPRs within 2 wait states.  CPU only (cross-compiled code)."""
import importlib.util
import os
import re
import shutil
import subprocess

import pytest

from helpers import ROOT

spec = importlib.util.spec_from_file_location("check_store_hazards", os.path.join(ROOT, "tools", "check_store_hazards.py"))
chk = importlib.util.module_from_spec(spec)
spec.loader.exec_module(chk)
CSRC = os.path.join(ROOT, "dbs-gym_amd", "csrc")


def _fn(lines):
    """a synthetic llvm-objdump listing of one function"""
    out = ["0000000000001000 <f>:"]
    addr = 0x1000
    for ln in lines:
        insn, tgt = ln if isinstance(ln, tuple) else (ln, None)
        out.append(f"\t{insn}  // {addr:012X}: 00000000" + (f" <f+0x{tgt:x}>" if tgt is not None else ""))
        addr += 4
    return "\n".join(out)


def _branch(insn, target_off):
    return (insn, target_off)


def _hz(lines):
    funcs = chk.parse(_fn(lines))
    return chk.find_hazards(funcs)


def test_detects_valu_write_right_after_wide_store():
    assert _hz(["buffer_store_dwordx4 v[4:7], v0, s[8:11], s2 offen", "v_pk_add_f32 v[4:5], v[8:9], v[10:11]"])
    assert _hz(["global_store_dwordx4 v[0:1], v[4:7], off", "s_mov_b32 s0, 1", "v_mov_b32_e32 v7, 0"])


def test_wait_states_and_unrelated_registers_are_safe():
    assert not _hz(["buffer_store_dwordx4 v[4:7], v0, s[8:11], 0 offen", "s_nop 1", "v_mov_b32_e32 v4, 0"])
    assert not _hz(["buffer_store_dwordx4 v[4:7], v0, s[8:11], 0 offen", "s_mov_b32 s0, 1", "s_mov_b32 s1, 1",
                    "v_mov_b32_e32 v4, 0"])
    assert not _hz(["buffer_store_dwordx4 v[4:7], v0, s[8:11], 0 offen", "v_mov_b32_e32 v8, 0"])
    assert not _hz(["buffer_store_dwordx2 v[4:5], v0, s[8:11], 0 offen", "v_mov_b32_e32 v4, 0"])   # 8 bytes
    assert not _hz(["global_store_dwordx4 v[0:1], v[4:7], off", "v_mov_b32_e32 v0, 0"])   # address, not data


def test_follows_branch_successors():
    # store; s_cbranch to +0x10 (the v_mov writing v5): the taken path has 1 wait state
    lines = ["buffer_store_dwordx4 v[4:7], v0, s[8:11], 0 offen", _branch("s_cbranch_execz 2", 0x10),
             "s_nop 7", "s_nop 7", "v_mov_b32_e32 v5, 0"]
    assert _hz(lines)
    lines = ["buffer_store_dwordx4 v[4:7], v0, s[8:11], 0 offen", _branch("s_branch 2", 0x10),
             "v_mov_b32_e32 v5, 0", "s_endpgm", "s_nop 0", "v_mov_b32_e32 v5, 0"]
    assert not _hz(lines[:4] + ["s_nop 1", "v_mov_b32_e32 v5, 0"])   # taken path passes s_nop 1 first


@pytest.mark.parametrize("name", ["libkura.so", "libkura_debug.so"])
def test_shipped_libraries_are_hazard_free(name):
    lib = os.path.join(CSRC, name)
    if not os.path.exists(lib):
        pytest.skip(f"{name} not built")
    n, hz, _census = chk.check_library(lib)
    assert n > 100            # the records' wide stores are there
    assert not hz, hz[:5]


def test_old_sgpr_soffset_store_form_is_flagged(tmp_path):
    """The round-2 record-store form (profiles/r04_sgpr_soffset_store.patch)
    built from today's source: the gate must fail on it."""
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    d = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "dbs-gym_amd", "csrc"), d / "dbs-gym_amd" / "csrc",
                    ignore=shutil.ignore_patterns("*.so"))
    shutil.copytree(os.path.join(ROOT, "include"), d / "include")
    # the patch's one change, applied by pattern so that edits elsewhere in the
    # file (which move its line numbers) do not break the test
    src = d / "dbs-gym_amd" / "csrc" / "kura_kernels.hip"
    text = src.read_text()
    old = re.compile(r"(raw_buffer_store_b128\(__builtin_bit_cast\(v4u32, v\), rs, )opaque_vgpr\(voff\) \+ soff, 0,")
    assert len(old.findall(text)) == 1, "store_rec_b128's record-store line not found"
    src.write_text(old.sub(r"\1voff, soff,", text))
    import __graft_entry__ as ge
    lib = str(tmp_path / "libkura_sgpr.so")
    subprocess.run([ge.HIPCC, *ge.HIP_FLAGS, "-o", lib, str(d / "dbs-gym_amd" / "csrc" / "kura_kernels.hip")],
                   check=True, capture_output=True)
    _n, hz, _census = chk.check_library(lib)
    assert hz, "the checker did not flag the SGPR-soffset store form"
    assert any(h[2] == "buffer_store_dwordx4" for h in hz)


def test_spilled_mask_census_reads_compiler_listings():
    """The round-4 lost-store shape: a store under an
    exec mask restored from a spill lane is counted; a mask that is
    overwritten after the restore, or one computed in place, is not."""
    asm = "\n".join(["f:", "\tv_readlane_b32 s0, v252, 59", "\tv_readlane_b32 s1, v252, 60",
                     "\ts_and_saveexec_b64 s[22:23], s[0:1]", "\tflat_store_dword v[12:13], v163",
                     "\ts_or_b64 exec, exec, s[22:23]",
                     "\tv_readlane_b32 s0, v252, 61", "\tv_readlane_b32 s1, v252, 62", "\ts_mov_b32 s1, 0",
                     "\ts_and_saveexec_b64 s[22:23], s[0:1]", "\tflat_store_dword v[12:13], v160",
                     "\ts_or_b64 exec, exec, s[22:23]",
                     "\ts_and_saveexec_b64 s[22:23], s[14:15]", "\tflat_store_dword v[12:13], v162",
                     "\ts_or_b64 exec, exec, s[22:23]"])
    r = chk.find_spilled_store_masks(chk.parse_asm(asm))
    assert [(n, v, k) for n, _i, v, k in r] == [("f", "v252", 1)]


@pytest.mark.parametrize("name", ["libkura.so", "libkura_debug.so"])
def test_spilled_mask_census_within_reviewed_baseline(name):
    """the census is gated against its reviewed baseline
    (tools/store_mask_baseline.json; sites mapped by tools/store_mask_sites.py,
    executed by tests/test_gpu_store_sites.py): a kernel edit that adds a
    store of this shape fails the build until it is reviewed."""
    import json
    lib = os.path.join(CSRC, name)
    if not os.path.exists(lib):
        pytest.skip(f"{name} not built")
    base = json.load(open(chk.BASELINE))["stores_per_function"]
    _n, _hz, sm = chk.check_library(lib)
    assert chk.over_baseline(lib, sm, base) == []
    # one more store in a known function, or a site in a new one, is over
    extra = sm + [(sm[0][0], 0, "v250", 1), ("new_fn", 0, "v250", 1)]
    over = chk.over_baseline(lib, extra, base)
    assert [f for f, _k, _b in over] == sorted([sm[0][0], "new_fn"])
