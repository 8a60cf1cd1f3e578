#!/usr/bin/env python3
"""Per-kernel VALU issue cost from the ISA.

gfx950 does not issue every VALU instruction in the same time: tools/micro/valubench.hip
(profiles/r03/micro/valubench_*.txt, 4 waves per SIMD, independent instructions) measured
~2.1 cycles per wave64 instruction for the VOP1/VOP2 integer forms (v_xor / v_or / v_and /
v_add_u32 / right shifts / v_mov), ~2.35 for their VOP3 encodings and v_bitop3, and ~4.1 for
SDWA, DPP, left shifts (v_lshlrev_b32), v_perm, v_bfe / v_bfi, v_alignbit / v_alignbyte,
v_add3 / v_lshl_add / v_and_or, the 24-bit multiplies, v_max_u32, 64-bit ops (v_lshl_add_u64,
v_mov_b64, v_add_co with its carry in VCC) and any instruction with an SGPR operand.

This tool disassembles the built library (llvm-objdump of the gfx950 code object inside
walrus_amd/libwalrus_rs2.so), classifies every VALU instruction of each kernel by that table and
writes, per kernel, the static counts per class and the mean issue cycles per VALU instruction.
The kernels' hot code is straight-line (fully unrolled transforms and compression rounds), so
the static mix stands for the executed one; bench.py multiplies it with the PMC's executed VALU
count (SQ_INSTS_VALU) for the cycle-weighted issue fraction.  (The PMC has no cycle-weighted
VALU counter to check it against on gfx950: SQ_ACTIVE_INST_VALU, nominally VALU quad-cycles,
equals SQ_INSTS_VALU to 0.02 % for every kernel, profiles/r05/v2_pmc_summary.txt.)

usage: python3 tools/isa_mix.py [LIB] [OUT.json]   (default: the in-tree library ->
       profiles/isa_mix.json)
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"

# cycles per wave64 instruction per SIMD (valubench, 4 waves/SIMD)
C_FAST, C_VOP3, C_SLOW = 2.1, 2.35, 4.1
SLOW = {
    "v_lshlrev_b32", "v_lshl_add_u32", "v_lshl_add_u64", "v_lshl_or_b32", "v_and_or_b32",
    "v_or3_b32", "v_xad_u32", "v_perm_b32", "v_bfe_u32", "v_bfe_i32", "v_bfi_b32",
    "v_alignbit_b32", "v_alignbyte_b32", "v_add3_u32", "v_mul_u32_u24", "v_mul_hi_u32_u24",
    "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_mad_u64_u32", "v_max_u32", "v_min_u32",
    "v_max_i32", "v_min_i32", "v_mov_b64", "v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32",
    "v_subb_co_u32", "v_subrev_co_u32", "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64",
    "v_cndmask_b32", "v_readlane_b32", "v_readfirstlane_b32", "v_writelane_b32",
    "v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32", "v_pk_add_u16", "v_pk_mov_b32",
}
SGPR = re.compile(r"(?<![a-z_])(s\d+|s\[\d+:\d+\]|vcc|vcc_lo|vcc_hi|exec|m0|ttmp\d+)(?![\w])")


def classify(mn: str, ops: str) -> str:
    base = mn.split("_e32")[0].split("_e64")[0].split("_sdwa")[0].split("_dpp")[0]
    if "_sdwa" in mn or "_sel:" in ops or "sel:" in ops:
        return "sdwa"
    if "_dpp" in mn or "quad_perm" in ops or "row_" in ops or "bound_ctrl" in ops:
        return "dpp"
    if base.startswith("v_cmp"):
        return "slow"  # writes an SGPR pair / VCC
    if base in SLOW:
        return "slow"
    # an SGPR (or VCC / EXEC / M0) source operand: the destination is the first operand
    srcs = ops.split(",", 1)[1] if "," in ops else ""
    if SGPR.search(srcs):
        return "sgpr"
    if mn.endswith("_e64") or base.startswith("v_bitop3") or base.startswith("v_xor3") or \
            base.startswith("v_lshl") or base.startswith("v_add3"):
        return "vop3"
    return "fast"


CYC = {"fast": C_FAST, "vop3": C_VOP3, "slow": C_SLOW, "sgpr": C_SLOW, "sdwa": C_SLOW,
       "dpp": C_SLOW}


def code_object(lib: str, tmp: str) -> str:
    """The gfx950 code object bundled in the shared library."""
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={lib}"],
                   capture_output=True)
    out = os.path.join(tmp, "co.elf")
    # the library embeds one fat binary per translation unit; llvm-objdump --offloading
    # extracts every bundle next to the input, so work on a copy in tmp
    cp = os.path.join(tmp, os.path.basename(lib))
    subprocess.run(["cp", lib, cp], check=True)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", cp], capture_output=True, cwd=tmp)
    objs = sorted(f for f in os.listdir(tmp) if "gfx950" in f)
    return [os.path.join(tmp, f) for f in objs] or [out]


def demangle(names):
    res = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True)
    return res.stdout.splitlines()


def mix_of(objs):
    kernels = {}
    cur = None
    for obj in objs:
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", obj],
                             capture_output=True, text=True).stdout
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                cur = m.group(1)
                kernels.setdefault(cur, {})
                continue
            if cur is None:
                continue
            t = line.strip()
            if not t.startswith("v_"):
                continue
            t = t.split("//")[0].strip()
            parts = t.split(None, 1)
            mn, ops = parts[0], parts[1] if len(parts) > 1 else ""
            if mn.startswith(("v_mfma", "v_smfma")):
                continue
            c = classify(mn, ops)
            d = kernels[cur]
            d[c] = d.get(c, 0) + 1
            d.setdefault("_mn", {})
            d["_mn"][mn] = d["_mn"].get(mn, 0) + 1
    names = [k for k in kernels if kernels[k]]
    dem = demangle(names)
    out = {}
    for raw, nice in zip(names, dem):
        d = kernels[raw]
        tot = sum(v for k, v in d.items() if k != "_mn")
        if not tot:
            continue
        cyc = sum(CYC[k] * v for k, v in d.items() if k != "_mn") / tot
        short = re.sub(r"^void ", "", nice)
        short = re.sub(r"^rs2::", "", short)
        short = re.sub(r"\(.*$", "", short)
        top = sorted(d["_mn"].items(), key=lambda kv: -kv[1])[:12]
        out.setdefault(short, {"valu_static": tot, "cycles_per_valu": round(cyc, 4),
                               "classes": {k: v for k, v in d.items() if k != "_mn"},
                               "top": dict(top)})
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "walrus_amd", "libwalrus_rs2.so")
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "isa_mix.json")
    with tempfile.TemporaryDirectory() as tmp:
        objs = code_object(lib, tmp)
        mix = mix_of(objs)
    doc = {"source": os.path.relpath(lib, ROOT),
           "cycles": {"fast": C_FAST, "vop3": C_VOP3, "slow": C_SLOW, "sgpr": C_SLOW,
                      "sdwa": C_SLOW, "dpp": C_SLOW},
           "note": "static VALU mix per kernel, classes priced by tools/micro/valubench "
                   "(profiles/r03/micro/valubench_*.txt); cycles_per_valu = mean issue cycles "
                   "per wave64 VALU instruction on one SIMD",
           "kernels": mix}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k in sorted(mix):
        if any(s in k for s in ("decode_kernel<512", "pipe_kernel<512", "leaf_hash", "merkle_trees")):
            print(f"{k:60s} {mix[k]['valu_static']:7d} VALU  {mix[k]['cycles_per_valu']:.3f} cyc")


if __name__ == "__main__":
    main()
