"""Steady-state VALU instruction mix of the batched decode kernels, from their compiled ISA (tools only).

Compiles vd_decode_pk<HARD,B32> and vd_decode_pk<SOFT8,B16> (the bench's headline kernels, batched form)
to gfx950 assembly and weighs the basic blocks of the 96-stage group loop by how often they run per group:
the three block bodies (32 stages each) once, the traceback bodies (ds_read_u8 chains) once per TBS
blocks (5 words per pass for HARD, 6 for SOFT8), the fairness controller's blocks every other group,
everything else in the loop once.  Output per
kernel: VALU instructions per chunk-stage (a chunk's 64 states for one stage; two chunks per wave), by
opcode, and the same with per-opcode issue costs from a vd_ubench12 log (cycles, relative to v_fma_f32 at 2
cycles: MI355X_MICROARCH.md), i.e. the VALU cycles a chunk-stage needs.  bench.py reads the JSON this writes
(profiles/<round>/valu_model.json) for roofline.valu.cycle_model.

Usage: python tools/isa_mix.py <ubench12.log> <out.json>
"""
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc")
KERNELS = {"hard_b32": "vd::HARD, vd::B32", "soft8_b16": "vd::SOFT8, vd::B16"}
TBS = 5  # words per traceback pass (PkLds: 5 at 8 waves per SIMD, 6 at 7; set per kernel in main)
TBS_OF = {"hard_b32": 5, "soft8_b16": 6}
# ubench12 row name for an opcode (issue cost); opcodes not measured take the 4-cycle class of bit/int ops
UB = {"v_add_f32": "add_f32", "v_sub_f32": "sub_f32", "v_fma_f32": "fma_f32", "v_max_f32": "max_f32",
      "v_add_u32": "add_u32", "v_sub_u32": "sub_u32", "v_sub_u32_dpp": "sub_u32_dpp", "v_pk_max_u16": "pk_max_u16",
      "v_and_b32": "and_b32", "v_xad_u32": "xad_u32", "v_lshl_or_b32": "lshl_or_b32", "v_or3_b32": "or3_b32",
      "v_xor_b32": "xor_b32", "v_lshlrev_b32": "lshlrev_b32", "v_lshrrev_b32": "lshrrev_b32",
      "v_bitop3_b32": "bitop3_b32", "v_lshl_add_u32": "lshl_add_u32", "v_bfe_u32": "bfe_u32", "v_bfi_b32": "bfi_b32",
      "v_perm_b32": "perm_b32", "v_mul_u32_u24": "mul_u32_u24", "v_cndmask_b32": "cndmask_b32",
      "v_readfirstlane_b32": "readfirstlane", "v_and_or_b32": "and_or_b32", "v_lshrrev_b32_sdwa": "lshr_sdwa",
      "v_add3_u32": "add3_u32", "v_max_i32": "max_i32", "v_add_u32_dpp": "sub_u32_dpp"}


def compile_isa():
    tu = "#include \"vd_kernel_pk.h\"\n" + "".join(
        f"template __global__ void vd::vd_decode_pk<{a}, 32, false>(const void*, void*, vd::Geom);\n" for a in KERNELS.values())
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "mix.hip")
        open(p, "w").write(tu)
        s = os.path.join(d, "mix.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                        "-w", "-I", CSRC, p, "-o", s], check=True, capture_output=True, timeout=900)
        return open(s).read()


def blocks_of(asm, sym):
    i = asm.index("\n" + sym + ":")
    body = asm[i:asm.index(".Lfunc_end", i)].split("\n")
    # a block: (label, opcodes, loop header?, inside a loop?) from the compiler's "Loop Header" / "in Loop"
    # annotations on the label line
    out, cur, name, hdr, inl = [], [], "entry", False, False
    for line in body:
        st = line.strip()
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):", st)
        if m:
            out.append((name, cur, hdr, inl))
            cur, name, hdr, inl = [], m.group(1), "Loop Header" in st, "Loop" in st
        elif st and not st.startswith((";", ".")):
            cur.append(st.split()[0])
    out.append((name, cur, hdr, inl))
    return out


def group_mix(blocks):
    """per-group dynamic VALU counts by opcode over the group loop's blocks"""
    start = next(k for k, b in enumerate(blocks) if b[2])
    mix = Counter()
    for name, ins, _, inl in blocks[start:]:
        c = Counter(ins)
        if "s_endpgm" in c:
            break
        if not inl:  # after the group loop (the guard check, the split's pass epilogue): once per kernel
            continue
        if any(op.startswith(("ds_read_u8", "ds_read_u16")) for op in c):
            w = 1.0 / TBS  # a traceback body: one pass per TBS blocks
        elif "s_setprio" in c or "v_add_u32_dpp" in c or "global_load_dword" in c or "global_store_dword" in c:
            w = 0.5  # the fairness controller: every other group head
        else:
            w = 1.0
        for op, n in c.items():
            if op.startswith("v_"):
                mix[re.sub(r"_e(32|64)$", "", op)] += w * n
    return mix


def costs(log):
    """cycles per opcode from a vd_ubench12 log (ns per unit per SIMD), scaled so that v_fma_f32 = 2"""
    ns = {}
    for line in open(log):
        m = re.match(r"^(\S+)\s+([0-9.]+) ns$", line.strip())
        if m:
            ns[m.group(1)] = float(m.group(2))
    ref = ns["fma_f32"] / 2.0
    return {op: round(ns[u] / ref, 2) for op, u in UB.items() if u in ns}, ns


def main():
    log, out = sys.argv[1], sys.argv[2]
    asm = compile_isa()
    cyc, ns = costs(log)
    res = {"what": __doc__.split("\n\n")[0], "ubench_log": os.path.relpath(log, ROOT), "cycles_per_opcode": cyc,
           "kernels": {}}
    for name, args in KERNELS.items():
        sym = next(s for s in re.findall(r"\n(_ZN2vd12vd_decode_pk\w+):", asm)
                   if s.startswith("_ZN2vd12vd_decode_pkILi%dELi%d" % ((0, 0) if name == "hard_b32" else (2, 1))))
        global TBS
        TBS = TBS_OF[name]
        mix = group_mix(blocks_of(asm, sym))
        per = {op: n / (96 * 2) for op, n in mix.items()}  # a group: 96 stages of two chunks
        total = sum(per.values())
        unknown = sorted(op for op in per if op not in cyc)
        cycles = sum(n * cyc.get(op, 4.0) for op, n in per.items())
        res["kernels"][name] = {"symbol": sym, "valu_per_chunk_stage": round(total, 3),
                                "valu_cycles_per_chunk_stage": round(cycles, 3),
                                "opcodes_at_default_4_cycles": unknown,
                                "mix_per_chunk_stage": {op: round(n, 4) for op, n in sorted(per.items(), key=lambda x: -x[1])}}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(k, v["valu_per_chunk_stage"], "VALU /chunk-stage,", v["valu_cycles_per_chunk_stage"], "cycles; default-4:",
              v["opcodes_at_default_4_cycles"])


if __name__ == "__main__":
    main()
