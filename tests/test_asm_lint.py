"""Static checks of the kernels' inline assembly (CPU).

Round 2 found the renormalisation asm (`s_sub_u32` inside VD_TG_RN, vd_kernel_tg.h) without an "scc"
clobber: where the compiler kept a branch condition in SCC across the statement, the branch followed the
subtraction's borrow instead (profiles/r02/scc_clobber_check.log) and an LDS ring store went one slot
below the wave's ring.  The decode tests only catch such a bug when the register allocation happens to
expose it, so the rules are checked on the source and on the compiled code:
  * every asm statement whose instructions write SCC, VCC, EXEC or M0 implicitly (or name them as a
    destination) declares that register clobbered;
  * every physical VGPR an asm template names is a declared clobber or a "{vN}" operand constraint;
  * in the compiled kernels no SCC reader follows the renormalisation's s_sub_u32 before an SCC writer,
    and the same scan finds such readers in a scratch copy without the clobber (the scan is not vacuous).
"""
import glob
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc")
SRC = sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip")) +
             glob.glob(os.path.join(ROOT, "tools", "*.hip")) + glob.glob(os.path.join(ROOT, "tools", "*.h")))
# SOP1/SOP2/SOPC instructions that write SCC (the ones the kernels could plausibly use)
SCC_WRITERS = re.compile(r"\bs_(add|sub|addc|subb|and|or|xor|andn2|orn2|nand|nor|xnor|lshl|lshr|ashr|bfe|"
                         r"min|max|cmp|bitcmp|not|abs|absdiff|cselect)\w*")
# instructions writing VCC / EXEC / M0 without naming them as an operand
VCC_WRITERS = re.compile(r"\bv_(cmp_\w+_e32|cmp_class_\w+_e32|add_co_u32\w*|sub_co_u32\w*|subrev_co_u32\w*|"
                         r"addc_co_u32\w*|subb_co_u32\w*|subbrev_co_u32\w*|div_scale\w*)\b|\bvcc\b")
EXEC_WRITERS = re.compile(r"\b(v_cmpx_\w+|s_\w+_saveexec_b\d+|s_\w+_wrexec_b\d+)\b|\bexec\b")
M0_WRITERS = re.compile(r"\bm0\b")
PHYS_VGPR = re.compile(r"(?<!\[)\bv(\d+)\b|\bv\[(\d+):(\d+)\]")  # not a named operand %[v0]


def _macros(text):
    """#define NAME "..." string macros (with line continuations), for expanding asm templates"""
    out = {}
    for m in re.finditer(r"#define\s+(\w+)(\([^)]*\))?\s+((?:[^\n]*\\\n)*[^\n]*)", text):
        out[m.group(1)] = m.group(3).replace("\\\n", " ")
    return out


def _asm_statements(text):
    """(line, statement text) of every asm(...) / asm volatile(...) statement, parentheses balanced"""
    for m in re.finditer(r"\basm\s*(volatile\s*)?\(", text):
        i, depth = m.end(), 1
        while depth and i < len(text):
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        yield text.count("\n", 0, m.start()) + 1, text[m.start():i]


def _split(stmt):
    """(template strings, constraint/clobber part) of an asm statement: split at the first ':' outside the
    string literals (templates contain ':' themselves, e.g. offset:%[o])"""
    body = stmt[stmt.index("(") + 1:-1]
    inq = False
    for i, ch in enumerate(body):
        if ch == '"' and (i == 0 or body[i - 1] != "\\"):
            inq = not inq
        elif ch == ":" and not inq:
            return body[:i], body[i + 1:]
    return body, ""


def _statements():
    for path in SRC:
        text = open(path).read()
        macros = _macros(text)
        for line, stmt in _asm_statements(text):
            tmpl, rest = _split(stmt)
            expanded = tmpl
            for name in re.findall(r"\b[A-Z][A-Z0-9_]+\b", tmpl):
                expanded += " " + macros.get(name, "")
            expanded = expanded.replace("\\n", " ").replace("\\t", " ")  # the templates' escape sequences
            yield f"{os.path.relpath(path, ROOT)}:{line}", stmt, expanded, rest


def test_sources_scanned():
    names = [os.path.basename(p) for p in SRC]
    assert "vd_kernel_tg.h" in names and "vd_capi.hip" in names and "vd_ablate.hip" in names


def test_scc_writing_asm_declares_scc():
    bad = [w for w, stmt, tmpl, rest in _statements() if SCC_WRITERS.search(tmpl) and '"scc"' not in rest]
    assert not bad, "asm writing SCC without a \"scc\" clobber: " + ", ".join(bad)


def _saves_m0(tmpl):
    """M0 is reserved: the compiler ignores an "m0" clobber, so a statement that writes M0 must save it first
    and restore it last (s_mov_b32 %[t], m0 ... s_mov_b32 m0, %[t])"""
    ins = [i.strip() for i in re.split(r"\s{2,}|\n|\\n", tmpl.replace('"', " ")) if i.strip()]
    m = re.match(r"s_mov_b32 (%\[\w+\]), m0$", ins[0]) if ins else None
    return bool(m) and ins[-1] == f"s_mov_b32 m0, {m.group(1)}"


@pytest.mark.parametrize("reg,pat", [("vcc", VCC_WRITERS), ("exec", EXEC_WRITERS), ("m0", M0_WRITERS)])
def test_vcc_exec_m0_writing_asm_declares_them(reg, pat):
    bad = [w for w, stmt, tmpl, rest in _statements() if pat.search(tmpl) and f'"{reg}"' not in rest
           and not (reg == "m0" and _saves_m0(tmpl))]
    assert not bad, f"asm writing {reg} without a \"{reg}\" clobber: " + ", ".join(bad)


def test_m0_save_restore_rule_is_not_vacuous():
    hits = [w for w, stmt, tmpl, rest in _statements() if M0_WRITERS.search(tmpl)]
    assert hits and all(_saves_m0(t) for w, s, t, r in _statements() if M0_WRITERS.search(t))
    assert not _saves_m0("s_mov_b32 m0, %[b]  ds_write_addtid_b32 %[v]")


def test_physical_vgprs_are_declared():
    bad = []
    for w, stmt, tmpl, rest in _statements():
        for m in PHYS_VGPR.finditer(tmpl):
            regs = [int(m.group(1))] if m.group(1) else list(range(int(m.group(2)), int(m.group(3)) + 1))
            for r in regs:
                if f'"v{r}"' not in rest and "{v%d}" % r not in rest:
                    bad.append(f"{w} v{r}")
    assert not bad, "asm naming a VGPR that is neither clobbered nor a {vN} operand: " + ", ".join(bad)


def test_lint_sees_the_renormalisation_asm():
    # the rules are not vacuous: the statements that carry VD_TG_RN are found and expand to s_sub_u32
    path = os.path.join(CSRC, "vd_kernel_tg.h")
    text = open(path).read()
    assert SCC_WRITERS.search(_macros(text)["VD_TG_RN"].replace("\\n", " ").replace("\\t", " "))
    hits = [s for w, s, t, r in _statements() if w.startswith("gpu-accelerated") and "VD_TG_RN" in s]
    assert len(hits) == 2 and all('"scc"' in s for s in hits)


# ---- the compiled kernels ----
_TU = """#include "vd_kernel_pk.h"
template __global__ void vd::vd_decode_pk<vd::HARD, vd::B32>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_pk<vd::FP32, vd::F16>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_pk<vd::SOFT8, vd::B32>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_tg<vd::FP32, vd::F16, 32>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_tg<vd::HARD, vd::B32, 32>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_tg<vd::SOFT8, vd::B16, 32>(const void*, void*, vd::Geom);
template __global__ void vd::vd_decode_tg<vd::SOFT16, vd::B32, 16>(const void*, void*, vd::Geom);
"""


def _compile(csrc_dir, out_dir):
    tu = os.path.join(out_dir, "isa_probe.hip")
    with open(tu, "w") as f:
        f.write(_TU)
    s = os.path.join(out_dir, "isa_probe.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-w", "-I", csrc_dir, tu, "-o", s], check=True, capture_output=True, timeout=600)
    return open(s).read()


def scc_reads_after_renorm(asm):
    """per kernel: SCC readers reached from a renormalisation s_sub_u32 (the VBASE subtraction) before any
    SCC writer, on the straight-line text"""
    out = {}
    for m in re.finditer(r"\n(_ZN2vd12vd_decode_(?:tg|pk)\w+):[^\n]*\n", asm):
        i = m.end()
        body = [l.split(";")[0].strip() for l in asm[i:asm.index(".Lfunc_end", i)].split("\n")]
        hits = 0
        for k, l in enumerate(body):
            # the VBASE subtraction: s_sub_u32 s, s, VBASE (tg, pk HARD / SOFT4 / FP32), or s_sub_u32 s, K, s with
            # K = VBASE - 0x10001 (pk SOFT8's merged clear + renormalisation)
            if not (l.startswith("s_sub_u32") and re.search(r"(, (0x4b2\w+|0x1f001f00|0x20102010|0x100|0x10000|256|65536)$|"
                                                            r"^s_sub_u32 s\d+, 0x64036403, s\d+$)", l)):
                continue
            for l2 in body[k + 1:k + 60]:
                if l2.startswith(("s_cbranch_scc", "s_cselect", "s_addc", "s_subb", "s_cmov")):
                    hits += 1
                    break
                if SCC_WRITERS.match(l2):
                    break
        out[m.group(1)] = hits
    return out


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_compiled_kernels_do_not_branch_on_the_renormalisation_borrow():
    with tempfile.TemporaryDirectory() as d:
        product = scc_reads_after_renorm(_compile(CSRC, d))
        scratch_src = os.path.join(d, "csrc")
        shutil.copytree(CSRC, scratch_src)
        p = os.path.join(scratch_src, "vd_kernel_tg.h")
        s = open(p).read()
        old = 'VD_TG_RN : [V] "+{v60}"(V), [w] "+v"(word), [sr] "=&s"(sr) : VD_TG_IN : "scc");'
        assert s.count(old) == 2
        open(p, "w").write(s.replace(old, old.replace(' : "scc");', ");")))
        scratch = scc_reads_after_renorm(_compile(scratch_src, d))
    assert len(product) == 7 and all(v == 0 for v in product.values()), product
    # without the clobber the compiler does branch on SCC right after the subtraction
    assert sum(scratch.values()) > 0, scratch
