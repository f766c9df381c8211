"""Static lint of the kernels' inline assembly (CPU): every asm statement that runs a scalar ALU instruction
writing SCC must declare "scc" clobbered.

Round 2 found the renormalisation asm (`s_sub_u32` inside VD_TG_RN, vd_kernel_tg.h) without it: where the
compiler kept a branch condition in SCC across the statement, the branch followed the subtraction's
borrow instead (profiles/r02/scc_clobber_check.log).  The decode tests only catch such a bug when the
register allocation happens to expose it, so the rule is checked on the source."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc", f)
       for f in ("vd_kernel_tg.h", "vd_kernels.h", "vd_pack.h", "vd_mt.h", "vd_capi.hip")]
# SOP1/SOP2/SOPC instructions that write SCC (the ones the kernels could plausibly use)
SCC_WRITERS = re.compile(r"\bs_(add|sub|addc|subb|and|or|xor|andn2|orn2|nand|nor|xnor|lshl|lshr|ashr|bfe|"
                         r"min|max|cmp|bitcmp|not|abs|absdiff|cselect)\w*")


def _writes_scc(template):
    """a template (escape sequences as written in the source) runs an SCC-writing instruction"""
    return bool(SCC_WRITERS.search(template.replace("\\n", " ").replace("\\t", " ")))


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


def test_scc_writing_asm_declares_scc():
    bad = []
    for path in SRC:
        if not os.path.exists(path):
            continue
        text = open(path).read()
        macros = _macros(text)
        for line, stmt in _asm_statements(text):
            expanded = stmt
            for name in re.findall(r"\b[A-Z][A-Z0-9_]+\b", stmt):
                expanded += " " + macros.get(name, "")
            expanded = expanded.replace("\\n", " ").replace("\\t", " ")  # the templates' escape sequences
            if SCC_WRITERS.search(expanded) and '"scc"' not in stmt:
                bad.append(f"{os.path.basename(path)}:{line}")
    assert not bad, "asm writing SCC without a \"scc\" clobber: " + ", ".join(bad)


def test_lint_sees_the_renormalisation_asm():
    # the rule is not vacuous: the statements that carry VD_TG_RN are found and expand to s_sub_u32
    text = open(SRC[0]).read()
    macros = _macros(text)
    assert _writes_scc(macros["VD_TG_RN"])
    hits = [s for _, s in _asm_statements(text) if "VD_TG_RN" in s]
    assert len(hits) >= 3 and all('"scc"' in s for s in hits)
