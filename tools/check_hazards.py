#!/usr/bin/env python3
"""Static check of the hand-placed wait states in a decode kernel's assembly (tools only).

usage: python tools/check_hazards.py <file.s> <kernel symbol substring>

Checks, on the straight-line text of the kernel (every path is a superset of the textual order inside a
basic block; the kernels' stage code is branch-free): a DPP read of a VGPR needs 2 wait states after the
last VALU write of it, v_permlane*_swap 2, v_readfirstlane 1.  s_nop N counts N+1 wait states, every
other instruction 1.  Prints the violations (exit 1 if any) and the s_nop count.
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines, on = [], False
    for raw in open(path):
        l = raw.split(";")[0].strip()
        if not on:
            if raw.startswith(sym) or (sym in raw and raw.rstrip().endswith(":") and not raw.startswith(".")):
                on = True
            continue
        if raw.startswith(".Lfunc_end"):
            break
        if not l or l.startswith(".") or l.endswith(":"):
            continue
        lines.append(l)
    lastw = {}
    viol = 0
    for i, l in enumerate(lines):
        parts = l.replace(",", " ").split()
        op = parts[0]
        regs = re.findall(r"\bv(\d+)\b|v\[(\d+):(\d+)\]", " ".join(parts[1:]))
        srcs = set()
        toks = [t for t in parts[1:] if t.startswith("v")]
        # sources: every VGPR operand after the destination
        for t in toks[1:] if op.startswith("v_") else toks:
            m = re.match(r"v(\d+)$", t)
            if m:
                srcs.add(int(m.group(1)))
            m = re.match(r"v\[(\d+):(\d+)\]$", t)
            if m:
                srcs.update(range(int(m.group(1)), int(m.group(2)) + 1))
        need = 2 if "_dpp" in op or "permlane" in op else 1 if op.startswith("v_readfirstlane") else 0
        if "permlane" in op:  # both operands are read
            srcs = set()
            for t in toks:
                m = re.match(r"v(\d+)$", t)
                if m:
                    srcs.add(int(m.group(1)))
        if need:
            check = srcs if "permlane" in op or op.startswith("v_readfirstlane") else (
                {int(re.match(r"v(\d+)$", toks[1]).group(1))} if len(toks) > 1 and re.match(r"v(\d+)$", toks[1]) else set())
            for r in check:
                if r not in lastw:
                    continue
                ws = 0
                for k in range(lastw[r] + 1, i):
                    o = lines[k].split()
                    ws += int(o[1]) + 1 if o[0] == "s_nop" else 1
                if ws < need:
                    viol += 1
                    print(f"VIOLATION v{r}: {lines[lastw[r]]}  ->  {l}  ({ws} < {need})")
        if op.startswith("v_") and toks:
            d = toks[0]
            m = re.match(r"v(\d+)$", d)
            if m:
                lastw[int(m.group(1))] = i
            m = re.match(r"v\[(\d+):(\d+)\]$", d)
            if m:
                for r in range(int(m.group(1)), int(m.group(2)) + 1):
                    lastw[r] = i
            if "permlane" in op:  # swaps write both operands
                for t in toks[:2]:
                    m = re.match(r"v(\d+)$", t)
                    if m:
                        lastw[int(m.group(1))] = i
    nops = sum(1 for l in lines if l.startswith("s_nop"))
    print(f"{len(lines)} instructions, {nops} s_nop, {viol} violations")
    sys.exit(1 if viol else 0)


if __name__ == "__main__":
    main()
