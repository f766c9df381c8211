#!/usr/bin/env python3
"""Per-kernel PMC table for the ablation driver (tools only): python tools/pmc_abl.py <dir>"""
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "*", "*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        n = row["Kernel_Name"]
        if "vd_decode" not in n:
            continue
        n = n.split("(")[0].replace("void vd::", "")
        vals[n][row["Counter_Name"]].append(float(row["Counter_Value"]))
cols = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
        "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_IFETCH"]
print("%-34s" % "kernel (per wave; /5088 stages)" + "".join("%11s" % c.replace("SQ_", "")[:10] for c in cols))
for n in sorted(vals):
    v = vals[n]
    w = sum(v["SQ_WAVES"]) / max(1, len(v["SQ_WAVES"])) or 6400
    row = []
    for c in cols:
        x = v.get(c)
        row.append(sum(x) / len(x) / w / 5088 if x else float("nan"))
    print("%-34s" % n[:34] + "".join("%11.3f" % r for r in row))
