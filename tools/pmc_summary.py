#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (counter_collection.csv) per decode kernel.

usage: python tools/pmc_summary.py <pmc dir with one sub-dir per pass> <out.json>

Per kernel name: mean of every counter over its dispatches, and the derived HBM traffic per
launch.  Units and gfx950 corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of a wide coalesced
streaming read on gfx950, so `traffic_bytes` doubles it (the decode kernels' input loads are
coalesced streaming reads); WRITE_SIZE is taken as is.  SQ cycle counters count quad-cycles.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

DECODE = {"vd::vd_decode_pk<0, 0, 32, false": "hard_b32", "vd::vd_decode_tg<0, 0, 32>": "hard_b32_tg",
          "vd::vd_decode_pk<2, 1, 32, false": "soft8_b16", "vd::vd_decode_tg<2, 1, 32>": "soft8_b16_tg",
          "vd::vd_decode_pk<10, 1, 32, false": "soft8_b16_llr",
          "vd::vd_decode_pk<4, 2, 32, false": "fp32_f16", "vd::vd_decode_tg<4, 2, 32>": "fp32_f16_tg",
          "vd::vd_decode_pk<1, 1, 32, false": "soft4_b16", "vd::vd_decode_tg<1, 1, 32>": "soft4_b16_tg",
          "vd::vd_decode_tg<3, 0, 32>": "soft16_b32", "vd::vd_decode_pk<0, 0, 16, false": "hard_b32_ob16",
          "vd::vd_decode_tg<0, 0, 16>": "hard_b32_ob16_tg",
          "vd::vd_decode_tg<10, 1, 32>": "soft8_b16_llr_tg"}


def short(name):
    for k, v in DECODE.items():
        if k in name:
            return v
    return None


def main():
    root, out = sys.argv[1], sys.argv[2]
    # --batches N: each dispatch decoded N batches (vd_run_device_batch); counters and durations per batch
    nb = int(sys.argv[sys.argv.index("--batches") + 1]) if "--batches" in sys.argv else 1
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]) / nb)
    # kernel durations of the passes run with --kernel-trace (the GRBM pass): the clock of that run
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "*", "*kernel_trace.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k is not None:
                    durs[k].append((float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) / nb)
    res = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        r = {"counters_mean_per_dispatch": m, "dispatches": max(len(v) for v in cs.values()), "batches_per_dispatch": nb,
             "per": "batch" if nb > 1 else "dispatch"}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            fetch = m["FETCH_SIZE"] * 1024 * 2  # KiB, x2 gfx950 streaming-read correction
            write = m["WRITE_SIZE"] * 1024
            r["fetch_bytes_corrected"] = fetch
            r["write_bytes"] = write
            r["traffic_bytes"] = fetch + write
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_BUSY_CYCLES" in m and "SQ_WAVES" in m:
            r["valu_active_per_wave_quadcycles"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVES"]
        if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
            r["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        if "SQ_INSTS_LDS" in m and "SQ_WAVES" in m:
            r["lds_insts_per_wave"] = m["SQ_INSTS_LDS"] / m.get("SQ_WAVES", 1)
        if durs.get(k):
            d = sorted(durs[k])
            r["pmc_run_kernel_ns_median"] = d[len(d) // 2]
            if "GRBM_GUI_ACTIVE" in m:  # summed over the 8 XCDs
                r["pmc_run_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / (sum(d) / len(d))
        res[k] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, r in res.items():
        print(k, {x: r[x] for x in r if x != "counters_mean_per_dispatch"})
        print("   ", {c: round(v, 1) for c, v in r["counters_mean_per_dispatch"].items()})


if __name__ == "__main__":
    main()
