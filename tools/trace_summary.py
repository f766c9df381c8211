"""Per-kernel, per-grid dispatch durations from a rocprofv3 --kernel-trace CSV (kernel_trace.csv):
separates the bench's K-batch launches (vd_decode_tg: 1600 K workgroups x 256; vd_decode_pk: 800 K, two
chunks per wave) from its single launches and side measurements, which --stats averages together.  usage: python tools/trace_summary.py <run_kernel_trace.csv>"""
import collections
import csv
import sys


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "vd_decode_tg" not in name and "vd_decode_pk" not in name:
            continue
        tmpl = ("tg<" if "vd_decode_tg" in name else "pk<") + name.split("<", 1)[1].split(">", 1)[0] + ">"
        wgs = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        d[(tmpl, wgs)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'vd_decode_tg/pk<CH, CORE, OB, ..>':34s} {'workgroups':>10s} {'calls':>6s} {'avg us':>10s} {'min us':>10s} {'batches':>8s} {'avg us/batch':>12s}")
    for (tmpl, wgs), v in sorted(d.items()):
        per = 800 if tmpl.startswith("pk<") and "false" in tmpl else 1600  # batched pk: 8 chunks per workgroup
        nb = wgs // per if wgs % per == 0 else 1
        avg = sum(v) / len(v) / 1e3
        print(f"{tmpl:34s} {wgs:10d} {len(v):6d} {avg:10.1f} {min(v) / 1e3:10.1f} {nb:8d} {avg / nb:12.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
