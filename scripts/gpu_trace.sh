# rocprofv3 kernel trace + stats of the default bench command (the profile the bench line cites)
# usage: gpurun --timeout 600 -- bash scripts/gpu_trace.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}
mkdir -p $O
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/bench.log 2> $O/bench.err || { echo rc=$?; tail $O/bench.err; exit 1; }
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
t=$(find $O/trace -name "*kernel_trace.csv" | head -1); python3 tools/trace_summary.py $t > $O/kernel_trace_by_grid.txt
python3 - "$t" > $O/single_launch_gaps.txt <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "vd_decode" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# consecutive dispatches of the same kernel and grid: duration and the gap to the previous one's end
prev = {}
st = collections.defaultdict(list)
for r in rows:
    k = (r["Kernel_Name"].split("(")[0][-60:], r["Grid_Size_X"])
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if k in prev:
        st[k].append((e - s, s - prev[k]))
    prev[k] = e
for k, v in st.items():
    v.sort()
    d = [x[0] for x in v]; g = sorted(x[1] for x in v)
    print(k, "n", len(v), "dur us median %.1f" % (d[len(d)//2] / 1e3), "gap us median %.1f min %.1f" % (g[len(g)//2] / 1e3, g[0] / 1e3))
PY
cat $O/kernel_trace_by_grid.txt; cat $O/single_launch_gaps.txt; tail -1 $O/bench.log | cut -c1-300
