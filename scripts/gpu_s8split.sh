# SOFT8 single-batch launch: tg segments against the packed split kernel (VD_PK_SPLIT=2), bench data and random
# usage: gpurun --timeout 900 -- bash scripts/gpu_s8split.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s8split}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-llr --no-pcie --no-channel"
timeout -k 10 300 $B > $O/bench_default.log 2>&1 || { echo bench_rc=$?; tail $O/bench_default.log; exit 1; }
VD_PK_SPLIT=2 timeout -k 10 300 $B > $O/bench_s8split.log 2>&1 || { echo bench2_rc=$?; tail $O/bench_s8split.log; exit 1; }
for w in default s8split; do tail -1 $O/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['config']['kernel_ms'], d['config']['single_launch'])"; done
timeout -k 10 200 python tools/study/s8split_random.py > $O/random.log 2>&1 || { echo rnd_rc=$?; tail $O/random.log; exit 1; }
cat $O/random.log
