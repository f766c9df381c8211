# bench.py and the bench-condition A/B tool on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-benchab2}
mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other"
timeout -k 10 300 tools/vd_benchab 10 10 > $O/benchab.log 2>&1 && \
timeout -k 10 300 $B > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 300 tools/vd_benchab 10 10 > $O/benchab2.log 2>&1 && \
timeout -k 10 300 $B > $O/bench2.json 2> $O/bench2.err
echo rc=$?
cat $O/benchab.log $O/benchab2.log
for f in $O/bench1.json $O/bench2.json; do python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['config']['kernel_ms'], d['config']['ber'])"; done
