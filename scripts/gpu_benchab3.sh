# what makes bench.py's kernels slower than the A/B tool's: data noise, split
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-benchab3}
mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other"
timeout -k 10 300 tools/vd_benchab 6 10 0.04 1 > $O/ab_noisy.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 6 10 0.0 0.0 > $O/ab_clean.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 6 10 0.001 0.3 > $O/ab_low.log 2>&1 && \
VD_NO_SPLIT=1 timeout -k 10 300 $B > $O/bench_nosplit.json 2> $O/bench_nosplit.err && \
timeout -k 10 300 $B > $O/bench.json 2> $O/bench.err
echo rc=$?
cat $O/ab_noisy.log $O/ab_clean.log $O/ab_low.log
for f in $O/bench_nosplit.json $O/bench.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['kernel_ms'])"; done
