# One GPU call: parity tests, bench line, rocprofv3 kernel-trace summary, ablation timings.
# usage (from this container): gpurun --timeout 900 -- bash scripts/gpu_round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-llr --no-pcie --no-channel > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -5 $O/kernel_stats.csv
timeout -k 10 120 tools/vd_ablate 5 > $O/ablate.log 2>&1
echo abl_rc=$?
cat $O/ablate.log
