# One GPU call: bench line, rocprofv3 kernel-trace summary of the timed kernels (side measurements off,
# so the per-kernel averages are the bench's launches only), then the PMC passes.
# usage: gpurun --timeout 900 -- bash scripts/gpu_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-llr --no-pcie --no-channel > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
tail -1 $O/prof.log
head -5 $O/kernel_stats.csv
bash scripts/gpu_pmc.sh ${TAG}_pmc
