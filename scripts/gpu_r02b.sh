# Round-2: new fairness board + barrier split protocol: all GPU tests, split A/B (codeword and random
# data), ablation incl. board load flavour, bench, HBM traffic of the bench kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log
[ -f $O/tests.log ] && grep -q " passed" $O/tests.log || exit 1
timeout -k 10 120 tools/vd_splitab 10 0.04 > $O/splitab_bsc04.log 2>&1 && \
timeout -k 10 120 tools/vd_splitab 10 0.5 > $O/splitab_random.log 2>&1 && \
timeout -k 10 200 tools/vd_ablate 5 > $O/ablate.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-400 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other > $O/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other > $O/pmc_write.log 2>&1
echo rc=$?
head -3 $O/splitab_bsc04.log $O/splitab_random.log
cat $O/ablate.log | head -40
