# GPU call: decode parity tests, swap-stage study, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_llr.py tests/test_gpu_cli.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/vd_swapab 15 > gpurun_out/swapab.log 2>&1 && cat gpurun_out/swapab.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.log 2>&1
echo bench_rc=$?
tail -1 gpurun_out/quick_bench.log | cut -c1-700
