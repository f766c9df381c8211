# GPU call: split-launch tests, then the bench with and without splitting
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|re-decoded|passed|failed" gpurun_out/split_tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-llr --no-pcie --no-channel > gpurun_out/split_bench.log 2>&1 || exit 1
tail -1 gpurun_out/split_bench.log | cut -c1-420
VD_NO_SPLIT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-llr --no-pcie --no-channel > gpurun_out/nosplit_bench.log 2>&1 || exit 1
tail -1 gpurun_out/nosplit_bench.log | cut -c1-420
