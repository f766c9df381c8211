set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_llr.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/llr.log 2>&1
echo rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/llr.log | tail -25
