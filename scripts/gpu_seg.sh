# segment launches: 3-mode single-launch A/B with clock stamps, then the split/guard/stream GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-seg}
mkdir -p $O
timeout -k 10 120 tools/vd_splitab 10 0.04 > $O/splitab.log 2>&1
echo splitab_rc=$?
cat $O/splitab.log | head -30
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_guard.py tests/test_gpu_streams.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head
