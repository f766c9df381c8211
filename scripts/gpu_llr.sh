set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-llr}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_llr.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-channel --no-other > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['kernel_ms'], d['config']['llr_input'])"
