set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-benchtest}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bench.py -x -v -m gpu --timeout 280 --timeout-method thread > $O/tests.log 2>&1
echo rc=$?; tail -3 $O/tests.log
