# final-tree check: every GPU test, then the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['kernel_ms'], d['roofline']['int_op_roofline'], {k: v['gbps'] for k, v in d['config']['other_configs'].items()})"
