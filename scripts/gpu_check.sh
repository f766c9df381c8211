# GPU tests, smoke() and the driver's bench command on the current tree (no profiling passes).
# usage (from this container): gpurun --timeout 1100 -- bash scripts/gpu_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | tail -60; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
cat $O/smoke.log
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], c['ber'], {k: v['gbps'] for k, v in c['other_configs'].items()}, c['single_launch'], c['final_gather'], d['cpu_baseline']['matches_gpu'], c['parity']['all_match'], c['parity']['mismatching_paths'], c['parity']['seconds'])"
