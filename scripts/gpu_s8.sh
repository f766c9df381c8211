# SOFT8 packed kernel: its GPU tests, then the bench (parity block over every path).
# usage: gpurun --timeout 900 -- bash scripts/gpu_s8.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s8}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_pk.py -x -v -m gpu -k "s8" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo test_rc=$rc; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | tail -60; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], {k: v['gbps'] for k, v in c['other_configs'].items()}, c['single_launch'], c['parity']['all_match'], c['parity']['mismatching_paths'])"
