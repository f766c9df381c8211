# round 6: full GPU suite, smoke, the driver's bench command, packed-kernel ablations (tools/vd_pkab)
# usage: gpurun --timeout 1150 -- bash scripts/gpu_r06_suite.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $O/tests_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests_gpu.log | tail -60; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], {k: v['gbps'] for k, v in c['other_configs'].items()}, {k: v['gbps'] for k, v in c['single_launch'].items()}, c['parity']['all_match'], c['parity']['mismatching_paths'], d['roofline']['int_op_roofline'])"
timeout -k 10 200 tools/vd_pkab 6 20 > $O/ablate_batched.log 2>&1 || { echo pkab_rc=$?; exit 1; }
cat $O/ablate_batched.log
echo all_rc=0
