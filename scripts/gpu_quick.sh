# quick check of the packed kernels after a change: their GPU tests, the A/B tool, the bench
# usage: gpurun --timeout 900 -- bash scripts/gpu_quick.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pk.py tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | tail -60; exit 1; }
timeout -k 10 200 tools/vd_pkab 8 20 > $O/ablate_batched.log 2>&1 || { echo pkab_rc=$?; exit 1; }
cat $O/ablate_batched.log
timeout -k 10 300 python bench.py > $O/bench.log 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], {k: v['gbps'] for k, v in c['other_configs'].items()}, {k: v['gbps'] for k, v in c['single_launch'].items()}, c['llr_input']['fused_gbps'], c['llr_input']['fused_batched']['gbps'], c['parity']['all_match'], c['parity']['mismatching_paths'])"
