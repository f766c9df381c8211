# round-5 measurement pass: GPU tests, smoke, bench (parity block), vd_ubench12 at 8 waves per SIMD, the
# packed kernels' component ablations (tools/vd_pkab), PMC passes of the bench's kernels.
# usage: gpurun --timeout 1150 -- bash scripts/gpu_r05.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05}
O=gpurun_out/$T
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo test_rc=$rc; tail -2 $O/tests.log
  [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | tail -60; exit 1; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
fi
timeout -k 10 300 python bench.py > $O/bench.log 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], {k: v['gbps'] for k, v in c['other_configs'].items()}, {k: v['gbps'] for k, v in c['single_launch'].items()}, c['llr_input']['fused_gbps'], c['llr_input']['fused_batched']['gbps'], c['parity']['all_match'], c['parity']['mismatching_paths'])"
timeout -k 10 200 tools/vd_ubench12 8 > $O/ubench12.log 2>&1 || { echo ubench_rc=$?; exit 1; }
timeout -k 10 200 tools/vd_pkab 8 20 > $O/ablate_batched.log 2>&1 || { echo pkab_rc=$?; exit 1; }
cat $O/ablate_batched.log
bash scripts/gpu_pmc.sh $T/main hard_b32,soft8_b16 > $O/pmc_main.log 2>&1 || { echo pmc_main_rc=$?; tail $O/pmc_main.log; exit 1; }
bash scripts/gpu_pmc.sh $T/other soft16_b32,fp32_f16,soft8_b16_llr > $O/pmc_other.log 2>&1 || { echo pmc_other_rc=$?; tail $O/pmc_other.log; exit 1; }
tail -3 $O/pmc_main.log
echo all_rc=0
