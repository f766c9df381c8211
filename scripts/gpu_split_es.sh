# split single-batch launches (vd_decode_pk, early-stop re-decodes): packed + split GPU tests, SOFT8 random /
# zeros study (tg segment launch vs packed split), bench with VD_PK_SPLIT=0 and default (single_launch block)
# usage: gpurun --timeout 900 -- bash scripts/gpu_split_es.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-es}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pk.py tests/test_gpu_split.py tests/test_gpu_llr.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | tail -60; exit 1; }
timeout -k 10 200 python tools/study/s8split_random.py > $O/random.log 2>&1 || { echo rnd_rc=$?; tail $O/random.log; exit 1; }
grep -v amdgpu.ids $O/random.log
B="python bench.py --no-cpu-baseline --no-pcie --no-channel"
for m in 0 1; do
  VD_PK_SPLIT=$m timeout -k 10 300 $B > $O/bench_pksplit$m.log 2>&1 || { echo bench_rc=$?; tail $O/bench_pksplit$m.log; exit 1; }
  tail -1 $O/bench_pksplit$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('VD_PK_SPLIT=$m', d['value'], c['kernel_ms'], {k: (v['kernel_ms'], v['gbps'], v['split_redecodes_per_launch']) for k, v in c['single_launch'].items()}, c['llr_input']['fused_gbps'], c['parity']['all_match'])"
done
echo all_rc=0
