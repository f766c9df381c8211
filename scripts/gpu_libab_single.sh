# same-box A/B of two builds through bench.py's single-launch side measurement (20 launches of one 32M-bit
# batch per workload), alternating: gpurun -- bash scripts/gpu_libab_single.sh <tag> <other lib> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-libabs}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel"
for r in $(seq 1 ${3:-3}); do
  timeout -k 10 240 $B > $O/new_$r.log 2>&1 || { echo new_rc=$?; tail $O/new_$r.log; exit 1; }
  VITDEC_LIB=$2 timeout -k 10 240 $B > $O/old_$r.log 2>&1 || { echo old_rc=$?; tail $O/old_$r.log; exit 1; }
  for w in new old; do tail -1 $O/${w}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', {k: v['kernel_ms'] for k, v in d['config']['single_launch'].items()}, d['config']['kernel_ms'])"; done
done
echo all_rc=0
