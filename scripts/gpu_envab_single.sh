# same-box A/B of an environment switch through bench.py's single-launch side measurement, alternating:
# gpurun -- bash scripts/gpu_envab_single.sh <tag> <VAR> [rounds]   (VAR=1 against VAR=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-envab}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel"
for r in $(seq 1 ${3:-3}); do
  for v in 1 0; do
    env $2=$v timeout -k 10 240 $B > $O/${v}_$r.log 2>&1 || { echo rc=$? v=$v; tail $O/${v}_$r.log; exit 1; }
    tail -1 $O/${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2=$v', {k: v['kernel_ms'] for k, v in d['config']['single_launch'].items()}, d['config']['kernel_ms'])"
  done
done
echo all_rc=0
