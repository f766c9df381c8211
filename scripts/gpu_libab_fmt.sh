# same-box A/B of two builds of libvitdec.so through bench.py's timed region on chosen workloads (batched
# launches of 100 distinct resident batches), alternating: gpurun -- bash scripts/gpu_libab_fmt.sh <tag> <other lib>
# [rounds] [workloads]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-libabf}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-parity --workloads ${4:-fp32_f16,soft8_b16,hard_b32}"
for r in $(seq 1 ${3:-3}); do
  timeout -k 10 240 $B > $O/new_$r.log 2>&1 || { echo new_rc=$?; tail $O/new_$r.log; exit 1; }
  VITDEC_LIB=$2 timeout -k 10 240 $B > $O/old_$r.log 2>&1 || { echo old_rc=$?; tail $O/old_$r.log; exit 1; }
  for w in new old; do tail -1 $O/${w}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['config']['kernel_ms'], d['config']['kernel_gbps'])"; done
done
echo all_rc=0
