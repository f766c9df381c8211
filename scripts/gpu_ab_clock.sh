# same-box A/B of two builds of the packed kernels' split single launches (tools/vd_pkclock_old / _new):
# gpurun -- bash scripts/gpu_ab_clock.sh <tag> [pairs] [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abclock}
mkdir -p $O
for r in $(seq 1 ${2:-3}); do
  for v in old new; do
    timeout -k 10 200 tools/vd_pkclock_$v ${3:-10} > $O/${v}_$r.log 2>&1 || { echo ${v}_rc=$?; tail $O/${v}_$r.log; exit 1; }
    grep "launch" $O/${v}_$r.log | sed "s/^/$v $r: /" | cut -c1-150
  done
done
echo all_rc=0
