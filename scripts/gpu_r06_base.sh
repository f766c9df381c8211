# round 6 baseline: per-batch kernel time at the driver's K = 20 against K = 100 (same box, alternating),
# the two-stream step at K = 20 and 100, and the wave timeline of 20-batch launches
# usage: gpurun --timeout 900 -- bash scripts/gpu_r06_base.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-base}
mkdir -p $O
F="--no-cpu-baseline --no-llr --no-pcie --no-channel --no-other --no-parity"
for i in 1 2; do
  for K in 20 100; do
    timeout -k 10 200 python bench.py --steps $K --warmup 5 $F > $O/bench_k${K}_$i.log 2> $O/bench_k${K}_$i.err || { echo bench_rc=$?; tail $O/bench_k${K}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_k${K}_$i.log'.replace('.log','.log'))) if False else None" 2>/dev/null
    tail -1 $O/bench_k${K}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('K=$K run $i', d['value'], d['ms_per_step'], c['kernel_ms'])"
  done
done
timeout -k 10 120 tools/vd_concur 10 20 > $O/concur_k20.log 2>&1 || { echo concur_rc=$?; exit 1; }
cat $O/concur_k20.log
timeout -k 10 200 tools/vd_concur 6 100 > $O/concur_k100.log 2>&1 || { echo concur_rc=$?; exit 1; }
cat $O/concur_k100.log
timeout -k 10 200 tools/vd_pkclock 10 > $O/pkclock.log 2>&1 || { echo pkclock_rc=$?; exit 1; }
grep -A9 "batched" $O/pkclock.log
echo all_rc=0
