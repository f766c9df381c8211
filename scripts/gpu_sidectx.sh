# the side kernels timed as the bench's timed region (fresh process each, 100-batch launches):
# gpurun -- bash scripts/gpu_sidectx.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sidectx}
mkdir -p $O
for W in fp32_f16 soft16_b32 soft8_b16_llr soft8_b16 hard_b32,soft8_b16,fp32_f16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other --workloads $W > $O/$W.log 2>&1 || { echo rc=$? $W; tail $O/$W.log; exit 1; }
  tail -1 $O/$W.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$W', c['kernel_ms'], c.get('launch', {}).get('batches_per_launch'))"
done
echo all_rc=0
