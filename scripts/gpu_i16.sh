# int32-pattern / 16-stage-field variant (ABL I16) against the product kernel, and the bench on distinct
# resident batches.  usage: gpurun -- bash scripts/gpu_i16.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-i16}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate 7 "i16,soft8/b16 full,fp32/f16 full,soft4/b16 full,soft8/b32 full" > $O/ablate.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 6 10 > $O/benchab.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
cat $O/ablate.log $O/benchab.log
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], c['ber'], c['launch'], {k: v['gbps'] for k, v in c['other_configs'].items()}, d['cpu_baseline']['matches_gpu'])"
