# final tree: PMC passes + kernel trace, then the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final4}
mkdir -p $O
bash scripts/gpu_pmc2.sh ${1:-final4}/p > $O/pmc2.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -6 $O/pmc2.log
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], c['ber'], {k: v['gbps'] for k, v in c['other_configs'].items()}, d['cpu_baseline']['matches_gpu'])"
