# the default bench line (driver's command), and a short variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bench3}
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other > $O/bench_short.log 2> $O/bench_short.err
echo rc=$?
for f in $O/bench.log $O/bench_short.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['warmup_steps_run'], {k: v['gbps'] for k, v in d['config'].get('other_configs', {}).items()})"; done
