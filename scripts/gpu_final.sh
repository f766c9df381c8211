# final-tree measurements: PMC passes for all five kernels, the driver's bench, and the same bench under
# rocprofv3 --kernel-trace --stats: gpurun --timeout 1100 -- bash scripts/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
bash scripts/gpu_pmc_all.sh ${1:-final}/pmc > $O/pmc_all.log 2>&1 || { echo pmc_rc=$?; tail $O/pmc_all.log; exit 1; }
tail -2 $O/pmc_all.log
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], {k: v['gbps'] for k, v in c['other_configs'].items()}, c['single_launch'], c['llr_input']['fused_batched'], d['roofline']['valu'].get('cycle_model_pct'), d['cpu_baseline']['matches_gpu'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/trace.log 2>&1 || { echo trace_rc=$?; tail $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -4 $O/kernel_stats.csv
echo all_rc=0
