# round-end rehearsal on the current tree: every GPU test, smoke(), the driver's bench command, and the same
# bench under rocprofv3 --kernel-trace --stats.  usage: gpurun --timeout 1100 -- bash scripts/gpu_r04.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r04}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || { grep -E "FAILED|ERROR" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke_rc=$?; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'kernel_ms', c.get('kernel_ms'))
print('parity', c['parity']['all_match'], c['parity'].get('mismatching_paths'), 'cpu matches', d['cpu_baseline']['matches_gpu'])
print('other', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in c['other_configs'].items()}))
print('single', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in c['single_launch'].items()}))
print('llr', json.dumps(c['llr_input'])[:300])
" $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py > $O/trace.log 2>&1 || { echo trace_rc=$?; tail $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -8 $O/kernel_stats.csv | cut -c1-200
echo all_rc=0
