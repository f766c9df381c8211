# chosen GPU test files, then the bench line: gpurun -- bash scripts/gpu_tb.sh <tag> <test files...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-tb}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']
print('value', d['value'], 'kernel_ms', c.get('kernel_ms'))
print('parity', c['parity']['all_match'], c['parity'].get('mismatching_paths'))
print('other', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in c['other_configs'].items()}))
print('single', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in c['single_launch'].items()}))
" $O/bench.json
echo all_rc=0
