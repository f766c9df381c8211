# packed split single launches: GPU tests (packed + split suites), then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pks}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pk.py tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value', d['value'], 'kernel_ms', d['config'].get('kernel_ms'))
p=d['config']['parity']; print('parity', p['all_match'], p.get('mismatching_paths'))
print('other', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in d['config']['other_configs'].items()}))
print('single', json.dumps(d['config']['single_launch'])[:400])
" $O/bench.json
echo all_rc=0
