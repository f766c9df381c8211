# packed SOFT4 / FP32 kernels: GPU tests vs oracle, then the bench line with its parity block
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pk4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pk.py -x -q --timeout 300 --timeout-method thread > $O/tests_pk.log 2>&1 || { echo tests_rc=$?; tail -30 $O/tests_pk.log; exit 1; }
tail -2 $O/tests_pk.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench_rc=$?; tail $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('value', d['value'], 'kernel_ms', d['config'].get('kernel_ms'))
print('parity', json.dumps(d['config']['parity'])[:600])
print('other', json.dumps({k:(v['kernel_ms'],v['gbps']) for k,v in d['config']['other_configs'].items()}))
print('single', json.dumps(d['config']['single_launch'])[:400])
" $O/bench.json
echo all_rc=0
