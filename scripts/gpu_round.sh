# round-end rehearsal on the final tree: GPU tests, smoke(), PMC passes + kernel trace, the driver's bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
bash scripts/gpu_pmc.sh ${1:-round}/p > $O/pmc2.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
cat $O/smoke.log; tail -4 $O/pmc2.log
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['kernel_ms'], c['ber'], {k: v['gbps'] for k, v in c['other_configs'].items()}, d['cpu_baseline']['matches_gpu'], d['roofline']['valu'].get('cycle_model_pct'))"
