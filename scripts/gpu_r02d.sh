# all GPU tests (slow included), ablation of the exchange choice, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r02d}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 300 tools/vd_ablate 9 "tg soft8/b16 full,tg hard/b32 full,tg fp32/f16 full,q5,ACS only" > $O/ablate.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo rc=$?
cat $O/ablate.log
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], {k: v['gbps'] for k, v in d['config']['other_configs'].items()})"
