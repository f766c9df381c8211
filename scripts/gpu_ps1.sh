# paired-state kernel: GPU tests (no slow) on the default family (ps), then the bench with each family
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ps1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
B="python bench.py --no-cpu-baseline --no-pcie --no-llr --no-channel"
VD_KERNEL=ps timeout -k 10 300 $B > $O/bench_ps.log 2>&1 && VD_KERNEL=tg timeout -k 10 300 $B > $O/bench_tg.log 2>&1 && VD_KERNEL=ps timeout -k 10 300 $B > $O/bench_ps2.log 2>&1
echo rc=$?
for f in bench_ps bench_tg bench_ps2; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['config']['kernel_ms'], {k: v['gbps'] for k, v in d['config']['other_configs'].items()})"; done
