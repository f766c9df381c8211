# quick check after a kernel change: GPU tests (no slow), ablation with exact twins, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed\|error" $O/tests.log || exit 1
timeout -k 10 300 tools/vd_ablate ${2:-5} > $O/ablate.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-channel > $O/bench.log 2>&1
echo rc=$?
grep -v "^===\|kernel span\|wave \|clock\|cycles/stage\|progress\|SIMDs" $O/ablate.log | head -45
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['kernel_ms'], d['config']['kernel_gbps'])"
