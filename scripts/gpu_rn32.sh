# renormalisation once per block (product) vs every 16 stages (ABL 27): twins, A/B, all GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rn32}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 300 tools/vd_ablate 5 "rn16,soft16/b32 full,fp32/f16 full" 8 > $O/ablate_batched.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 8 20 > $O/benchab.log 2>&1
echo rc=$?
cat $O/ablate_batched.log; tail -8 $O/benchab.log
