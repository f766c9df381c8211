# M_B32 with the LDS xor-32 exchange: GPU tests, bench-condition A/B, ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s32}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q " failed\| error" $O/tests.log || exit 1
timeout -k 10 300 tools/vd_benchab 8 10 > $O/benchab.log 2>&1 && \
timeout -k 10 300 tools/vd_ablate 9 "tg hard/b32,tg soft8/b16 full" > $O/ablate.log 2>&1
echo rc=$?
cat $O/benchab.log; grep -v "^===" $O/ablate.log
