# SOFT8 table rows from the two soft values (product) against (A, B) rows (ABL 30): twins, A/B, GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-s01}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate 5 "soft8/b16 full,ab rows,soft8/b16 -tabbuild" 8 > $O/ablate_batched.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 8 20 > $O/benchab.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo rc=$?
cat $O/ablate_batched.log; tail -7 $O/benchab.log; tail -2 $O/tests.log
