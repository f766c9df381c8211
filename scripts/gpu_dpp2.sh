# GPU call: parity of the two-op DPP stage, A/B timing against the three-op stage, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dpp2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/vd_ablate 8 > $O/ablate.log 2>&1 || exit 1
grep "full\|3-op" $O/ablate.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-400
