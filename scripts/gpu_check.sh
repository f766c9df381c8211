# GPU call: the full-size parity tests, then the bench line (all side measurements)
# usage: gpurun --timeout 900 -- bash scripts/gpu_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m "gpu and slow" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -6 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
rc=$?
tail -1 $O/bench.log
exit $rc
