# fast GPU parity tests, then the ablation timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/tests_fast.log 2>&1
rc=$?
echo test_rc=$rc
tail -4 gpurun_out/tests_fast.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 tools/vd_ablate ${1:-8} > gpurun_out/ablate.log 2>&1
echo abl_rc=$?
head -40 gpurun_out/ablate.log
