# tagged kernel: fast parity tests then ablation timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tg1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/tg1/tests.log 2>&1
rc=$?
echo test_rc=$rc
tail -15 gpurun_out/tg1/tests.log
timeout -k 10 120 tools/vd_ablate 8 > gpurun_out/tg1/ablate.log 2>&1
echo abl_rc=$?
cat gpurun_out/tg1/ablate.log
