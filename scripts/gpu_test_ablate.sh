set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/t3.log 2>&1
echo test_rc=$?
tail -5 gpurun_out/t3.log
timeout -k 10 120 tools/vd_ablate 10 > gpurun_out/ablate3.log 2>&1
echo abl_rc=$?
cat gpurun_out/ablate3.log
