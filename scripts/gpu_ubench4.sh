set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/vd_ubench4 > gpurun_out/ubench4.log 2>&1
echo rc=$?
cat gpurun_out/ubench4.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/t4.log 2>&1
echo test_rc=$?
tail -3 gpurun_out/t4.log
