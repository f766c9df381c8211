set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/vd_ubench10 > gpurun_out/ubench10.log 2>&1
echo rc=$?
cat gpurun_out/ubench10.log
