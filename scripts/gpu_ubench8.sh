set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/vd_ubench8 > gpurun_out/ubench8.log 2>&1
echo rc=$?
cat gpurun_out/ubench8.log
