set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/vd_ubench9 > gpurun_out/ubench9.log 2>&1
echo rc=$?
cat gpurun_out/ubench9.log
