set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 tools/vd_ubench2 > gpurun_out/ubench2.log 2>&1
echo rc=$?
cat gpurun_out/ubench2.log
