set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 tools/vd_acs_ubench > gpurun_out/acs_ubench.log 2>&1
echo rc=$?
cat gpurun_out/acs_ubench.log
