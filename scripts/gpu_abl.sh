set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/vd_ablate ${1:-8} > gpurun_out/ablate.log 2>&1
echo abl_rc=$?
cat gpurun_out/ablate.log
