set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/vd_ablate 5 > gpurun_out/ablate4.log 2>&1
echo abl_rc=$?
cat gpurun_out/ablate4.log
true
echo rc=$?
true
