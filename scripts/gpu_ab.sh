set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/vd_abtest ${1:-15} > gpurun_out/ab.log 2>&1
echo ab_rc=$?
cat gpurun_out/ab.log
