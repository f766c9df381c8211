set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chains
timeout -k 10 300 tools/vd_chains 15 > gpurun_out/chains/chains.log 2>&1; echo rc=$?; cat gpurun_out/chains/chains.log
