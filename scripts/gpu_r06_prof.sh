# round 6 profiles on the final tree: PMC passes (scripts/gpu_pmc.sh) and the kernel trace + stats of the
# default bench command (scripts/gpu_trace.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc.sh ${1:-prof}_pmc && bash scripts/gpu_trace.sh ${1:-prof}_trace
