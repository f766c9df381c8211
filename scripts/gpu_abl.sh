# ablation / exact-twin timing run: gpurun -- bash scripts/gpu_abl.sh <tag> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abl}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate ${2:-5} > $O/ablate.log 2>&1
echo rc=$?
grep -v "^===\|kernel span\|wave \|clock\|cycles/stage\|progress\|SIMDs" $O/ablate.log
