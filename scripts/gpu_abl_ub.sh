# ablation run + ubench12 at 4 and 7 waves: gpurun -- bash scripts/gpu_abl_ub.sh <tag> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ablub}
mkdir -p $O
timeout -k 10 120 tools/vd_ubench12 4 > $O/ub_w4.log 2>&1 && timeout -k 10 120 tools/vd_ubench12 7 > $O/ub_w7.log 2>&1 && \
timeout -k 10 300 tools/vd_ablate ${2:-5} > $O/ablate.log 2>&1
echo rc=$?
paste $O/ub_w4.log $O/ub_w7.log | awk -F'\t' '{print $1 " | " $2}' | sed 's/  */ /g' | tail -20
grep -v "^===\|kernel span\|wave \|clock\|cycles/stage\|progress\|SIMDs" $O/ablate.log
