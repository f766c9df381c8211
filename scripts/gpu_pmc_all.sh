# PMC passes for the metric's workloads and for the other formats (one call)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc.sh ${1:-pmcall}/main hard_b32,soft8_b16 && \
bash scripts/gpu_pmc.sh ${1:-pmcall}/other soft16_b32,fp32_f16,soft8_b16_llr
echo all_rc=$?
