# round-4 PMC passes (all kernels the bench reports) + component ablations of the batched kernels:
# gpurun --timeout 1100 -- bash scripts/gpu_pmc_r04.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc4}
mkdir -p $O
bash scripts/gpu_pmc.sh ${1:-pmc4}/main hard_b32,soft8_b16 > $O/pmc_main.log 2>&1 || { echo pmc_main_rc=$?; tail $O/pmc_main.log; exit 1; }
bash scripts/gpu_pmc.sh ${1:-pmc4}/other soft16_b32,fp32_f16,soft8_b16_llr > $O/pmc_other.log 2>&1 || { echo pmc_other_rc=$?; tail $O/pmc_other.log; exit 1; }
timeout -k 10 400 tools/vd_ablate 5 "tg " 8 > $O/ablate_batched.log 2>&1 || { echo ablate_rc=$?; tail $O/ablate_batched.log; exit 1; }
tail -3 $O/pmc_main.log; tail -3 $O/pmc_other.log; grep -i "ACS only\|full" $O/ablate_batched.log | head
echo all_rc=0
