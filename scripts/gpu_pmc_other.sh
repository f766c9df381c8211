set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc4}
mkdir -p $O
bash scripts/gpu_pmc.sh ${1:-pmc4}/other soft16_b32,fp32_f16,soft8_b16_llr > $O/pmc_other.log 2>&1 || { echo pmc_other_rc=$?; tail $O/pmc_other.log; exit 1; }
tail -3 $O/pmc_other.log
echo all_rc=0
