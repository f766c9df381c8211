# round-end measurement, part b: PMC passes of the bench's kernels and of the other formats, rocprofv3 kernel
# trace + stats of the default bench command
# usage: gpurun --timeout 1150 -- bash scripts/gpu_final_b.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
bash scripts/gpu_pmc.sh $1/main hard_b32,soft8_b16 > $O/pmc_main.log 2>&1 || { echo pmc_main_rc=$?; tail $O/pmc_main.log; exit 1; }
tail -3 $O/pmc_main.log
bash scripts/gpu_pmc.sh $1/other soft16_b32,fp32_f16,soft8_b16_llr > $O/pmc_other.log 2>&1 || { echo pmc_other_rc=$?; tail $O/pmc_other.log; exit 1; }
bash scripts/gpu_trace.sh $1/trace > $O/trace.log 2>&1 || { echo trace_rc=$?; tail $O/trace.log; exit 1; }
tail -12 $O/trace.log
echo all_rc=0
