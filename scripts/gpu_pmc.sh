# PMC passes + kernel-trace summary over the bench (one counter group per rocprofv3 run, each bounded).
# usage: gpurun -- bash scripts/gpu_pmc.sh <tag> [workloads]   (workloads: bench.py --workloads, default the metric's)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
W=${2:-hard_b32,soft8_b16}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --warm-s 0.3 --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel --no-other --workloads $W"
run() { timeout -s KILL 120 rocprofv3 $3 --pmc $1 -d $O/pmc/$2 -o run --output-format csv -- $B > $O/pmc_$2.log 2>&1; }
run "FETCH_SIZE" fetch && \
run "WRITE_SIZE" write && \
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" sqa --kernel-trace && \
run "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" sqb && \
run "SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_IOPS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU" sqc && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel --no-other --workloads $W > $O/trace.log 2>&1
echo rc=$?
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
mkdir -p $O/pmc_raw
for d in $O/pmc/*; do f=$(find $d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp $f $O/pmc_raw/$(basename $d)_counter_collection.csv; done
python3 tools/pmc_summary.py $O/pmc $O/pmc_summary.json --batches 3
head -6 $O/kernel_stats.csv
# LDS-array activity (last: a counter the box does not know ends only this pass)
run "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS" sqd && \
f=$(find $O/pmc/sqd -name "*counter_collection.csv" | head -1) && cp $f $O/pmc_raw/sqd_counter_collection.csv && \
python3 tools/pmc_summary.py $O/pmc $O/pmc_summary.json --batches 3 > /dev/null
echo sqd_rc=$?
