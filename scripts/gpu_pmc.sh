# PMC passes over the bench (one counter group per rocprofv3 run, each under its own time limit).
# usage: gpurun -- bash scripts/gpu_pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
O=gpurun_out/$TAG
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-llr --no-pcie --no-channel"
run() { timeout -s KILL 120 rocprofv3 --pmc $1 -d $O/$2 -o run --output-format csv -- $B > $O/$2.log 2>&1; }
run "FETCH_SIZE" fetch && \
run "WRITE_SIZE" write && \
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" sqa && \
run "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" sqb && \
run "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_IFETCH" sqc
echo rc=$?
find $O -name "*counter_collection.csv" | head
