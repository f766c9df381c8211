# PMC passes over the ablation driver (one counter group per rocprofv3 run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_abl}
mkdir -p $O
run() { timeout -s KILL 120 rocprofv3 --pmc $1 -d $O/$2 -o run --output-format csv -- tools/vd_ablate 1 > $O/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" sqa && \
run "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" sqb && \
run "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_IFETCH" sqc
echo rc=$?
