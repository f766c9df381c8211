set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() { timeout -k 10 240 rocprofv3 --pmc $1 -d gpurun_out/pmc_$2 -o run --output-format csv -- $B > gpurun_out/pmc_$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" a && \
run "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_IFETCH SQ_ACTIVE_INST_SCA" b && \
run "GRBM_GUI_ACTIVE SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS" c && \
run "FETCH_SIZE" d && run "WRITE_SIZE" e
echo rc=$?
