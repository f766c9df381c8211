set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 tools/vd_ablate 10 > gpurun_out/ablate.log 2>&1 && \
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; \
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o run --output-format csv -- tools/vd_ablate 1 > gpurun_out/pmc1.log 2>&1
echo rc=$?
cat gpurun_out/ablate.log
