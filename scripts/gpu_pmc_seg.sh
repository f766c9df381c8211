# PMC passes over tools/vd_abx1 (product kernels only): batched launches (grid 1600 x K) and single-batch
# segment launches (grid 1792) of HARD/b32 and SOFT8/b16, to compare how the two launch kinds spend cycles.
# gpurun -- bash scripts/gpu_pmc_seg.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcseg}
mkdir -p $O
run() { timeout -s KILL 120 rocprofv3 --pmc $1 -d $O/pmc/$2 -o run --output-format csv -- tools/vd_abx1 1 4 > $O/pmc_$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" a && \
run "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE" b && \
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- tools/vd_abx1 1 4 > $O/trace.log 2>&1
echo rc=$?
mkdir -p $O/raw
for d in $O/pmc/* $O/trace; do f=$(find $d -name "*.csv" | head -5); for x in $f; do cp $x $O/raw/$(basename $d)_$(basename $x); done; done
ls $O/raw
