# round 6 study: the SOFT8 ring skew (slot s keeps position p' at dword p' ^ s). GPU suite on the changed tree,
# same-box A/B against the previous kernels (tools/vd_pkab_old / _new, "full" only, alternating), and the
# LDS counter pass over the bench's SOFT8 batches.  usage: gpurun --timeout 1150 -- bash scripts/gpu_skew.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-skew}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $O/tests_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests_gpu.log | tail -60; exit 1; }
for r in 1 2 3 4; do
  for v in old new; do
    timeout -k 10 200 tools/vd_pkab_$v 4 20 > $O/ab_${v}_$r.log 2>&1 || { echo ${v}_rc=$?; tail $O/ab_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $O/ab_${v}_$r.log)"
  done
done
B="python3 bench.py --steps 3 --warmup 1 --warm-s 0.3 --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel --no-other --workloads hard_b32,soft8_b16"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/pmc/sqd -o run --output-format csv -- $B > $O/pmc_sqd.log 2>&1 || { echo pmc_rc=$?; tail $O/pmc_sqd.log; exit 1; }
f=$(find $O/pmc/sqd -name "*counter_collection.csv" | head -1) && cp $f $O/sqd_counter_collection.csv
echo all_rc=0
