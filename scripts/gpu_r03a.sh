# occupancy / launch-size study, SOFT16 label-region parity, ablations:
# gpurun -- bash scripts/gpu_r03a.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r03a}
mkdir -p $O
timeout -k 10 300 tools/vd_occab 8 32 > $O/occab.log 2>&1 || { echo occab_rc=$?; cat $O/occab.log; exit 1; }
cat $O/occab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo tests_rc=$?; tail -30 $O/tests_gpu.log; exit 1; }
tail -3 $O/tests_gpu.log
timeout -k 10 300 tools/vd_ablate 5 "tg " 8 > $O/ablate.log 2>&1 || { echo ablate_rc=$?; tail $O/ablate.log; exit 1; }
cat $O/ablate.log
echo all_rc=0
