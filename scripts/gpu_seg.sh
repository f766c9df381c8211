# single-launch modes (plain / pieces / thirds, 6 or 3 warm-up blocks): gpurun -- bash scripts/gpu_seg.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-seg}
mkdir -p $O
timeout -k 10 300 tools/vd_splitab 10 0.04 > $O/splitab_bsc04.log 2>&1 || { echo rc=$?; cat $O/splitab_bsc04.log; exit 1; }
cat $O/splitab_bsc04.log
timeout -k 10 300 tools/vd_splitab 4 0.08 > $O/splitab_bsc08.log 2>&1 || { echo rc=$?; cat $O/splitab_bsc08.log; exit 1; }
grep -E "exact|median|re-decoded" $O/splitab_bsc08.log
echo all_rc=0
