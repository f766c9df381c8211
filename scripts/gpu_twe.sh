# early table writes (ABL TWE): exact twins on random input for every core, bench-condition A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-twe}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate 3 "twe" > $O/ablate.log 2>&1 && \
timeout -k 10 300 tools/vd_ablate 3 "twe" 4 > $O/ablate_batched.log 2>&1 && \
timeout -k 10 300 tools/vd_benchab 8 20 > $O/benchab.log 2>&1
echo rc=$?
cat $O/ablate.log $O/ablate_batched.log; tail -8 $O/benchab.log
