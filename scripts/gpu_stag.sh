set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-stag}
mkdir -p $O
timeout -k 10 300 tools/vd_benchab 8 10 > $O/benchab.log 2>&1 && \
timeout -k 10 300 tools/vd_ablate 9 "tg soft8/b16 full,tg hard/b32 full,staggered" > $O/ablate.log 2>&1
echo rc=$?
cat $O/benchab.log $O/ablate.log
