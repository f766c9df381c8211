set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-capiab}
mkdir -p $O
timeout -k 10 300 tools/vd_capiab 6 10 > $O/capiab.log 2>&1
echo rc=$?
cat $O/capiab.log
