set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ub12b}
mkdir -p $O
timeout -k 10 120 tools/vd_ubench12 3 > $O/w3.log 2>&1 && timeout -k 10 120 tools/vd_ubench12 4 > $O/w4.log 2>&1 && timeout -k 10 120 tools/vd_ubench12 7 > $O/w7.log 2>&1
echo rc=$?
paste $O/w3.log $O/w4.log $O/w7.log | awk -F'\t' '{print $1 " |w4 " $2 " |w7 " $3}' | sed 's/  */ /g' | tail -22
