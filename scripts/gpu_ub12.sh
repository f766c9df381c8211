set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ub12
timeout -k 10 120 tools/vd_ubench12 7 > gpurun_out/ub12/w7.log 2>&1 && timeout -k 10 120 tools/vd_ubench12 8 > gpurun_out/ub12/w8.log 2>&1 && timeout -k 10 120 tools/vd_ubench12 4 > gpurun_out/ub12/w4.log 2>&1
echo rc=$?
paste gpurun_out/ub12/w4.log gpurun_out/ub12/w7.log gpurun_out/ub12/w8.log | awk -F'\t' '{print $2 "   |w4 " $1 "   |w8 " $3}' | sed 's/  */ /g'
