# instruction-cost microbenchmark (tools/vd_ubench12) at 7 and 8 waves per SIMD: gpurun -- bash scripts/gpu_ubench.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ubench}
mkdir -p $O
timeout -k 10 200 tools/vd_ubench12 7 > $O/ubench7.log 2>&1 && timeout -k 10 200 tools/vd_ubench12 8 > $O/ubench8.log 2>&1
echo rc=$?
paste $O/ubench7.log $O/ubench8.log | cut -c1-110
