# bench-condition A/B of kernel variants: gpurun -- bash scripts/gpu_benchab.sh <tag> [groups] [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-benchab}
mkdir -p $O
timeout -k 10 300 tools/vd_benchab ${2:-8} ${3:-10} > $O/benchab.log 2>&1
echo rc=$?
cat $O/benchab.log
