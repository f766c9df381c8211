# GPU tests + vd_benchab A/B: gpurun -- bash scripts/gpu_ab.sh <tag> [groups] [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo tests_rc=$?; tail -30 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
timeout -k 10 400 tools/vd_benchab ${2:-8} ${3:-20} > $O/benchab.log 2>&1 || { echo benchab_rc=$?; tail $O/benchab.log; exit 1; }
cat $O/benchab.log
echo all_rc=0
