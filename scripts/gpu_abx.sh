# A/B of kernel variants (tools/vd_abx: batched and segment launches) + the GPU parity tests of the soft/hard
# kernels: gpurun --timeout 900 -- bash scripts/gpu_abx.sh <tag> [rounds] [batches] [pytest -k expression]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abx}
mkdir -p $O
timeout -k 10 420 tools/vd_abx ${2:-6} ${3:-20} > $O/abx.log 2>&1 || { echo abx_rc=$?; tail $O/abx.log; exit 1; }
cat $O/abx.log
if [ -n "$4" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$4" > $O/tests_gpu.log 2>&1 || { echo tests_rc=$?; tail -30 $O/tests_gpu.log; exit 1; }
  tail -2 $O/tests_gpu.log
fi
echo all_rc=0
