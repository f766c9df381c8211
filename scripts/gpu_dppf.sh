# DPP stage form per core: bench-condition A/B (12 groups) and the GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dppf}
mkdir -p $O
timeout -k 10 400 tools/vd_benchab 12 20 > $O/benchab.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo rc=$?
tail -7 $O/benchab.log; tail -2 $O/tests.log
