set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/f2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pk.py -x -v -m gpu -k two_chain --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_envab_single.sh f2ab VD_F2 3
