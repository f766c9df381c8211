# Round-2 first check: counter list, GPU tests (no slow), bench, WRITE_SIZE of the ablation variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo list_rc=$?
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo test_rc=$?; tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-600 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_abl_w -o run --output-format csv -- tools/vd_ablate 1 > $O/pmc_abl_w.log 2>&1
echo pmc_rc=$?
