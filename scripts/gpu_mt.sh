# GPU call: channel-source parity tests, then the timing probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mt.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/mt_tests.log 2>&1
rc=$?
tail -15 gpurun_out/mt_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/mt_probe.py > gpurun_out/mt_probe.log 2>&1
echo probe_rc=$?
cat gpurun_out/mt_probe.log
mkdir -p gpurun_out/mtprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mtprof -o run --output-format csv -- python3 tools/mt_probe.py > gpurun_out/mtprof/log 2>&1
echo prof_rc=$?
find gpurun_out/mtprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/mtprof/kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/mtprof/kernel_stats.csv | head -12
