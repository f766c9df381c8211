# parity tests, bench line, ablation + clock stamps (one GPU call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/full_t.log 2>&1
echo test_rc=$?
tail -3 gpurun_out/full_t.log
timeout -k 10 300 python bench.py > gpurun_out/full_bench.log 2>&1
echo bench_rc=$?
tail -2 gpurun_out/full_bench.log
timeout -k 10 120 tools/vd_ablate 5 > gpurun_out/full_ablate.log 2>&1
echo abl_rc=$?
cat gpurun_out/full_ablate.log
