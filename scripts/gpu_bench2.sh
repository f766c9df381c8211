set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-bench}
mkdir -p $O
timeout -k 10 300 python bench.py ${2:-} > $O/bench.log 2>&1
echo rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['config']['step_minus_kernels_us'], d['roofline']['frac'])"
