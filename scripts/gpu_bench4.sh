set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bench4}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-channel > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['kernel_ms'], c['two_streams'], c['llr_input']['fused_gbps'], {k: v['gbps'] for k, v in c['other_configs'].items()})"
