# bench kernel time per batch against the number of resident batches K (distinct inputs)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ksweep}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other"
for k in 10 20 50 100 200; do
  timeout -k 10 200 $B --steps $k > $O/k$k.json 2> $O/k$k.err || exit 1
  python3 -c "import json; d=json.load(open('$O/k$k.json')); print($k, d['value'], d['config']['kernel_ms'], d['config']['ber'])"
done
