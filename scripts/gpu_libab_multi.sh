# same-box A/B of several builds through bench.py's single-launch side measurement and timed region,
# alternating round by round: gpurun -- bash scripts/gpu_libab_multi.sh <tag> <rounds> <lib> [<lib> ...]
# (the tree's own library is measured as "head")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-libabm}
R=${2:-2}
shift 2
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel"
for r in $(seq 1 $R); do
  timeout -k 10 240 $B > $O/head_$r.log 2>&1 || { echo head_rc=$?; tail $O/head_$r.log; exit 1; }
  tail -1 $O/head_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('head', {k: v['kernel_ms'] for k, v in d['config']['single_launch'].items()}, d['config']['kernel_ms'])"
  for L in "$@"; do
    n=$(basename $(dirname $L))
    VITDEC_LIB=$L timeout -k 10 240 $B > $O/${n}_$r.log 2>&1 || { echo ${n}_rc=$?; tail $O/${n}_$r.log; exit 1; }
    tail -1 $O/${n}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', {k: v['kernel_ms'] for k, v in d['config']['single_launch'].items()}, d['config']['kernel_ms'])"
  done
done
echo all_rc=0
