# exchange-variant ablation, split stamps, interleaved tg/ps bench: gpurun -- bash scripts/gpu_r02c.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02c}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate 5 "tg soft8/b16 full,q5,q4,tg soft8/b16 ACS only" > $O/ablate.log 2>&1 && \
timeout -k 10 120 tools/vd_splitab 10 0.04 > $O/splitab_bsc04.log 2>&1 && \
for i in 1 2 3 4; do
  k=tg; [ $((i % 2)) = 0 ] && k=ps
  VD_KERNEL=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-llr --no-pcie --no-channel --no-other > $O/bench_$k$i.json 2> $O/bench_$k$i.err || exit 1
  python -c "import json,sys; r=json.load(open('$O/bench_$k$i.json')); print('$k', r['value'], r['config']['kernel_ms'])"
done
echo rc=$?
cat $O/ablate.log; cat $O/splitab_bsc04.log
