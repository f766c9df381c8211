# round-2 profile set: PMC passes + kernel trace (gpu_pmc2.sh), ablation, then the default bench line
# reading the fresh PMC summary and ablation log.  gpurun -- bash scripts/gpu_final2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final2}
mkdir -p $O
bash scripts/gpu_pmc2.sh $1 > $O/pmc_script.log 2>&1 || { echo pmc failed; cat $O/pmc_script.log; exit 1; }
timeout -k 10 400 tools/vd_ablate 9 "tg hard/b32 full,tg soft8/b16 full,tg fp32/f16 full,ACS only,-readout,-tabreads,-tabbuild,-traceback,-loads,-fairness,q5,all-dpp" > $O/ablate.log 2>&1 || exit 1
mkdir -p profiles/r02 && cp $O/pmc_summary.json $O/ablate.log profiles/r02/ && \
timeout -k 10 400 python bench.py > $O/bench.log 2> $O/bench.err
echo rc=$?
tail -4 $O/pmc_script.log
tail -1 $O/bench.log
