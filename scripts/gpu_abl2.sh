# component ablations of the product kernel, single unsplit launches and batched launches (8 batches)
# usage: gpurun -- bash scripts/gpu_abl2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abl2}
mkdir -p $O
F="tg hard/b32,tg soft8/b16,tg fp32/f16 full,tg soft16/b32 full,tg soft16/b32 ACS only"
timeout -k 10 300 tools/vd_ablate 9 "$F" > $O/ablate.log 2>&1 && \
timeout -k 10 300 tools/vd_ablate 5 "$F" 8 > $O/ablate_batched.log 2>&1
echo rc=$?
cat $O/ablate.log $O/ablate_batched.log
