# split warm-up 6 vs 3 blocks (tools/build/ab_warm3): single launches on the bench data, random / zeros input
# usage: gpurun --timeout 1100 -- bash scripts/gpu_warm3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-warm3}
mkdir -p $O
bash scripts/gpu_libab_multi.sh $1/ab 2 tools/build/ab_warm3/libvitdec.so > $O/ab.log 2>&1 || { echo ab_rc=$?; tail $O/ab.log; exit 1; }
grep "^head\|^ab_" $O/ab.log
timeout -k 10 200 python tools/study/s8split_random.py > $O/random_head.log 2>&1 || { echo rnd_rc=$?; exit 1; }
VITDEC_LIB=tools/build/ab_warm3/libvitdec.so timeout -k 10 200 python tools/study/s8split_random.py > $O/random_warm3.log 2>&1 || { echo rnd3_rc=$?; exit 1; }
grep -h "VD_PK_SPLIT=1\|equal" $O/random_head.log $O/random_warm3.log
echo all_rc=0
