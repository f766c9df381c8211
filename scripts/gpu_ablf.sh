# filtered ablation run: gpurun -- bash scripts/gpu_ablf.sh <tag> <rounds> <filter>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ablf}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate ${2:-5} "$3" > $O/ablate.log 2>&1
echo rc=$?
cat $O/ablate.log
