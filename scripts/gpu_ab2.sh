# same-box A/B of two builds of the packed kernels (tools/vd_pkab_old vs tools/vd_pkab_new, one variant
# each), alternating processes: gpurun -- bash scripts/gpu_ab2.sh <tag> [pairs] [K]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab2}
mkdir -p $O
for r in $(seq 1 ${2:-4}); do
  for v in old new; do
    timeout -k 10 200 tools/vd_pkab_$v 4 ${3:-20} > $O/${v}_$r.log 2>&1 || { echo ${v}_rc=$?; tail $O/${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $O/${v}_$r.log)"
  done
done
echo all_rc=0
