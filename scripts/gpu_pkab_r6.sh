# round 6 kernel-variant A/B (tools/vd_pkab_r6: variants alternate round by round, exact ones compared)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pkab}
mkdir -p $O
timeout -k 10 300 tools/vd_pkab_r6 8 20 > $O/pkab_k20.log 2>&1 || { echo rc=$?; cat $O/pkab_k20.log; exit 1; }
cat $O/pkab_k20.log
timeout -k 10 300 tools/vd_pkab_r6 4 100 > $O/pkab_k100.log 2>&1 || { echo rc=$?; cat $O/pkab_k100.log; exit 1; }
cat $O/pkab_k100.log
