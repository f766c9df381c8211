# launch-tail study: any-order launches, two streams, split last batch (tools/vd_anyorder)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-anyorder}
mkdir -p $O
timeout -k 10 200 tools/vd_anyorder 12 20 > $O/anyorder_k20.log 2>&1 || { echo rc=$?; cat $O/anyorder_k20.log; exit 1; }
cat $O/anyorder_k20.log
timeout -k 10 200 tools/vd_anyorder 6 100 > $O/anyorder_k100.log 2>&1 || { echo rc=$?; cat $O/anyorder_k100.log; exit 1; }
cat $O/anyorder_k100.log
