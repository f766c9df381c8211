set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-probe}
mkdir -p $O
timeout -k 10 300 python tools/bench_probe.py 2.0 > $O/probe.log 2>&1 && timeout -k 10 300 tools/vd_capiab 4 10 > $O/capiab.log 2>&1
echo rc=$?
cat $O/probe.log $O/capiab.log
