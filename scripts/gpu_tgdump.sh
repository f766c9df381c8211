set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 tools/vd_tgdump tools/dbg_in1m.bin gpurun_out/dbg_a.bin 6400 0 && \
timeout -k 10 60 tools/vd_tgdump tools/dbg_in1m.bin gpurun_out/dbg_b.bin 6400 1 && \
timeout -k 10 60 tools/vd_tgdump tools/dbg_in1m.bin gpurun_out/dbg_c.bin 1 0
echo rc=$?
