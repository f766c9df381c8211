# SOFT16 (vd_decode_tg<SOFT16,B32>): component ablations in 20-batch launches, and the same-box A/B of this
# tree's library against the previous commit's (tools/build/oldlib) through bench.py's timed region
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-soft16}
mkdir -p $O
timeout -k 10 300 tools/vd_ablate 5 soft16 20 > $O/ablate_soft16.log 2>&1 || { echo ablate_rc=$?; tail $O/ablate_soft16.log; exit 1; }
cat $O/ablate_soft16.log
OLD=tools/build/oldlib/gpu-accelerated-viterbi-decoder_amd/lib/libvitdec.so
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-llr --no-pcie --no-channel --no-other --workloads soft16_b32,fp32_f16"
for r in 1 2 3; do
  timeout -k 10 240 $B > $O/new_$r.log 2>&1 || { echo new_rc=$?; tail $O/new_$r.log; exit 1; }
  VITDEC_LIB=$OLD timeout -k 10 240 $B > $O/old_$r.log 2>&1 || { echo old_rc=$?; tail $O/old_$r.log; exit 1; }
  for w in new old; do tail -1 $O/${w}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['config']['kernel_ms'], d['config']['kernel_gbps'])"; done
done
echo all_rc=0
