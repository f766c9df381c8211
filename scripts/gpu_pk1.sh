# A/B (study): single-batch HARD launches on vd_decode_pk (VD_PK_SINGLE=1) vs the segment launches of
# vd_decode_tg; bench.py's config.single_launch of both workloads, variants alternating, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pk1}
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    VD_PK_SINGLE=$v timeout -k 10 300 python -u bench.py --no-parity > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo rc=$? v=$v; tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('pk_single=$v', json.dumps(d['config']['single_launch']))" $O/b_${v}_$r.json
  done
done
echo all_rc=0
