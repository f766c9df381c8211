#!/bin/bash
# Scratch build of the product library with the round-2 bug re-introduced (test infrastructure only):
# the renormalisation asm in vd_kernel_tg.h without its "scc" clobber.  tests/test_gpu_guard.py runs it
# through the LDS guard check to show the check catches that bug.  Output: tools/build/scc_scratch/lib/,
# with BUILD_RECORD: the product's build-record line (vd_build_info format: hash of the product sources the
# scratch copy was made from, then their paths) -- the test refuses a scratch library whose record no longer
# matches the tree (vitdec.build_mismatch), so a stale build is never loaded.
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
B=$HERE/build/scc_scratch
rm -rf "$B/pkg" "$B/include" "$B/lib"
mkdir -p "$B/pkg" "$B/lib"
PKG="$ROOT/gpu-accelerated-viterbi-decoder_amd"
REC=$(make -s -C "$PKG" print-build-record)
cp -r "$ROOT/gpu-accelerated-viterbi-decoder_amd/csrc" "$B/pkg/csrc"
cp -r "$ROOT/include" "$B/include"
python3 - "$B/pkg/csrc/vd_kernel_tg.h" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
old = 'VD_TG_RN : [V] "+{v60}"(V), [w] "+v"(word), [sr] "=&s"(sr) : VD_TG_IN : "scc");'
assert s.count(old) == 2, "renormalisation asm statements not found"
open(p, "w").write(s.replace(old, 'VD_TG_RN : [V] "+{v60}"(V), [w] "+v"(word), [sr] "=&s"(sr) : VD_TG_IN);'))
PY
H=${HIPCC:-/opt/rocm/bin/hipcc}
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -w"
cd "$B/pkg"
$H $F -c csrc/vd_capi.hip -o "$B/vd_capi.o" & p1=$!
$H $F -c csrc/vd_host.cpp -o "$B/vd_host.o" & p2=$!
$H $F -c csrc/vd_mtjump.cpp -o "$B/vd_mtjump.o" & p3=$!
wait $p1 && wait $p2 && wait $p3
$H --offload-arch=gfx950 -shared -o "$B/lib/libvitdec.so" "$B/vd_capi.o" "$B/vd_host.o" "$B/vd_mtjump.o"
echo "$REC" > "$B/lib/BUILD_RECORD"
echo "built $B/lib/libvitdec.so ($REC)"
