#!/bin/bash
# Scratch build of the product library with the round-2 bug re-introduced (test infrastructure only):
# the renormalisation asm in vd_kernel_tg.h without its "scc" clobber.  tests/test_gpu_guard.py runs it
# through the LDS guard check to show the check catches that bug.  Output: tools/build/scc_scratch/lib/,
# with BUILD_RECORD: the product's build-record line (vd_build_info format: hash of the product sources the
# scratch copy was made from, then their paths) -- the test refuses a scratch library whose record no longer
# matches the tree (vitdec.build_mismatch), so a stale build is never loaded; SCC_EVIDENCE: the count of SCC
# readers after a renormalisation in the scratch ISA.
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
# ISA evidence: SCC readers after a renormalisation in the scratch copy's compiled tg kernels
# (tests/test_asm_lint.py's scan).  Whether the bug shows at run time depends on the compiler keeping SCC
# live across the un-clobbered asm; the guard test asserts violations only when this count is non-zero.
python3 - "$ROOT" "$B/pkg/csrc" "$B/SCC_EVIDENCE" <<'PY' & p4=$!
import os, sys, tempfile
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import test_asm_lint as t
with tempfile.TemporaryDirectory() as d:
    r = t.scc_reads_after_renorm(t._compile(sys.argv[2], d))
open(sys.argv[3], "w").write(f"{sum(r.values())}\n")
PY
wait $p1 && wait $p2 && wait $p3 && wait $p4
$H --offload-arch=gfx950 -shared -o "$B/lib/libvitdec.so" "$B/vd_capi.o" "$B/vd_host.o" "$B/vd_mtjump.o"
mv "$B/SCC_EVIDENCE" "$B/lib/SCC_EVIDENCE"
echo "$REC" > "$B/lib/BUILD_RECORD"
echo "built $B/lib/libvitdec.so ($REC)"
