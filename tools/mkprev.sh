# Regenerate tools/vd_tg_prev.h (namespace vd::old) from the committed kernel header, for vd_abtest.
# usage: bash tools/mkprev.sh [git-rev]   (default HEAD)
set -e
cd "$(dirname "$0")/.."
git show ${1:-HEAD}:gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h |
  sed -e 's|#include "vd_kernels.h"|#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernels.h"|' \
      -e 's|#include "vd_pack.h"|#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_pack.h"|' \
      -e 's|^namespace vd {|namespace vd { namespace old {|' \
      -e 's|^}  // namespace vd$|} }  // namespace vd::old|' > tools/vd_tg_prev.h
