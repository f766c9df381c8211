// vd_segplan.h -- host-side segment tables of segment launches (vd_kernel_tg.h "segment launches"):
// the first chunk of every workgroup, then the chunk count.  Shared by the C-ABI (vd_capi.hip) and the
// timing tools.
#pragma once
#include <cstdint>
#include <vector>
#include "vd_kernels.h"

namespace vd {

// Segment tables for kChunks chunks on nsimd SIMDs (8 waves per SIMD at most):
//  pieces: 6 whole chunks per SIMD (workgroups of 4) and the remaining nsimd/4 chunks in 4 pieces each
//          (one workgroup per chunk): 7 waves per SIMD, one of them a quarter chunk (round 2's split);
//  thirds: 8 workgroups per CU, each 3 chunks in 4 segments of 3/4 chunk, except one workgroup per CU of 4
//          chunks (segments of 1 chunk): 8 waves per SIMD for the whole launch.  Workgroups go to the 8
//          XCDs round robin (workgroup g to XCD g % 8, its n = g / 8-th there); the 4-chunk ones are those
//          with n / 32 == (n % 32) % 8: four in every aligned 32 consecutive n (one per aligned 8) and one
//          per residue class of n mod 32, so one per CU whether the XCD deals its 256 workgroups to its 32
//          CUs round robin (CU = n % 32) or 8 at a time (CU = n / 8); tests/cxx/segplan_check.cpp checks both.
inline std::vector<uint32_t> seg_table(int nsimd, bool thirds)
{
    std::vector<uint32_t> t{0u};
    const uint32_t nch = kChunks;
    if (!thirds) {
        const uint32_t rem = nch % (uint32_t)nsimd, nwhole = nch - rem;
        if (rem == 0 || rem * kWaves != (uint32_t)nsimd || nch / (uint32_t)nsimd + 1 > 8) return {};
        for (uint32_t c = kWaves; c <= nwhole; c += kWaves) t.push_back(c);
        for (uint32_t c = nwhole + 1; c <= nch; c++) t.push_back(c);
        return t;
    }
    const uint32_t nwg = 2u * (uint32_t)nsimd;  // 8 workgroups of 4 waves per CU
    if (nch < 3 * nwg || nch - 3 * nwg != nwg / 8 || nwg % 256 != 0) return {};
    for (uint32_t g = 0; g < nwg; g++) {
        const uint32_t n = g / 8;  // the workgroup's index within its XCD's sequence
        const bool four = n / 32 == (n % 32) % 8;
        t.push_back(t.back() + (four ? 4u : 3u));
    }
    return t.back() == nch ? t : std::vector<uint32_t>{};
}

}  // namespace vd
