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
//  sevenths: 7 workgroups per CU, 4 of 4 whole chunks and 3 of 3 chunks in 4 segments of 3/4 chunk: 7 waves
//          per SIMD for the whole launch (4 of 1 chunk, 3 of 3/4 chunk, their progress kept even by the fairness
//          controller in fractions of each wave's work), speculative starts only in the 3-chunk workgroups
//          (3 x 3/7 of them: a third of thirds' warm-up work).  Workgroup g goes to XCD g % 8 as its
//          n = g / 8-th; the 4-chunk ones are those with (n % 7) % 2 == 0: a CU receives n = c + 32 k
//          (k = 0..6) when its XCD deals round robin, whose n % 7 = (c + 4 k) % 7 take every residue once,
//          or 7 consecutive n when dealt 7 at a time: 4 four-chunk and 3 three-chunk workgroups per CU either
//          way (tests/cxx/segplan_check.cpp).
enum SegMode : int { kSegPieces = 0, kSegThirds = 1, kSegSevenths = 2 };
inline std::vector<uint32_t> seg_table(int nsimd, int mode)
{
    std::vector<uint32_t> t{0u};
    const uint32_t nch = kChunks;
    if (mode == kSegSevenths) {
        const uint32_t nwg = 7u * (uint32_t)nsimd / 4u;  // 7 workgroups of 4 waves per CU
        if (nsimd % 32 != 0) return {};
        for (uint32_t g = 0; g < nwg; g++) {
            const uint32_t n = g / 8;
            t.push_back(t.back() + ((n % 7) % 2 == 0 ? 4u : 3u));
        }
        return t.back() == nch ? t : std::vector<uint32_t>{};
    }
    const bool thirds = mode == kSegThirds;
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
