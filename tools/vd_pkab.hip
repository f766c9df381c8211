// vd_pkab.hip -- timing-only A/B of vd_decode_pk variants in batched launches (not part of the product): the
// bench's timed region (K distinct resident 32M-bit batches per launch) for HARD/b32 (K=7 codeword through a
// BSC, p = 0.04 unless given), SOFT8/b16 (BPSK codeword + Gaussian noise at Eb/N0 2 dB, quantised like
// SoftDecisionPacker(SOFT8)) and FP32/f16 (the same noisy values as floats, BASELINE configs[4]).  Variants alternate round by round with a rotating order; every exact variant's
// words are compared with variant 0's (last batch).  Component ablations (ABL bits, vd_kernel_tg.h) give
// wrong words by design and are labelled so.
// Usage: vd_pkab [rounds] [batches per launch] [HARD flip probability, default 0.04]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "build/abl/vd_kernel_pk.h"  // the product kernel + tools-only ablation bits (tools/abl/gen_abl.py)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
// NW 0: the product's layout for the format (7 waves per SIMD for SOFT8 and FP32, 8 otherwise)
template <int CH, int CORE, int ABL, int NW = 0>
constexpr KFn pk() { return (KFn)vd::vd_decode_pk<CH, CORE, 32, false, NW ? NW : ((vd::PkFmt<CH>::P2 || (CH & 7) == vd::FP32) ? 7 : 8), ABL>; }
struct Variant { const char* name; KFn hard, soft8, fp32; bool exact; };
#define VD_PKAB_ALL(NAME, ABL, NW, EXACT) \
    {NAME, pk<vd::HARD, vd::B32, ABL, NW>(), pk<vd::SOFT8, vd::B16, ABL, NW>(), pk<vd::FP32, vd::F16, ABL, NW>(), EXACT}
#ifndef VD_PKAB_VARIANTS
#define VD_PKAB_VARIANTS                                                                          \
    VD_PKAB_ALL("full", 0, 0, true), VD_PKAB_ALL("ACS only (ablation)", vd::kAblAcsOnly, 0, false), \
    VD_PKAB_ALL("-traceback (ablation)", vd::kAblNoTraceback, 0, false),                          \
    VD_PKAB_ALL("-read-out (ablation)", vd::kAblNoReadout, 0, false),                             \
    VD_PKAB_ALL("-table build (ablation)", vd::kAblNoTabBuild, 0, false),                         \
    VD_PKAB_ALL("-table reads (ablation)", vd::kAblNoTabReads, 0, false),                         \
    VD_PKAB_ALL("-input loads (ablation)", vd::kAblNoLoads, 0, false),                            \
    VD_PKAB_ALL("LDS exchanges as DPP (ablation)", vd::kAblNoLdsX, 0, false),                     \
    VD_PKAB_ALL("ACS only, LDS exchanges as DPP", vd::kAblAcsOnly | vd::kAblNoLdsX, 0, false),    \
    VD_PKAB_ALL("8 waves/SIMD, 5 words per traceback", 0, 8, true),                                \
    VD_PKAB_ALL("7 waves/SIMD, 6 words per traceback", 0, 7, true),                                \
    VD_PKAB_ALL("6 waves/SIMD, 8 words per traceback", 0, 6, true),
#endif

static double median(std::vector<float> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 6, K = argc > 2 ? atoi(argv[2]) : 20;
    const double pbsc = argc > 3 ? atof(argv[3]) : 0.04;  // HARD: flip probability of the binary symmetric channel
    const size_t N = 32000000;  // coded stages per batch (the bench's 32M-bit input)
    std::mt19937 rng(7);
    std::vector<uint8_t> o0(N), o1(N);
    uint32_t reg = 0;
    for (size_t t = 0; t < N; t++) {
        reg = ((reg >> 1) | ((rng() & 1u) << 6)) & 127u;
        o0[t] = __builtin_popcount(reg & 0171u) & 1u;
        o1[t] = __builtin_popcount(reg & 0133u) & 1u;
    }
    std::vector<uint32_t> hh(N / 16 + 64, 0u);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (size_t t = 0; t < N; t++) {
        uint32_t a = o0[t] ^ (U(rng) < pbsc), b = o1[t] ^ (U(rng) < pbsc);
        hh[t / 16] |= (a << (31 - 2 * (t % 16))) | (b << (30 - 2 * (t % 16)));
    }
    const double sigma = std::sqrt(1.0 / (2.0 * 0.5 * std::pow(10.0, 0.2)));
    std::normal_distribution<double> G(0.0, sigma);
    auto q8 = [&](double x) { long v = std::lround(x * 40.0); v = std::min(127L, std::max(-128L, v)); return (uint32_t)(uint8_t)(int8_t)v; };
    std::vector<uint32_t> hs(N / 2 + 64, 0u);
    std::vector<float> hf(2 * N + 64, 0.0f);
    for (size_t t = 0; t < N; t++) {
        const double x0 = (o0[t] ? -1.0 : 1.0) + G(rng), x1 = (o1[t] ? -1.0 : 1.0) + G(rng);
        const uint32_t s0 = q8(x0), s1 = q8(x1);
        hs[t / 2] |= ((s0 << 8) | s1) << (16 * ((t % 2) ^ 1));
        hf[2 * t] = (float)x0;
        hf[2 * t + 1] = (float)x1;
    }
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t strF = (hf.size() * 4 + 255) / 256 * 256;
    const size_t ostr = (g.packNum * 4 + 255) / 256 * 256;
    char *bH, *bS, *bF, *bO;
    CK(hipMalloc(&bH, strH * K));
    CK(hipMalloc(&bS, strS * K));
    CK(hipMalloc(&bF, strF * K));
    CK(hipMalloc(&bO, ostr * K));
    for (int k = 0; k < K; k++) {
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bF + k * strF, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
    }
    vd::Geom gb = g;
    gb.nbatch = (uint32_t)K;
    gb.outStride = ostr;
    const unsigned grid = 800u * (unsigned)K;  // two chunks per wave, 4 waves per workgroup
    printf("TBS: 8 waves %d, 7 waves %d, 6 waves %d\n", vd::PkLds<8>::TBS, vd::PkLds<7>::TBS, vd::PkLds<6>::TBS);
    const Variant vs[] = {VD_PKAB_VARIANTS};
    const int nv = sizeof(vs) / sizeof(vs[0]);
    hipEvent_t ev[4];
    for (auto& evi : ev) CK(hipEventCreate(&evi));
    std::vector<std::vector<float>> th(nv), ts(nv), tf(nv);
    for (int r = 0; r < rounds + 1; r++)
        for (int vi = 0; vi < nv; vi++) {
            const int v = (vi + r) % nv;
            vd::Geom gh = gb, gS = gb, gF = gb;
            gh.inStride = strH;
            gS.inStride = strS;
            gF.inStride = strF;
            CK(hipEventRecord(ev[0]));
            hipLaunchKernelGGL(vs[v].hard, dim3(grid), dim3(256), 0, 0, bH, bO, gh);
            CK(hipEventRecord(ev[1]));
            hipLaunchKernelGGL(vs[v].soft8, dim3(grid), dim3(256), 0, 0, bS, bO, gS);
            CK(hipEventRecord(ev[2]));
            hipLaunchKernelGGL(vs[v].fp32, dim3(grid), dim3(256), 0, 0, bF, bO, gF);
            CK(hipEventRecord(ev[3]));
            CK(hipEventSynchronize(ev[3]));
            float a, b, c;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            CK(hipEventElapsedTime(&c, ev[2], ev[3]));
            if (r) { th[v].push_back(a / K); ts[v].push_back(b / K); tf[v].push_back(c / K); }
        }
    std::vector<uint32_t> ref(g.packNum), got(g.packNum);
    for (int w = 0; w < 3; w++)
        for (int v = 0; v < nv; v++) {
            if (v && !vs[v].exact) continue;
            vd::Geom gg = gb;
            gg.inStride = w == 2 ? strF : w ? strS : strH;
            CK(hipMemset(bO, 0, ostr * K));
            hipLaunchKernelGGL(w == 2 ? vs[v].fp32 : w ? vs[v].soft8 : vs[v].hard, dim3(grid), dim3(256), 0, 0, w == 2 ? bF : w ? bS : bH, bO, gg);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(v ? got.data() : ref.data(), bO + (K - 1) * ostr, g.packNum * 4, hipMemcpyDeviceToHost));
            if (v) {
                size_t bad = 0;
                for (size_t k = 0; k < ref.size(); k++) bad += ref[k] != got[k];
                printf("exact twin %s %-40.40s: %zu words differ\n", w == 2 ? "fp32 " : w ? "soft8" : "hard ", vs[v].name, bad);
            }
        }
    printf("%d rounds, %d batches per launch; ms per 32M-bit batch (median)\n", rounds, K);
    printf("%-36s %9s %9s %9s\n", "variant", "hard_b32", "soft8_b16", "fp32_f16");
    for (int v = 0; v < nv; v++) printf("%-36.36s %9.4f %9.4f %9.4f\n", vs[v].name, median(th[v]), median(ts[v]), median(tf[v]));
    return 0;
}
