// vd_abx.hip -- timing-only A/B of kernel variants (not part of the product), both launch kinds the product
// uses: batched launches (bench.py's timed region: K distinct resident batches per launch) and single-batch
// segment launches (the reference run()'s unit of work, vd_run_device: the product's "pieces" table).
// Workloads: HARD/b32 (K=7 codeword through a BSC, p = 0.04) and SOFT8/b16 (BPSK codeword + Gaussian noise
// at Eb/N0 2 dB, quantised like SoftDecisionPacker(SOFT8)).  Variants alternate round by round with a
// rotating order, so clock and thermal drift hit all alike; every variant's words are checked against the
// product kernel's (batched: last batch; segment launch: the whole output).
// Usage: vd_abx [rounds] [batches per launch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_pk.h"
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_segplan.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
#define PK(A) (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, (A)>

template <int ABL>
struct V {
    static constexpr KFn hard = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, ABL>;
    static constexpr KFn soft8 = (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, ABL>;
};
// a variant: kernels, and the segment table (vd_segplan.h SegMode) + warm-up blocks of its segment launches
struct Variant { const char* name; KFn hard, soft8; int seg = vd::kSegPieces; uint32_t warm = vd::kSplitWarm; KFn hardBatched = nullptr; };
#ifndef VD_ABX_VARIANTS
#define VD_ABX_VARIANTS                                                                                      \
    {"vd_decode_pk full", V<0>::hard, V<0>::soft8, vd::kSegPieces, vd::kSplitWarm, PK(0)},                  \
    {"pk -traceback", V<0>::hard, V<0>::soft8, vd::kSegPieces, vd::kSplitWarm, PK(vd::kAblNoTraceback)},     \
    {"pk -loads", V<0>::hard, V<0>::soft8, vd::kSegPieces, vd::kSplitWarm, PK(vd::kAblNoLoads)},             \
    {"pk loads two groups ahead", V<0>::hard, V<0>::soft8, vd::kSegPieces, vd::kSplitWarm, PK(vd::kAblLoad2)},
#endif

static double median(std::vector<float> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 6, K = argc > 2 ? atoi(argv[2]) : 20;
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
        uint32_t a = o0[t] ^ (U(rng) < 0.04), b = o1[t] ^ (U(rng) < 0.04);
        hh[t / 16] |= (a << (31 - 2 * (t % 16))) | (b << (30 - 2 * (t % 16)));
    }
    const double sigma = std::sqrt(1.0 / (2.0 * 0.5 * std::pow(10.0, 0.2)));
    std::normal_distribution<double> G(0.0, sigma);
    auto q8 = [&](double x) { long v = std::lround(x * 40.0); v = std::min(127L, std::max(-128L, v)); return (uint32_t)(uint8_t)(int8_t)v; };
    std::vector<uint32_t> hs(N / 2 + 64, 0u);
    for (size_t t = 0; t < N; t++) {
        const uint32_t s0 = q8((o0[t] ? -1.0 : 1.0) + G(rng)), s1 = q8((o1[t] ? -1.0 : 1.0) + G(rng));
        hs[t / 2] |= ((s0 << 8) | s1) << (16 * ((t % 2) ^ 1));
    }
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    CK(hipMalloc(&g.stats, 4));
    CK(hipMemset(g.stats, 0, 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* tabd[3];
    unsigned gridT[3];
    for (int m = 0; m < 3; m++) {
        const std::vector<uint32_t> tab = vd::seg_table(4 * cus, m);
        if (tab.empty()) { printf("no segment table %d for %d CUs\n", m, cus); return 1; }
        CK(hipMalloc(&tabd[m], tab.size() * 4));
        CK(hipMemcpy(tabd[m], tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        gridT[m] = (unsigned)(tab.size() - 1);
    }
    // K distinct resident copies per workload (nothing served from another batch's cache lines)
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t ostr = (g.packNum * 4 + 255) / 256 * 256;
    char *bH, *bS, *bO, *bO2;
    CK(hipMalloc(&bH, strH * K));
    CK(hipMalloc(&bS, strS * K));
    CK(hipMalloc(&bO, ostr * K));
    CK(hipMalloc(&bO2, ostr * K));
    for (int k = 0; k < K; k++) {
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    vd::Geom gb = g, gs = g;
    gb.nbatch = (uint32_t)K;
    gb.outStride = ostr;
    const unsigned gridB = 1600u * (unsigned)K;
    const Variant vs[] = {VD_ABX_VARIANTS};
    const int nv = sizeof(vs) / sizeof(vs[0]);
    hipEvent_t ev[5];
    for (auto& evi : ev) CK(hipEventCreate(&evi));
    std::vector<std::vector<float>> tbh(nv), tbs(nv), tsh(nv), tss(nv);
    for (int r = 0; r < rounds + 1; r++)
        for (int vi = 0; vi < nv; vi++) {
            const int v = (vi + r) % nv;
            vd::Geom gh = gb, gS = gb;
            gh.inStride = strH;
            gS.inStride = strS;
            CK(hipEventRecord(ev[0]));
            if (vs[v].hardBatched) hipLaunchKernelGGL(vs[v].hardBatched, dim3(gridB / 2), dim3(256), 0, 0, bH, bO, gh);
            else hipLaunchKernelGGL(vs[v].hard, dim3(gridB), dim3(256), 0, 0, bH, bO, gh);
            CK(hipEventRecord(ev[1]));
            hipLaunchKernelGGL(vs[v].soft8, dim3(gridB), dim3(256), 0, 0, bS, bO, gS);
            CK(hipEventRecord(ev[2]));
            vd::Geom gv = gs;
            gv.seg = tabd[vs[v].seg];
            gv.segWarm = vs[v].warm;
            const unsigned gridS = gridT[vs[v].seg];
            for (int k = 0; k < K; k++) hipLaunchKernelGGL(vs[v].hard, dim3(gridS), dim3(256), 0, 0, bH + k * strH, bO2 + k * ostr, gv);
            CK(hipEventRecord(ev[3]));
            for (int k = 0; k < K; k++) hipLaunchKernelGGL(vs[v].soft8, dim3(gridS), dim3(256), 0, 0, bS + k * strS, bO2 + k * ostr, gv);
            CK(hipEventRecord(ev[4]));
            CK(hipEventSynchronize(ev[4]));
            float a, b, c, d;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            CK(hipEventElapsedTime(&c, ev[2], ev[3]));
            CK(hipEventElapsedTime(&d, ev[3], ev[4]));
            if (r) { tbh[v].push_back(a / K); tbs[v].push_back(b / K); tsh[v].push_back(c / K); tss[v].push_back(d / K); }
        }
    // exact twins against the product (variant 0): batched (last batch) and segment launch outputs
    std::vector<uint32_t> ref(g.packNum), got(g.packNum);
    for (int w = 0; w < 2; w++)
        for (int kind = 0; kind < 2; kind++)
            for (int v = 0; v < nv; v++) {
                vd::Geom gg = kind == 0 ? gb : gs;
                if (kind == 0) gg.inStride = w ? strS : strH;
                else { gg.seg = tabd[vs[v].seg]; gg.segWarm = vs[v].warm; }
                const unsigned gridS = gridT[vs[v].seg];
                CK(hipMemset(bO, 0, ostr * K));
                KFn f = w ? vs[v].soft8 : vs[v].hard;
                const char* in = w ? bS : bH;
                if (kind == 0 && w == 0 && vs[v].hardBatched) hipLaunchKernelGGL(vs[v].hardBatched, dim3(gridB / 2), dim3(256), 0, 0, in, bO, gg);
                else if (kind == 0) hipLaunchKernelGGL(f, dim3(gridB), dim3(256), 0, 0, in, bO, gg);
                else hipLaunchKernelGGL(f, dim3(gridS), dim3(256), 0, 0, in, bO + (K - 1) * ostr, gg);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(v ? got.data() : ref.data(), bO + (K - 1) * ostr, g.packNum * 4, hipMemcpyDeviceToHost));
                if (v) {
                    size_t bad = 0;
                    for (size_t k = 0; k < ref.size(); k++) bad += ref[k] != got[k];
                    printf("exact twin %s %-8s %-40.40s: %zu words differ\n", w ? "soft8" : "hard ", kind ? "segment" : "batched", vs[v].name, bad);
                }
            }
    uint32_t redec = 0;
    CK(hipMemcpy(&redec, g.stats, 4, hipMemcpyDeviceToHost));
    const double bits = (double)(g.packNum * 32);
    printf("%d rounds, %d batches per launch / %d segment launches per round; segment re-decodes %u\n", rounds, K, K, redec);
    printf("%-36s %9s %9s %8s | %9s %9s %8s   (ms per 32M-bit batch, Gb/s of the hard+soft8 pair)\n", "variant", "b.hard", "b.soft8",
           "b.Gb/s", "s.hard", "s.soft8", "s.Gb/s");
    for (int v = 0; v < nv; v++) {
        const double a = median(tbh[v]), b = median(tbs[v]), c = median(tsh[v]), d = median(tss[v]);
        printf("%-36.36s %9.4f %9.4f %8.1f | %9.4f %9.4f %8.1f\n", vs[v].name, a, b, 2 * bits / ((a + b) * 1e-3) / 1e9, c, d,
               2 * bits / ((c + d) * 1e-3) / 1e9);
    }
    return 0;
}
