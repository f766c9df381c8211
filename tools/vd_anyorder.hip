// vd_anyorder.hip -- launch-tail study (tools only): the bench step's two batched launches (HARD/b32 and
// SOFT8/b16, K batches each) on one stream, back to back as the bench issues them, against
//  * the first launch with hipExtAnyOrderLaunch (no barrier behind it: the second kernel's workgroups may
//    start while the first one's last waves drain),
//  * both on two streams at once,
//  * each workload as K - 1 batched batches + the last batch as a split single-batch launch behind it
//    (any-order), so that the finer split waves fill the batched launch's tail.
// Prints ms per step (median / min over rounds) and checks every variant's words against the plain one.
// Inputs as tools/vd_pkab.  Usage: vd_anyorder [rounds] [K]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_pk.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 10, K = argc > 2 ? atoi(argv[2]) : 20;
    const size_t N = 32000000;
    std::mt19937 rng(7);
    std::vector<uint32_t> hh(N / 16 + 64, 0u), hs(N / 2 + 64, 0u);
    uint32_t reg = 0;
    std::normal_distribution<double> G(0.0, std::sqrt(1.0 / (2.0 * 0.5 * std::pow(10.0, 0.2))));
    auto q8 = [&](double x) { long v = std::lround(x * 40.0); v = std::min(127L, std::max(-128L, v)); return (uint32_t)(uint8_t)(int8_t)v; };
    for (size_t t = 0; t < N; t++) {
        reg = ((reg >> 1) | ((rng() & 1u) << 6)) & 127u;
        const uint32_t o0 = __builtin_popcount(reg & 0171u) & 1u, o1 = __builtin_popcount(reg & 0133u) & 1u;
        const double x0 = (o0 ? -1.0 : 1.0) + G(rng), x1 = (o1 ? -1.0 : 1.0) + G(rng);
        hh[t / 16] |= ((uint32_t)(x0 < 0) << (31 - 2 * (t % 16))) | ((uint32_t)(x1 < 0) << (30 - 2 * (t % 16)));
        hs[t / 2] |= ((q8(x0) << 8) | q8(x1)) << (16 * ((t % 2) ^ 1));
    }
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t ostr = ((N - 64) / 32 * 4 + 255) / 256 * 256;
    char *bH, *bS, *oH, *oS;
    CK(hipMalloc(&bH, strH * K));
    CK(hipMalloc(&bS, strS * K));
    CK(hipMalloc(&oH, ostr * K));
    CK(hipMalloc(&oS, ostr * K));
    for (int k = 0; k < K; k++) {  // distinct batches: every batch its own rotation of the words
        std::rotate(hh.begin(), hh.begin() + 1, hh.end() - 64);
        std::rotate(hs.begin(), hs.begin() + 1, hs.end() - 64);
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    g.outStride = ostr;
    uint32_t *fa, *fb, *st;
    CK(hipMalloc(&fa, vd::kFairBoardWords * 4));
    CK(hipMalloc(&fb, vd::kFairBoardWords * 4));
    CK(hipMalloc(&st, 8));
    CK(hipMemset(fa, 0xFF, vd::kFairBoardWords * 4));
    CK(hipMemset(fb, 0xFF, vd::kFairBoardWords * 4));
    CK(hipMemset(st, 0, 8));
    vd::Geom gh = g, gs = g;
    gh.inStride = strH;
    gs.inStride = strS;
    gh.fair = fa;
    gs.fair = fb;
    // split single batch (vd_capi.hip launch_decode, Form::PkSplit): tail workgroups for nchunks mod SIMDs
    const uint32_t tailc = 6400u % (4u * cus);
    vd::Geom ghs = gh, gss = gs;
    ghs.nbatch = gss.nbatch = 1;
    ghs.stats = gss.stats = st;
    ghs.tailWG = gss.tailWG = (6400u - tailc) / 4u;
    const unsigned gsplit = ghs.tailWG + tailc;
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    auto hard = [&](hipStream_t s, uint32_t fl, int nb) {
        vd::Geom x = gh;
        x.nbatch = nb;
        hipExtLaunchKernelGGL((vd::vd_decode_pk<vd::HARD, vd::B32, 32, false>), dim3(800u * nb), dim3(256), 0, s, nullptr, nullptr, fl, (const void*)bH, (void*)oH, x);
    };
    auto soft = [&](hipStream_t s, uint32_t fl, int nb) {
        vd::Geom x = gs;
        x.nbatch = nb;
        hipExtLaunchKernelGGL((vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false>), dim3(800u * nb), dim3(256), 0, s, nullptr, nullptr, fl, (const void*)bS, (void*)oS, x);
    };
    auto hard_split = [&](hipStream_t s, uint32_t fl) {
        hipExtLaunchKernelGGL((vd::vd_decode_pk<vd::HARD, vd::B32, 32, true>), dim3(gsplit), dim3(256), 0, s, nullptr, nullptr, fl,
                              (const void*)(bH + (K - 1) * strH), (void*)(oH + (K - 1) * ostr), ghs);
    };
    auto soft_split = [&](hipStream_t s, uint32_t fl) {
        hipExtLaunchKernelGGL((vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true>), dim3(gsplit), dim3(256), 0, s, nullptr, nullptr, fl,
                              (const void*)(bS + (K - 1) * strS), (void*)(oS + (K - 1) * ostr), gss);
    };
    const uint32_t AO = hipExtAnyOrderLaunch;
    const char* names[] = {"one stream, back to back (bench)", "one stream, HARD any-order",
                           "one stream, both any-order", "two streams, concurrent",
                           "one stream, K-1 batched + split last, any-order",
                           "one stream, K-1 batched + split last, plain"};
    const int NV = 6;
    auto step = [&](int v) {
        switch (v) {
        case 0: hard(sa, 0, K); soft(sa, 0, K); break;
        case 1: hard(sa, AO, K); soft(sa, 0, K); break;
        case 2: hard(sa, AO, K); soft(sa, AO, K); break;
        case 3:
            CK(hipStreamWaitEvent(sb, e0, 0));
            hard(sa, 0, K);
            soft(sb, 0, K);
            CK(hipEventRecord(e2, sb));
            CK(hipStreamWaitEvent(sa, e2, 0));
            break;
        case 4: hard(sa, AO, K - 1); hard_split(sa, AO); soft(sa, AO, K - 1); soft_split(sa, 0); break;
        case 5: hard(sa, 0, K - 1); hard_split(sa, 0); soft(sa, 0, K - 1); soft_split(sa, 0); break;
        }
    };
    // reference words (plain launches), then every variant's words against them
    std::vector<uint32_t> rH(ostr / 4 * K), rS(ostr / 4 * K), xH(ostr / 4 * K), xS(ostr / 4 * K);
    step(0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(rH.data(), oH, ostr * K, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rS.data(), oS, ostr * K, hipMemcpyDeviceToHost));
    for (int v = 1; v < NV; v++) {
        CK(hipMemset(oH, 0, ostr * K));
        CK(hipMemset(oS, 0, ostr * K));
        CK(hipEventRecord(e0, sa));
        step(v);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(xH.data(), oH, ostr * K, hipMemcpyDeviceToHost));
        CK(hipMemcpy(xS.data(), oS, ostr * K, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < rH.size(); i++) bad += (rH[i] != xH[i]) + (rS[i] != xS[i]);
        printf("words differing from the plain launches, %-48s: %zu\n", names[v], bad);
    }
    for (int i = 0; i < 3; i++) step(0);  // clock ramp
    CK(hipDeviceSynchronize());
    std::vector<std::vector<float>> t(NV);
    for (int r = 0; r < rounds; r++)
        for (int vi = 0; vi < NV; vi++) {
            const int v = (vi + r) % NV;
            CK(hipEventRecord(e0, sa));
            step(v);
            CK(hipEventRecord(e1, sa));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / K);
        }
    uint32_t redec[2];
    CK(hipMemcpy(redec, st, 8, hipMemcpyDeviceToHost));
    printf("K = %d batches per launch, %d rounds; ms per step (one HARD + one SOFT8 batch), median / min "
           "(split re-decodes %u, cap exits %u)\n", K, rounds, redec[0], redec[1]);
    for (int v = 0; v < NV; v++) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-52s: %.4f / %.4f\n", names[v], t[v][t[v].size() / 2], t[v][0]);
    }
    return 0;
}
