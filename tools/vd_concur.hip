// vd_concur.hip -- timing study (tools only): the bench step's two batched launches (HARD/b32 and SOFT8/b16, K
// batches each) back to back on one stream against the same two launches on two streams at once.
// Inputs as tools/vd_pkab.  Usage: vd_concur [rounds] [K]
#include <hip/hip_runtime.h>
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
    const int rounds = argc > 1 ? atoi(argv[1]) : 10, K = argc > 2 ? atoi(argv[2]) : 100;
    const size_t N = 32000000;
    std::mt19937 rng(7);
    std::vector<uint32_t> hh(N / 16 + 64, 0u), hs(N / 2 + 64, 0u);
    uint32_t reg = 0;
    std::normal_distribution<double> G(0.0, std::sqrt(1.0 / (2.0 * 0.5 * std::pow(10.0, 0.2))));
    auto q8 = [&](double x) { long v = std::lround(x * 40.0); v = std::min(127L, std::max(-128L, v)); return (uint32_t)(uint8_t)(int8_t)v; };
    for (size_t t = 0; t < N; t++) {
        reg = ((reg >> 1) | ((rng() & 1u) << 6)) & 127u;
        const uint32_t o0 = __builtin_popcount(reg & 0171u) & 1u, o1 = __builtin_popcount(reg & 0133u) & 1u;
        hh[t / 16] |= (o0 << (31 - 2 * (t % 16))) | (o1 << (30 - 2 * (t % 16)));
        const uint32_t s0 = q8((o0 ? -1.0 : 1.0) + G(rng)), s1 = q8((o1 ? -1.0 : 1.0) + G(rng));
        hs[t / 2] |= ((s0 << 8) | s1) << (16 * ((t % 2) ^ 1));
    }
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t ostr = ((N - 64) / 32 * 4 + 255) / 256 * 256;
    char *bH, *bS, *oH, *oS;
    CK(hipMalloc(&bH, strH * K));
    CK(hipMalloc(&bS, strS * K));
    CK(hipMalloc(&oH, ostr * K));
    CK(hipMalloc(&oS, ostr * K));
    for (int k = 0; k < K; k++) {
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    g.nbatch = K;
    g.outStride = ostr;
    uint32_t *fa, *fb;
    CK(hipMalloc(&fa, vd::kFairBoardWords * 4));
    CK(hipMalloc(&fb, vd::kFairBoardWords * 4));
    CK(hipMemset(fa, 0xFF, vd::kFairBoardWords * 4));
    CK(hipMemset(fb, 0xFF, vd::kFairBoardWords * 4));
    vd::Geom gh = g, gs = g;
    gh.inStride = strH;
    gs.inStride = strS;
    gh.fair = fa;
    gs.fair = fb;  // (two kernels on one SIMD: separate boards)
    const unsigned grid = 800u * K;
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    auto hard = [&](hipStream_t s) { hipLaunchKernelGGL((vd::vd_decode_pk<vd::HARD, vd::B32, 32, false>), dim3(grid), dim3(256), 0, s, bH, oH, gh); };
    auto soft = [&](hipStream_t s) { hipLaunchKernelGGL((vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false>), dim3(grid), dim3(256), 0, s, bS, oS, gs); };
    for (int i = 0; i < 3; i++) { hard(sa); soft(sa); }  // clock ramp
    CK(hipDeviceSynchronize());
    std::vector<float> tseq, tcon;
    for (int r = 0; r < rounds; r++) {
        for (int mode = 0; mode < 2; mode++) {
            const bool con = (mode + r) % 2 == 1;
            CK(hipEventRecord(e0, sa));
            if (con) {
                CK(hipStreamWaitEvent(sb, e0, 0));
                hard(sa);
                soft(sb);
                CK(hipEventRecord(e2, sb));
                CK(hipStreamWaitEvent(sa, e2, 0));
            } else {
                hard(sa);
                soft(sa);
            }
            CK(hipEventRecord(e1, sa));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            (con ? tcon : tseq).push_back(t / K);
        }
    }
    std::sort(tseq.begin(), tseq.end());
    std::sort(tcon.begin(), tcon.end());
    printf("K = %d batches per launch, %d rounds; ms per step (one HARD + one SOFT8 batch), median / min\n", K, rounds);
    printf("one stream, back to back : %.4f / %.4f\n", tseq[tseq.size() / 2], tseq[0]);
    printf("two streams, concurrent  : %.4f / %.4f\n", tcon[tcon.size() / 2], tcon[0]);
    return 0;
}
