// vd_occab.hip -- timing study (not part of the product): how the per-batch time of the product kernels
// depends on (1) waves per SIMD and (2) batches per launch.
//  (1) batched launches of `steps` distinct batches with the resident workgroups per CU capped at 8, 7, 6, 5
//      (dynamic LDS padding on top of the kernel's static LDS), variants alternating launch by launch;
//  (2) launches of n = 1, 2, 4, 8, 16, 32 batches at full occupancy: t(n) = a + b / n separates the
//      per-batch rate (a) from the once-per-launch ramp and tail (b).
// Input: a K=7 codeword through a BSC (HARD, p = 0.04) / BPSK + AWGN at 2 dB (SOFT8), as vd_benchab.
// Usage: vd_occab [rounds] [steps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);

static double median(std::vector<float> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 8, steps = argc > 2 ? atoi(argv[2]) : 32;
    const size_t N = 32000000;
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
    // FP32 input (2 floats per stage): BPSK + AWGN at 2 dB, unscaled (the kernel clamps to [-8, 7])
    std::vector<float> hf(2 * N + 128, 0.0f);
    for (size_t t = 0; t < N; t++) {
        hf[2 * t] = (float)((o0[t] ? -1.0 : 1.0) + G(rng)) * 4.0f;
        hf[2 * t + 1] = (float)((o1[t] ? -1.0 : 1.0) + G(rng)) * 4.0f;
    }
    vd::Geom g{};
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t ostr = (g.packNum * 4 + 255) / 256 * 256;
    char *bH, *bS, *bO;
    CK(hipMalloc(&bH, strH * steps));
    CK(hipMalloc(&bS, strS * steps));
    CK(hipMalloc(&bO, ostr * steps));
    for (int k = 0; k < steps; k++) {
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    const KFn kh = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32>, ks = (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32>;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    auto run = [&](int nb, size_t pad, float& th, float& ts) {
        vd::Geom gh = g, gs = g;
        gh.nbatch = gs.nbatch = (uint32_t)nb;
        gh.inStride = strH; gs.inStride = strS; gh.outStride = gs.outStride = ostr;
        const unsigned grid = 1600u * (unsigned)nb;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kh, dim3(grid), dim3(256), pad, 0, bH, bO, gh);
        CK(hipEventRecord(e1));
        hipLaunchKernelGGL(ks, dim3(grid), dim3(256), pad, 0, bS, bO, gs);
        CK(hipEventRecord(e2));
        CK(hipEventSynchronize(e2));
        CK(hipEventElapsedTime(&th, e0, e1));
        CK(hipEventElapsedTime(&ts, e1, e2));
        th /= nb;
        ts /= nb;
    };
    // warm the clock up
    for (int i = 0; i < 20; i++) { float a, b; run(steps, 0, a, b); }
    // (1) occupancy
    const int occ[] = {8, 7, 6, 5};
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)kh));
    const size_t lds_wg = fa.sharedSizeBytes;
    std::vector<float> oh[4], os[4];
    for (int r = 0; r < rounds; r++)
        for (int vi = 0; vi < 4; vi++) {
            const int v = (vi + r) % 4;
            const size_t pad = occ[v] == 8 ? 0 : (163840 / occ[v] - lds_wg) / 256 * 256;
            float a, b;
            run(steps, pad, a, b);
            oh[v].push_back(a); os[v].push_back(b);
        }
    printf("(1) batched launches of %d batches, workgroups per CU capped by LDS padding; ms per batch (median of %d)\n", steps, rounds);
    for (int v = 0; v < 4; v++) {
        const size_t pad = occ[v] == 8 ? 0 : (163840 / occ[v] - lds_wg) / 256 * 256;
        printf("  %d waves/SIMD (pad %5zu B): hard %.4f  soft8 %.4f\n", occ[v], pad, median(oh[v]), median(os[v]));
    }
    // (2) batches per launch
    std::vector<int> ns;
    for (int n = 1; n <= steps; n *= 2) ns.push_back(n);
    std::vector<std::vector<float>> nh(ns.size()), nsv(ns.size());
    for (int r = 0; r < rounds; r++)
        for (size_t vi = 0; vi < ns.size(); vi++) {
            const size_t v = (vi + r) % ns.size();
            float a, b;
            run(ns[v], 0, a, b);
            nh[v].push_back(a); nsv[v].push_back(b);
        }
    printf("(2) batches per launch at full occupancy; ms per batch (median of %d)\n", rounds);
    for (size_t v = 0; v < ns.size(); v++) printf("  n %3d: hard %.4f  soft8 %.4f\n", ns[v], median(nh[v]), median(nsv[v]));
    // least squares t = a + b/n
    for (int w = 0; w < 2; w++) {
        double sx = 0, sy = 0, sxx = 0, sxy = 0;
        for (size_t v = 0; v < ns.size(); v++) {
            const double x = 1.0 / ns[v], y = median(w ? nsv[v] : nh[v]);
            sx += x; sy += y; sxx += x * x; sxy += x * y;
        }
        const double m = (double)ns.size(), b = (m * sxy - sx * sy) / (m * sxx - sx * sx), a = (sy - b * sx) / m;
        printf("  fit %s: t(n) = %.4f + %.4f / n ms (per-launch ramp + tail %.1f us)\n", w ? "soft8" : "hard ", a, b, b * 1e3);
    }
    // (3) FP32 input (8 B per stage): `steps` distinct resident batches against one batch read `steps` times
    //     (input stride 0: after the first batch it comes from the caches), SOFT8 alongside
    {
        const size_t strF = (hf.size() * 4 + 255) / 256 * 256;
        char* bF;
        CK(hipMalloc(&bF, strF * steps));
        for (int k = 0; k < steps; k++) CK(hipMemcpy(bF + k * strF, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
        const KFn kf = (KFn)vd::vd_decode_tg<vd::FP32, vd::F16, 32>;
        std::vector<float> tf[3];
        for (int r = 0; r < rounds; r++)
            for (int v = 0; v < 3; v++) {
                vd::Geom q = g;
                q.nbatch = (uint32_t)steps;
                q.outStride = ostr;
                q.inStride = v == 0 ? strF : v == 1 ? 0 : strS;
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(v < 2 ? kf : ks, dim3(1600u * steps), dim3(256), 0, 0, v < 2 ? bF : bS, bO, q);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                tf[v].push_back(ms / steps);
            }
        printf("(3) %d-batch launches, ms per batch: fp32/f16 distinct inputs %.4f, fp32/f16 one input (stride 0) %.4f, soft8/b16 distinct %.4f\n",
               steps, median(tf[0]), median(tf[1]), median(tf[2]));
        CK(hipFree(bF));
    }
    return 0;
}
