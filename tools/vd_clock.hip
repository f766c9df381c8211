// vd_clock.hip -- in-kernel clock of batched launches (not part of the product).  Is the decode kernel's
// time set by its issue cycles or by the clock the chip holds under it?  For the headline kernels (HARD/b32,
// SOFT8/b16) and some component ablations (vd_kernel_tg.h kAbl*, outputs of ablations are wrong), batched
// launches over distinct resident codeword inputs (bench conditions, as tools/vd_benchab), each built with
// kAblClock: every wave stamps s_memtime / s_memrealtime at its start and end.  Per variant: ms per batch,
// median in-kernel clock (delta memtime / delta realtime x 100 MHz, MI355X_MICROARCH.md 'DVFS give-back'
// item 6), and SIMD cycles per wave-stage = launch time x clock x 1024 SIMDs / wave-stages.
// Usage: vd_clock [groups] [batches per launch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "build/abl/vd_kernel_tg.h"  // the product kernel + tools-only ablation bits (tools/abl/gen_abl.py)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
struct Variant { const char* name; KFn fn; int in; };  // in: 0 HARD, 1 SOFT8, 2 FP32

int main(int argc, char** argv)
{
    const int groups = argc > 1 ? atoi(argv[1]) : 6, steps = argc > 2 ? atoi(argv[2]) : 16;
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
    // FP32: the same noisy BPSK values as floats scaled like the packer's FP32 path (x 40000 / 2^13 here:
    // the kernel clamps to [-8, 7]), two per stage
    std::vector<float> hf(2 * N + 128, 0.0f);
    {
        std::mt19937 r2(11);
        std::normal_distribution<double> G2(0.0, sigma);
        for (size_t t = 0; t < N; t++) {
            hf[2 * t] = (float)(((o0[t] ? -1.0 : 1.0) + G2(r2)) * 4.0);
            hf[2 * t + 1] = (float)(((o1[t] ? -1.0 : 1.0) + G2(r2)) * 4.0);
        }
    }
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t strF = (hf.size() * 4 + 255) / 256 * 256;
    void *bH, *bS, *bF, *out;
    CK(hipMalloc(&bH, strH * steps));
    CK(hipMalloc(&bS, strS * steps));
    CK(hipMalloc(&bF, strF * steps));
    // outputs at stride 0 (timing only): the clock stamps sit at out + 16 MiB + 48 B per launch wave
    const size_t outBytes = (16u << 20) + (size_t)6400 * steps * 48;
    CK(hipMalloc(&out, outBytes));
    for (int k = 0; k < steps; k++) {
        CK(hipMemcpy((char*)bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy((char*)bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy((char*)bF + k * strF, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
    }
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    g.nbatch = (uint32_t)steps;
    g.outStride = 0;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    constexpr int C = vd::kAblClock;
    const Variant vs[] = {
        {"hard  full", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, C>, 0},
        {"hard  ACS only", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, C | vd::kAblAcsOnly>, 0},
        {"hard  -tabreads", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, C | vd::kAblNoTabReads>, 0},
        {"hard  -traceback", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, C | vd::kAblNoTraceback>, 0},
        {"hard  -tabbuild", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, C | vd::kAblNoTabBuild>, 0},
        {"soft8 full", (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, C>, 1},
        {"soft8 ACS only", (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, C | vd::kAblAcsOnly>, 1},
        {"soft8 -tabreads", (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, C | vd::kAblNoTabReads>, 1},
        {"fp32  full", (KFn)vd::vd_decode_tg<vd::FP32, vd::F16, 32, C>, 2},
        {"fp32  ACS only", (KFn)vd::vd_decode_tg<vd::FP32, vd::F16, 32, C | vd::kAblAcsOnly>, 2},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    const unsigned grid = 1600u * (unsigned)steps;
    const size_t waves = (size_t)6400 * steps;
    // wave-stages of one batch: every chunk decodes (words + 2) blocks of 32 stages
    double wstages = 0;
    for (uint32_t c = 0; c < 6400; c++) wstages += 32.0 * (g.packNum / 6400 + (c < g.packNum % 6400 ? 1 : 0) + 2);
    wstages *= steps;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto launch = [&](const Variant& v) {
        vd::Geom gg = g;
        gg.inStride = v.in == 2 ? strF : v.in == 1 ? strS : strH;
        hipLaunchKernelGGL(v.fn, dim3(grid), dim3(256), 0, 0, v.in == 2 ? bF : v.in == 1 ? bS : bH, out, gg);
    };
    // warm-up: 0.5 s of launches (the clock ramps from idle)
    {
        CK(hipEventRecord(e0));
        float ms = 0;
        while (ms < 500.0f) {
            for (int i = 0; i < 4; i++) launch(vs[0]);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        }
    }
    std::vector<std::vector<double>> tms(nv), mhz(nv);
    std::vector<uint64_t> d(waves * 6);
    for (int r = 0; r < groups; r++)
        for (int vi = 0; vi < nv; vi++) {
            const int v = (vi + r) % nv;
            launch(vs[v]);  // one untimed launch of this variant first (same clock regime)
            CK(hipEventRecord(e0));
            launch(vs[v]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(d.data(), (char*)out + (16u << 20), d.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> m;
            for (size_t w = 0; w < waves; w++) {
                const uint64_t* e = &d[6 * w];
                if (e[3] > e[2]) m.push_back((double)(e[1] - e[0]) / (double)(e[3] - e[2]) * 100.0);
            }
            std::sort(m.begin(), m.end());
            tms[v].push_back(ms / steps);
            mhz[v].push_back(m[m.size() / 2]);
        }
    printf("batched launches of %d batches (codeword input, distinct copies), %d groups, medians\n", steps, groups);
    printf("%-18s %9s %9s %9s %14s\n", "variant", "ms/batch", "Gb/s", "MHz", "cycles/w-s");
    for (int v = 0; v < nv; v++) {
        std::sort(tms[v].begin(), tms[v].end());
        std::sort(mhz[v].begin(), mhz[v].end());
        const double t = tms[v][tms[v].size() / 2], f = mhz[v][mhz[v].size() / 2];
        const double cyc = t * 1e-3 * steps * f * 1e6 * 1024.0 / wstages;
        printf("%-18s %9.4f %9.1f %9.0f %14.2f\n", vs[v].name, t, (double)(g.packNum * 32) / (t * 1e-3) / 1e9, f, cyc);
    }
    return 0;
}
