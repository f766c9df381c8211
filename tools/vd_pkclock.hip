// vd_pkclock.hip -- timeline of single-batch split launches of vd_decode_pk (tools only): every wave stamps
// s_memrealtime at its start, after its first pass and at its end (kAblClock), with its hardware slot.
// Prints, per kernel, the launch time (HIP events), the spread of wave start and end times, the waves' own
// durations (whole-chunk and tail waves apart), the re-decoded waves, and the same per-wave figures for a
// batched launch (8 waves per SIMD, two chunks per wave) for comparison.  Inputs as tools/vd_pkab.
// Usage: vd_pkclock [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
#include <vector>
#include <map>
#include <algorithm>
#include "build/abl/vd_kernel_pk.h"  // the product kernel + tools-only ablation bits (tools/abl/gen_abl.py)
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);

static double pct(std::vector<double> v, double p)
{
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
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
    const int K = 20;  // batches of the batched comparison launch
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    char *bH, *bS, *bO;
    CK(hipMalloc(&bH, strH * K));
    CK(hipMalloc(&bS, strS * K));
    for (int k = 0; k < K; k++) {
        CK(hipMemcpy(bH + k * strH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bS + k * strS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    const size_t ostr = ((N - 64) / 32 * 4 + 255) / 256 * 256;
    const size_t maxWaves = 800u * K * 4;
    const size_t obytes = std::max(ostr * K, (size_t)16 << 20) + maxWaves * 64;
    CK(hipMalloc(&bO, obytes));
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    uint32_t* stats;
    CK(hipMalloc(&stats, 4));
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const double us_per_tick = 1000.0 / rate_khz;
    printf("s_memrealtime: %d kHz\n", rate_khz);

    struct Case { const char* name; KFn f; const char* in; size_t istr; bool split; unsigned grid = 0; };
    constexpr int C = vd::kAblClock;
    const Case cases[] = {
        {"HARD/b32 split", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, C>, bH, strH, true},
        {"SOFT8/b16 split", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 7, C>, bS, strS, true},
        {"HARD/b32 batched x20", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C>, bH, strH, false},
        {"SOFT8/b16 batched x20", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 8, C>, bS, strS, false},
        {"HARD/b32 batched, one generation of 6 WG per CU", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C>, bH, strH, false, 1536},
        {"HARD/b32 batched, one generation of 7 WG per CU", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C>, bH, strH, false, 1792},
        {"HARD/b32 batched, one generation of 8 WG per CU", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C>, bH, strH, false, 2048},
        {"SOFT8/b16 batched, one generation of 7 WG per CU", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 8, C>, bS, strS, false, 1792},
        {"HARD/b32 batched + fairness, one generation of 7 WG per CU", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C | vd::kAblFairAll>, bH, strH, false, 1792},
        {"SOFT8/b16 batched + fairness, one generation of 7 WG per CU", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 8, C | vd::kAblFairAll>, bS, strS, false, 1792},
        {"HARD/b32 batched + fairness, one generation of 8 WG per CU", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C | vd::kAblFairAll>, bH, strH, false, 2048},
        {"SOFT8/b16 batched + fairness, one generation of 8 WG per CU", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 8, C | vd::kAblFairAll>, bS, strS, false, 2048},
        {"HARD/b32 batched + fairness x20", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, C | vd::kAblFairAll>, bH, strH, false},
        {"SOFT8/b16 batched, one generation of 8 WG per CU", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 8, C>, bS, strS, false, 2048},
        {"HARD/b32 split (no stamps)", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, 0>, bH, strH, true},
        {"SOFT8/b16 split (no stamps)", (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 7, 0>, bS, strS, true},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    {  // clock ramp: about 2 s of batched launches before anything is timed (profiles/r02/clock_ramp.log)
        vd::Geom gw = g;
        gw.nbatch = K;
        gw.inStride = strH;
        gw.outStride = ostr;
        for (int i = 0; i < 800; i++)
            hipLaunchKernelGGL((vd::vd_decode_pk<vd::HARD, vd::B32, 32, false, 8, 0>), dim3(800u * K), dim3(256), 0, 0, bH, bO, gw);
        CK(hipDeviceSynchronize());
    }
    for (const Case& c : cases) {
        vd::Geom gg = g;
        unsigned grid;
        if (c.split) {
            gg.stats = stats;
            gg.tailWG = (6400u - 256u) / 4u;
            grid = gg.tailWG + 256u;
        } else {
            gg.nbatch = K;
            gg.inStride = c.istr;
            gg.outStride = ostr;
            grid = c.grid ? c.grid : 800u * K;
        }
        const size_t stampOff = std::max((size_t)gg.nbatch * gg.outStride, (size_t)16 << 20);
        CK(hipMemset(bO + stampOff, 0, maxWaves * 64));
        std::vector<float> ms;
        for (int r = 0; r < reps + 1; r++) {
            CK(hipMemset(stats, 0, 4));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(c.f, dim3(grid), dim3(256), 0, 0, c.in, bO, gg);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        uint32_t nre = 0;
        CK(hipMemcpy(&nre, stats, 4, hipMemcpyDeviceToHost));
        printf("\n%s: grid %u, launch %.4f ms (median of %d; min %.4f), re-decoded parts %u\n", c.name, grid,
               ms[ms.size() / 2], reps, ms[0], c.split ? nre : 0u);
        if (strstr(c.name, "no stamps")) continue;
        const size_t nw = (size_t)grid * 4;
        std::vector<uint64_t> st(nw * 8);
        CK(hipMemcpy(st.data(), bO + stampOff, nw * 64, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, tend = 0;
        for (size_t w = 0; w < nw; w++) {
            if (!st[8 * w]) continue;
            t0 = std::min(t0, st[8 * w]);
            tend = std::max(tend, st[8 * w + 2]);
        }
        std::vector<double> s_all, e_all, d_whole, d_tail, d_p0, late;
        std::map<uint64_t, std::vector<size_t>> simd;
        int multi = 0, nst = 0;
        for (size_t w = 0; w < nw; w++) {
            const uint64_t* d = &st[8 * w];
            if (!d[0]) continue;
            nst++;
            const double s = (d[0] - t0) * us_per_tick, e = (d[2] - t0) * us_per_tick;
            s_all.push_back(s);
            e_all.push_back(e);
            const bool tail = c.split && w / 4 >= gg.tailWG;
            (tail ? d_tail : d_whole).push_back(e - s);
            if (d[1]) d_p0.push_back((d[1] - t0) * us_per_tick - s);
            if (d[5] > 1) {
                multi++;
                late.push_back((d[2] - d[1]) * us_per_tick);
            }
            const uint32_t hw = (uint32_t)d[3], xcc = (uint32_t)d[4] & 0xF;
            const uint64_t key = ((uint64_t)xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) |
                                 (((hw >> 8) & 0xF) << 2) | ((hw >> 4) & 3);
            simd[key].push_back(w);
        }
        printf("  stamped waves %d, span %.2f us (first start -> last end)\n", nst, (tend - t0) * us_per_tick);
        printf("  start  us: p0 %.2f p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f\n", pct(s_all, 0), pct(s_all, .1),
               pct(s_all, .5), pct(s_all, .9), pct(s_all, .99), pct(s_all, 1));
        printf("  end    us: p0 %.2f p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f\n", pct(e_all, 0), pct(e_all, .1),
               pct(e_all, .5), pct(e_all, .9), pct(e_all, .99), pct(e_all, 1));
        printf("  wave duration us (%s): p10 %.2f p50 %.2f p90 %.2f max %.2f\n", c.split ? "whole-chunk" : "all",
               pct(d_whole, .1), pct(d_whole, .5), pct(d_whole, .9), pct(d_whole, 1));
        if (!d_tail.empty())
            printf("  wave duration us (tail):        p10 %.2f p50 %.2f p90 %.2f max %.2f\n", pct(d_tail, .1),
                   pct(d_tail, .5), pct(d_tail, .9), pct(d_tail, 1));
        if (c.split)
            printf("  first pass us: p50 %.2f p90 %.2f max %.2f; waves with re-decodes %d (extra us p50 %.2f max %.2f)\n",
                   pct(d_p0, .5), pct(d_p0, .9), pct(d_p0, 1), multi, pct(late, .5), pct(late, 1));
        // per SIMD: waves, busy span, and the sum of wave durations
        std::map<int, int> wps;
        std::vector<double> simd_end, simd_start, simd_spread;
        for (auto& kv : simd) {
            wps[(int)kv.second.size()]++;
            double smin = 1e30, emax = 0, ewmin = 1e30, ewmax = 0;
            for (size_t w : kv.second) {
                smin = std::min(smin, (st[8 * w] - t0) * us_per_tick);
                emax = std::max(emax, (st[8 * w + 2] - t0) * us_per_tick);
                if (!c.split || w / 4 < gg.tailWG) {
                    ewmin = std::min(ewmin, (st[8 * w + 2] - t0) * us_per_tick);
                    ewmax = std::max(ewmax, (st[8 * w + 2] - t0) * us_per_tick);
                }
            }
            simd_start.push_back(smin);
            simd_end.push_back(emax);
            simd_spread.push_back(ewmax - ewmin);
        }
        if (c.split) {
            int shown = 0;
            for (auto& kv : simd) {
                if (shown++ == 2) break;
                printf("  SIMD %llx:", (unsigned long long)kv.first);
                for (size_t w : kv.second)
                    printf(" [wg %zu w %zu: %.2f-%.2f]", w / 4, w % 4, (st[8 * w] - t0) * us_per_tick, (st[8 * w + 2] - t0) * us_per_tick);
                printf("\n");
            }
        }
        printf("  within a SIMD, last minus first end of its whole-chunk waves us: p10 %.2f p50 %.2f p90 %.2f\n",
                   pct(simd_spread, .1), pct(simd_spread, .5), pct(simd_spread, .9));
        printf("  SIMDs %zu; waves per SIMD:", simd.size());
        for (auto& kv : wps) printf(" %d x%d", kv.first, kv.second);
        printf("\n  SIMD first start us: p50 %.2f max %.2f; SIMD last end us: p0 %.2f p50 %.2f max %.2f\n",
               pct(simd_start, .5), pct(simd_start, 1), pct(simd_end, 0), pct(simd_end, .5), pct(simd_end, 1));
        // wave-blocks (one wave, both halves, one 32-stage block) per SIMD: batched waves run 2 chunks in lockstep
        // (157 + 2 blocks), split whole-chunk waves 78 + 6 + 2, tail waves about 29
        const double wb = c.split ? (6.0 * 86 + 29) : (double)nst / simd.size() * 159.0;
        printf("  wave-blocks per SIMD %.0f: %.4f us per wave-block at the SIMD median end\n", wb, pct(simd_end, .5) / wb);
    }
    // same-box A/B of the fairness controller on split launches (variants alternate round by round)
    struct Ab { const char* name; KFn hard, soft8; };
    const Ab ab[] = {
        {"product (LDS for 7 waves, fairness at every group head)", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, 0>,
         (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 7, 0>},
        {"at every other group head (round 5's first form)", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, vd::kAblFair2>,
         (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 7, vd::kAblFair2>},
        {"no fairness controller", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, vd::kAblNoFair>,
         (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 7, vd::kAblNoFair>},
        {"LDS laid out for 8 waves per SIMD (5 words per traceback)", (KFn)vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 8, 0>,
         (KFn)vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, true, 8, 0>},
    };
    const int na = sizeof(ab) / sizeof(ab[0]);
    std::vector<std::vector<float>> ah(na), as(na);
    vd::Geom gs = g;
    gs.stats = stats;
    gs.tailWG = (6400u - 256u) / 4u;
    const unsigned sgrid = gs.tailWG + 256u;
    for (int r = 0; r < 3 * reps + 1; r++)
        for (int vi = 0; vi < na; vi++) {
            const int v = (vi + r) % na;
            for (int w = 0; w < 2; w++) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(w ? ab[v].soft8 : ab[v].hard, dim3(sgrid), dim3(256), 0, 0, w ? bS : bH, bO, gs);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (r) (w ? as : ah)[v].push_back(t);
            }
        }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("\nsplit launches, %d rounds, ms (median)\n%-52s %9s %9s\n", 3 * reps, "variant", "hard_b32", "soft8_b16");
    for (int v = 0; v < na; v++) printf("%-52s %9.4f %9.4f\n", ab[v].name, med(ah[v]), med(as[v]));
    return 0;
}
