// vd_splitab.hip -- timing-only A/B of single launches (the reference run()'s unit of work, one 32M-bit
// batch per launch): plain (one chunk per wave), "pieces" and "thirds" segment launches (vd_kernel_tg.h
// "segment launches", tables from vd_segplan.h), isolated and back to back, with per-wave clock stamps
// (kAblClock): waves per SIMD, SIMD and XCD end times, clocks.  The modes' decoded words are compared.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <map>
#include <algorithm>
#include "build/abl/vd_kernel_tg.h"  // the product kernel + tools-only ablation bits (tools/abl/gen_abl.py)
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_segplan.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
int main(int argc, char** argv)
{
    const size_t N = 32000000, inBytes = 2 * N / 8;  // HARD
    void *in, *out;
    CK(hipMalloc(&in, inBytes));
    CK(hipMalloc(&out, (16u << 20) + 8192 * 48));
    // a K=7 (0171, 0133) codeword through a binary symmetric channel (flip probability argv[2], default
    // 0.04, about what 2 dB gives hard decisions), HARD format: stage t -> bits 31-2(t%16), 30-2(t%16)
    std::vector<uint32_t> h(inBytes / 4, 0u);
    const double pflip = argc > 2 ? atof(argv[2]) : 0.04;
    const uint32_t thr = (uint32_t)(pflip * 4294967296.0);
    uint32_t x = 12345, reg = 0;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
    for (size_t t = 0; t < N; t++) {
        reg = ((reg >> 1) | ((rnd() & 1u) << 6)) & 127u;
        uint32_t o0 = __builtin_popcount(reg & 0171u) & 1u, o1 = __builtin_popcount(reg & 0133u) & 1u;
        if (rnd() < thr) o0 ^= 1u;
        if (rnd() < thr) o1 ^= 1u;
        h[t / 16] |= (o0 << (31 - 2 * (t % 16))) | (o1 << (30 - 2 * (t % 16)));
    }
    CK(hipMemcpy(in, h.data(), inBytes, hipMemcpyHostToDevice));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    g.scale = 1.0f;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    uint32_t* stats;
    CK(hipMalloc(&stats, 4));
    CK(hipMemset(stats, 0, 4));
    // modes: plain; pieces and thirds with 6 and 3 warm-up blocks per speculative segment
    constexpr int NM = 5;
    const char* names[NM] = {"plain", "pieces", "pieces-w3", "thirds", "thirds-w3"};
    const bool thirdsOf[NM] = {false, false, false, true, true};
    const uint32_t warmOf[NM] = {0, 6, 3, 6, 3};
    uint32_t* tab[NM] = {nullptr};
    unsigned grid[NM] = {1600, 0, 0, 0, 0};
    for (int m = 1; m < NM; m++) {
        std::vector<uint32_t> t = vd::seg_table(4 * cus, thirdsOf[m] ? vd::kSegThirds : vd::kSegPieces);
        if (t.empty()) { printf("no %s table for %d CUs\n", names[m], cus); return 1; }
        CK(hipMalloc(&tab[m], t.size() * 4));
        CK(hipMemcpy(tab[m], t.data(), t.size() * 4, hipMemcpyHostToDevice));
        grid[m] = (unsigned)(t.size() - 1);
    }
    auto launch = [&](KFn f, int m) {
        vd::Geom q = g;
        if (m) { q.seg = tab[m]; q.stats = stats; q.segWarm = warmOf[m]; }
        hipLaunchKernelGGL(f, dim3(grid[m]), dim3(256), 0, 0, in, out, q);
    };
    KFn f0 = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, 0>, fc = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, vd::kAblClock>;
    // the modes decode the same words
    {
        std::vector<uint32_t> a(g.packNum), b(g.packNum);
        for (int m = 0; m < NM; m++) {
            CK(hipMemset(out, 0, g.packNum * 4));
            launch(f0, m);
            CK(hipMemcpy(m ? b.data() : a.data(), out, g.packNum * 4, hipMemcpyDeviceToHost));
            if (m) {
                size_t bad = 0;
                for (size_t k = 0; k < a.size(); k++) bad += a[k] != b[k];
                printf("exact twin %s vs plain: %zu of %zu words differ\n", names[m], bad, a.size());
            }
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<float> t[NM], tb[NM];
    for (int r = 0; r < rounds + 2; r++)
        for (int m = 0; m < NM; m++) {
            CK(hipEventRecord(e0)); launch(f0, m); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) t[m].push_back(ms);
            // back to back (as a caller streams batches): 20 launches between two events
            CK(hipEventRecord(e0)); for (int k = 0; k < 20; k++) launch(f0, m); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) tb[m].push_back(ms / 20);
        }
    for (int m = 0; m < NM; m++) {
        std::sort(t[m].begin(), t[m].end()); std::sort(tb[m].begin(), tb[m].end());
        printf("%-7s isolated median %.4f ms  back to back (20) median %.4f ms per launch -> %.1f Gb/s\n", names[m],
               t[m][t[m].size() / 2], tb[m][tb[m].size() / 2], (double)(N - 64) / (tb[m][tb[m].size() / 2] * 1e-3) / 1e9);
    }
    uint32_t redec = 0; CK(hipMemcpy(&redec, stats, 4, hipMemcpyDeviceToHost));
    printf("re-decoded segments over all segment launches: %u\n", redec);
    for (int m = 1; m < NM; m++) {  // re-decodes per launch by mode
        CK(hipMemset(stats, 0, 4));
        for (int k = 0; k < 10; k++) launch(f0, m);
        CK(hipMemcpy(&redec, stats, 4, hipMemcpyDeviceToHost));
        printf("  %-9s re-decoded segments in 10 launches: %u\n", names[m], redec);
    }
    for (int m = 0; m < NM; m++) {
        const int nw = (int)grid[m] * 4;
        for (int r = 0; r < 3; r++) launch(fc, m);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> d(nw * 6);
        CK(hipMemcpy(d.data(), (char*)out + (16u << 20), d.size() * 8, hipMemcpyDeviceToHost));
        uint64_t r0 = ~0ull, r1 = 0;
        for (int w = 0; w < nw; w++) { if (d[6 * w + 2] == 0) continue; r0 = std::min(r0, d[6 * w + 2]); r1 = std::max(r1, d[6 * w + 3]); }
        std::map<uint32_t, std::vector<int>> bysimd;
        for (int w = 0; w < nw; w++) {
            uint32_t hw = (uint32_t)d[6 * w + 4], xc = (uint32_t)d[6 * w + 5] & 7;
            bysimd[(xc << 16) | (hw & 0xFFF0)].push_back(w);
        }
        std::map<int, int> hist; std::vector<double> simdEnd;
        for (auto& kv : bysimd) {
            hist[(int)kv.second.size()]++;
            double e = 0;
            for (int w : kv.second) e = std::max(e, (d[6 * w + 3] - r0) / 100.0);
            simdEnd.push_back(e);
        }
        std::sort(simdEnd.begin(), simdEnd.end());
        printf("=== %s: span %.1f us, SIMDs %zu, waves/SIMD:", names[m], (r1 - r0) / 100.0, bysimd.size());
        for (auto& kv : hist) printf(" %d:%d", kv.first, kv.second);
        printf("\n    SIMD end us: min %.1f p10 %.1f med %.1f p90 %.1f max %.1f\n", simdEnd[0], simdEnd[simdEnd.size() / 10],
               simdEnd[simdEnd.size() / 2], simdEnd[simdEnd.size() * 9 / 10], simdEnd.back());
        std::vector<double> st, we; std::map<uint32_t, std::vector<double>> xend, xmhz;
        for (int w = 0; w < nw; w++) {
            if (d[6 * w + 2] == 0) continue;
            st.push_back((d[6 * w + 2] - r0) / 100.0);
            we.push_back((d[6 * w + 3] - r0) / 100.0);
            const uint32_t xc = (uint32_t)d[6 * w + 5] & 7;
            xend[xc].push_back((d[6 * w + 3] - r0) / 100.0);
            xmhz[xc].push_back((double)(d[6 * w + 1] - d[6 * w]) / (double)(d[6 * w + 3] - d[6 * w + 2]) * 100.0);
        }
        std::sort(st.begin(), st.end()); std::sort(we.begin(), we.end());
        printf("    wave start us: min %.1f med %.1f max %.1f; wave end us: min %.1f p10 %.1f med %.1f max %.1f\n", st[0],
               st[st.size() / 2], st.back(), we[0], we[we.size() / 10], we[we.size() / 2], we.back());
        for (auto& kv : xend) { auto a = kv.second, b = xmhz[kv.first]; std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
            printf("    XCD %u: wave end med %.1f max %.1f, clock med %.0f MHz\n", kv.first, a[a.size() / 2], a.back(), b[b.size() / 2]); }
    }
    return 0;
}
