// vd_splitab.hip -- timing-only A/B of the split launch (vd_kernel_tg.h "split chunks") against the
// plain launch, interleaved, plus per-wave clock stamps (ABL 32) of both: waves per SIMD and when
// each SIMD's last wave ends.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <map>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
int main(int argc, char** argv)
{
    const size_t N = 32000000, inBytes = 2 * N / 8;  // HARD
    void *in, *out;
    CK(hipMalloc(&in, inBytes));
    CK(hipMalloc(&out, (16u << 20) + 7168 * 48));
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
    auto launch = [&](KFn f, bool split) {
        vd::Geom q = g;
        if (split) { q.nwhole = 6144; q.stats = stats; }
        hipLaunchKernelGGL(f, dim3(split ? 1792 : 1600), dim3(256), 0, 0, in, out, q);
    };
    KFn f0 = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, 0>, f32 = (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, 32>;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<float> t[2];
    for (int r = 0; r < rounds + 2; r++)
        for (int s = 0; s < 2; s++) {
            CK(hipEventRecord(e0)); launch(f0, s); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) t[s].push_back(ms);
        }
    for (int s = 0; s < 2; s++) { std::sort(t[s].begin(), t[s].end());
        printf("%-8s median %.4f ms  min %.4f ms\n", s ? "split" : "plain", t[s][t[s].size() / 2], t[s][0]); }
    // back to back (the reference run()'s unit of work, one launch per batch, as a caller streams batches):
    // per launch wall time between events around 20 launches, against the kernel span the clock stamps of
    // single launches show below; the difference is the launch-to-launch gap
    for (int s = 0; s < 2; s++) {
        std::vector<float> tb;
        for (int r = 0; r < rounds; r++) {
            CK(hipEventRecord(e0)); for (int k = 0; k < 20; k++) launch(f0, s); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); tb.push_back(ms / 20);
        }
        std::sort(tb.begin(), tb.end());
        printf("%-8s back to back (20 launches): median %.4f ms per launch\n", s ? "split" : "plain", tb[tb.size() / 2]);
    }
    uint32_t redec = 0; CK(hipMemcpy(&redec, stats, 4, hipMemcpyDeviceToHost));
    printf("re-decoded split chunks over all split launches: %u\n", redec);
    for (int s = 0; s < 2; s++) {
        const int nw = s ? 7168 : 6400;
        for (int r = 0; r < 3; r++) launch(f32, s);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> d(nw * 6);
        CK(hipMemcpy(d.data(), (char*)out + (16u << 20), d.size() * 8, hipMemcpyDeviceToHost));
        uint64_t r0 = ~0ull, r1 = 0;
        for (int w = 0; w < nw; w++) { if (d[6 * w + 2] == 0) continue; r0 = std::min(r0, d[6 * w + 2]); r1 = std::max(r1, d[6 * w + 3]); }
        std::map<uint32_t, std::vector<int>> bysimd;
        for (int w = 0; w < nw; w++) {
            uint32_t hw = (uint32_t)d[6 * w + 4], xc = (uint32_t)d[6 * w + 5] & 7;
            uint32_t key = (xc << 16) | (hw & 0xFFF0);
            bysimd[key].push_back(w);
        }
        std::map<int, int> hist; std::vector<double> simdEnd; std::map<int, std::vector<double>> endByCount;
        int piecesPerSimdMax = 0; std::map<int, int> pieceHist;
        for (auto& kv : bysimd) {
            hist[(int)kv.second.size()]++;
            double e = 0; int pc = 0;
            for (int w : kv.second) { e = std::max(e, (d[6 * w + 3] - r0) / 100.0); if (s && w >= 6144) pc++; }
            simdEnd.push_back(e); endByCount[(int)kv.second.size()].push_back(e);
            pieceHist[pc]++; piecesPerSimdMax = std::max(piecesPerSimdMax, pc);
        }
        std::sort(simdEnd.begin(), simdEnd.end());
        printf("=== %s: span %.1f us, SIMDs %zu, waves/SIMD:", s ? "split" : "plain", (r1 - r0) / 100.0, bysimd.size());
        for (auto& kv : hist) printf(" %d:%d", kv.first, kv.second);
        printf("\n    SIMD end us: min %.1f p10 %.1f med %.1f p90 %.1f max %.1f\n", simdEnd[0], simdEnd[simdEnd.size() / 10],
               simdEnd[simdEnd.size() / 2], simdEnd[simdEnd.size() * 9 / 10], simdEnd.back());
        for (auto& kv : endByCount) { auto v = kv.second; std::sort(v.begin(), v.end());
            printf("    SIMDs with %d waves: %zu, end med %.1f max %.1f\n", kv.first, v.size(), v[v.size() / 2], v.back()); }
        {   // start skew and clock: wave start times, per-XCD median end and clock (s_memtime / s_memrealtime)
            std::vector<double> st; std::map<uint32_t, std::vector<double>> xend, xmhz;
            for (int w = 0; w < nw; w++) {
                if (d[6 * w + 2] == 0) continue;
                st.push_back((d[6 * w + 2] - r0) / 100.0);
                const uint32_t xc = (uint32_t)d[6 * w + 5] & 7;
                xend[xc].push_back((d[6 * w + 3] - r0) / 100.0);
                xmhz[xc].push_back((double)(d[6 * w + 1] - d[6 * w]) / (double)(d[6 * w + 3] - d[6 * w + 2]) * 100.0);
            }
            std::sort(st.begin(), st.end());
            printf("    wave start us: min %.1f p10 %.1f med %.1f p90 %.1f max %.1f\n", st[0], st[st.size() / 10], st[st.size() / 2],
                   st[st.size() * 9 / 10], st.back());
            for (auto& kv : xend) { auto a = kv.second, b = xmhz[kv.first]; std::sort(a.begin(), a.end()); std::sort(b.begin(), b.end());
                printf("    XCD %u: wave end med %.1f max %.1f, clock med %.0f MHz\n", kv.first, a[a.size() / 2], a.back(), b[b.size() / 2]); }
        }
        if (s) { printf("    piece waves per SIMD:"); for (auto& kv : pieceHist) printf(" %d:%d", kv.first, kv.second); printf("\n");
            std::vector<double> pe; for (int w = 6144; w < nw; w++) pe.push_back((d[6 * w + 3] - r0) / 100.0);
            std::sort(pe.begin(), pe.end()); printf("    piece wave end us: min %.1f med %.1f max %.1f\n", pe[0], pe[pe.size() / 2], pe.back()); }
    }
    return 0;
}
