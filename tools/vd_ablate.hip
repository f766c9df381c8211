// vd_ablate.hip -- timing-only ablation driver for the decode kernels (not part of the product).
// Builds every ABL variant of the two headline kernels and times them interleaved in one process
// (cdna_hip_programming.md 5.4 rule 24) on random 32M-bit inputs.  Outputs of ABL != 0 are wrong.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>
#include <string>
#include "build/abl/vd_kernel_tg.h"  // the product kernel + tools-only ablation bits (tools/abl/gen_abl.py)

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using KFn = void (*)(const void*, void*, vd::Geom);
struct Var { const char* name; KFn fn; int grid; int block = 256; int ref = -1; };  // ref: exact twin

template <int ABL> void tgb(std::vector<Var>& v, const char* n) { v.push_back({n, (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, ABL>, 1600}); }
template <int ABL> void tgs(std::vector<Var>& v, const char* n) { v.push_back({n, (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, ABL>, 1600}); }
template <int ABL> void tgf(std::vector<Var>& v, const char* n) { v.push_back({n, (KFn)vd::vd_decode_tg<vd::FP32, vd::F16, 32, ABL>, 1600}); }
template <int ABL> void tgi(std::vector<Var>& v, const char* n) { v.push_back({n, (KFn)vd::vd_decode_tg<vd::SOFT16, vd::B32, 32, ABL>, 1600}); }

int main(int argc, char** argv)
{
    const size_t N = 32000000, inputNum = 2 * N;
    const size_t inBytes = inputNum * 4;  // FP32 (largest)
    // argv[3] = nb > 1: batched launches (bench conditions) of nb batches, each its own copy of the random
    // input (distinct addresses); only the vd_decode_tg variants run then
    const int nb = argc > 3 ? std::max(1, atoi(argv[3])) : 1;
    const size_t outStride = (size_t)4 << 20;
    void *in, *out;
    CK(hipMalloc(&in, inBytes * nb));
    CK(hipMalloc(&out, std::max((size_t)(16u << 20) + 6400 * 48, outStride * nb)));
    std::vector<uint32_t> h(inBytes / 4);
    uint32_t x = 12345;
    for (auto& w : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; w = x; }
    for (int b = 0; b < nb; b++) CK(hipMemcpy((char*)in + b * inBytes, h.data(), inBytes, hipMemcpyHostToDevice));
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    if (nb > 1) { g.nbatch = (uint32_t)nb; g.inStride = inBytes; g.outStride = outStride; }
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    std::vector<Var> v;
    // component ablations of the product kernels (vd_kernel_tg.h kAbl*): what each part of the kernel
    // costs, and the ACS-only instruction-mix ceiling bench.py quotes
    tgb<0>(v, "tg hard/b32 full"); tgb<vd::kAblNoTraceback>(v, "tg hard/b32 -traceback");
    tgb<vd::kAblNoLoads>(v, "tg hard/b32 -loads"); tgb<vd::kAblNoFair>(v, "tg hard/b32 -fairness");
    tgb<vd::kAblNoTabReads>(v, "tg hard/b32 -tabreads"); tgb<vd::kAblNoReadout>(v, "tg hard/b32 -readout");
    tgb<vd::kAblNoTabBuild>(v, "tg hard/b32 -tabbuild");
    tgb<vd::kAblAcsOnly>(v, "tg hard/b32 ACS only");
    tgs<0>(v, "tg soft8/b16 full"); tgs<vd::kAblNoTraceback>(v, "tg soft8/b16 -traceback");
    tgs<vd::kAblNoLoads>(v, "tg soft8/b16 -loads"); tgs<vd::kAblNoFair>(v, "tg soft8/b16 -fairness");
    tgs<vd::kAblNoTabReads>(v, "tg soft8/b16 -tabreads"); tgs<vd::kAblNoReadout>(v, "tg soft8/b16 -readout");
    tgs<vd::kAblNoTabBuild>(v, "tg soft8/b16 -tabbuild");
    tgs<vd::kAblAcsOnly>(v, "tg soft8/b16 ACS only");
    tgi<0>(v, "tg soft16/b32 full"); tgi<vd::kAblNoTabBuild>(v, "tg soft16/b32 -tabbuild");
    tgi<vd::kAblNoReadout>(v, "tg soft16/b32 -readout"); tgi<vd::kAblNoTraceback>(v, "tg soft16/b32 -traceback");
    tgi<vd::kAblNoTabReads>(v, "tg soft16/b32 -tabreads"); tgi<vd::kAblAcsOnly>(v, "tg soft16/b32 ACS only");
    tgf<0>(v, "tg fp32/f16 full"); tgf<vd::kAblNoTabBuild>(v, "tg fp32/f16 -tabbuild");
    tgf<vd::kAblNoLoads>(v, "tg fp32/f16 -loads"); tgf<vd::kAblAcsOnly>(v, "tg fp32/f16 ACS only");
    // balanced grid (every SIMD the same waves): 6144 chunks; the rate is per 6144-chunk launch
    v.push_back({"tg soft8/b16 6144 chunks", (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, 0>, 1536});
    // variants that must decode exactly like the full kernel: outputs compared word for word below
    auto twin = [&](const char* a, const char* b) {
        int ia = -1, ib = -1;
        for (size_t i = 0; i < v.size(); i++) { if (!strcmp(v[i].name, a)) ia = (int)i; if (!strcmp(v[i].name, b)) ib = (int)i; }
        if (ia >= 0 && ib >= 0) v[ib].ref = ia;
    };
    // optional filter (argv[2]): comma-separated name substrings; a kept variant keeps its exact twin
    if (argc > 2) {
        std::vector<int> keep(v.size(), 0);
        std::string f = argv[2];
        for (size_t i = 0; i < v.size(); i++) {
            size_t a = 0;
            while (a <= f.size()) {
                size_t b = f.find(',', a); if (b == std::string::npos) b = f.size();
                const std::string k = f.substr(a, b - a);
                if (!k.empty() && strstr(v[i].name, k.c_str())) keep[i] = 1;
                a = b + 1;
            }
        }
        for (size_t i = 0; i < v.size(); i++) if (keep[i] && v[i].ref >= 0) keep[v[i].ref] = 1;
        std::vector<Var> w; std::vector<int> idx(v.size(), -1);
        for (size_t i = 0; i < v.size(); i++) if (keep[i]) { idx[i] = (int)w.size(); w.push_back(v[i]); }
        for (auto& x : w) if (x.ref >= 0) x.ref = idx[x.ref];
        v.swap(w);
    }
    if (nb > 1) {  // batched: vd_decode_tg variants only, grid x nb, times per batch
        std::vector<Var> w; std::vector<int> idx(v.size(), -1);
        for (size_t i = 0; i < v.size(); i++)
            if (!strncmp(v[i].name, "tg ", 3) && strstr(v[i].name, "6144") == nullptr) { idx[i] = (int)w.size(); w.push_back(v[i]); }
        for (auto& y : w) { y.ref = y.ref >= 0 ? idx[y.ref] : -1; y.grid *= nb; }
        v.swap(w);
        printf("batched launches: %d batches per launch, distinct input copies; times per batch\n", nb);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<std::vector<float>> t(v.size());
    for (int r = 0; r < rounds + 2; r++)
        for (size_t i = 0; i < v.size(); i++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v[i].fn, dim3(v[i].grid), dim3(v[i].block), 0, 0, in, out, g);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t[i].push_back(ms / nb);
        }
    for (size_t i = 0; i < v.size(); i++) {
        std::sort(t[i].begin(), t[i].end());
        printf("%-26s median %.4f ms  min %.4f ms  -> %.1f Gb/s\n", v[i].name, t[i][t[i].size() / 2], t[i][0],
               (double)(N - 64) / (t[i][t[i].size() / 2] * 1e-3) / 1e9);
    }
    // exact twins: the same decoded words as the full kernel
    {
        const size_t nb = g.packNum * 4;
        std::vector<uint32_t> a(nb / 4), b(nb / 4);
        for (size_t i = 0; i < v.size(); i++) {
            if (v[i].ref < 0) continue;
            const Var& r = v[v[i].ref];
            CK(hipMemset(out, 0, nb));
            hipLaunchKernelGGL(r.fn, dim3(r.grid), dim3(r.block), 0, 0, in, out, g);
            CK(hipMemcpy(a.data(), out, nb, hipMemcpyDeviceToHost));
            CK(hipMemset(out, 0, nb));
            hipLaunchKernelGGL(v[i].fn, dim3(v[i].grid), dim3(v[i].block), 0, 0, in, out, g);
            CK(hipMemcpy(b.data(), out, nb, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t k = 0; k < a.size(); k++) bad += a[k] != b[k];
            printf("exact twin %-30s vs %-22s: %zu of %zu words differ\n", v[i].name, r.name, bad, a.size());
        }
    }
    // per-wave clock stamps of the full kernel (kAblClock)
    if (argc <= 2 && nb == 1)  // not with a filter
    for (KFn f : {(KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, vd::kAblClock>}) {
        printf("=== tg full\n");
        for (int r = 0; r < 3; r++) hipLaunchKernelGGL(f, dim3(1600), dim3(256), 0, 0, in, out, g);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> d(6400 * 6);
        CK(hipMemcpy(d.data(), (char*)out + (16u << 20), d.size() * 8, hipMemcpyDeviceToHost));
        uint64_t c0 = ~0ull, r0 = ~0ull, r1 = 0; std::vector<double> cyc, mhz, startus, endus;
        for (int w = 0; w < 6400; w++) { r0 = std::min(r0, d[6 * w + 2]); r1 = std::max(r1, d[6 * w + 3]); }
        std::vector<int> per_simd(8 * 64 * 4 * 4 * 4, 0);
        for (int w = 0; w < 6400; w++) {
            const uint64_t* e = &d[6 * w];
            cyc.push_back((double)(e[1] - e[0]));
            mhz.push_back((double)(e[1] - e[0]) / (double)(e[3] - e[2]) * 100.0);
            startus.push_back((e[2] - r0) / 100.0); endus.push_back((e[3] - r0) / 100.0);
        }
        auto pr = [](const char* n, std::vector<double> v) { std::sort(v.begin(), v.end());
            printf("%-22s min %.1f  p10 %.1f  med %.1f  p90 %.1f  max %.1f\n", n, v[0], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back()); };
        printf("kernel span (realtime) %.1f us\n", (r1 - r0) / 100.0);
        pr("wave cycles", cyc); pr("clock MHz", mhz); pr("wave start us", startus); pr("wave end us", endus);
        printf("cycles/stage (median wave, 5088 stages): %.2f\n", [&]{ auto v = cyc; std::sort(v.begin(), v.end()); return v[v.size()/2] / 5088.0; }());
        // waves per (xcc, se, cu, simd) from HW_ID: wave_id[3:0] simd_id[5:4] cu_id[11:8] sh_id[12] se_id[15:13]
        std::vector<int> cnt(8 * 8 * 2 * 16 * 4, 0);
        for (int w = 0; w < 6400; w++) {
            uint32_t h = (uint32_t)d[6 * w + 4], x = (uint32_t)d[6 * w + 5] & 7;
            int simd = (h >> 4) & 3, cu = (h >> 8) & 15, sh = (h >> 12) & 1, se = (h >> 13) & 7;
            cnt[(((x * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd]++;
        }
        std::vector<int> hist(16, 0); int used = 0;
        for (int c : cnt) if (c) { used++; hist[std::min(c, 15)]++; }
        std::vector<uint32_t> fb(vd::kFairBoardWords);
        CK(hipMemcpy(fb.data(), g.fair, fb.size() * 4, hipMemcpyDeviceToHost));
        int nz = 0; for (auto x : fb) nz += x != vd::kFairEmpty;
        printf("progress board slots still taken after run: %d\n", nz);
        printf("SIMDs used %d; waves-per-SIMD histogram:", used);
        for (int i = 0; i < 16; i++) if (hist[i]) printf(" %d:%d", i, hist[i]);
        printf("\n");
    }
    return 0;
}
