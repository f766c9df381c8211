// vd_benchab.hip -- timing-only A/B of kernel variants under bench conditions (not part of the product):
// per step one 32M-bit HARD batch (int32 core) and one 32M-bit SOFT8 batch (int16 core), batched launches
// over distinct resident copies (the variant table; split launches in the side sections),
// codeword data (HARD: K=7 codeword through a BSC, p = 0.04; SOFT8: BPSK codeword + Gaussian noise at
// Eb/N0 2 dB, quantised like SoftDecisionPacker(SOFT8)), K steps back to back with the launches grouped
// per workload as bench.py does.  Variants alternate step group by step group, so clock and thermal drift
// hit both alike.  Usage: vd_benchab [groups] [steps per group] [BSC p] [noise scale]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h"
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_segplan.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);

struct Variant { const char* name; KFn hard, soft8; };

int main(int argc, char** argv)
{
    const int groups = argc > 1 ? atoi(argv[1]) : 8, steps = argc > 2 ? atoi(argv[2]) : 10;
    const double pflip = argc > 3 ? atof(argv[3]) : 0.04, nscale = argc > 4 ? atof(argv[4]) : 1.0;
    const size_t N = 32000000;  // coded stages per batch (the bench's 32M-bit input: 16M stages x 2)
    const size_t stages = N / 2 * 2;
    (void)stages;
    // codeword
    std::mt19937 rng(7);
    std::vector<uint8_t> o0(N), o1(N);
    uint32_t reg = 0;
    for (size_t t = 0; t < N; t++) {
        reg = ((reg >> 1) | ((rng() & 1u) << 6)) & 127u;
        o0[t] = __builtin_popcount(reg & 0171u) & 1u;
        o1[t] = __builtin_popcount(reg & 0133u) & 1u;
    }
    // HARD: BSC p = 0.04, 16 stages per word, MSB first
    std::vector<uint32_t> hh(N / 16 + 64, 0u);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (size_t t = 0; t < N; t++) {
        uint32_t a = o0[t] ^ (U(rng) < pflip), b = o1[t] ^ (U(rng) < pflip);
        hh[t / 16] |= (a << (31 - 2 * (t % 16))) | (b << (30 - 2 * (t % 16)));
    }
    // SOFT8: BPSK (bit 0 -> +1), rate 1/2 at Eb/N0 2 dB, scaled by 40000 / 2^8 and clamped like the packer's
    // 8-bit code; 2 stages per word, stage g in the 16-bit half g ^ 1: s0 high byte, s1 low byte
    const double sigma = nscale * std::sqrt(1.0 / (2.0 * 0.5 * std::pow(10.0, 0.2)));
    std::normal_distribution<double> G(0.0, sigma);
    auto q8 = [&](double x) { long v = std::lround(x * 40.0); v = std::min(127L, std::max(-128L, v)); return (uint32_t)(uint8_t)(int8_t)v; };
    std::vector<uint32_t> hs(N / 2 + 64, 0u);
    for (size_t t = 0; t < N; t++) {
        const uint32_t s0 = q8((o0[t] ? -1.0 : 1.0) + G(rng)), s1 = q8((o1[t] ? -1.0 : 1.0) + G(rng));
        const uint32_t half = (s0 << 8) | s1;
        hs[t / 2] |= half << (16 * ((t % 2) ^ 1));
    }
    void *inH, *inS, *out;
    CK(hipMalloc(&inH, hh.size() * 4));
    CK(hipMalloc(&inS, hs.size() * 4));
    CK(hipMalloc(&out, 16u << 20));
    CK(hipMemcpy(inH, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(inS, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
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
    {   // single launches: the product's segment table (round 2's pieces)
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        const std::vector<uint32_t> t = vd::seg_table(4 * cus, vd::kSegPieces);
        uint32_t* tb; CK(hipMalloc(&tb, t.size() * 4));
        CK(hipMemcpy(tb, t.data(), t.size() * 4, hipMemcpyHostToDevice));
        g.seg = tb;
    }
    g.stats = stats;
    const Variant vs[] = {
        {"product (xor-32 by ds_bpermute)", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, 0>, (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, 0>},
        {"LDS stages: exchange V, subtract after", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, vd::kAblPostExchange>, (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, vd::kAblPostExchange>},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    // bench conditions (bench.py): each workload's `steps` batches as one batched launch, every batch its
    // own resident copy of the input (distinct addresses: nothing is served from a previous batch's
    // cache lines), outputs at their own stride
    const size_t strH = (hh.size() * 4 + 255) / 256 * 256, strS = (hs.size() * 4 + 255) / 256 * 256;
    const size_t ostr = (g.packNum * 4 + 255) / 256 * 256;
    void *bH, *bS, *bO;
    CK(hipMalloc(&bH, strH * steps));
    CK(hipMalloc(&bS, strS * steps));
    CK(hipMalloc(&bO, ostr * steps));
    for (int k = 0; k < steps; k++) {
        CK(hipMemcpy((char*)bH + k * strH, inH, hh.size() * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy((char*)bS + k * strS, inS, hs.size() * 4, hipMemcpyDeviceToDevice));
    }
    vd::Geom gh = g, gs = g;
    gh.seg = gs.seg = nullptr;
    gh.nbatch = gs.nbatch = (uint32_t)steps;
    gh.inStride = strH; gs.inStride = strS; gh.outStride = gs.outStride = ostr;
    const unsigned gridB = 1600u * (unsigned)steps;
    hipEvent_t ev[3];
    for (int i = 0; i < 3; i++) CK(hipEventCreate(&ev[i]));
    std::vector<std::vector<float>> th(nv), ts(nv);
    // the variant order rotates from group to group: a fixed order favoured whichever variant ran last
    // (0.5-1 %, profiles/r02/benchab_dpp_forms_8w.log)
    for (int r = 0; r < groups + 1; r++)
        for (int vi = 0; vi < nv; vi++) {
            const int v = (vi + r) % nv;
            CK(hipEventRecord(ev[0]));
            hipLaunchKernelGGL(vs[v].hard, dim3(gridB), dim3(256), 0, 0, bH, bO, gh);
            CK(hipEventRecord(ev[1]));
            hipLaunchKernelGGL(vs[v].soft8, dim3(gridB), dim3(256), 0, 0, bS, bO, gs);
            CK(hipEventRecord(ev[2]));
            CK(hipEventSynchronize(ev[2]));
            float a, b;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            if (r) { th[v].push_back(a / steps); ts[v].push_back(b / steps); }
        }
    // exact twins: every variant's words equal the product kernel's (last batch of the launch)
    {
        std::vector<uint32_t> a(g.packNum), b(g.packNum);
        for (int w = 0; w < 2; w++)
            for (int v = 0; v < nv; v++) {
                CK(hipMemset(bO, 0, ostr * steps));
                if (w == 0) hipLaunchKernelGGL(vs[v].hard, dim3(gridB), dim3(256), 0, 0, bH, bO, gh);
                else hipLaunchKernelGGL(vs[v].soft8, dim3(gridB), dim3(256), 0, 0, bS, bO, gs);
                CK(hipMemcpy(v ? b.data() : a.data(), (char*)bO + (steps - 1) * ostr, g.packNum * 4, hipMemcpyDeviceToHost));
                if (v) {
                    size_t bad = 0;
                    for (size_t k = 0; k < a.size(); k++) bad += a[k] != b[k];
                    printf("exact twin %s %-40.40s: %zu words differ\n", w ? "soft8" : "hard ", vs[v].name, bad);
                }
            }
    }
    // the product kernels with the two workloads on two streams (independent batches overlap their
    // launch tails) against the same launches on one stream, alternating
    {
        hipStream_t sa, sb;
        CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        hipEvent_t e0, e1, eb;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&eb));
        vd::Geom g2 = g;
        void* out2; CK(hipMalloc(&out2, 16u << 20));
        std::vector<float> t1, t2;
        for (int r = 0; r < groups + 1; r++) {
            for (int mode = 0; mode < 2; mode++) {
                CK(hipEventRecord(e0, sa));
                CK(hipStreamWaitEvent(sb, e0, 0));
                for (int k = 0; k < steps; k++) {
                    hipLaunchKernelGGL(vs[0].hard, dim3(1792), dim3(256), 0, sa, inH, out, g);
                    hipLaunchKernelGGL(vs[0].soft8, dim3(1792), dim3(256), 0, mode ? sb : sa, inS, out2, g2);
                }
                CK(hipEventRecord(eb, sb));
                CK(hipStreamWaitEvent(sa, eb, 0));
                CK(hipEventRecord(e1, sa));
                CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) (mode ? t2 : t1).push_back(ms / steps);
            }
        }
        std::sort(t1.begin(), t1.end()); std::sort(t2.begin(), t2.end());
        const double a = t1[t1.size() / 2], b = t2[t2.size() / 2];
        printf("step on one stream %.4f ms (%.1f Gb/s), two streams %.4f ms (%.1f Gb/s)\n", a,
               2.0 * (double)(g.packNum * 32) / (a * 1e-3) / 1e9, b, 2.0 * (double)(g.packNum * 32) / (b * 1e-3) / 1e9);
    }
    // one launch per workload decoding `steps` batches (Geom::nbatch, inputs at stride 0, outputs at stride
    // 0 -- timing only) against `steps` split launches, alternating
    {
        hipEvent_t e0, e1, e2;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
        vd::Geom gb = g;
        gb.seg = nullptr; gb.nbatch = (uint32_t)steps;
        const unsigned gridb = 1600u * (unsigned)steps;
        std::vector<float> th1, ts1, thb, tsb;
        for (int r = 0; r < groups + 1; r++) {
            for (int mode = 0; mode < 2; mode++) {
                CK(hipEventRecord(e0));
                if (mode) hipLaunchKernelGGL(vs[0].hard, dim3(gridb), dim3(256), 0, 0, inH, out, gb);
                else for (int k = 0; k < steps; k++) hipLaunchKernelGGL(vs[0].hard, dim3(1792), dim3(256), 0, 0, inH, out, g);
                CK(hipEventRecord(e1));
                if (mode) hipLaunchKernelGGL(vs[0].soft8, dim3(gridb), dim3(256), 0, 0, inS, out, gb);
                else for (int k = 0; k < steps; k++) hipLaunchKernelGGL(vs[0].soft8, dim3(1792), dim3(256), 0, 0, inS, out, g);
                CK(hipEventRecord(e2));
                CK(hipEventSynchronize(e2));
                float a, b; CK(hipEventElapsedTime(&a, e0, e1)); CK(hipEventElapsedTime(&b, e1, e2));
                if (r) { (mode ? thb : th1).push_back(a / steps); (mode ? tsb : ts1).push_back(b / steps); }
            }
        }
        for (auto* v : {&th1, &ts1, &thb, &tsb}) std::sort(v->begin(), v->end());
        const double h1 = th1[th1.size() / 2], s1 = ts1[ts1.size() / 2], hb = thb[thb.size() / 2], sb = tsb[tsb.size() / 2];
        printf("per batch: split launches hard %.4f soft8 %.4f ms (%.1f Gb/s); batched launch hard %.4f soft8 %.4f ms (%.1f Gb/s)\n",
               h1, s1, 2.0 * (double)(g.packNum * 32) / ((h1 + s1) * 1e-3) / 1e9, hb, sb,
               2.0 * (double)(g.packNum * 32) / ((hb + sb) * 1e-3) / 1e9);
    }
    uint32_t redec = 0;
    CK(hipMemcpy(&redec, stats, 4, hipMemcpyDeviceToHost));
    printf("%d groups x %d steps, BSC p %.3f, noise x %.2f, variants: batched launches, distinct inputs; split re-decodes: %u\n", groups, steps,
           pflip, nscale, redec);
    for (int v = 0; v < nv; v++) {
        std::sort(th[v].begin(), th[v].end());
        std::sort(ts[v].begin(), ts[v].end());
        const double mh = th[v][th[v].size() / 2], ms = ts[v][ts[v].size() / 2];
        printf("%-42s hard %.4f ms  soft8 %.4f ms  step %.4f ms -> %.1f Gb/s (soft8 %.1f)\n", vs[v].name, mh, ms, mh + ms,
               2.0 * (double)(g.packNum * 32) / ((mh + ms) * 1e-3) / 1e9, (double)(g.packNum * 32) / (ms * 1e-3) / 1e9);
    }
    return 0;
}
