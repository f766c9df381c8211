// vd_abtest.hip -- timing-only A/B of the current tagged kernel against the previous commit's copy
// (tools/vd_tg_prev.h, namespace vd::old), interleaved in one process on identical random inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h"
#include "vd_tg_prev.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using KFn = void (*)(const void*, void*, vd::Geom);
struct Var { const char* name; KFn fn; };
int main(int argc, char** argv)
{
    const size_t N = 32000000, inBytes = 2 * N * 4;
    void *in, *out;
    CK(hipMalloc(&in, inBytes));
    CK(hipMalloc(&out, 16u << 20));
    std::vector<uint32_t> h(inBytes / 4);
    uint32_t x = 12345;
    for (auto& w : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; w = x; }
    CK(hipMemcpy(in, h.data(), inBytes, hipMemcpyHostToDevice));
    vd::Geom g;
    g.packNum = (N - 64) / 32;
    g.nchunks = 6400;
    g.availStages = N;
    CK(hipMalloc(&g.fair, vd::kFairBoardWords * 4));
    CK(hipMemset(g.fair, 0xFF, vd::kFairBoardWords * 4));
    std::vector<Var> v = {
        {"new hard/b32", (KFn)vd::vd_decode_tg<vd::HARD, vd::B32, 32, 0>}, {"old hard/b32", (KFn)vd::old::vd_decode_tg<vd::HARD, vd::B32, 32, 0>},
        {"new soft8/b16", (KFn)vd::vd_decode_tg<vd::SOFT8, vd::B16, 32, 0>}, {"old soft8/b16", (KFn)vd::old::vd_decode_tg<vd::SOFT8, vd::B16, 32, 0>},
        {"new fp32/f16", (KFn)vd::vd_decode_tg<vd::FP32, vd::F16, 32, 0>}, {"old fp32/f16", (KFn)vd::old::vd_decode_tg<vd::FP32, vd::F16, 32, 0>}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<std::vector<float>> t(v.size());
    for (int r = 0; r < rounds + 2; r++)
        for (size_t i = 0; i < v.size(); i++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v[i].fn, dim3(1600), dim3(256), 0, 0, in, out, g);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t[i].push_back(ms);
        }
    for (size_t i = 0; i < v.size(); i++) {
        std::sort(t[i].begin(), t[i].end());
        printf("%-16s median %.4f ms  min %.4f ms  -> %.1f Gb/s\n", v[i].name, t[i][t[i].size() / 2], t[i][0],
               (double)(N - 64) / (t[i][t[i].size() / 2] * 1e-3) / 1e9);
    }
    return 0;
}
