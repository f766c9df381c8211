// vd_acs_ubench.hip -- cost of the ACS stage body, built up one feature at a time (timing only).
// Same geometry as the product (1600 workgroups x 4 waves, 5088 stages per wave); results are stored
// so nothing is dead.  F bits: 1 = metric from the LDS table, 2 = LDS exchanges for q=4,5 (else DPP),
// 4 = decision bit + accumulate, 8 = per-block overhead (renormalise, pack word, ring store),
// 16 = one traceback-like dependent LDS chain of 64 reads per 14 blocks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "vd_sc_kernel.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int F>
__global__ __launch_bounds__(256) void acs_kernel(float* out, int nblk)
{
    __shared__ float4 tab_all[4][96];
    __shared__ __attribute__((aligned(256))) uint32_t ring_all[4][15 * 64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* tab = tab_all[wv];
    uint32_t* ring = ring_all[wv];
    const float* tabf = (const float*)tab;
    int L4[6];
    vd::sfor<6>([&](auto K) { constexpr int k = decltype(K)::value; L4[k] = vd::own_label(lane, k) * 4; });
    const int bp_addr = (lane ^ 32) * 4;
    if (lane < 32) for (int i = 0; i < 3; i++) tab[i * 32 + lane] = make_float4(-1.f - lane % 3, -(float)(lane % 2), (float)(lane % 2), 1.f + lane % 3);
    vd::wave_sync();
    float pm = 0.f;
    uint32_t sink = 0;
    uint32_t tbQ = (uint32_t)(wv * 15 * 256 + 256 + lane * 4);
    auto block = [&](auto PHc, int j) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int TB0 = PH / 2;
        float acc = 0.f;
        uint32_t hi16 = 0, word = 0;
        vd::sfor<32>([&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int K = (PH + i) % 6;
            constexpr int Q = (K + 5) % 6;
            const float m = (F & 1) ? tabf[(TB0 * 32 + i) * 4 + (L4[K] >> 2)] : (float)(L4[K] - 6);
            const float oth = (F & 2) ? vd::xchgf<Q>(pm, bp_addr) : vd::xchgf<Q, 2>(pm, bp_addr);
            const float t1 = pm + m, t2 = oth - m;
            pm = fmaxf(t1, t2);
            if constexpr (F & 4) {
                float bit = vd::clamp01(t1 - t2);
                acc = (i == 0 || i == 16) ? bit : __builtin_fmaf(acc, 2.0f, bit);
                if constexpr (i == 15) hi16 = (uint32_t)acc;
                if constexpr (i == 31) word = (hi16 << 16) | (uint32_t)acc;
            }
        });
        if constexpr (F & 8) {
            pm -= __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, pm)));
            word = ~word;
            vd::wave_sync();
            ring[(j % 14) * 64 + lane] = word;
        } else {
            sink ^= word;
        }
        if constexpr (F & 16) {
            if (j % 14 == 13 && lane < 14) {
                vd::wave_sync();
                uint32_t Q = tbQ;
                vd::sfor<64>([&](auto S) {
                    constexpr int s = decltype(S)::value;
                    uint32_t w = *(const uint32_t*)((const char*)ring_all + Q);
                    uint32_t d = (uint32_t)((int)(w << (31 - (s & 31))) >> 31);
                    Q = Q ^ (d & (4u << (s % 6)));
                });
                sink ^= Q;
            }
        }
    };
    for (int j = 0; j < nblk; j += 3) {
        block(std::integral_constant<int, 0>{}, j);
        block(std::integral_constant<int, 2>{}, j + 1);
        block(std::integral_constant<int, 4>{}, j + 2);
    }
    out[blockIdx.x * 256 + threadIdx.x] = pm + (float)sink;
}

int main()
{
    float* out;
    CK(hipMalloc(&out, 1600 * 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    struct V { const char* n; void (*k)(float*, int); };
    V vs[] = {
        {"dpp-only add/sub/max", acs_kernel<0>},
        {"+ LDS metric table", acs_kernel<1>},
        {"+ LDS xchg q4,q5", acs_kernel<3>},
        {"+ decisions", acs_kernel<7>},
        {"+ per-block overhead", acs_kernel<15>},
        {"+ traceback chain", acs_kernel<31>},
        {"dpp-only + decisions", acs_kernel<4>},
        {"table + decisions (dpp xchg)", acs_kernel<5>},
    };
    const int nblk = 159;  // 5088 stages
    for (auto& v : vs) {
        std::vector<float> t;
        for (int r = 0; r < 12; r++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.k, dim3(1600), dim3(256), 0, 0, out, nblk);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        double ms = t[t.size() / 2];
        // per SIMD: 7 waves (6.25 avg) x 5088 stages
        printf("%-32s %.4f ms   %.1f cyc/wave-stage (7 waves/SIMD @2.4GHz)\n", v.n, ms, ms * 1e-3 * 2.4e9 / (7.0 * 5088));
    }
    return 0;
}
