// vd_chains.hip -- microbenchmark (not part of the product): the ACS recursion with its table reads, one
// trellis chain per wave at 8 waves per SIMD (the product) against two independent chains per wave at 4
// waves per SIMD (the same 32 chains per CU and LDS per chain), interleaved instruction by instruction.
// Every 6 stages: 4 DPP stages (two-op form) and 2 LDS exchanges (ds_swizzle xor 16, ds_bpermute xor 32);
// the branch metric of every stage from a per-chain LDS table, one ds_read_b64 per two stages, 4 stages
// ahead.  Prints ns per chain-stage per SIMD (lower is better).  Usage: vd_chains [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f2v __attribute__((ext_vector_type(2)));
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

#define DPP1(CTRL) asm volatile("v_sub_f32 %2, %0, %3\n\tv_add_f32 %1, %0, %3\n\ts_nop 0\n\tv_max_f32_dpp %0, %2, %1 " CTRL " row_mask:0xf bank_mask:0xf" : "+v"(V0), "=&v"(a0), "=&v"(b0) : "v"(m0))
#define DPP2(CTRL) asm volatile("v_sub_f32 %4, %0, %6\n\tv_sub_f32 %5, %1, %7\n\tv_add_f32 %2, %0, %6\n\tv_add_f32 %3, %1, %7\n\t" \
                                "v_max_f32_dpp %0, %4, %2 " CTRL " row_mask:0xf bank_mask:0xf\n\tv_max_f32_dpp %1, %5, %3 " CTRL " row_mask:0xf bank_mask:0xf" \
                                : "+v"(V0), "+v"(V1), "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1) : "v"(m0), "v"(m1))

template <int NC>
__global__ __launch_bounds__(256) void chains(float* out, int groups, int tabStride)
{
    extern __shared__ float lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* tab0 = lds + wv * NC * tabStride;
    float* tab1 = tab0 + tabStride;
    for (int i = lane; i < NC * tabStride; i += 64) tab0[i] = (float)((i * 37) % 17) - 8.0f;
    __builtin_amdgcn_s_barrier();
    const int pa5 = 4 * (lane ^ 32);
    float V0 = 12582912.0f + lane, V1 = 12582912.0f + 64 - lane;
    typedef __attribute__((address_space(3))) const volatile f2v* lptr;
    const __attribute__((address_space(3))) char* t0 = (const __attribute__((address_space(3))) char*)tab0 + 8 * (lane & 7);
    const __attribute__((address_space(3))) char* t1 = (const __attribute__((address_space(3))) char*)tab1 + 8 * (lane & 7);
    for (int g = 0; g < groups; g++) {
        f2v e0[96], e1[96];
        auto issue = [&](auto Rc) {
            constexpr int r = decltype(Rc)::value;
            if constexpr ((r / 6) % 2 == 0) {
                e0[r] = *(lptr)(t0 + 8 * r);
                if constexpr (NC == 2) e1[r] = *(lptr)(t1 + 8 * r);
            }
        };
        sfor<4>([&](auto X) { issue(X); });
        sfor<96>([&](auto I) {
            constexpr int r = decltype(I)::value, K = r % 6, Q = (K + 5) % 6;
            constexpr int RP = (r / 6) % 2 ? r - 6 : r;
            const float m0 = (r / 6) % 2 ? e0[RP].y : e0[RP].x;
            const float m1 = NC == 2 ? ((r / 6) % 2 ? e1[RP].y : e1[RP].x) : 0.0f;
            float a0, b0, a1, b1;
            if constexpr (NC == 1) {
                if constexpr (Q == 0) DPP1("quad_perm:[1,0,3,2]");
                else if constexpr (Q == 1) DPP1("quad_perm:[2,3,0,1]");
                else if constexpr (Q == 2) DPP1("row_half_mirror");
                else if constexpr (Q == 3) DPP1("row_ror:8");
                else {
                    const float p0 = Q == 4 ? __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, V0), 0x401F))
                                            : __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(pa5, __builtin_bit_cast(int, V0)));
                    asm volatile("v_add_f32 %1, %0, %3\n\tv_sub_f32 %2, %4, %3\n\tv_max_f32 %0, %1, %2" : "+v"(V0), "=&v"(a0), "=&v"(b0) : "v"(m0), "v"(p0));
                }
            } else {
                if constexpr (Q == 0) DPP2("quad_perm:[1,0,3,2]");
                else if constexpr (Q == 1) DPP2("quad_perm:[2,3,0,1]");
                else if constexpr (Q == 2) DPP2("row_half_mirror");
                else if constexpr (Q == 3) DPP2("row_ror:8");
                else {
                    float p0, p1;
                    if constexpr (Q == 4) {
                        p0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, V0), 0x401F));
                        p1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, V1), 0x401F));
                    } else {
                        p0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(pa5, __builtin_bit_cast(int, V0)));
                        p1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(pa5, __builtin_bit_cast(int, V1)));
                    }
                    asm volatile("v_add_f32 %2, %0, %6\n\tv_add_f32 %3, %1, %7\n\tv_sub_f32 %4, %8, %6\n\tv_sub_f32 %5, %9, %7\n\t"
                                 "v_max_f32 %0, %2, %4\n\tv_max_f32 %1, %3, %5"
                                 : "+v"(V0), "+v"(V1), "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1) : "v"(m0), "v"(m1), "v"(p0), "v"(p1));
                }
            }
            if constexpr (r + 4 < 96) issue(std::integral_constant<int, r + 4>{});
            if constexpr (r % 32 == 31) {  // renormalise (keeps V in range; as the product, once per block)
                const float s0 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, V0)));
                V0 = V0 - s0 + 12582912.0f;
                if constexpr (NC == 2) {
                    const float s1 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, V1)));
                    V1 = V1 - s1 + 12582912.0f;
                }
            }
        });
    }
    out[blockIdx.x * 256 + threadIdx.x] = V0 + (NC == 2 ? V1 : 0.0f);
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int groups = 64;           // 6144 stages per chain
    const int tabStride = 416;       // floats per chain table (the product's 4 x 104 dwords)
    float* out;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    // nc chains per wave, wg workgroups of 4 waves per CU (the LDS per workgroup padded so exactly that many
    // fit): wg waves per SIMD
    auto run = [&](int nc, int wg) {
        const size_t lds = 163840 / wg / 256 * 256;
        const int grid = cus * wg;
        CK(hipEventRecord(e0));
        if (nc == 1) hipLaunchKernelGGL(chains<1>, dim3(grid), dim3(256), lds, 0, out, groups, tabStride);
        else hipLaunchKernelGGL(chains<2>, dim3(grid), dim3(256), lds, 0, out, groups, tabStride);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double cs = (double)wg * nc * groups * 96;  // chain-stages per SIMD
        return ms * 1e6 / cs;
    };
    const int cfg[][2] = {{1, 8}, {1, 7}, {1, 6}, {2, 8}, {2, 7}, {2, 6}, {2, 4}};
    for (int i = 0; i < 2; i++)
        for (auto& c : cfg) run(c[0], c[1]);
    // settled: each configuration runs back to back for ~0.4 s first (the power-limited clock of a long
    // launch sequence), then timed
    for (auto& c : cfg) {
        double t = 0;
        while (t < 0.4e9) t += run(c[0], c[1]) * (double)c[1] * c[0] * groups * 96;
        std::vector<double> a;
        for (int r = 0; r < reps; r++) a.push_back(run(c[0], c[1]));
        std::sort(a.begin(), a.end());
        printf("ns per chain-stage per SIMD: %d chain(s) x %d waves: %.3f\n", c[0], c[1], a[a.size() / 2]);
    }
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)chains<1>)); printf("NC 1: %d VGPRs\n", fa.numRegs);
    CK(hipFuncGetAttributes(&fa, (const void*)chains<2>)); printf("NC 2: %d VGPRs\n", fa.numRegs);
    return 0;
}
