// vd_pack.h -- the reference's SoftDecisionPacker on the GPU (src/viterbiDF.h:98-167).
//
// quant(v*scale) per channel type, bit-exact with the reference's x86 host code:
//   HARD    v > 0 ? 1 : 0
//   SOFT4/8 q = (int)lrintf(v) -- the long is NARROWED to int before saturating to [-8,7] / [-128,127]
//   SOFT16  q = lrintf(v) saturated as a long to [-32768, 32767]
// lrintf rounds half to even and, on x86-64 glibc, returns LONG_MIN ("integer indefinite") for NaN and
// for |v| >= 2^63; the narrowing keeps the low 32 bits.  Codes are packed MSB-first, dataPerPack per
// 32-bit word (32 / 8 / 4 / 2).  FP32 passes v*scale through.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vd {

// (int)lrintf(v) for |v| >= 2^31: the low 32 bits of the 64-bit rounded value (v is integral there;
// v - 2^32 floor(v / 2^32) is exact, a multiple of 256 below 2^32), 0 for NaN and |v| >= 2^63
__device__ __forceinline__ int narrow_lrintf_x86_big(float v)
{
    if (!(__builtin_fabsf(v) < 9.2233720368547758e18f)) return 0;
    const float r = __builtin_fmaf(-4294967296.0f, __builtin_floorf(v * 2.3283064365386963e-10f), v);  // [0, 2^32)
    return (int)(uint32_t)r;
}
// channel code of one scaled value (CH = HARD 0, SOFT4 1, SOFT8 2, SOFT16 3)
template <int CH>
__device__ __forceinline__ uint32_t pack_code(float v)
{
    if constexpr (CH == 0) {
        return v > 0.0f ? 1u : 0u;
    } else if constexpr (CH == 3) {
        // lrintf saturated as a long: |v| < 2^63 rounds and clamps (v_cvt_i32 saturates), NaN and
        // |v| >= 2^63 are LONG_MIN -> -32768
        int q = __builtin_amdgcn_fmed3f(__builtin_rintf(v), -32768.0f, 32767.0f);
        if (!(__builtin_fabsf(v) < 9.2233720368547758e18f)) q = -32768;
        return (uint32_t)q & 0xFFFFu;
    } else {
        constexpr int lo = CH == 1 ? -8 : -128, hi = CH == 1 ? 7 : 127;
        int q;
        if (__builtin_expect(__builtin_fabsf(v) < 2147483648.0f, 1))
            q = (int)__builtin_rintf(v);  // exact: integral and in int range
        else
            q = narrow_lrintf_x86_big(v);
        q = q < lo ? lo : (q > hi ? hi : q);
        return (uint32_t)q & (CH == 1 ? 0xFu : 0xFFu);
    }
}
// signed soft value (or hard bit) the decoder sees for a code (viterbiBM.cuh:15-153)
template <int CH>
__device__ __forceinline__ int code_value(uint32_t c)
{
    if constexpr (CH == 0) return (int)c;
    else if constexpr (CH == 1) return (int)(c << 28) >> 28;
    else if constexpr (CH == 2) return (int)(c << 24) >> 24;
    else return (int)(c << 16) >> 16;
}

// one thread per packed 32-bit word (FP32: per value); n values, missing tail values pack as 0.0f
template <int CH>
__global__ __launch_bounds__(256) void pack_llr(const float* __restrict__ v, uint64_t n, float scale, void* __restrict__ out)
{
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (CH == 4) {
        if (w < n) ((float*)out)[w] = scale == 1.0f ? v[w] : v[w] * scale;
    } else {
        constexpr int per = CH == 0 ? 32 : CH == 1 ? 8 : CH == 2 ? 4 : 2;
        constexpr int width = CH == 0 ? 1 : CH == 1 ? 4 : CH == 2 ? 8 : 16;
        const uint64_t nw = (n + per - 1) / per;
        if (w >= nw) return;
        const uint64_t i0 = w * per;
        uint32_t acc = 0;
        if (i0 + per <= n) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4* p = (const f4*)(v + i0);  // i0 * 4 bytes is a multiple of 16 (per >= 4)
            if constexpr (per == 2) {
                const float2 x = *(const float2*)(v + i0);
                acc = (pack_code<CH>(x.x * scale) << 16) | pack_code<CH>(x.y * scale);
            } else {
#pragma unroll
                for (int q = 0; q < per / 4; q++) {
                    const f4 x = __builtin_nontemporal_load(p + q);
                    acc = (acc << width) | pack_code<CH>(x.x * scale);
                    acc = (acc << width) | pack_code<CH>(x.y * scale);
                    acc = (acc << width) | pack_code<CH>(x.z * scale);
                    acc = (acc << width) | pack_code<CH>(x.w * scale);
                }
            }
        } else {
            for (int j = 0; j < per; j++) {
                const float x = i0 + j < n ? v[i0 + j] : 0.0f;
                acc = (acc << width) | pack_code<CH>(x * scale);
            }
        }
        ((uint32_t*)out)[w] = acc;
    }
}

}  // namespace vd
