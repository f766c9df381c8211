// vd_synth.h -- device-resident synthetic channel source for benchmarks and large-N tests.
//
// Same chain as the reference harness (RandBitGen | ConvolutionalEncoder(7,0171,0133) |
// AddNoise(10^(-snr/5)) | SoftDecisionPacker(type, 40000), viterbiDF.h:20-167), but generated on the
// GPU from a counter-based hash so each rank can fill its own 32M-bit batch in HBM in well under a
// millisecond.  The random streams are NOT the reference's mt19937 streams (the host harness in
// vd_host.cpp reproduces those); decode parity never depends on which source made the input.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vd {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint32_t synth_bit(uint64_t seed, int64_t i)
{
    return i < 0 ? 0u : (uint32_t)(splitmix64(seed * 0x632BE59BD9B4E019ull + (uint64_t)i) >> 63);
}
__device__ __forceinline__ float synth_normal(uint64_t seed, uint64_t v)
{
    uint64_t h = splitmix64((seed ^ 0xD1B54A32D192ED03ull) * 0x9E3779B97F4A7C15ull + v);
    float u1 = ((uint32_t)(h >> 40) + 1u) * (1.0f / 16777216.0f);  // (0,1]
    float u2 = (uint32_t)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);   // [0,1)
    return sqrtf(-2.0f * __logf(u1)) * __cosf(6.2831853071795864f * u2);
}
// encoded value v (0..2N-1) of the rate-1/2 K=7 code, out0 (0171) first (viterbiDF.h:49-60)
__device__ __forceinline__ uint32_t synth_code(uint64_t seed, uint64_t v)
{
    int64_t i = (int64_t)(v >> 1);
    uint32_t r = 0;  // bit6 = newest input
#pragma unroll
    for (int d = 0; d < 7; d++) r |= synth_bit(seed, i - d) << (6 - d);
    uint32_t poly = (v & 1) ? 0133u : 0171u;
    return __builtin_popcount(r & poly) & 1u;
}
__device__ __forceinline__ float synth_value(uint64_t seed, uint64_t v, float sigma, int noiseless)
{
    float base = synth_code(seed, v) ? 1.0f : -1.0f;
    return noiseless ? base : base + synth_normal(seed, v) * sigma;
}
template <int CH>
__device__ __forceinline__ uint32_t synth_quant(float v)
{
    if constexpr (CH == 0) return v > 0.0f ? 1u : 0u;
    else {
        constexpr int lo = CH == 1 ? -8 : CH == 2 ? -128 : -32768;
        constexpr int hi = CH == 1 ? 7 : CH == 2 ? 127 : 32767;
        constexpr uint32_t mask = CH == 1 ? 0xFu : CH == 2 ? 0xFFu : 0xFFFFu;
        int q = (int)rintf(fminf(fmaxf(v, -1.0e9f), 1.0e9f));
        q = q < lo ? lo : (q > hi ? hi : q);
        return (uint32_t)q & mask;
    }
}

// one thread per packed 32-bit word (FP32: per value); bits_out written by the first pass
template <int CH>
__global__ void synth_pack(uint64_t seed, uint64_t nvalues, float sigma, int noiseless, void* packed)
{
    constexpr int per = CH == 0 ? 32 : CH == 1 ? 8 : CH == 2 ? 4 : CH == 3 ? 2 : 1;
    constexpr int width = CH == 0 ? 1 : CH == 1 ? 4 : CH == 2 ? 8 : 16;
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nwords = nvalues / per;
    if (w >= nwords) return;
    if constexpr (CH == 4) {
        ((float*)packed)[w] = synth_value(seed, w, sigma, noiseless) * 40000.0f;
    } else {
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < per; j++) {
            float v = synth_value(seed, w * per + j, sigma, noiseless) * 40000.0f;
            acc = (acc << width) | synth_quant<CH>(v);
        }
        ((uint32_t*)packed)[w] = acc;
    }
}

__global__ void synth_bits(uint64_t seed, uint64_t n, uint8_t* bits)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) bits[i] = (uint8_t)synth_bit(seed, (int64_t)i);
}

}  // namespace vd
