// vd_mt.h -- the reference harness's channel source on the GPU, bit-exact with its host generators:
// RandBitGen (std::mt19937 + uniform_int_distribution<int>(0,1)), ConvolutionalEncoder(7, 0171, 0133)
// and AddNoise (std::mt19937 + normal_distribution<float>, Marsaglia polar), src/viterbiDF.h:20-95,
// seeded as in src/main.cpp:131-137.  The libstdc++ 11 semantics restated in SURVEY.md §8c:
//   bit              = mt() >> 31
//   u                = float(mt()) / 2^32, clamped to nextafter(1, 0)        (generate_canonical<float>)
//   x, y             = 2u - 1 (one float rounding); reject r2 = x*x + y*y > 1 or == 0
//   draw 2q, 2q + 1  = y*m*sigma + 0, x*m*sigma + 0,  m = sqrtf(-2 logf(r2) / r2)   (q-th accepted pair)
// logf is glibc's (see glibc_logf below); products and sums are single roundings, never contracted.
//
// Parallel generation: each stream is cut into segments of L outputs; segment starts come from the
// jump-ahead of vd_mtjump (a radix-R tree of jumps computed on the GPU: mt_xseq + mt_jump), then one
// workgroup per segment runs the engine (mt_bits, mt_noise).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vd {
namespace mt {

constexpr int kN = 624, kM = 397, kNX = 20592, kQW = 624, kMexp = 19937;
constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    return y ^ (y >> 18);
}
__device__ __forceinline__ uint32_t twist1(uint32_t a, uint32_t b, uint32_t c)  // x_{k+624} from x_k, x_{k+1}, x_{k+397}
{
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
// one twist, workgroup-parallel: cur (624 words, x_n ..) -> nxt (x_{n+624} ..), three dependent phases
__device__ __forceinline__ void twist_wg(const uint32_t* cur, uint32_t* nxt)
{
    const int t = threadIdx.x;
    if (t < 227) nxt[t] = twist1(cur[t], cur[t + 1], cur[t + kM]);
    __syncthreads();
    if (t < 227) nxt[227 + t] = twist1(cur[227 + t], cur[228 + t], nxt[t]);
    __syncthreads();
    if (t < 170) {
        const int i = 454 + t;
        nxt[i] = twist1(cur[i], i == kN - 1 ? nxt[0] : cur[i + 1], nxt[i - 227]);
    }
    __syncthreads();
}

__constant__ double kLogfTab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
// glibc 2.35 logf, x86-64 FMA variant (the one selected on FMA/AVX2 hosts; e_logf.c of the ARM
// optimized-routines, table __logf_data).  Constants read from this image's libm; the restatement
// matches the host logf on every normal float in (0, 1] (tests/test_mt_logf.py).  Valid for normal
// positive finite x (r2 of the polar method is one).
__device__ __forceinline__ float glibc_logf(float x)
{
    const uint32_t ix = __builtin_bit_cast(uint32_t, x);
    if (ix == 0x3f800000u) return 0.0f;
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (tmp >> 19) & 15, k = (int32_t)tmp >> 23;
    const double z = (double)__builtin_bit_cast(float, ix - (tmp & 0xff800000u));
    const double r = __builtin_fma(z, kLogfTab[i][0], -1.0);
    const double y0 = __builtin_fma((double)k, 0x1.62e42fefa39efp-1, kLogfTab[i][1]);
    double y = __builtin_fma(r, 0x1.5575b0be00b6ap-2, -0x1.ffffef20a4123p-2);
    const double r2 = r * r;
    y = __builtin_fma(r2, -0x1.00ea348b88334p-2, y);
    y = __builtin_fma(r2, y, y0 + r);
    return (float)y;
}

// ---------------------------------------------------------------- kernels
// std::mt19937(seed)'s array, before its first output (one thread)
__global__ void mt_seed(uint32_t seed, uint32_t* st)
{
    if (threadIdx.x != 0) return;
    uint32_t v = seed;
    st[0] = v;
    for (int i = 1; i < kN; i++) {
        v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
        st[i] = v;
    }
}
// raw words x_0 .. x_{kNX-1} of the states st[src(b)], src(b) = b * srcStep, into xs[b]
__global__ __launch_bounds__(kThreads) void mt_xseq(const uint32_t* __restrict__ st, uint32_t srcStep,
                                                     uint32_t* __restrict__ xs)
{
    __shared__ uint32_t buf[2][kN];
    const uint32_t* s = st + (size_t)blockIdx.x * srcStep * kN;
    uint32_t* o = xs + (size_t)blockIdx.x * kNX;
    for (int i = threadIdx.x; i < kN; i += kThreads) buf[0][i] = s[i];
    __syncthreads();
    for (int b = 0; b * kN < kNX; b++) {
        const uint32_t* cur = buf[b & 1];
        for (int i = threadIdx.x; i < kN; i += kThreads) o[b * kN + i] = cur[i];
        if ((b + 1) * kN < kNX) twist_wg(cur, buf[(b + 1) & 1]);
    }
}
// jump: st[src + c * dstStep] ^= slice of q_c(A) st[src], for the jump polynomials q_c of one tree
// level (R - 1 of them, kQW words each).  Grid: (nsrc, R - 1, slices), one wave per workgroup: lane t
// accumulates the state words j = t + 64 k (k < 10), so each set coefficient costs one address add,
// five ds_read2st64_b32 and ten XORs for all 624 words; the coefficient loop is scalar.  A slice is sw
// poly words (the host picks sw so that narrow tree levels still launch enough workgroups).
constexpr int kSliceWords = 64;  // largest slice
__global__ __launch_bounds__(64) void mt_jump(const uint32_t* __restrict__ xs, const uint32_t* __restrict__ polys,
                                              uint32_t srcStep, uint32_t dstStep, uint32_t nstates, int sw,
                                              uint32_t* __restrict__ st)
{
    constexpr int NXL = 32 * kSliceWords + 640;
    __shared__ uint32_t xl[NXL];
    const uint32_t src = blockIdx.x * srcStep, dst = src + (blockIdx.y + 1) * dstStep;
    if (dst >= nstates) return;
    const int w0 = blockIdx.z * sw;
    if (w0 >= kQW) return;
    const int nwq = min(sw, kQW - w0);
    const uint32_t* x = xs + (size_t)blockIdx.x * kNX + 32 * w0;
    const int nl = 32 * nwq + 640, nx = min(nl, kNX - 32 * w0);
    for (int i = threadIdx.x; i < nl; i += 64) xl[i] = i < nx ? x[i] : 0u;
    const uint32_t* q = polys + (size_t)blockIdx.y * kQW + w0;
    __syncthreads();
    const int t = threadIdx.x;
    uint32_t acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < nwq; w++) {
        uint32_t bits = __builtin_amdgcn_readfirstlane(q[w]);
        while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t* row = xl + 32 * w + b + t;
#pragma unroll
            for (int k = 0; k < 10; k++) acc[k] ^= row[64 * k];
        }
    }
    uint32_t* o = st + (size_t)dst * kN;
#pragma unroll
    for (int k = 0; k < 10; k++)
        if (t + 64 * k < kN && acc[k]) atomicXor(o + t + 64 * k, acc[k]);
}

// RandBitGen: bit n = output n >> 31 for n < nbits; segment m = outputs [m L, (m + 1) L)
__global__ __launch_bounds__(kThreads) void mt_bits(const uint32_t* __restrict__ st, uint64_t L, uint64_t nbits,
                                                     uint8_t* __restrict__ bits)
{
    __shared__ uint32_t buf[2][kN];
    const uint64_t n0 = (uint64_t)blockIdx.x * L;
    const uint64_t n1 = min(n0 + L, nbits);
    for (int i = threadIdx.x; i < kN; i += kThreads) buf[0][i] = st[(size_t)blockIdx.x * kN + i];
    __syncthreads();
    int p = 0;
    for (uint64_t b = n0; b < n1; b += kN) {
        twist_wg(buf[p], buf[p ^ 1]);
        p ^= 1;
        for (int i = threadIdx.x; i < kN; i += kThreads)
            if (b + i < n1) bits[b + i] = (uint8_t)(temper(buf[p][i]) >> 31);
    }
}

// uniform in [0, 1) as generate_canonical<float, 24>(mt19937)
__device__ __forceinline__ float canon(uint32_t y)
{
    const float u = __fmul_rn((float)y, 0x1p-32f);
    return u >= 1.0f ? 0x1.fffffep-1f : u;
}
// r2 of a polar attempt (accept: 0 < r2 <= 1)
__device__ __forceinline__ bool polar_accept(uint32_t o1, uint32_t o2)
{
    const float x = __fsub_rn(__fmul_rn(2.0f, canon(o1)), 1.0f);
    const float y = __fsub_rn(__fmul_rn(2.0f, canon(o2)), 1.0f);
    const float r2 = __fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y));
    return !(r2 > 1.0f || r2 == 0.0f);
}
// one polar attempt from outputs (u1, u2); returns accepted, and the multiplier m
__device__ __forceinline__ bool polar(uint32_t o1, uint32_t o2, float& x, float& y, float& m)
{
    x = __fsub_rn(__fmul_rn(2.0f, canon(o1)), 1.0f);
    y = __fsub_rn(__fmul_rn(2.0f, canon(o2)), 1.0f);
    const float r2 = __fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y));
    if (r2 > 1.0f || r2 == 0.0f) return false;
    // sqrtf, not __fsqrt_rn: on this toolchain the latter lowers to the 1-ulp v_sqrt_f32, sqrtf to the
    // correctly rounded sequence (v_sqrt_f32 + two fma corrections) that matches the host
    m = sqrtf(__fdiv_rn(__fmul_rn(-2.0f, glibc_logf(r2)), r2));
    return true;
}
// AddNoise's draws.  Attempt a uses outputs 2a, 2a + 1; segment m = attempts [m L/2, (m + 1) L/2).
// PASS 0 counts the accepted attempts of each segment; PASS 1 (after scan_counts) writes draws
// 2q, 2q + 1 = y*m*sigma + 0, x*m*sigma + 0 of the q-th accepted attempt, q < nvalues / 2, into
// values; mt_add_base then adds the BPSK symbols.
template <int PASS>
__global__ __launch_bounds__(kThreads) void mt_noise(const uint32_t* __restrict__ st, uint64_t L,
                                                      uint32_t* __restrict__ counts, uint64_t nvalues, float sigma,
                                                      float* __restrict__ values)
{
    __shared__ uint32_t buf[2][kN];
    __shared__ uint32_t wsum[kThreads / 64 + 1];
    const uint64_t npairs = nvalues / 2;
    for (int i = threadIdx.x; i < kN; i += kThreads) buf[0][i] = st[(size_t)blockIdx.x * kN + i];
    uint64_t q = PASS ? counts[blockIdx.x] : 0;  // accepted attempts before this segment
    if (PASS && q >= npairs) return;  // uniform: nothing of this segment is used
    uint32_t cnt = 0;
    __syncthreads();
    int p = 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t b = 0; b < L; b += kN) {
        twist_wg(buf[p], buf[p ^ 1]);
        p ^= 1;
        // 312 attempts per block (pairs of consecutive outputs), two rounds of 256 threads
        for (int r0 = 0; r0 < kN / 2; r0 += kThreads) {
            const int a = r0 + threadIdx.x;
            const bool in = a < kN / 2 && b + 2 * a < L;
            if constexpr (PASS == 0) {
                cnt += in && polar_accept(temper(buf[p][2 * a]), temper(buf[p][2 * a + 1]));
            } else {
                bool ok = false;
                float x = 0.f, y = 0.f, m = 0.f;
                if (in) ok = polar(temper(buf[p][2 * a]), temper(buf[p][2 * a + 1]), x, y, m);
                const uint64_t bal = __ballot(ok);
                const uint32_t before = __builtin_popcountll(bal & ((1ull << lane) - 1));
                if (lane == 0) wsum[wv] = __builtin_popcountll(bal);
                __syncthreads();
                uint32_t off = 0, tot = 0;
                for (int k = 0; k < kThreads / 64; k++) {
                    off += k < wv ? wsum[k] : 0;
                    tot += wsum[k];
                }
                const uint64_t qq = q + off + before;
                if (ok && qq < npairs) {
                    float2 d;
                    d.x = __fadd_rn(__fmul_rn(__fmul_rn(y, m), sigma), 0.0f);
                    d.y = __fadd_rn(__fmul_rn(__fmul_rn(x, m), sigma), 0.0f);
                    *(float2*)(values + 2 * qq) = d;
                }
                q += tot;
                __syncthreads();
            }
        }
    }
    if constexpr (PASS == 0) {
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
        if (lane == 0) wsum[wv] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t s = 0;
            for (int k = 0; k < kThreads / 64; k++) s += wsum[k];
            counts[blockIdx.x] = s;
        }
    }
}
// exclusive scan of nseg segment counts in place (one workgroup); total at counts[nseg]
__global__ __launch_bounds__(1024) void scan_counts(uint32_t* counts, uint32_t nseg)
{
    __shared__ unsigned long long part[1024];
    const uint32_t per = (nseg + 1023) / 1024, t = threadIdx.x;
    unsigned long long s = 0;
    for (uint32_t i = t * per; i < min(nseg, (t + 1) * per); i++) s += counts[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        unsigned long long run = 0;
        for (int k = 0; k < 1024; k++) {
            const unsigned long long v = part[k];
            part[k] = run;
            run += v;
        }
        counts[nseg] = (uint32_t)(run > 0xFFFFFFFFull ? 0xFFFFFFFFull : run);
    }
    __syncthreads();
    unsigned long long run = part[t];
    for (uint32_t i = t * per; i < min(nseg, (t + 1) * per); i++) {
        const uint32_t v = counts[i];
        counts[i] = (uint32_t)run;
        run += v;
    }
}
// value = base + draw (AddNoise, viterbiDF.h:86-93), or base alone for stddev = +inf (:79-85);
// 1024 values (512 bits) per workgroup, four per thread
template <bool NOISE>
__global__ __launch_bounds__(256) void mt_add_base(const uint8_t* __restrict__ bits, uint64_t nvalues,
                                                   float* __restrict__ values)
{
    __shared__ uint8_t bl[512 + 8];  // bits i0-8 .. i0+511
    const uint64_t v0 = (uint64_t)blockIdx.x * 1024, i0 = v0 / 2, nb = nvalues / 2;
    const int t = threadIdx.x;
    for (int k = t; k < 520; k += 256) {
        const int64_t i = (int64_t)i0 - 8 + k;
        bl[k] = (i >= 0 && (uint64_t)i < nb) ? bits[i] : 0;
    }
    __syncthreads();
    const uint64_t v = v0 + 4 * t;
    if (v >= nvalues) return;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int li = (4 * t + e) / 2 + 8;  // bit (v + e) / 2
        uint32_t r = 0;
#pragma unroll
        for (int d = 0; d < 7; d++) r |= (uint32_t)bl[li - d] << (6 - d);
        o[e] = (__builtin_popcount(r & ((e & 1) ? 0133u : 0171u)) & 1) ? 1.0f : -1.0f;
    }
    if (v + 4 <= nvalues) {
        float4 w = NOISE ? *(const float4*)(values + v) : float4{0.f, 0.f, 0.f, 0.f};
        w.x = NOISE ? __fadd_rn(o[0], w.x) : o[0];
        w.y = NOISE ? __fadd_rn(o[1], w.y) : o[1];
        w.z = NOISE ? __fadd_rn(o[2], w.z) : o[2];
        w.w = NOISE ? __fadd_rn(o[3], w.w) : o[3];
        *(float4*)(values + v) = w;
    } else {
        for (int e = 0; e < 4 && v + e < nvalues; e++) values[v + e] = NOISE ? __fadd_rn(o[e], values[v + e]) : o[e];
    }
}

}  // namespace mt
}  // namespace vd
