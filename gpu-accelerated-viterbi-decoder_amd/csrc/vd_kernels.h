// vd_kernels.h -- device code of the MI355X (gfx950) Viterbi decoder.
//
// Hot path of the reference (alireza-md93/GPU-Accelerated-Viterbi-Decoder): the fused
// branch-metric + add-compare-select + traceback kernel `viterbi_core` (src/viterbi/viterbi.cu:144-207,
// viterbiBM.cuh, viterbiACS.cuh, viterbiTB.cuh), re-designed for CDNA4 wave64.  Not a translation:
//
//  * State layout.  A wave64 lane holds ONE trellis state (the reference: a warp32 lane holds two).
//    Lane p holds, after stage t, the state rotr6(p, t%6).  Under that rotation the radix-2 butterfly
//    of every stage pairs lanes p and p^(1<<q), q = (t%6+5)%6, so each stage needs one xor-lane
//    exchange: DPP quad_perm (q=0,1), DPP row_half_mirror+quad_perm (q=2), DPP row_ror:8 (q=3),
//    ds_swizzle xor-16 (q=4), ds_bpermute xor-32 (q=5).
//  * Metric cores.  int32 (M_B32): one stream chunk per wave.  int16x2 (M_B16) and fp16x2 (M_FP16):
//    two chunks per wave, chunk 2w in the low and chunk 2w+1 in the high half of every lane, so one
//    v_pk_add/v_pk_sub/v_pk_max advances two chunks.
//  * Survivors.  No register exchange: each stage's decision ("took the exchanged predecessor") is
//    shifted into a per-lane 32-bit word; one word per lane per 32-stage block goes to an LDS ring.
//    Output words are traced back lane-parallel (TB words at a time) in POSITION space, where a
//    traceback step is p ^= d << q -- no state arithmetic.
//  * Branch metrics.  Per 32-stage block, 32 lanes compute the 4 branch metrics of one stage each
//    into an LDS table; every stage each lane reads the metric of its own transition with one
//    ds_read_b32 whose base register depends only on (lane, t%6).
//
// Decode semantics (bit-exact with the reference for every valid option): see DESIGN.md and
// oracle/vd_oracle.c.  Tie rules, in own/exchanged terms: M_B16 -> exchanged wins, M_FP16 -> own
// wins, M_B32 -> exchanged wins except at t%6==0 where the odd predecessor wins (lanes >= 32 keep own).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

namespace vd {

enum Ch : int { HARD = 0, SOFT4 = 1, SOFT8 = 2, SOFT16 = 3, FP32 = 4 };
enum Core : int { B32 = 0, B16 = 1, F16 = 2 };

constexpr int kChunks = 6400;  // reference blocksNum_total = 16*400 (viterbi.cu:19)
constexpr int kTB = 16;        // output words traced back per batch

struct Geom {
    uint64_t packNum;      // output words of bpp bits (getMessageLen / bpp)
    uint64_t availStages;  // stages readable from the input buffer
    uint32_t nchunks;
};

// ---------------------------------------------------------------- compile-time loop helper
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f)
{
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------- trellis helpers
__device__ __forceinline__ int rotr6(int v, int r) { return ((v >> r) | (v << (6 - r))) & 63; }
__device__ __forceinline__ int par7(int v) { return __builtin_popcount(v & 127) & 1; }
// label (o0<<1|o1) of the transition into the state at position p from its OWN predecessor, stage phase k
__device__ __forceinline__ int own_label(int p, int k)
{
    int T = rotr6(p, k), O = rotr6(p, (k + 5) % 6);
    int R = (T << 1) | (O & 1);  // R bit6 = newest input, bit0 = dropped bit (viterbiDF.h:49-60 encoder)
    return (par7(R & 0171) << 1) | par7(R & 0133);
}

// xor-lane exchange along position bit Q (see header)
template <int Q>
__device__ __forceinline__ int xchg(int x, int bp_addr)
{
    if constexpr (Q == 0) return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);   // quad_perm 1,0,3,2
    else if constexpr (Q == 1) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);  // quad_perm 2,3,0,1
    else if constexpr (Q == 2) {
        int y = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);  // row_half_mirror: i -> 7-i
        return __builtin_amdgcn_mov_dpp(y, 0x1B, 0xF, 0xF, true);    // quad_perm 3,2,1,0 => i^4
    } else if constexpr (Q == 3) return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);  // row_ror:8
    else if constexpr (Q == 4) return __builtin_amdgcn_ds_swizzle(x, 0x401F);  // bitmask mode xor 0x10
    else return __builtin_amdgcn_ds_bpermute(bp_addr, x);                     // lane ^ 32
}

// ---------------------------------------------------------------- decision accumulation
// acc = 2*acc + (a CMP b): the compare lands in VCC and v_addc_co_u32 shifts it in as the carry, one
// VALU op per decision instead of the select/or/shift sequence the compiler builds otherwise.
__device__ __forceinline__ uint32_t dec_ge_i32(uint32_t acc, int a, int b)
{
    asm("v_cmp_ge_i32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
    return acc;
}
// low halves (int16)
__device__ __forceinline__ uint32_t dec_ge_i16lo(uint32_t acc, uint32_t a, uint32_t b)
{
    asm("v_cmp_ge_i16 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
    return acc;
}
// high halves (int16), read through SDWA word selects
__device__ __forceinline__ uint32_t dec_ge_i16hi(uint32_t acc, uint32_t a, uint32_t b)
{
    asm("v_cmp_ge_i16_sdwa vcc, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
        : "+v"(acc) : "v"(a), "v"(b) : "vcc");
    return acc;
}
__device__ __forceinline__ uint32_t dec_gt_f16lo(uint32_t acc, uint32_t a, uint32_t b)
{
    asm("v_cmp_gt_f16 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
    return acc;
}
__device__ __forceinline__ uint32_t dec_gt_f16hi(uint32_t acc, uint32_t a, uint32_t b)
{
    asm("v_cmp_gt_f16_sdwa vcc, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
        : "+v"(acc) : "v"(a), "v"(b) : "vcc");
    return acc;
}

// ---------------------------------------------------------------- channel input -> branch metrics
// For stage g: A = BM[label 3] = s0+s1 and B = BM[label 2] = s0-s1 (BM[0] = -A, BM[1] = -B).
// Reference: viterbiBM.cuh:15-153 (formats), viterbi.h:80-87 (values per 32-bit word).
template <int CH>
struct In;

template <>
struct In<HARD> {  // 16 stages per word, stage g -> bits 31-2(g%16) (s0) and 30-2(g%16) (s1)
    using raw_t = uint32_t;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        return g < avail ? __builtin_nontemporal_load(&((const uint32_t*)p)[g >> 4]) : 0u;
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, int& A, int& B)
    {
        int sh = 30 - 2 * (int)(g & 15);
        int r0 = (w >> (sh + 1)) & 1, r1 = (w >> sh) & 1;
        A = r0 + r1 - 1;  // 1 - #mismatches against (1,1)
        B = r0 - r1;      // against (1,0)
    }
};
template <>
struct In<SOFT4> {  // 4 stages per word, byte g%4 from the MSB: high nibble s0, low nibble s1
    using raw_t = uint32_t;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        return g < avail ? __builtin_nontemporal_load(&((const uint32_t*)p)[g >> 2]) : 0u;
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, int& A, int& B)
    {
        int sh = 24 - 8 * (int)(g & 3);
        int s0 = (int)(w << (24 - sh)) >> 28;
        int s1 = (int)(w << (28 - sh)) >> 28;
        A = s0 + s1;
        B = s0 - s1;
    }
};
template <>
struct In<SOFT8> {  // 2 stages per word; the 16-bit half (g^1) holds s0 (high byte), s1 (low byte)
    using raw_t = uint32_t;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        return g < avail ? (uint32_t)__builtin_nontemporal_load(&((const uint16_t*)p)[g ^ 1]) : 0u;
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t, int& A, int& B)
    {
        int s0 = (int)(w << 16) >> 24;
        int s1 = (int)(w << 24) >> 24;
        A = s0 + s1;
        B = s0 - s1;
    }
};
template <>
struct In<SOFT16> {  // 1 stage per word: high 16 bits s0, low 16 bits s1
    using raw_t = uint32_t;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        return g < avail ? __builtin_nontemporal_load(&((const uint32_t*)p)[g]) : 0u;
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t, int& A, int& B)
    {
        int s0 = (int)w >> 16;
        int s1 = (int)(w << 16) >> 16;
        A = s0 + s1;
        B = s0 - s1;
    }
};
template <>
struct In<FP32> {  // 2 floats per stage, clamped to [-8,7]; BM = (int)(+-x0 +- x1) (truncation)
    using raw_t = float2;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 v = g < avail ? __builtin_nontemporal_load(&((const f2*)p)[g]) : f2{0.f, 0.f};
        return make_float2(v.x, v.y);
    }
    static __device__ __forceinline__ void ab(raw_t v, uint64_t, int& A, int& B)
    {
        float x0 = fminf(fmaxf(v.x, -8.0f), 7.0f);
        float x1 = fminf(fmaxf(v.y, -8.0f), 7.0f);
        A = (int)__fadd_rn(x0, x1);
        B = (int)__fsub_rn(x0, x1);
    }
};

// ---------------------------------------------------------------- chunk partition (viterbi.cu:156-165)
struct ChunkRange {
    uint64_t startWord;  // first output word (bpp units)
    uint32_t words;      // output words of this chunk
};
__device__ __forceinline__ ChunkRange chunk_range(const Geom& g, uint32_t c)
{
    ChunkRange r;
    if (c >= g.nchunks) { r.startWord = 0; r.words = 0; return r; }
    uint64_t base = g.packNum / g.nchunks, rem = g.packNum % g.nchunks;
    r.words = (uint32_t)(base + (c < rem ? 1 : 0));
    r.startWord = base * c + (c < rem ? c : rem);
    return r;
}

// ---------------------------------------------------------------- lane-parallel traceback
// Lane traces output word k (0-based within its chunk); block k+2 sits in ring slot l+1, block k+1
// in slot l (slots of slotB bytes, this chunk's 64 decision words at chunkOffB inside a slot).
// Position-space traceback: p_{t-1} = p_t ^ (d_t(p_t) << q_t); the decoded bit of stage t is bit
// q_t of p_{t-1} (the dropped bit of the predecessor state).  Reference: viterbiTB.cuh:4-21.
__device__ __forceinline__ uint32_t traceback_word(const char* ring, int slotB, int chunkOffB, int l, uint64_t k)
{
    const int e6 = (int)((95 + 32 * k) % 6);  // stage phase of the traceback start
    int MK[6], QS[6];
    sfor<6>([&](auto R) {
        constexpr int r = decltype(R)::value;
        int t6 = (e6 - r + 6) % 6;
        int q = (t6 + 5) % 6;
        MK[r] = 4 << q;
        QS[r] = q + 2;
    });
    uint32_t Q = (uint32_t)((l + 1) * slotB + chunkOffB);  // position 0 = state 0
    sfor<32>([&](auto I) {
        constexpr int i = decltype(I)::value;
        uint32_t w = *(const uint32_t*)(ring + Q);
        int d = (int)(w << (31 - i)) >> 31;  // bit i = stage 31-i of the block (stage 95+32k-i)
        Q ^= (uint32_t)(d & MK[i % 6]);
    });
    Q -= (uint32_t)slotB;
    uint32_t word = 0;
    sfor<32>([&](auto I) {
        constexpr int i = decltype(I)::value;
        uint32_t w = *(const uint32_t*)(ring + Q);
        int d = (int)(w << (31 - i)) >> 31;
        Q ^= (uint32_t)(d & MK[(i + 32) % 6]);
        word |= ((Q >> QS[(i + 32) % 6]) & 1u) << i;  // word bit i <-> stage 63+32k-i
    });
    return word;
}

// ================================================================ int32 core: one chunk per wave
template <int CH, int OB>
__global__ __launch_bounds__(64) void vd_decode_b32(const void* __restrict__ in, void* __restrict__ out, Geom geo)
{
    using IN = In<CH>;
    __shared__ int4 tab[32];                     // per stage: BM[0..3]
    __shared__ uint32_t ring[(kTB + 1) * 64];    // decision words, 64 per 32-stage block
    const int lane = threadIdx.x;
    const ChunkRange cr = chunk_range(geo, blockIdx.x);
    if (cr.words == 0) return;
    const uint64_t start = cr.startWord * OB;                      // first stage of the chunk
    const uint32_t S = OB == 32 ? cr.words : (cr.words + 1) / 2;  // 32-bit words traced back
    const uint32_t nblk = S + 2;                                   // 64 warm-up stages + S slides

    int L4[6];
    sfor<6>([&](auto K) {
        constexpr int k = decltype(K)::value;
        L4[k] = own_label(lane, k) * 4;
    });
    const int ebias = lane >= 32 ? 1 : 0;  // M_B32, t%6==0: lanes with p5=1 keep own on ties
    const int bp_addr = (lane ^ 32) * 4;
    const int* tabi = (const int*)tab;

    int pm = 0;
    uint32_t acc = 0;
    uint32_t kb = 0;
    typename IN::raw_t raw = IN::load(in, start + (uint64_t)(lane & 31), geo.availStages);

    for (uint32_t j = 0; j < nblk; j++) {
        if (lane < 32) {
            int A, B;
            IN::ab(raw, start + 32ull * j + lane, A, B);
            tab[lane] = make_int4(-A, -B, B, A);
        }
        if (j + 1 < nblk) raw = IN::load(in, start + 32ull * (j + 1) + (uint64_t)(lane & 31), geo.availStages);
        __syncthreads();

        auto run = [&](auto PHc) {
            constexpr int PH = decltype(PHc)::value;
            sfor<32>([&](auto I) {
                constexpr int i = decltype(I)::value;
                constexpr int K = (PH + i) % 6;
                constexpr int Q = (K + 5) % 6;
                const int m = tabi[i * 4 + (L4[K] >> 2)];
                const int oth = xchg<Q>(pm, bp_addr);
                const int t1 = pm + m, t2 = oth - m;
                pm = t1 > t2 ? t1 : t2;  // the survivor value does not depend on the tie rule
                if constexpr (K == 0) acc = dec_ge_i32(acc, t2 - t1, ebias);
                else acc = dec_ge_i32(acc, t2, t1);
            });
        };
        switch (j % 3) {
        case 0: run(std::integral_constant<int, 0>{}); break;
        case 1: run(std::integral_constant<int, 2>{}); break;
        default: run(std::integral_constant<int, 4>{}); break;
        }
        // decision-neutral renormalisation: keeps |pm| small for SOFT16 over long chunks
        pm -= __builtin_amdgcn_readfirstlane(pm);
        __syncthreads();
        if (j >= 1) ring[(j - 1 - kb) * 64 + lane] = acc;
        if (j >= 2 && (j - 1 - kb == (uint32_t)kTB || j == nblk - 1)) {
            __syncthreads();
            const uint32_t nw = j - 1 - kb;  // words kb .. j-2
            if ((uint32_t)lane < nw) {
                const uint64_t k = kb + lane;
                uint32_t w = traceback_word((const char*)ring, 256, 0, lane, k);
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[cr.startWord + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + cr.startWord;
                    o[2 * k] = (uint16_t)(w >> 16);
                    if (2 * k + 1 < cr.words) o[2 * k + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            __syncthreads();
            ring[lane] = acc;  // block j becomes slot 0 of the next batch
            kb = j - 1;
        }
    }
}

// ================================================================ packed cores: two chunks per wave
template <int CORE>
struct Pk;
template <>
struct Pk<B16> {
    typedef short v2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ uint32_t cvt(int a) { return (uint32_t)(uint16_t)(int16_t)a; }
    static __device__ __forceinline__ v2 as(uint32_t x) { return __builtin_bit_cast(v2, x); }
    static __device__ __forceinline__ uint32_t bits(v2 x) { return __builtin_bit_cast(uint32_t, x); }
    // one ACS for both halves; exchanged predecessor wins ties (viterbiACS.cuh:113-119,216-220)
    static __device__ __forceinline__ uint32_t acs(uint32_t own, uint32_t oth, uint32_t m, uint32_t& a0, uint32_t& a1)
    {
        v2 t1 = as(own) + as(m), t2 = as(oth) - as(m);
        a0 = dec_ge_i16lo(a0, bits(t2), bits(t1));
        a1 = dec_ge_i16hi(a1, bits(t2), bits(t1));
        return bits(__builtin_elementwise_max(t1, t2));
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return bits(as(a) - as(b)); }
};
template <>
struct Pk<F16> {
    typedef _Float16 v2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ uint32_t cvt(int a) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a); }
    static __device__ __forceinline__ v2 as(uint32_t x) { return __builtin_bit_cast(v2, x); }
    static __device__ __forceinline__ uint32_t bits(v2 x) { return __builtin_bit_cast(uint32_t, x); }
    // own predecessor wins ties (__hlt2_mask is strict, viterbiACS.cuh:147-157,250-256)
    static __device__ __forceinline__ uint32_t acs(uint32_t own, uint32_t oth, uint32_t m, uint32_t& a0, uint32_t& a1)
    {
        v2 t1 = as(own) + as(m), t2 = as(oth) - as(m);
        a0 = dec_gt_f16lo(a0, bits(t2), bits(t1));
        a1 = dec_gt_f16hi(a1, bits(t2), bits(t1));
        return bits(__builtin_elementwise_max(t1, t2));
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return bits(as(a) - as(b)); }
};

template <int CH, int CORE, int OB>
__global__ __launch_bounds__(64) void vd_decode_pk(const void* __restrict__ in, void* __restrict__ out, Geom geo)
{
    using IN = In<CH>;
    using P = Pk<CORE>;
    __shared__ uint4 tab[32];                     // per stage: BM[0..3] as (chunk lo, chunk hi) pairs
    __shared__ uint32_t ring[(kTB + 1) * 128];    // per block: 64 words chunk lo, 64 words chunk hi
    const int lane = threadIdx.x;
    const int half = lane >> 5, li = lane & 31;
    const ChunkRange c0 = chunk_range(geo, 2 * blockIdx.x), c1 = chunk_range(geo, 2 * blockIdx.x + 1);
    if (c0.words == 0 && c1.words == 0) return;
    const ChunkRange my = half ? c1 : c0;
    const uint32_t S0 = OB == 32 ? c0.words : (c0.words + 1) / 2;
    const uint32_t S1 = OB == 32 ? c1.words : (c1.words + 1) / 2;
    const uint32_t Smy = half ? S1 : S0;
    const uint32_t nblk = (S0 > S1 ? S0 : S1) + 2;
    const uint64_t start = my.startWord * OB;
    const uint64_t avail = my.words ? geo.availStages : 0;  // an empty chunk reads nothing

    int L4[6];
    sfor<6>([&](auto K) {
        constexpr int k = decltype(K)::value;
        L4[k] = own_label(lane, k) * 4;
    });
    const int bp_addr = (lane ^ 32) * 4;
    const uint32_t* tabu = (const uint32_t*)tab;

    uint32_t pm = 0, acc0 = 0, acc1 = 0;
    uint32_t kb = 0;
    typename IN::raw_t raw = IN::load(in, start + (uint64_t)li, avail);

    for (uint32_t j = 0; j < nblk; j++) {
        {
            int A, B;
            IN::ab(raw, start + 32ull * j + li, A, B);
            uint32_t a = P::cvt(A), b = P::cvt(B), na = P::cvt(-A), nb = P::cvt(-B);
            uint32_t pa = __shfl_xor(a, 32), pb = __shfl_xor(b, 32), pna = __shfl_xor(na, 32), pnb = __shfl_xor(nb, 32);
            if (half == 0)
                tab[li] = make_uint4(na | (pna << 16), nb | (pnb << 16), b | (pb << 16), a | (pa << 16));
        }
        if (j + 1 < nblk) raw = IN::load(in, start + 32ull * (j + 1) + (uint64_t)li, avail);
        __syncthreads();

        auto run = [&](auto PHc) {
            constexpr int PH = decltype(PHc)::value;
            sfor<32>([&](auto I) {
                constexpr int i = decltype(I)::value;
                constexpr int K = (PH + i) % 6;
                constexpr int Q = (K + 5) % 6;
                const uint32_t m = tabu[i * 4 + (L4[K] >> 2)];
                const uint32_t oth = (uint32_t)xchg<Q>((int)pm, bp_addr);
                pm = P::acs(pm, oth, m, acc0, acc1);
            });
        };
        switch (j % 3) {
        case 0: run(std::integral_constant<int, 0>{}); break;
        case 1: run(std::integral_constant<int, 2>{}); break;
        default: run(std::integral_constant<int, 4>{}); break;
        }
        // decision-neutral renormalisation of both halves by the metric of position 0
        pm = P::sub(pm, __builtin_amdgcn_readfirstlane(pm));
        __syncthreads();
        if (j >= 1) {
            ring[(j - 1 - kb) * 128 + lane] = acc0;
            ring[(j - 1 - kb) * 128 + 64 + lane] = acc1;
        }
        if (j >= 2 && (j - 1 - kb == (uint32_t)kTB || j == nblk - 1)) {
            __syncthreads();
            const uint32_t hi = (j - 1) < Smy ? (j - 1) : Smy;  // words kb .. min(j-1,S)-1 of my chunk
            const uint32_t nw = hi > kb ? hi - kb : 0;
            if ((uint32_t)li < nw) {
                const uint64_t k = kb + li;
                uint32_t w = traceback_word((const char*)ring, 512, half * 256, li, k);
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[my.startWord + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + my.startWord;
                    o[2 * k] = (uint16_t)(w >> 16);
                    if (2 * k + 1 < my.words) o[2 * k + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            __syncthreads();
            ring[lane] = acc0;
            ring[64 + lane] = acc1;
            kb = j - 1;
        }
    }
}

}  // namespace vd
