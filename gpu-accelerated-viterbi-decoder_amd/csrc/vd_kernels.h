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
//  * Metric cores.  Every core (M_B32, M_B16, M_FP16) runs in exact-integer fp32, one chunk per wave;
//    the metric type only selects the tie rule (see "fp32 core" below).  This file holds the shared
//    helpers and vd_decode_sc, the untagged kernel that SOFT16 uses; vd_kernel_tg.h holds the tagged
//    kernel every other input format uses.
//  * Survivors.  No register exchange: each stage's decision ("took the exchanged predecessor") is
//    the sign bit of a candidate difference, accumulated into one word per lane per 32-stage block
//    that goes to an LDS ring.  Output words are traced back lane-parallel (TB words at a time) in
//    POSITION space, where a traceback step is p ^= d << q -- no state arithmetic.
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
constexpr int kTBsc = 14;      // fp32 kernel: 14 words per batch keeps 7 four-wave workgroups per CU

struct Geom {
    uint64_t packNum;      // output words of bpp bits (getMessageLen / bpp)
    uint64_t availStages;  // stages readable from the input buffer
    uint32_t nchunks;
    uint32_t* fair;        // per-SIMD progress board (kFairBoardWords, empty at rest) or null
    float scale;           // LLR input (channel ids 8 + base): SoftDecisionPacker scale, else unused
    // split launch (vd_kernel_tg.h "split chunks"): chunks >= nwhole are decoded as kWaves pieces, one
    // workgroup each; 0 = every chunk whole
    uint32_t nwhole = 0;
    float* spec = nullptr;       // [chunk - nwhole][kSplitVecs][64] piece boundary metric vectors
    uint32_t* stats = nullptr;   // count of split pieces re-decoded (or null)
};
// Progress board of the fairness controller: per SIMD slot (XCC, SE, SH, CU, SIMD from the hardware
// wave id) kFairWaves 32-bit words, one per hardware wave slot of that SIMD (HW_ID.WAVE_ID): the blocks
// the wave in that slot has started, kFairEmpty when the slot is free.  Only issue priority depends on
// it; a collision (another kernel on the same SIMD) only perturbs priorities.
constexpr int kFairSlots = 8 * 8 * 2 * 16 * 4;
constexpr int kFairWaves = 16;
constexpr size_t kFairBoardWords = (size_t)kFairSlots * kFairWaves;
constexpr uint32_t kFairEmpty = 0xFFFFFFFFu;

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
template <int Q, int ABL = 0>
__device__ __forceinline__ int xchg(int x, int bp_addr)
{
    if constexpr ((ABL & 2) && Q >= 4) return __builtin_amdgcn_mov_dpp(x, 0x124, 0xF, 0xF, true);
    else if constexpr (Q == 0) return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);   // quad_perm 1,0,3,2
    else if constexpr (Q == 1) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);  // quad_perm 2,3,0,1
    else if constexpr (Q == 2) {
        int y = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);  // row_half_mirror: i -> 7-i
        return __builtin_amdgcn_mov_dpp(y, 0x1B, 0xF, 0xF, true);    // quad_perm 3,2,1,0 => i^4
    } else if constexpr (Q == 3) return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);  // row_ror:8
    else if constexpr (Q == 4) return __builtin_amdgcn_ds_swizzle(x, 0x401F);  // bitmask mode xor 0x10
    else return __builtin_amdgcn_ds_bpermute(bp_addr, x);                     // lane ^ 32
}

// ---------------------------------------------------------------- decision bits
// A stage's decision is the sign of a candidate difference, shifted into a per-lane word with pure
// VGPR ops (v_alignbit_b32 / v_pk_lshrrev_b16 + v_bfi_b32).  Routing it through VCC (v_cmp + v_addc)
// was measured 2.6x slower on gfx950: the VALU->SGPR->VALU dependency serialises every stage.
// ---------------------------------------------------------------- channel input -> branch metrics
// For stage g: A = BM[label 3] = s0+s1 and B = BM[label 2] = s0-s1 (BM[0] = -A, BM[1] = -B).
// Reference: viterbiBM.cuh:15-153 (formats), viterbi.h:80-87 (values per 32-bit word).
template <int CH>
struct In;

// Loads are unconditional (clamped address) so the compiler can count them with vmcnt(N) across
// the prefetch distance; stages past the input (only reachable by the O_B16 overrun and by the
// shorter chunk of a packed pair) read as zero words in ab().
__device__ __forceinline__ uint64_t clampg(uint64_t g, uint64_t avail) { return g < avail ? g : avail - 1; }

template <>
struct In<HARD> {  // 16 stages per word, stage g -> bits 31-2(g%16) (s0) and 30-2(g%16) (s1)
    using raw_t = uint32_t;
    static __device__ __forceinline__ raw_t load(const void* p, uint64_t g, uint64_t avail)
    {
        return __builtin_nontemporal_load(&((const uint32_t*)p)[clampg(g, avail) >> 4]);
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, uint64_t avail, int& A, int& B)
    {
        w = g < avail ? w : 0u;
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
        return __builtin_nontemporal_load(&((const uint32_t*)p)[clampg(g, avail) >> 2]);
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, uint64_t avail, int& A, int& B)
    {
        w = g < avail ? w : 0u;
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
        uint64_t c = clampg(g, avail);
        return (uint32_t)__builtin_nontemporal_load(&((const uint16_t*)p)[c ^ 1]);
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, uint64_t avail, int& A, int& B)
    {
        w = g < avail ? w : 0u;
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
        return __builtin_nontemporal_load(&((const uint32_t*)p)[clampg(g, avail)]);
    }
    static __device__ __forceinline__ void ab(raw_t w, uint64_t g, uint64_t avail, int& A, int& B)
    {
        w = g < avail ? w : 0u;
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
        f2 v = __builtin_nontemporal_load(&((const f2*)p)[clampg(g, avail)]);
        return make_float2(v.x, v.y);
    }
    static __device__ __forceinline__ void ab(raw_t v, uint64_t g, uint64_t avail, int& A, int& B)
    {
        if (g >= avail) v = make_float2(0.f, 0.f);
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


// ---------------------------------------------------------------- traceback, fp32 kernel ring format
// ring: per block slot 64 words (lane p), bit 31-s = take-bit of stage s.  `Q` is a byte offset from
// the (256-B aligned) ring array holding base + 4p, so a step is one ds_read at Q and one bitop3
// (Q ^= d & MK), and the ds_read address needs no add.  The decoded bits are not extracted per step:
// with b_t = bit q_t of p_{t-1} and p's bit q_t untouched between stages t+5 and t, b_t = b_{t+6} ^ d_t,
// so the word is the stride-6 prefix XOR of the collected decision bits D, seeded by the six bits
// of the position reached at the end of the convergence phase.
__device__ __forceinline__ uint32_t bitop3_xor_and(uint32_t a, uint32_t b, uint32_t c)
{
    return a ^ (b & c);  // v_bitop3_b32
}
__device__ __forceinline__ uint32_t traceback_word_sc(const char* ringb, uint32_t Q, uint64_t k)
{
    const int e6 = (int)((95 + 32 * k) % 6);  // stage phase of the traceback start
    uint32_t MK[6];
    sfor<6>([&](auto R) {
        constexpr int r = decltype(R)::value;
        int q = ((e6 - r + 6) % 6 + 5) % 6;
        MK[r] = 4u << q;
    });
    // convergence: block k+2, stages 95+32k .. 64+32k
    sfor<32>([&](auto I) {
        constexpr int i = decltype(I)::value;
        uint32_t w = *(const uint32_t*)(ringb + Q);
        uint32_t d = (uint32_t)((int)(w << (31 - i)) >> 31);  // bit i = stage 31-i of the block
        Q = bitop3_xor_and(Q, d, MK[i % 6]);
    });
    const uint32_t p = (Q >> 2) & 63u;  // position at stage 63+32k
    Q -= 256u;
    // emit: block k+1, stages 63+32k .. 32+32k; D bit j = take-bit at stage 63+32k-j
    uint32_t D = 0;
    sfor<32>([&](auto J) {
        constexpr int j = decltype(J)::value;
        uint32_t w = *(const uint32_t*)(ringb + Q);
        D = (D & ~(1u << j)) | (w & (1u << j));
        if constexpr (j < 31) {
            uint32_t d = (uint32_t)((int)(w << (31 - j)) >> 31);
            Q = bitop3_xor_and(Q, d, MK[(j + 32) % 6]);
        }
    });
    // seed: E_j = bit q(63+32k-j) of p for j < 6 = brev6(rotr6(p, (q0+1) % 6)), q0 = q(63+32k)
    const int q0 = ((e6 - 32 % 6 + 6) % 6 + 5) % 6;
    const int s = (q0 + 1) % 6;
    const uint32_t y = ((p >> s) | (p << (6 - s))) & 63u;
    const uint32_t E = __builtin_bitreverse32(y) >> 26;
    uint32_t X = D ^ E;
    X ^= X << 6;
    X ^= X << 12;
    X ^= X << 24;
    return X;  // word bit i <-> stage 63+32k-i
}

// ================================================================ fp32 core: one chunk per wave
// Every metric core (M_B32, M_B16, M_FP16) runs here in exact-integer fp32: branch metrics are
// integers of magnitude <= 65534, path metrics stay below 2^22 after the per-block renormalisation,
// so fp32 add/sub/max are exact and the decisions equal the reference's int32/int16/fp16 ones; the
// metric type only selects the tie rule.  fp32 because on gfx950 v_add/v_sub/v_fma_f32 issue every
// 2 cycles per wave64 while v_max, DPP, v_pk_* and integer shift/bitfield ops take 4 (tools/vd_ubench).
// Per stage: t1 = own + m, t2 = exchanged - m (DPP-fused or LDS permute), pm = max(t1, t2),
// bit = clamp(t1 - t2) (a 0.0/1.0 from v_sub_f32's clamp modifier), acc = fma(acc, 2, bit).
template <int CORE>
struct Tie;
// bit = NOT take (t1 > t2 strictly) : exchanged wins ties
template <> struct Tie<B16> { static constexpr bool kInvert = true; };
template <> struct Tie<B32> { static constexpr bool kInvert = true; };
// bit = take (t2 > t1 strictly) : own wins ties
template <> struct Tie<F16> { static constexpr bool kInvert = false; };

__device__ __forceinline__ float clamp01(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 1.0f); }

// ---------------------------------------------------------------- port-aware ACS stage (inline asm)
// gfx950 VALU issue model (tools/vd_ubench2/3): a wave64 op starts every 2 cycles on one of two
// ports and holds it for 4; add/sub/fma/fmac/cndmask/bitop3 may use either port, v_max only one,
// and DPP / VOP3P ops hold both.  The compiler's order (add, sub_dpp, max, sub, fmac) serialises
// at ~20 cycles a stage; this order keeps the DPP op alone and pairs max with the clamp-sub and the
// previous stage's fmac with this stage's add: ~12 cycles.  Registers: pm metric, m own branch
// metric, acc/bit decision accumulator (the fmac of stage t-1 runs in stage t), t1/t2 scratch.
// DPP issue: an s_nop 0 right before each DPP op is worth ~7 cycles a stage (tools/vd_ubench6:
// add,sub_dpp 21.1 -> add,s_nop,sub_dpp 14.1 cycles at 7 waves/SIMD); without it the DPP op stalls
// the SIMD.  The DPP source (previous max) is >= 2 VALU ops back, as the data hazard requires.
#define VD_DPP_CTRL_0 "quad_perm:[1,0,3,2]"
#define VD_DPP_CTRL_1 "quad_perm:[2,3,0,1]"
#define VD_DPP_CTRL_3 "row_ror:8"
template <int Q, bool OWN_WINS>
__device__ __forceinline__ void stage_dpp(float& pm, float& acc, float& bit, float m)
{
    float t1, t2;
    if constexpr (Q == 2) {
        float x;
        // x = pm[lane ^ 7 within 8]; t2 = x[lane ^ 3 within 4] - m  ==  pm[lane ^ 4] - m
        if constexpr (OWN_WINS)
            asm("v_fma_f32 %0, %0, 2.0, %1\n\ts_nop 0\n\tv_mov_b32_dpp %5, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32 %3, %2, %6\n\ts_nop 0\n\tv_sub_f32_dpp %4, %5, %6 quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_max_f32 %2, %3, %4\n\tv_sub_f32_e64 %1, %4, %3 clamp"
                : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2), "=&v"(x) : "v"(m));
        else
            asm("v_fma_f32 %0, %0, 2.0, %1\n\ts_nop 0\n\tv_mov_b32_dpp %5, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32 %3, %2, %6\n\ts_nop 0\n\tv_sub_f32_dpp %4, %5, %6 quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_max_f32 %2, %3, %4\n\tv_sub_f32_e64 %1, %3, %4 clamp"
                : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2), "=&v"(x) : "v"(m));
    } else {
#define VD_STAGE_DPP(CTRL, CL)                                                                                  \
    asm("v_fma_f32 %0, %0, 2.0, %1\n\tv_add_f32 %3, %2, %5\n\ts_nop 0\n\tv_sub_f32_dpp %4, %2, %5 " CTRL " row_mask:0xf bank_mask:0xf\n\t" \
        "v_max_f32 %2, %3, %4\n\t" CL                                                                            \
        : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2) : "v"(m))
        if constexpr (OWN_WINS) {
            if constexpr (Q == 0) VD_STAGE_DPP(VD_DPP_CTRL_0, "v_sub_f32_e64 %1, %4, %3 clamp");
            else if constexpr (Q == 1) VD_STAGE_DPP(VD_DPP_CTRL_1, "v_sub_f32_e64 %1, %4, %3 clamp");
            else VD_STAGE_DPP(VD_DPP_CTRL_3, "v_sub_f32_e64 %1, %4, %3 clamp");
        } else {
            if constexpr (Q == 0) VD_STAGE_DPP(VD_DPP_CTRL_0, "v_sub_f32_e64 %1, %3, %4 clamp");
            else if constexpr (Q == 1) VD_STAGE_DPP(VD_DPP_CTRL_1, "v_sub_f32_e64 %1, %3, %4 clamp");
            else VD_STAGE_DPP(VD_DPP_CTRL_3, "v_sub_f32_e64 %1, %3, %4 clamp");
        }
#undef VD_STAGE_DPP
    }
}
// exchanged metric already fetched (LDS permute); E: bit = clamp(t1 + e - t2) (M_B32 own-wins lanes)
template <bool OWN_WINS, bool EBIAS>
__device__ __forceinline__ void stage_lds(float& pm, float& acc, float& bit, float m, float oth, float e)
{
    float t1, t2;
    if constexpr (EBIAS) {
        float t1e;
        asm("v_fma_f32 %0, %0, 2.0, %1\n\tv_add_f32 %3, %2, %6\n\tv_sub_f32 %4, %7, %6\n\tv_add_f32 %5, %3, %8\n\t"
            "v_max_f32 %2, %3, %4\n\tv_sub_f32_e64 %1, %5, %4 clamp"
            : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2), "=&v"(t1e) : "v"(m), "v"(oth), "v"(e));
    } else if constexpr (OWN_WINS) {
        asm("v_fma_f32 %0, %0, 2.0, %1\n\tv_add_f32 %3, %2, %5\n\tv_sub_f32 %4, %6, %5\n\t"
            "v_max_f32 %2, %3, %4\n\tv_sub_f32_e64 %1, %4, %3 clamp"
            : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2) : "v"(m), "v"(oth));
    } else {
        asm("v_fma_f32 %0, %0, 2.0, %1\n\tv_add_f32 %3, %2, %5\n\tv_sub_f32 %4, %6, %5\n\t"
            "v_max_f32 %2, %3, %4\n\tv_sub_f32_e64 %1, %3, %4 clamp"
            : "+v"(acc), "+v"(bit), "+v"(pm), "=&v"(t1), "=&v"(t2) : "v"(m), "v"(oth));
    }
}

template <int Q, int ABL = 0>
__device__ __forceinline__ float xchgf(float x, int bp_addr)
{
    return __builtin_bit_cast(float, xchg<Q, ABL>(__builtin_bit_cast(int, x), bp_addr));
}

// Workgroups of kWaves independent waves (one chunk each): gfx950 admits a bounded number of
// workgroups per CU, so single-wave workgroups could not keep all 6400 chunks resident at once.
// Waves never synchronise with each other; LDS is partitioned per wave and wave_sync() only orders
// the wave's own LDS traffic (LDS instructions of one wave execute in order).
constexpr int kWaves = 4;
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t simd_slot()
{
    const uint32_t h = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));         // HW_ID
    const uint32_t x = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)) & 7u;  // XCC_ID
    return (((x * 8 + ((h >> 13) & 7u)) * 2 + ((h >> 12) & 1u)) * 16 + ((h >> 8) & 15u)) * 4 + ((h >> 4) & 3u);
}

// Fairness controller.  The SIMD arbiter favours the oldest wave, so left alone the waves sharing a
// SIMD finish up to 2x apart and the tail of the launch runs at low occupancy (tools/vd_ablate clock
// stamps).  At every 3-block group head each wave posts the blocks it has started to its own board word
// and sets its issue priority from its lag behind the mean of the SIMD's waves, read at the previous
// head.  Posting is a plain store and reading one 64-byte load (16 lanes): both stay in the XCD's L2
// (all waves of a SIMD are on one XCD), so the board adds no HBM or fabric traffic -- a returning atomic
// per group went past the L2 and cost 11 MB of writes per launch (profiles/r02).  LD1: read with
// agent-scope (sc1) loads instead of workgroup-scope (sc0) ones (tools, A/B).
template <bool LD1 = false>
struct Fair {
    uint32_t* mine = nullptr;   // this wave's word
    uint32_t* simd = nullptr;   // the SIMD's kFairWaves words
    uint32_t seen = kFairEmpty; // lane l < kFairWaves: word l as read at the previous group head

    __device__ __forceinline__ void begin(uint32_t* board, int lane)
    {
        if (!board) return;
        const uint32_t wid = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) & (kFairWaves - 1);
        simd = board + (size_t)simd_slot() * kFairWaves;
        mine = simd + wid;
        if (lane == 0) __hip_atomic_store(mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    // group head; j = blocks started so far (a multiple of 3)
    __device__ __forceinline__ void group(uint32_t j, int lane)
    {
        if (!mine) return;
        if (j > 0) {
            const bool act = lane < kFairWaves && seen != kFairEmpty;
            const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(act));
            uint32_t x = act ? seen : 0u;
            // sum of the 16 words: row_shr 1, 2, 4, 8 (lanes past the row edge add 0); lane 15 holds it
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
            const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
            // (own - mean) * n in blocks; own word read back as posted at the previous head (j - 3).
            // 32-bit scalar arithmetic (n <= 16, j < 2^26): 64-bit compares would run on the VALU.
            const int32_t d = (int32_t)(j - 3) * (int32_t)n - (int32_t)sum, n3 = 3 * (int32_t)n;
            if (d <= -n3) __builtin_amdgcn_s_setprio(3);
            else if (d <= 0) __builtin_amdgcn_s_setprio(2);
            else if (d <= n3) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (lane == 0) __hip_atomic_store(mine, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t* w = simd + (lane & (kFairWaves - 1));
        if constexpr (LD1) seen = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else seen = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void end(int lane)
    {
        if (mine && lane == 0) __hip_atomic_store(mine, kFairEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};
template <int CH, int CORE, int OB, int ABL = 0>
__global__ __launch_bounds__(64 * kWaves) void vd_decode_sc(const void* __restrict__ in, void* __restrict__ out, Geom geo)
{
    using IN = In<CH>;
    constexpr int TBS = kTBsc;
    __shared__ float4 tab_all[kWaves][96];                   // per stage of a 3-block group: BM[0..3]
    __shared__ __attribute__((aligned(256))) uint32_t ring_all[kWaves][(TBS + 1) * 64];  // bit 31-s = stage s
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* tab = tab_all[wv];
    uint32_t* ring = ring_all[wv];
    const ChunkRange cr = chunk_range(geo, blockIdx.x * kWaves + wv);
    if (cr.words == 0) return;
    // ABL & 32 (tools only): per-wave clock stamps at out + 16 MiB
    const uint64_t t_clk0 = (ABL & 32) ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t t_rt0 = (ABL & 32) ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t start = cr.startWord * OB;                      // first stage of the chunk
    const uint32_t S = OB == 32 ? cr.words : (cr.words + 1) / 2;  // 32-bit words traced back
    const uint32_t nblk = S + 2;                                   // 64 warm-up stages + S slides

    int L4[6];
    sfor<6>([&](auto K) {
        constexpr int k = decltype(K)::value;
        L4[k] = own_label(lane, k) * 4;
    });
    // M_B32 at t%6==0: lanes >= 32 (position bit 5 = 1) keep their own predecessor on ties
    const float ebias = (CORE == B32 && lane >= 32) ? 1.0f : 0.0f;
    const int bp_addr = (lane ^ 32) * 4;
    const float* tabf = (const float*)tab;
    const uint64_t avail = geo.availStages;
    const uint64_t li = (uint64_t)(lane & 31);

    float pm = 0.0f;
    uint32_t kb = 0;
    // fairness controller (see Fair; ABL & 256 disables)
    Fair<> fair;
    if constexpr (!(ABL & 256)) fair.begin(geo.fair, lane);
    // first traceback batch is shortened per workgroup so the waves sharing a SIMD do not all enter
    // their latency-bound traceback in the same block
    uint32_t tbn = TBS - 3 * (blockIdx.x & 3);
    // Input of a 3-block group is loaded one group ahead (~96 stages of compute, several loaded-HBM
    // round trips) and turned into the group's branch-metric table at the head of the group.
    typename IN::raw_t rA = IN::load(in, start + li, avail);
    typename IN::raw_t rB = IN::load(in, start + 32 + li, avail);
    typename IN::raw_t rC = IN::load(in, start + 64 + li, avail);

    // one 32-stage block j (stage phase 2j%6 = PH, table rows 32*TB0..); false after the last block
    auto block = [&](auto PHc, uint32_t j) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int TB0 = PH / 2;
        // decision bits: the fmac of stage t runs inside stage t+1 (see stage_dpp); acc restarts
        // at each 16-stage half so its value stays an exact integer below 2^16
        float acc = 0.0f, bit = 0.0f;
        uint32_t hi16 = 0, word = 0;
        sfor<32>([&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int K = (PH + i) % 6;
            constexpr int Q = (K + 5) % 6;
            const float m = (ABL & 4) ? (float)L4[K] : tabf[(TB0 * 32 + i) * 4 + (L4[K] >> 2)];
            constexpr bool OWN = !Tie<CORE>::kInvert;
            if constexpr (Q <= 3 || (ABL & 2)) {
                stage_dpp<(Q <= 3 ? Q : 3), OWN>(pm, acc, bit, m);
            } else {
                const float oth = xchgf<Q>(pm, bp_addr);
                stage_lds<OWN, CORE == B32 && K == 0>(pm, acc, bit, m, oth, ebias);
            }
            if constexpr (i == 16) {  // acc now holds stages 0..15
                hi16 = (uint32_t)acc;
                acc = 0.0f;
            }
        });
        acc = __builtin_fmaf(acc, 2.0f, bit);  // stage 31's accumulate
        word = (hi16 << 16) | (uint32_t)acc;
        if constexpr (ABL & 8) asm volatile("" ::"v"(word));
        // decision-neutral renormalisation by the metric of position 0 (keeps |pm| < 2^22)
        pm -= __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, pm)));
        if (Tie<CORE>::kInvert) word = ~word;  // ring holds take-bits
        wave_sync();
        if (j >= 1) ring[(j - 1 - kb) * 64 + lane] = word;
        if (j >= 2 && (j - 1 - kb == tbn || j == nblk - 1)) {
            wave_sync();
            const uint32_t nw = j - 1 - kb;  // words kb .. j-2
            if (!(ABL & 1) && (uint32_t)lane < nw) {
                const uint64_t k = kb + lane;
                const uint32_t Q0 = (uint32_t)(wv * (TBS + 1) * 256 + (lane + 1) * 256);
                uint32_t w = traceback_word_sc((const char*)ring_all, Q0, k);
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[cr.startWord + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + cr.startWord;
                    o[2 * k] = (uint16_t)(w >> 16);
                    if (2 * k + 1 < cr.words) o[2 * k + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            wave_sync();
            ring[lane] = word;  // block j becomes slot 0 of the next batch
            kb = j - 1;
            tbn = TBS;
        }
        return j + 1 < nblk;
    };
    for (uint32_t j = 0;; j += 3) {
        if constexpr (!(ABL & 256)) fair.group(j, lane);
        if (lane < 32) {
            int A, B;
            IN::ab(rA, start + 32ull * j + li, avail, A, B);
            tab[lane] = make_float4((float)-A, (float)-B, (float)B, (float)A);
            IN::ab(rB, start + 32ull * (j + 1) + li, avail, A, B);
            tab[32 + lane] = make_float4((float)-A, (float)-B, (float)B, (float)A);
            IN::ab(rC, start + 32ull * (j + 2) + li, avail, A, B);
            tab[64 + lane] = make_float4((float)-A, (float)-B, (float)B, (float)A);
        }
        if constexpr (!(ABL & 16)) {
            rA = IN::load(in, start + 32ull * (j + 3) + li, avail);
            rB = IN::load(in, start + 32ull * (j + 4) + li, avail);
            rC = IN::load(in, start + 32ull * (j + 5) + li, avail);
        }
        wave_sync();
        if (!block(std::integral_constant<int, 0>{}, j)) break;
        if (!block(std::integral_constant<int, 2>{}, j + 1)) break;
        if (!block(std::integral_constant<int, 4>{}, j + 2)) break;
        wave_sync();  // this group's table reads complete before the next group overwrites it
    }
    if constexpr (ABL & 8) asm volatile("" ::"v"(pm));
    if constexpr (!(ABL & 256)) fair.end(lane);  // slot free again
    if constexpr (ABL & 32) {
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            uint64_t* d = (uint64_t*)((char*)out + (16u << 20)) + 6 * (blockIdx.x * kWaves + wv);
            d[0] = t_clk0; d[1] = c1; d[2] = t_rt0; d[3] = r1;
            d[4] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_ID
            d[5] = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));  // XCC_ID
        }
    }
}


}  // namespace vd
