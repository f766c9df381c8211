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
//    the sign bit of a candidate difference, shifted into per-lane words with pure-VGPR ops; one
//    word per lane per 32-stage block (int32) or per 16-stage half-block (packed) goes to an LDS ring.
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
constexpr int kTB = 16;        // output words traced back per batch (packed kernel)
constexpr int kTBsc = 14;      // fp32 kernel: 14 words per batch keeps 7 four-wave workgroups per CU

struct Geom {
    uint64_t packNum;      // output words of bpp bits (getMessageLen / bpp)
    uint64_t availStages;  // stages readable from the input buffer
    uint32_t nchunks;
    unsigned long long* fair;  // per-SIMD progress board (kFairSlots words, zero at rest) or null
    float scale;               // LLR input (channel ids 8 + base): SoftDecisionPacker scale, else unused
    // split launch (vd_kernel_tg.h "split chunks"): chunks >= nwhole are decoded as kWaves pieces, one
    // workgroup each; 0 = every chunk whole
    uint32_t nwhole = 0;
    uint32_t epoch = 0;          // launch id carried by the split flags
    float* spec = nullptr;       // [chunk - nwhole][kWaves][64] published metric vectors
    uint32_t* flags = nullptr;   // [chunk - nwhole][16] split flags
    uint32_t* stats = nullptr;   // count of split chunks re-decoded whole (or null)
};
// progress board: one 64-bit word per SIMD slot, (waves << 32) + blocks started; indexed by
// (XCC, SE, SH, CU, SIMD) from the hardware wave id.  Only issue priority depends on it.
constexpr int kFairSlots = 8 * 8 * 2 * 16 * 4;

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

// ---------------------------------------------------------------- lane-parallel traceback
// Lane traces output word k (0-based within its chunk); block k+2 sits in ring slot l+1, block k+1
// in slot l.  Position-space traceback: p_{t-1} = p_t ^ (d_t(p_t) << q_t); the decoded bit of stage t
// is bit q_t of p_{t-1} (the dropped bit of the predecessor state).  Reference: viterbiTB.cuh:4-21.
// Ring formats:
//   PK=false (int32 core): slot = 64 words (lane p), bit 31-s = decision of stage s of the block.
//   PK=true  (packed cores): slot = 2 half-blocks x 64 words; half-block hb holds stages 16hb..16hb+15,
//            the low 16 bits for the chunk in the low metric halves, the high 16 bits for the other;
//            bit s' of a 16-bit half = stage 16hb+s'.  `Q` carries 2h (byte select of the half).
template <bool PK>
__device__ __forceinline__ uint32_t traceback_word(const char* ring, int h, int l, uint64_t k)
{
    constexpr int SLOTB = PK ? 512 : 256;
    const int e6 = (int)((95 + 32 * k) % 6);  // stage phase of the traceback start
    int MK[6], QS[6];
    sfor<6>([&](auto R) {
        constexpr int r = decltype(R)::value;
        int t6 = (e6 - r + 6) % 6;
        int q = (t6 + 5) % 6;
        MK[r] = 4 << q;
        QS[r] = q + 2;
    });
    uint32_t Q = (uint32_t)((l + 1) * SLOTB + (PK ? 2 * h : 0));  // position 0 = state 0
    uint32_t word = 0;
    sfor<64>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr int s = 31 - (i & 31);  // stage within the block
        int d;
        if constexpr (PK) {
            constexpr int off = (s >> 4) * 256;
            uint32_t w = *(const uint16_t*)(ring + Q + off);
            d = (int)(w << (31 - (s & 15))) >> 31;
        } else {
            uint32_t w = *(const uint32_t*)(ring + Q);
            d = (int)(w << s) >> 31;
        }
        Q ^= (uint32_t)(d & MK[i % 6]);
        if constexpr (i == 31) Q -= (uint32_t)SLOTB;
        if constexpr (i >= 32) word |= ((Q >> QS[i % 6]) & 1u) << (i - 32);  // word bit <-> stage 63+32k-(i-32)
    });
    return word;
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
    // Fairness: the SIMD arbiter favours the oldest wave, so left alone the waves sharing a SIMD
    // finish up to 2x apart and the tail runs at low occupancy (tools/vd_ablate clock stamps).
    // Each wave posts its progress to the SIMD's board word at every 3-block group and sets its
    // issue priority from its lag behind the SIMD mean (ABL & 256 disables).
    unsigned long long* fb = nullptr;
    unsigned long long fret = 0;
    uint32_t fadded = 0;
    if constexpr (!(ABL & 256)) {
        if (geo.fair) {
            fb = geo.fair + simd_slot();
            if (lane == 0) atomicAdd(fb, 1ull << 32);
        }
    }
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
        if constexpr (!(ABL & 256)) {
            if (fb) {
                if (j > 0) {
                    // board value returned at the previous group head (own add of 3 not included)
                    const uint64_t r = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(fret >> 32)) << 32) |
                                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)fret);
                    const int64_t n = (int64_t)(r >> 32), sum = (int64_t)(uint32_t)r + 3;
                    const int64_t d = (int64_t)j * n - sum;  // (own - mean) * n, in blocks
                    if (d <= -3 * n) __builtin_amdgcn_s_setprio(3);
                    else if (d <= 0) __builtin_amdgcn_s_setprio(2);
                    else if (d <= 3 * n) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(0);
                }
                if (lane == 0) fret = atomicAdd(fb, 3ull);
                fadded += 3;
            }
        }
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
    if constexpr (!(ABL & 256)) {
        if (fb && lane == 0) atomicAdd(fb, 0ull - ((1ull << 32) + fadded));  // board back to zero
    }
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

// ================================================================ packed cores: two chunks per wave
template <int CORE>
struct Pk;
template <>
struct Pk<B16> {
    typedef short v2 __attribute__((ext_vector_type(2)));
    static constexpr bool kInvert = true;  // sign(t2 - t1) = NOT take: exchanged wins ties
    static __device__ __forceinline__ uint32_t cvt(int a) { return (uint32_t)(uint16_t)(int16_t)a; }
    static __device__ __forceinline__ v2 as(uint32_t x) { return __builtin_bit_cast(v2, x); }
    static __device__ __forceinline__ uint32_t bits(v2 x) { return __builtin_bit_cast(uint32_t, x); }
    // one ACS for both halves (viterbiACS.cuh:113-119,216-220); d carries the decision in the sign bits
    static __device__ __forceinline__ uint32_t acs(uint32_t own, uint32_t oth, uint32_t m, uint32_t& d)
    {
        v2 t1 = as(own) + as(m), t2 = as(oth) - as(m);
        d = bits(t2 - t1);
        return bits(__builtin_elementwise_max(t1, t2));
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return bits(as(a) - as(b)); }
};
template <>
struct Pk<F16> {
    typedef _Float16 v2 __attribute__((ext_vector_type(2)));
    static constexpr bool kInvert = false;  // sign(t1 - t2) = take: own wins ties (__hlt2_mask is strict)
    static __device__ __forceinline__ uint32_t cvt(int a) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a); }
    static __device__ __forceinline__ v2 as(uint32_t x) { return __builtin_bit_cast(v2, x); }
    static __device__ __forceinline__ uint32_t bits(v2 x) { return __builtin_bit_cast(uint32_t, x); }
    // viterbiACS.cuh:147-157,250-256; metrics stay exact integers below 2048 in magnitude
    static __device__ __forceinline__ uint32_t acs(uint32_t own, uint32_t oth, uint32_t m, uint32_t& d)
    {
        v2 t1 = as(own) + as(m), t2 = as(oth) - as(m);
        d = bits(t1 - t2);
        return bits(__builtin_elementwise_max(t1, t2));
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return bits(as(a) - as(b)); }
};
// shift both halves right by one and insert the two sign bits of d at bits 15 and 31
__device__ __forceinline__ uint32_t pk_push(uint32_t acc, uint32_t d)
{
    typedef unsigned short u2 __attribute__((ext_vector_type(2)));
    uint32_t sh = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, acc) >> (u2){1, 1});
    return (d & 0x80008000u) | (sh & 0x7FFF7FFFu);
}

template <int CH, int CORE, int OB, int ABL = 0>
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

    uint32_t pm = 0, acc = 0, accLo = 0;
    uint32_t kb = 0;
    typename IN::raw_t raw = IN::load(in, start + (uint64_t)li, avail);

    for (uint32_t j = 0; j < nblk; j++) {
        {
            int A, B;
            IN::ab(raw, start + 32ull * j + li, avail, A, B);
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
                const uint32_t m = (ABL & 4) ? (uint32_t)L4[K] : tabu[i * 4 + (L4[K] >> 2)];
                const uint32_t oth = (uint32_t)xchg<Q, ABL>((int)pm, bp_addr);
                uint32_t d;
                pm = P::acs(pm, oth, m, d);
                if constexpr (!(ABL & 8)) acc = pk_push(acc, d);
                if constexpr (i == 15) accLo = acc;  // first half-block complete
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
            ring[(j - 1 - kb) * 128 + lane] = P::kInvert ? ~accLo : accLo;
            ring[(j - 1 - kb) * 128 + 64 + lane] = P::kInvert ? ~acc : acc;
        }
        if (j >= 2 && (j - 1 - kb == (uint32_t)kTB || j == nblk - 1)) {
            __syncthreads();
            const uint32_t hi = (j - 1) < Smy ? (j - 1) : Smy;  // words kb .. min(j-1,S)-1 of my chunk
            const uint32_t nw = hi > kb ? hi - kb : 0;
            if (!(ABL & 1) && (uint32_t)li < nw) {
                const uint64_t k = kb + li;
                uint32_t w = traceback_word<true>((const char*)ring, half, li, k);
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[my.startWord + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + my.startWord;
                    o[2 * k] = (uint16_t)(w >> 16);
                    if (2 * k + 1 < my.words) o[2 * k + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            __syncthreads();
            ring[lane] = P::kInvert ? ~accLo : accLo;
            ring[64 + lane] = P::kInvert ? ~acc : acc;
            kb = j - 1;
        }
    }
}

}  // namespace vd
