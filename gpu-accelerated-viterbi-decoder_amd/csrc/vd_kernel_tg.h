// vd_kernel_tg.h -- the decode kernel vd_decode_tg<CH, CORE, OB> (gfx950), one instantiation per input
// format x metric core x output width.  Reference hot path: viterbi_core (src/viterbi/viterbi.cu:144-207)
// with viterbiBM.cuh (branch metrics), viterbiACS.cuh:113-157,216-256 (ACS and tie rules) and
// viterbiTB.cuh:4-21 (traceback); bit-exact with it for every valid option.
//
// Tagged ACS: the survivor decision of every stage rides in the low bits of the path metric.  A metric
// word is V = metric * 2^S + h, an exact integer in fp32 (|V| < 2^24).  At stage j of a J-stage history
// field (S = J+1), the own candidate gets tag +c*2^j and the exchanged one -c*2^j, c = +1 where the
// reference's tie rule lets the own predecessor win ties, -1 where the exchanged one does:
//   t1 = V_own + (BM*2^S + c*2^j),  t2 = V_exch - (BM*2^S + c*2^j),  V' = max(t1, t2).
// The history h = sum of the chosen signed digits (+-2^i, i < j) satisfies |h| < 2^j, so on equal metrics
// the tag decides (the tie rule), and on unequal metrics (a difference of >= 2^S) neither tags nor history
// can flip the order: every decision equals the reference's int32/int16/fp16 decision, and the max copies
// the winner's history into the lane (a register exchange within the field).  V is kept in [2^23, 2^24)
// (base 1.25*2^23), where the fp32 ulp is 1 and the low mantissa bits are the low integer bits, and every
// field starts at 2^(S-1): after J stages the field 2^(S-1) + h is in (0, 2^S), its decision bits
// (h + 2^J - 1) / 2 are mantissa bits 1..J, and clearing it is one v_bitop3_b32.  Renormalising at the end
// of every 32-stage block keeps V in range (bounds below).
//
// SOFT16 (|BM| up to 65536: a metric spread near 2^21) leaves no room for the tags below 2^24, so its
// kernel runs the same scheme on int32 patterns (TgFmt::INT): V = metric * 2^S + 2^(S-1) + h with
// |V| < 2^31, integer add / DPP subtract / signed max, and the same bit-field read-out.
//
// Lane encoding.  Position p holds after stage t the trellis state rotr6(p, t%6); p lives in lane
// l = p0*1 ^ p1*2 ^ p2*7 ^ p3*8 ^ p4*16 ^ p5*32, so the butterfly partner p ^ (1<<q), q = (t%6+5)%6, is
// lane l ^ {1, 2, 7, 8, 16, 32}[q]: DPP quad_perm (xor 1, 2), row_half_mirror (xor 7) and row_ror:8
// (xor 8), each fused into the max; ds_swizzle (xor 16) and ds_bpermute (xor 32) fetch the partner's
// metric through the LDS crossbar (no memory access).
//
// LDS per wave: [guard | branch-metric table | guard | survivor ring | guard].  The guard words are
// written and checked only when Geom::check is set (tests: any out-of-bounds LDS store of the table or
// ring lands in a guard and is counted at kernel exit).
#pragma once
#include <type_traits>
#include "vd_kernels.h"
#include "vd_pack.h"

namespace vd {

// channel ids: HARD..FP32 = packed input (viterbiBM.cuh formats); 8 + base = float channel values
// quantised on the fly exactly like SoftDecisionPacker(base, scale) would have packed them (vd_pack.h)
constexpr int kLlr = 8;

template <int CH>
struct TgFmt {
    static constexpr bool INT = (CH & 7) == SOFT16;       // int32 metric patterns instead of fp32
    static constexpr int J = (CH & 7) == HARD ? 16 : 8;   // stages per history field
    static constexpr int S = J + 1;                       // metric scale 2^S
};
// Range.  The largest path metric never decreases (the best state's two successors get +-x, one of
// them >= it) and grows by at most BMmax per stage; every metric lies within D = (K-1)*(BMmax-BMmin) of
// the largest.  So R stages after a renormalisation (position 0 at the base, every metric within D of
// it) the metrics relative to the base are in [-D, D + R*BMmax], and the candidates t1/t2 add
// +-(BMmax + 1) more, in units of 2^S.  With the base at 1.25*2^23 (2,097,152 above 2^23 and 6,291,456
// below 2^24) and R = 32:
//   HARD (BMmax 1; 2^17 units: 16 below, 48 above):  [-14, 12+32+2] fits;
//   SOFT8 (BMmax 256; 2^9 units: 4096 below, 12288 above):  [-3329, 3072+8192+257] = [-3329, 11521] fits;
//   SOFT4/FP32 (BMmax 16):  [-209, 192+512+17] fits.
// SOFT16 (int32, base 0, BMmax 65536, 2^9 units, 2^22 each way): [-851,969, 786,432+2,097,152+65,537]
// fits, so |V +- E| < 2^31.  The CLI default SNR 15 (saturated soft values on the codeword: the best
// path gains BMmax every stage) is in the parity tests; tests/test_metric_range.py checks the bounds.

// Label-region table (the fp32 cores' table): one region of 96 entries per label, entry of stage
// t = 12m + 6o + K (period pair m, period o, phase K) at index 12m + 2K + o, so the entries of stages t and
// t+6 (o = 0, 1) are one ds_read_b64; the regions are 104 dwords apart (banks 0, 40, 16, 56: the four
// labels' reads in a lane group never share a bank).  Lane l builds the entries of the stage at index l
// (and lanes 0..31 index 64 + l) and writes them with ds_write_addtid_b32 (address = M0 + offset + 4 lane,
// no address VGPR: 2 cycles of the store path per 256 B instead of 6 per 512 B for ds_write2_b32 at
// scattered row addresses).  Against round 2's interleaved-row table: HARD 0.1627 -> 0.1582 ms, SOFT8
// 0.1655 -> 0.1632 ms per batch under bench conditions, exact twins (profiles/r03/benchab_label_regions.log).
// ALT (SOFT16, int32 patterns): the M_B32 upper position half needs the other tag sign at phase 0
// (E+[L] = BM[L]*2^S + 2^j, viterbiACS.cuh:137-142), and the fp32 cores' complementary-label trick needs
// a sign multiply the int32 core has no one-op form for.  So the phase-0 entries also exist with the +tag
// in an area after the regions: E+[L] of table index i = 12m + o (o = 0, 1) at dword ALT + i + 2L, written by
// the same lanes with ds_write_addtid_b32 under an EXEC mask (address M0 + offset + 4 lane: the +2L is the
// offset) and read as one ds_read_b64 per (t, t+6) pair like the regions.  The regions are then 98 dwords
// apart (banks 0, 34, 4, 38: still distinct for the four labels' pairs) so table + ALT (1,936 B) fit the
// 5,120 B of LDS a wave has at 8 waves per SIMD.
template <bool ALT>
struct TgTabLT {
    static constexpr int RW = ALT ? 98 : 104;  // dwords per label region
    static constexpr int REGION = RW * 4;      // bytes per label region
    static constexpr int ALT_OFF = 4 * REGION; // bytes: the +tag phase-0 area (ALT)
    static __host__ __device__ constexpr int index(int r) { return 12 * (r / 12) + 2 * (r % 6) + (r / 6) % 2; }
    static __host__ __device__ constexpr int row(int r) { return 4 * index(r); }
    // stage (within the group) whose entries table index i holds
    static __host__ __device__ constexpr int stage(int i) { return 12 * (i / 12) + 6 * (i % 2) + (i % 12) / 2; }
    static constexpr int BYTES = 4 * REGION + (ALT ? 4 * (12 * 7 + 8) : 0);
};
using TgTabL = TgTabLT<false>;
static_assert(TgTabL::stage(TgTabL::index(95)) == 95 && TgTabL::index(TgTabL::stage(64)) == 64, "index <-> stage");
static_assert(TgTabLT<true>::ALT_OFF % 8 == 0, "ALT pairs are ds_read_b64 aligned");
// ds_write_addtid_b32 x4: LDS[M0 + OFF + k R + 4 lane] = v_k for the active lanes.  M0 is a register the
// compiler reserves (it does not honour an "m0" clobber), so the statement saves and restores it.
template <int OFF, int R>
__device__ __forceinline__ void lds_write_addtid4(uint32_t base, float v0, float v1, float v2, float v3)
{
    uint32_t t;
    asm volatile("s_mov_b32 %[t], m0\n\ts_mov_b32 m0, %[b]\n\ts_nop 0\n\t"
                 "ds_write_addtid_b32 %[v0] offset:%[o0]\n\tds_write_addtid_b32 %[v1] offset:%[o1]\n\t"
                 "ds_write_addtid_b32 %[v2] offset:%[o2]\n\tds_write_addtid_b32 %[v3] offset:%[o3]\n\t"
                 "s_mov_b32 m0, %[t]"
                 : [t] "=&s"(t)
                 : [b] "s"(base), [v0] "v"(v0), [v1] "v"(v1), [v2] "v"(v2), [v3] "v"(v3), [o0] "i"(OFF),
                   [o1] "i"(OFF + R), [o2] "i"(OFF + 2 * R), [o3] "i"(OFF + 3 * R)
                 : "memory");
}

// Survivor ring: as many 256-B slots as fit next to the table in a wave's 5,120 B (8 workgroups of 4 waves
// per CU, so every SIMD holds 8 waves at <= 64 VGPRs); one traceback batch traces (slots - 1) words, and
// its VALU instructions cost the same whatever the number of words, so the longest ring is the cheapest:
// 13 slots with the fp32 cores' label-region table (1,664 B), 12 with SOFT16's (1,936 B).  8 waves beat 7
// with a longer ring by 1.4 % per batch (profiles/r02/benchab_8w.log).
constexpr int kGuardWords = 4;                 // guard words before the table, between table and ring, after the ring
constexpr uint32_t kGuardPattern = 0xA5C3E10Fu;
constexpr int kWaveLdsWords = 163840 / 4 / (8 * kWaves);  // 1,280: a wave's share at 8 workgroups per CU
template <int TABB>
struct TgLds {
    static constexpr int GW = kGuardWords;
    static constexpr int TAB = TABB / 4;                   // table words
    static constexpr int TBS = (kWaveLdsWords - 3 * GW - TAB) / 64 - 1;  // words per traceback batch
    static constexpr int RING = (TBS + 1) * 64;            // ring words
    // ring first, its 256-B slots aligned (the OR addressing of tg8_traceback): [ring | guard | table | guard |
    // guard], a wave's part a multiple of 64 words (word offsets within it)
    static constexpr int RING_OFF = 0, TAB_OFF = RING + GW;
    static constexpr int WAVE = (3 * GW + TAB + RING + 63) / 64 * 64;
    // guard word i (0 .. 3 GW - 1) of a wave's part
    static __device__ __forceinline__ int guard(int i) { return RING + (i < GW ? i : TAB + i); }
};
static_assert(TgLds<TgTabL::BYTES>::TBS == 12 && TgLds<TgTabLT<true>::BYTES>::TBS == 11, "ring lengths");
static_assert(kWaves * TgLds<TgTabL::BYTES>::WAVE * 4 <= 20480 && kWaves * TgLds<TgTabLT<true>::BYTES>::WAVE * 4 <= 20480,
              "8 workgroups of 4 waves per CU (160 KiB of LDS)");
static_assert(TgLds<TgTabL::BYTES>::WAVE % 64 == 0 && TgLds<TgTabLT<true>::BYTES>::WAVE % 64 == 0, "ring slots 256-B aligned");

__device__ __forceinline__ int tg_pos(int l)
{
    const int p2 = (l >> 2) & 1;
    return (l & ~7) | (p2 << 2) | ((((l >> 1) & 1) ^ p2) << 1) | ((l & 1) ^ p2);
}
// reference label (0..3) of position p's own predecessor branch at stage phase k, and its parity helper
__host__ __device__ constexpr int tg_par7(int v) { return (v & 1) ^ ((v >> 1) & 1) ^ ((v >> 2) & 1) ^ ((v >> 3) & 1) ^ ((v >> 4) & 1) ^ ((v >> 5) & 1) ^ ((v >> 6) & 1); }
__host__ __device__ constexpr int tg_label(int p, int k)
{
    const int T = ((p >> k) | (p << (6 - k))) & 63, r5 = (k + 5) % 6, O = ((p >> r5) | (p << (6 - r5))) & 63;
    const int R = (T << 1) | (O & 1);
    return (tg_par7(R & 0171) << 1) | tg_par7(R & 0133);
}
// label flip of the butterfly partner in the two LDS-exchange phases: 0 (checked at compile time)
static_assert(tg_label(32, 0) == 0 && tg_label(16, 5) == 0, "exchange partners share the label");

// ---------------------------------------------------------------- stages (inline asm, exact op order)
// The path metric V is pinned to v60 ("{v60}" constraints).
typedef float f2v __attribute__((ext_vector_type(2)));
// DPP stage, exchange lane xor {1,2,7,8}[Q].  The butterfly partner has the same branch label and tag
// in every DPP phase, so its V_exch - m is what this lane would compute from its own V: a = V + m,
// b = V - m, and the max takes b from the partner through the DPP operand, V' = max(a, dpp(b)).  b is
// read by DPP 2 slots after its write.  (The three-op form v_add, v_sub_f32_dpp, v_max decides the same;
// this one is 0.5-1 % faster, profiles/r02/benchab_dpp_forms_8w.log.)
template <int Q>
__device__ __forceinline__ void tg_stage_dpp2(float& V, float m)
{
    float a, b;
#define VD_TG_DPP2(MAX, CTRL)                                                                                \
    asm("v_sub_f32 %2, %0, %3\n\tv_add_f32 %1, %0, %3\n\ts_nop 0\n\t"                                      \
        MAX " %0, %2, %1 " CTRL " row_mask:0xf bank_mask:0xf"                                                  \
        : "+{v60}"(V), "=&v"(a), "=&v"(b) : "v"(m))
#define VD_TG_DPP2Q(MAX)                                                                                     \
    if constexpr (Q == 0) VD_TG_DPP2(MAX, "quad_perm:[1,0,3,2]");                                            \
    else if constexpr (Q == 1) VD_TG_DPP2(MAX, "quad_perm:[2,3,0,1]");                                       \
    else if constexpr (Q == 2) VD_TG_DPP2(MAX, "row_half_mirror");                                           \
    else VD_TG_DPP2(MAX, "row_ror:8");
    VD_TG_DPP2Q("v_max_f32_dpp")
#undef VD_TG_DPP2Q
#undef VD_TG_DPP2
}

// LDS-exchange stage: the partner's metric vp through the LDS crossbar (ds_swizzle / ds_bpermute), then
// V' = max(V + m, vp - m), the DPP stage's formula.  A VALU lane swap (v_permlane32_swap) costs about two
// DPP ops of issue; this costs three plain ops and one LDS round trip (profiles/r02/ablate.log).
__device__ __forceinline__ float tg_partner(float V, int paddr)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(paddr, __builtin_bit_cast(int, V)));
}
__device__ __forceinline__ float tg_swz16(float V)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, V), 0x401F));
}
// The stage with the subtraction before the exchange: b = V - m goes through the LDS crossbar, and
// since the exchange partners share the label and the tag (every core, except the M_B32 phase-0 stage
// with its per-half tag sign), the received value is V_partner - m.  After the exchange returns only the
// max is left, so the round trip's dependent chain is one op shorter; a = V + m issues while it is in
// flight.
template <bool X32, bool INT>
__device__ __forceinline__ void tg_stage_lds_pre(float& V, float m, int paddr)
{
    float a, b;
    if constexpr (INT) asm("v_sub_u32 %0, %1, %2" : "=v"(b) : "v"(V), "v"(m));
    else asm("v_sub_f32 %0, %1, %2" : "=v"(b) : "v"(V), "v"(m));
    const float bp = X32 ? tg_partner(b, paddr) : tg_swz16(b);
    if constexpr (INT) asm("v_add_u32 %0, %1, %2" : "=v"(a) : "v"(V), "v"(m));
    else asm("v_add_f32 %0, %1, %2" : "=v"(a) : "v"(V), "v"(m));
    if constexpr (INT) asm("v_max_i32 %0, %1, %2" : "={v60}"(V) : "v"(a), "v"(bp));
    else asm("v_max_f32 %0, %1, %2" : "={v60}"(V) : "v"(a), "v"(bp));
}
// M_B32 phase-0 stage (S32): V' = max(V + s*m, vp - s*m), s = -1 in the upper position half, where m is
// the entry of the complementary label (see the kernel)
__device__ __forceinline__ void tg_stage_lds_sg(float& V, float m, float vp, float sg)
{
    float t1, t2;
    asm("v_fma_f32 %1, %3, %5, %0\n\tv_fma_f32 %2, -%3, %5, %4\n\tv_max_f32 %0, %1, %2"
        : "+{v60}"(V), "=&v"(t1), "=&v"(t2) : "v"(m), "v"(vp), "v"(sg));
}

// int32 stages (TgFmt::INT): the same forms on integer patterns
template <int Q>
__device__ __forceinline__ void tg_stage_dpp_i2(float& V, float m)
{
    float a, b;
#define VD_TG_DPPI2(CTRL)                                                                                  \
    asm("v_sub_u32 %2, %0, %3\n\tv_add_u32 %1, %0, %3\n\ts_nop 0\n\tv_max_i32_dpp %0, %2, %1 " CTRL            \
        " row_mask:0xf bank_mask:0xf"                                                                      \
        : "+{v60}"(V), "=&v"(a), "=&v"(b) : "v"(m))
    if constexpr (Q == 0) VD_TG_DPPI2("quad_perm:[1,0,3,2]");
    else if constexpr (Q == 1) VD_TG_DPPI2("quad_perm:[2,3,0,1]");
    else if constexpr (Q == 2) VD_TG_DPPI2("row_half_mirror");
    else VD_TG_DPPI2("row_ror:8");
#undef VD_TG_DPPI2
}
__device__ __forceinline__ void tg_stage_lds_i(float& V, float m, float vp)
{
    float t1, t2;
    asm("v_add_u32 %1, %0, %3\n\tv_sub_u32 %2, %4, %3\n\tv_max_i32 %0, %1, %2"
            : "+{v60}"(V), "=&v"(t1), "=&v"(t2) : "v"(m), "v"(vp));
}

// ---------------------------------------------------------------- group traceback (reference viterbiTB.cuh:4-21)
// Ring slot = 64 words indexed by position; byte/half g of word p holds the take-bits of history field
// g along the survivor ending at p (register exchange within the field).  Tracing word k from state
// 0 at the end of stage 95+32k: per field, look up the bits at the position of the current state T,
// then, with the stride-6 structure of position-space traceback (bit q_t of the position is touched
// only by the stage-t decision, every 6 stages), the field's decoded bits are the stride-6 suffix XOR
// of (bits ^ T << (J-6)) and the state at the field start is its low 6 bits.  M_B32 keeps its raw
// phase-0 bits (own-wins tag in the upper position half), which already are the decoded bits there.
// One dependent LDS read per J stages instead of one per stage.
//
// Constants of the traceback of word k: they depend on the stage phase of its emit block,
// ph = 2 ((k + 1) % 3), only: the bit offsets (+ J - 6, see below) of the position of a state at the three
// odd field-end phases, and (M_B32) the phase-0 mask of field-start phase ph.  When every traceback batch
// starts at a multiple of 3 words, ph is the lane's (k = kb + lane): tb_pack(lane) computes the constants
// once per kernel into 5-bit fields of one word, tb_unpack reads them back.
struct TbC {
    uint32_t off[3];
    uint32_t m50;
};
template <int J, bool FIX5>
__device__ __forceinline__ TbC tb_direct(int k)
{
    const int ph = 2 * ((k + 1) % 3);
    TbC c;
    c.off[0] = 5 - ph + J - 6;
    c.off[1] = (ph <= 2 ? 3 - ph : 9 - ph) + J - 6;
    c.off[2] = (ph == 0 ? 1 : 7 - ph) + J - 6;
    c.m50 = FIX5 ? 0x41041041u << ((12 - ph) % 6) : 0u;
    return c;
}
template <int J, bool FIX5>
__device__ __forceinline__ uint32_t tb_pack(int lane)
{
    const int ph = 2 * ((lane + 1) % 3);
    const TbC c = tb_direct<J, false>(lane);
    return c.off[0] | c.off[1] << 5 | c.off[2] << 10 | (FIX5 ? (uint32_t)((12 - ph) % 6) << 15 : 0u);
}
template <bool FIX5>
__device__ __forceinline__ TbC tb_unpack(uint32_t tbk)
{
    TbC c;  // v_bfe_u32 takes its offset from bits 4:0 of the operand
    c.off[0] = tbk;
    c.off[1] = tbk >> 5;
    c.off[2] = tbk >> 10;
    c.m50 = FIX5 ? 0x41041041u << ((tbk >> 15) & 31u) : 0u;
    return c;
}
template <int J, bool FIX5>
__device__ __forceinline__ uint32_t traceback_word_tg(const char* ringb, uint32_t slot1, const TbC& tc)
{
    constexpr int G = 32 / J;
    // position of state T at a field end of stage phase s (odd) is rotl6(T, s) = bits [6-s, 12-s) of
    // T | T << 6.  TX = T * (2^(J-6) + 2^J) holds that pair shifted by J - 6: its bits [J-6, J) are the
    // T << (J-6) the field's XOR needs, so one multiply serves both (the copy above bit J is masked off
    // below).
    const uint32_t* const off = tc.off;
    uint32_t m5[3] = {0u, 0u, 0u};  // M_B32: bits of phase-0 stages for field start phase ph + 2d
    if constexpr (FIX5) {
        // 0x41041041 << ((12 - ph - 2d) % 6).  The mask has period 6, so in bits 0..29 (a field has J <= 16)
        // a shift by (s - 2) mod 6 is a right shift by 2 of the shift by s, whatever s in {0, 2, 4}.
        m5[0] = tc.m50;
        m5[1] = m5[0] >> 2;
        m5[2] = m5[0] >> 4;
    }
    constexpr uint32_t JM = (1u << J) - 1u;
    uint32_t T = 0, nat = 0;
    auto field = [&](auto BOc, auto Gc, uint32_t slot) {
        constexpr int BO = decltype(BOc)::value;  // 0: emit block, 2: convergence block
        constexpr int g = decltype(Gc)::value;
        constexpr int c = (BO + J * g + J - 1) % 6;
        if constexpr (J < 6) {
            // 4-stage fields (vd_decode_pk's SOFT4 / FP32 kernels; nibble g of the ring word): every stage of
            // the field touches a different position bit, so no suffix XOR; the field's decoded bits are
            // W ^ (T >> (6 - J)) and the state at the field start keeps the low 6 - J bits of T (offsets:
            // tb_direct<6, .>, TX = T | T << 6)
            const uint32_t p = __builtin_amdgcn_ubfe(T * 65u, off[c / 2], 6u);
            const uint32_t W = (uint32_t)(*(const uint8_t*)(ringb + slot + 4 * p + g / 2) >> (4 * (g % 2))) & JM;
            uint32_t Y = W ^ (T >> (6 - J));
            if constexpr (FIX5) {
                constexpr int d = ((BO + J * g) % 6) / 2;
                Y = (m5[d] & W) | (~m5[d] & Y);
            }
            T = ((T << J) | Y) & 63u;
            return Y;
        } else {
            const uint32_t TX = T * ((1u << (J - 6)) | (1u << J));
            const uint32_t p = __builtin_amdgcn_ubfe(TX, off[c / 2], 6u);
            uint32_t W;
            if constexpr (J == 8) W = *(const uint8_t*)(ringb + slot + 4 * p + g);
            else W = *(const uint16_t*)(ringb + slot + 4 * p + 2 * g);
            // the stride-6 suffix XOR of the field's J bits of W ^ T << (J-6) (bits >= J of Y: the copy of T)
            uint32_t Y = W ^ TX;
            if constexpr (J == 8) {
                Y ^= __builtin_amdgcn_ubfe(Y, 6u, 2u);
            } else {
                Y ^= __builtin_amdgcn_ubfe(Y, 6u, 10u);
                Y ^= __builtin_amdgcn_ubfe(Y, 12u, 4u);
            }
            if constexpr (FIX5) {
                constexpr int d = ((BO + J * g) % 6) / 2;
                Y = (m5[d] & W) | (~m5[d] & Y);
            }
            T = Y & 63u;
            return Y & JM;
        }
    };
    sfor<G>([&](auto I) {  // convergence: block k+2, fields G-1 .. 0
        constexpr int g = G - 1 - decltype(I)::value;
        (void)field(std::integral_constant<int, 2>{}, std::integral_constant<int, g>{}, slot1);
    });
    sfor<G>([&](auto I) {  // emit: block k+1
        constexpr int g = G - 1 - decltype(I)::value;
        nat |= field(std::integral_constant<int, 0>{}, std::integral_constant<int, g>{}, slot1 - 256u) << (J * g);
    });
    return __builtin_bitreverse32(nat);  // word bit i <-> stage 63+32k-i
}
// J = 8 (the fp32 cores' SOFT4 / SOFT8 / FP32 and SOFT16's int32 patterns): the same recursion in 2-cycle ops
// on the ring-first layout (vd_decode_pk's pk8_traceback for one chain).  base = the LDS byte address of the
// emit slot (256-B aligned; the convergence block is the next slot); sft[c] = TbC::off[c] - 2, so
// (TX >> sft) & 0xFC is 4 times the position of the state (TX = T * 260: T in bits 2..7 and 8..13); a field:
// the address by v_lshrrev + v_bitop3 ((t & 0xFC) | base), the byte by ds_read_u8 at a constant offset, Y = W ^
// TX with the stride-6 fold Y ^= (Y >> 6) & 3, M_B32's raw phase-0 bits back in (v_bitop3 select), the next TX
// = (Y & 63) * 260, the byte into the word (v_perm) -- where traceback_word_tg's v_bfe / v_lshl_add / v_bfi /
// v_lshl_or take 4 cycles each
template <bool FIX5>
__device__ __forceinline__ uint32_t tg8_traceback(uint32_t base, const uint32_t (&sft)[3], const uint32_t (&m5)[3])
{
    uint32_t TX = 0, nat = 0;
    auto step = [&](auto EMc, auto Gc) {
        constexpr bool EM = decltype(EMc)::value;
        constexpr int g = decltype(Gc)::value;
        constexpr int BO = EM ? 0 : 2;
        constexpr int c = (BO + 8 * g + 7) % 6;
        constexpr int off = (EM ? 0 : 256) + g;
        const uint32_t A = __builtin_amdgcn_bitop3_b32(TX >> (sft[c / 2] & 31u), 0xFCu, base, 0xEA);
        const uint32_t W = *(const __attribute__((address_space(3))) uint8_t*)(uintptr_t)(A + off);
        uint32_t Y = W ^ TX;
        Y = __builtin_amdgcn_bitop3_b32(Y, Y >> 6, 3u, 0x78);  // Y ^ ((Y >> 6) & 3)
        if constexpr (FIX5) Y = __builtin_amdgcn_bitop3_b32(m5[((BO + 8 * g) % 6) / 2], W, Y, 0xCA);
        if constexpr (!(EM && g == 0)) TX = __mul24(Y & 63u, 260u);
        if constexpr (EM) nat = __builtin_amdgcn_perm(Y, nat, (0x03020100u & ~(0xFFu << (8 * g))) | (4u << (8 * g)));
    };
    sfor<4>([&](auto I) { step(std::false_type{}, std::integral_constant<int, 3 - decltype(I)::value>{}); });
    sfor<4>([&](auto I) { step(std::true_type{}, std::integral_constant<int, 3 - decltype(I)::value>{}); });
    return __builtin_bitreverse32(nat);  // word bit i <-> stage 63+32k-i
}

// ---------------------------------------------------------------- channel input through a buffer resource
// Formats as In<CH> (viterbiBM.cuh:15-153).  The resource of a 96-stage group starts at the group's
// first stage and ends at the last whole word of the caller's data, so reads past the input return
// zero -- the reference window's "no data" -- with no per-lane address or range arithmetic.  Row r of
// the group (stage 32r + li) reads at voff(li) + r * RB.
template <int CH>
struct TgIn;
template <>
struct TgIn<HARD> {  // 16 stages per word; stage g -> bits 31-2(g%16), 30-2(g%16); g%16 = li%16
    static constexpr bool FAB = false;  // ab() gives ints
    using raw_t = uint32_t;
    static constexpr int RB = 8;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages / 4; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 4u * (uint32_t)(li >> 4); }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        return __builtin_amdgcn_raw_buffer_load_b32(rs, vo + R * RB, 0, 0);
    }
    static __device__ __forceinline__ void ab(raw_t w, int li, int& A, int& B, float)
    {
        const int sh = 30 - 2 * (li & 15);
        const int r0 = (w >> (sh + 1)) & 1, r1 = (w >> sh) & 1;
        A = r0 + r1 - 1;
        B = r0 - r1;
    }
};
template <>
struct TgIn<SOFT4> {  // 4 stages per word, byte g%4 from the MSB: high nibble s0, low nibble s1
    static constexpr bool FAB = false;  // ab() gives ints
    using raw_t = uint32_t;
    static constexpr int RB = 32;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 4u * (uint32_t)(li >> 2); }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        return __builtin_amdgcn_raw_buffer_load_b32(rs, vo + R * RB, 0, 0);
    }
    static __device__ __forceinline__ void ab(raw_t w, int li, int& A, int& B, float)
    {
        const int sh = 24 - 8 * (li & 3);
        const int s0 = (int)(w << (24 - sh)) >> 28, s1 = (int)(w << (28 - sh)) >> 28;
        A = s0 + s1;
        B = s0 - s1;
    }
};
template <>
struct TgIn<SOFT8> {  // 2 stages per word; the 16-bit half g^1 holds s0 (high byte), s1 (low byte)
    static constexpr bool FAB = false;  // ab() gives ints
    using raw_t = uint32_t;
    static constexpr int RB = 64;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages * 2; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 2u * (uint32_t)(li ^ 1); }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, vo + R * RB, 0, 0);
    }
    static __device__ __forceinline__ void ab(raw_t w, int, int& A, int& B, float)
    {
        const int s0 = (int)(w << 16) >> 24, s1 = (int)(w << 24) >> 24;
        A = s0 + s1;
        B = s0 - s1;
    }
    // the two soft values as floats (sign-extending byte converts): the table row is then six exact FMAs,
    // E[3], E[2] = s1 * +-2^S + (s0 * 2^S + tag), E[0], E[1] = s1 * -+2^S + (-s0 * 2^S + tag)
    static constexpr bool S01 = true;
    static __device__ __forceinline__ void s01(raw_t w, float& s0, float& s1)
    {
        // one sign-extending byte convert each (left to itself the compiler shifted byte 1 up to byte 3
        // first: one VALU op more per table row)
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(s0) : "v"(w));
        asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(s1) : "v"(w));
    }
};
template <>
struct TgIn<SOFT16> {  // 1 stage per word: high 16 bits s0, low 16 bits s1
    static constexpr bool FAB = false;  // ab() gives ints
    using raw_t = uint32_t;
    static constexpr int RB = 128;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages * 4; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 4u * (uint32_t)li; }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        return __builtin_amdgcn_raw_buffer_load_b32(rs, vo + R * RB, 0, 0);
    }
    static __device__ __forceinline__ void ab(raw_t w, int, int& A, int& B, float)
    {
        const int s0 = (int)w >> 16, s1 = (int)(w << 16) >> 16;
        A = s0 + s1;
        B = s0 - s1;
    }
};
template <>
struct TgIn<FP32> {  // 2 floats per stage, clamped to [-8,7]; BM = (int)(+-x0 +- x1) (truncation)
    // abf(): (A, B) as floats, truncated in fp32 (v_trunc_f32: one op where int conversion and back take
    // two).  trunc gives -0 where (float)(int) gives +0, which the table's fma(A, 2^S, tag) cannot see.
    static constexpr bool FAB = true;
    using raw_t = float2;
    static constexpr int RB = 256;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages * 8; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 8u * (uint32_t)li; }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        const f2v v = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, vo + R * RB, 0, 0));
        return make_float2(v.x, v.y);
    }
    static __device__ __forceinline__ void ab(raw_t v, int, int& A, int& B, float)
    {
        const float x0 = fminf(fmaxf(v.x, -8.0f), 7.0f), x1 = fminf(fmaxf(v.y, -8.0f), 7.0f);
        A = (int)__fadd_rn(x0, x1);
        B = (int)__fsub_rn(x0, x1);
    }
    static __device__ __forceinline__ void abf(raw_t v, int, float& A, float& B, float)
    {
        const float x0 = fminf(fmaxf(v.x, -8.0f), 7.0f), x1 = fminf(fmaxf(v.y, -8.0f), 7.0f);
        A = __builtin_truncf(__fadd_rn(x0, x1));
        B = __builtin_truncf(__fsub_rn(x0, x1));
    }
};
template <class T, class = void>
struct HasS01 : std::false_type {};
template <class T>
struct HasS01<T, std::void_t<decltype(T::S01)>> : std::bool_constant<T::S01> {};
// float channel values (2 per stage, 8 bytes), quantised as SoftDecisionPacker(BASE, scale) would
template <int BASE>
struct TgInLlr {
    // SOFT4 / SOFT8: the soft values straight in fp32 (abf), no integer round trip
    static constexpr bool FAB = BASE == SOFT4 || BASE == SOFT8;
    using raw_t = float2;
    static constexpr int RB = 256;
    static __device__ __forceinline__ uint64_t bytes(uint64_t stages) { return stages * 8; }
    static __device__ __forceinline__ uint32_t voff(int li) { return 8u * (uint32_t)li; }
    template <int R>
    static __device__ __forceinline__ raw_t load(__amdgpu_buffer_rsrc_t rs, uint32_t vo)
    {
        return TgIn<FP32>::template load<R>(rs, vo);
    }
    // (float)code_value(pack_code(v)) for SOFT4 / SOFT8: rint clamped in fp32 when |v| < 2^31 (exact there),
    // else the x86 narrowing path of pack_code
    static __device__ __forceinline__ float soft(float v)
    {
        constexpr float lo = BASE == SOFT4 ? -8.0f : -128.0f, hi = BASE == SOFT4 ? 7.0f : 127.0f;
        if (__builtin_expect(__builtin_fabsf(v) < 2147483648.0f, 1))
            return __builtin_amdgcn_fmed3f(__builtin_rintf(v), lo, hi);
        return (float)code_value<BASE>(pack_code<BASE>(v));
    }
    static __device__ __forceinline__ void abf(raw_t v, int, float& A, float& B, float scale)
    {
        const float s0 = soft(v.x * scale), s1 = soft(v.y * scale);
        A = s0 + s1;
        B = s0 - s1;
    }
    static __device__ __forceinline__ void ab(raw_t v, int li, int& A, int& B, float scale)
    {
        if constexpr (BASE == FP32) {
            TgIn<FP32>::ab(make_float2(v.x * scale, v.y * scale), li, A, B, scale);
        } else if constexpr (BASE == SOFT4 || BASE == SOFT8) {
            // the integer rows of vd_decode_pk: the float codes of soft() (exact small integers) converted
            // once, instead of the x86 narrowing path of pack_code for every value (profiles/r05: the fused
            // SOFT8 batched launch spent 18 us per batch more than the packed input's)
            float fa, fb;
            abf(v, li, fa, fb, scale);
            A = (int)fa;
            B = (int)fb;
        } else {
            const int s0 = code_value<BASE>(pack_code<BASE>(v.x * scale));
            const int s1 = code_value<BASE>(pack_code<BASE>(v.y * scale));
            if constexpr (BASE == HARD) {
                A = s0 + s1 - 1;  // 1 - #mismatches against (1,1)
                B = s0 - s1;      // against (1,0)
            } else {
                A = s0 + s1;
                B = s0 - s1;
            }
        }
    }
};
template <> struct TgIn<kLlr + HARD> : TgInLlr<HARD> {};
template <> struct TgIn<kLlr + SOFT4> : TgInLlr<SOFT4> {};
template <> struct TgIn<kLlr + SOFT8> : TgInLlr<SOFT8> {};
template <> struct TgIn<kLlr + SOFT16> : TgInLlr<SOFT16> {};
template <> struct TgIn<kLlr + FP32> : TgInLlr<FP32> {};
// resource for the 96 stages from g0 (g0 a multiple of 16).
// The range min(max(availBytes - off, 0), 2^32 - 1) is computed on the scalar unit with 32-bit halves
// (SCC carries the borrow): gfx950 has no scalar 64-bit compare, and hipcc's vector compare plus its
// VCC -> scalar select stalled every group head.
template <int CH>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tg_rsrc(const void* in, uint64_t g0, uint64_t availBytes)
{
    const uint64_t off = TgIn<CH>::bytes(g0);
    // the operands are wave-uniform; readfirstlane keeps them in SGPRs where the compiler's divergence
    // analysis cannot see it (a no-op on values already scalar)
    const uint32_t ol = __builtin_amdgcn_readfirstlane((uint32_t)off), oh = __builtin_amdgcn_readfirstlane((uint32_t)(off >> 32));
    const uint32_t al = __builtin_amdgcn_readfirstlane((uint32_t)availBytes);
    const uint32_t ah = __builtin_amdgcn_readfirstlane((uint32_t)(availBytes >> 32));
    uint32_t lo, hi;
    asm("s_sub_u32 %[lo], %[al], %[ol]\n\t"
        "s_subb_u32 %[hi], %[ah], %[oh]\n\t"  // SCC = borrow: the group starts past the data
        "s_cselect_b32 %[lo], 0, %[lo]\n\t"
        "s_cselect_b32 %[hi], 0, %[hi]\n\t"
        "s_cmp_lg_u32 %[hi], 0\n\t"
        "s_cselect_b32 %[lo], -1, %[lo]"
        : [lo] "=&s"(lo), [hi] "=&s"(hi)
        : [al] "s"(al), [ah] "s"(ah), [ol] "s"(ol), [oh] "s"(oh)
        : "scc");
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)in + ((uint64_t)oh << 32 | ol)), (short)0, (int)lo, 0x00020000);
}

// ---------------------------------------------------------------- segment launches
// A launch of 6400 chunks on 1024 SIMDs, one chunk per wave, puts 7 waves on a quarter of the SIMDs and
// 6 on the rest, and the 7-wave SIMDs set the kernel time.  In a segment launch (Geom::seg) workgroup g
// decodes the consecutive chunks [seg[g], seg[g+1]) as kWaves segments of about equal length, one per
// wave; a segment may end in one chunk and continue at the start of the next (each chunk part is a
// "run").  A segment that starts at a chunk start is exact.  One that starts inside a chunk starts
// kSplitWarm blocks before its first word's emit block from equal metrics; at that boundary block it
// records its renormalised metric vector (its start vector), and the segment to its left records its own
// vector at the same block (its end vector).  Equal vectors mean every later decision of the segment
// equals the exact decode's (the recursion and the tie rules depend only on metric differences; V at a
// block start is VBASE + (metric - metric of position 0) * 2^S with cleared fields), so a segment is
// verified when its left neighbour is and the two vectors agree.  After each pass every segment that ran
// publishes its two vectors in its own (now dead) table LDS, the workgroup synchronises (s_barrier) and
// every wave evaluates the same checks.  Each unverified segment takes its left neighbour's end vector
// into a register, a second barrier lets everyone finish reading, and the unverified segments re-decode
// their first run from its boundary block (their later runs start at chunk starts and are exact).  The
// first unverified segment always restarts from an exact vector, so every pass verifies at least one
// more: at most kWaves - 1 re-decode passes, no timeouts, no flags.  Writes of a later pass follow the
// barriers, so the last (verified) decode of every word is the one that stays.  Block boundaries inside
// a chunk are multiples of 3 (the group length, 96 stages = 16 trellis periods) so every run uses the
// same position <-> state map there.  The vectors never leave the workgroup's LDS, so concurrent launches
// share no storage.  The host's tables (vd_capi.hip plan_split): 256 workgroups of one chunk in 4 pieces
// after 1536 of 4 whole chunks (7 waves per SIMD, round 2's split), or 1792 workgroups of 3 chunks and
// 256 of 4 (8 waves of 3/4 chunk or 1 chunk per SIMD, their progress kept even by the fairness controller
// in fractions of their work).
constexpr int kSplitWarm = 6;                // default warm-up blocks of a speculative segment (Geom::segWarm)
constexpr int kSplitMinWords = 64;           // chunks of fewer 32-bit words are not split (host side)
constexpr int kSegSnap = 8;                  // a boundary this close to a chunk start or end moves onto it
// a workgroup's chunks (at most kWaves) and their 32-bit word counts; wave-uniform, in scalar registers
struct SegWG {
    uint32_t c0;
    int k;
    uint32_t warm;  // warm-up blocks of a segment that starts inside a chunk (3 or 6)
    uint32_t W0, W1, W2, W3;
    __host__ __device__ __forceinline__ uint32_t W(int i) const { return i == 0 ? W0 : i == 1 ? W1 : i == 2 ? W2 : W3; }
    __host__ __device__ __forceinline__ uint32_t cum(int i) const  // words of chunks 0 .. i-1
    {
        return (i > 0 ? W0 : 0u) + (i > 1 ? W1 : 0u) + (i > 2 ? W2 : 0u) + (i > 3 ? W3 : 0u);
    }
};
struct SegPos {
    int i;       // chunk within the workgroup (k: the end)
    uint32_t a;  // local word; a > 0: (a + 1) % 3 == 0 and a >= kSegSnap > warm
};
// boundary q (0 .. kWaves) of the workgroup's segments
__host__ __device__ __forceinline__ SegPos seg_bound(const SegWG& w, int q)
{
    if (q == 0) return {0, 0u};
    if (q == kWaves) return {w.k, 0u};
    const uint32_t x = (uint32_t)q * w.cum(w.k) / kWaves;
    int i = 0;
    while (i + 1 < w.k && w.cum(i + 1) <= x) i++;
    const uint32_t a = x - w.cum(i);
    if (a < kSegSnap) return {i, 0u};
    if (w.W(i) - a < kSegSnap) return {i + 1, 0u};
    return {i, a - (a + 1) % 3};
}
// one run: chunk c0 + i, frame word 0 = chunk word s0, emits words [E, words) of the frame; Xspec / Xcmp:
// the frame blocks of its left / right boundary (-1: none)
struct RunGeo {
    int i;
    uint32_t s0, words, E;
    int Xspec, Xcmp;
};
__host__ __device__ __forceinline__ RunGeo seg_run(const SegWG& w, SegPos b0, SegPos b1, int r)
{
    RunGeo g;
    g.i = b0.i + r;
    const uint32_t a = r == 0 ? b0.a : 0u, W = w.W(g.i);
    const uint32_t b = g.i == b1.i ? b1.a : W;
    g.s0 = a == 0 ? 0u : a + 1 - w.warm;
    g.words = b - g.s0;
    g.E = a - g.s0;
    g.Xspec = a == 0 ? -1 : (int)(a + 1 - g.s0);
    g.Xcmp = b == W ? -1 : (int)(b + 1 - g.s0);
    return g;
}
__host__ __device__ __forceinline__ int seg_nruns(SegPos b0, SegPos b1) { return b1.i - b0.i + (b1.a != 0 ? 1 : 0); }

// ================================================================ the kernel: one chunk per wave
template <int CH, int CORE, int OB>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(8))) void vd_decode_tg(const void* __restrict__ in_all, void* __restrict__ out_all, Geom geo)
{
    using IN = TgIn<CH>;
    using FMT = TgFmt<CH>;
    constexpr bool INT = FMT::INT;
    static_assert(!INT || CORE == B32, "int32 patterns: SOFT16 on the int32 core only");
    // M_B32 on the fp32 patterns (S32): its phase-0 tie rule differs between the position halves (upper
    // half: own wins, tag +2^j).  Instead of rows holding both tag signs, the upper lanes read the entry of
    // the complementary label in the ordinary row (tag -2^j) and negate it: BM[3-L] = -BM[L], so
    // -(BM[3-L]*2^S - 2^j) = BM[L]*2^S + 2^j.  The stage then forms V + s*e and V_partner - s*e with
    // s = -1 in the upper half (v_fma, as cheap as v_add), and the M_B32 table is the M_B16 one.  SOFT16
    // (INT) keeps the pair rows: each lane reads its own tag sign's half.
    constexpr bool S32 = CORE == B32 && !INT;
    // the label-region table (TgTabLT; SOFT16 with its +tag phase-0 area) written with ds_write_addtid_b32
    using TT = TgTabLT<INT>;
    using LL = TgLds<TT::BYTES>;
    constexpr int J = FMT::J, S = FMT::S;
    __shared__ __attribute__((aligned(256))) uint32_t lds[kWaves * LL::WAVE];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pos = tg_pos(lane);
    uint32_t* const wlds = lds + wv * LL::WAVE;
    char* const tabb = (char*)(wlds + LL::TAB_OFF);
    uint32_t* const ring = wlds + LL::RING_OFF;
    const uint32_t ringl = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(const char*)ring;  // LDS address
    // This wave's work: chunk blockIdx.x * kWaves + wv, or, in a segment launch (Geom::seg), segment wv of
    // the workgroup's chunks -- see "segment launches" above.
    // A batched launch (Geom::nbatch > 1) decodes chunk c of batch b at launch chunk b * nchunks + c.
    const bool split = geo.seg != nullptr;
    const int piece = split ? wv : -1;
    const uint32_t gchunk = blockIdx.x * kWaves + wv;
    const uint32_t batch = geo.nbatch > 1 && !split ? gchunk / geo.nchunks : 0u;
    const void* const in = (const char*)in_all + batch * geo.inStride;
    void* const out = (char*)out_all + batch * geo.outStride;
    auto words32 = [&](uint32_t c) {  // 32-bit words traced back in chunk c
        const uint32_t w = chunk_range(geo, c).words;
        return OB == 32 ? w : (w + 1) / 2;
    };
    SegWG sw;
    if (split) {
        sw.c0 = geo.seg[blockIdx.x];
        sw.k = (int)(geo.seg[blockIdx.x + 1] - sw.c0);
        sw.warm = geo.segWarm;
        sw.W0 = words32(sw.c0);
        sw.W1 = sw.k > 1 ? words32(sw.c0 + 1) : 0u;
        sw.W2 = sw.k > 2 ? words32(sw.c0 + 2) : 0u;
        sw.W3 = sw.k > 3 ? words32(sw.c0 + 3) : 0u;
    } else {
        sw.c0 = gchunk - batch * geo.nchunks;
        sw.k = 1;
        sw.warm = 0u;
        sw.W0 = words32(sw.c0);
        sw.W1 = sw.W2 = sw.W3 = 0u;
        if (sw.W0 == 0) return;  // an empty chunk (never in a segment launch: its chunks have >= kSplitMinWords words)
    }
    // this wave's segment [b0, b1) and the segments whose start is exact (a chunk start)
    const SegPos b0 = split ? seg_bound(sw, wv) : SegPos{0, 0u}, b1 = split ? seg_bound(sw, wv + 1) : SegPos{1, 0u};
    const int nrun = seg_nruns(b0, b1);
    // guard words (Geom::check): a uniform branch, nothing when off
    if (geo.check && lane < 3 * kGuardWords) wlds[LL::guard(lane)] = kGuardPattern;

    // per-lane LDS byte offset of this position's entry in a phase-K row (row offsets are compile-time)
    const bool upper5 = (pos >> 5) & 1;
    int aK[6];
    constexpr int LSTR = TT::REGION;  // bytes between the entries of two labels
    sfor<6>([&](auto KK) {
        constexpr int K = decltype(KK)::value;
        aK[K] = LSTR * own_label(pos, K);
    });
    if constexpr (S32) aK[0] = upper5 ? 3 * LSTR - aK[0] : aK[0];  // upper half: the complementary label 3 - L
    // INT, label regions: the upper half's phase-0 entries come from the +tag area
    if constexpr (INT) aK[0] = upper5 ? TgTabLT<true>::ALT_OFF + 8 * own_label(pos, 0) : aK[0];
    const float sg0 = upper5 ? -1.0f : 1.0f;                  // S32: sign of the phase-0 entry
    const int pa5 = 4 * (lane ^ 32);           // ds_bpermute address of the xor-32 partner
    const uint32_t tbk = tb_pack<J, CORE == B32>(lane);  // traceback constants of word kb + lane (kb % 3 == 0)
    // table-build roles: lane l builds the entries at table index l (stage sA) and, lanes 0..31, index
    // 64 + l (stage sB).  (Writing a group's entries a block ahead, when they are dead, measured no
    // faster: profiles/r02/ablate_twe.log.)
    const uint64_t li = (uint64_t)(lane & 31);
    const int sA = TgTabL::stage(lane), sB = TgTabL::stage(64 + (int)li);
    const float tagv = (float)(1 << (sA % J)), tagvB = (float)(1 << (sB % J));
    const float tg0A = CORE == F16 ? tagv : -tagv;  // tag of the row's own class (stage sA)
    const float tg0B = CORE == F16 ? tagvB : -tagvB;
    const uint32_t tabl = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)tabb;  // LDS address

    // V lives in [2^23, 2^24), where the fp32 ulp is 1 and the low mantissa bits ARE the low integer
    // bits: V = 1.25*2^23 + metric*2^S + 2^(S-1) + h.  The 2^(S-1) offset keeps the history field
    // 2^(S-1) + h in (0, 2^S), so read-out and clearing are bit operations on the pattern.
    // INT: V = metric*2^S + 2^(S-1) + h as an int32, no base needed.
    constexpr uint32_t VBASE = (INT ? 0u : 0x4B200000u) + (1u << (S - 1));  // 1.25*2^23 + 2^(S-1)
    const uint32_t fnm = ~((1u << S) - 1u), fhf = 1u << (S - 1);  // field clear: (p & fnm) | fhf
    Fair fair;  // fairness controller (vd_kernels.h)
    // In a batched launch only the last batch's waves run the controller: earlier batches' waves are
    // followed by more work on their SIMD, so evening out progress buys nothing there and costs issue
    // (1.6 % per batch, profiles/r02/benchab_fair2.log).
    fair.begin(batch + 1 < geo.nbatch ? nullptr : geo.fair, lane);
    // fairness progress: blocks started, or in a segment launch the fraction of the segment's pass-0
    // blocks started, scaled to 2^20 (its waves differ in length)
    uint32_t fscale = 1u;
    if (split) {
        uint32_t tot = 0;
        for (int r = 0; r < nrun; r++) tot += seg_run(sw, b0, b1, r).words + 2;
        fscale = (1u << 20) / (tot ? tot : 1u);
    }
    const uint64_t availB = IN::bytes(geo.availStages);
    const uint32_t vo1 = IN::voff(sA), vo2 = IN::voff(sB);
    // segment workgroups (uniform bookkeeping): bit q of `verified` = segment q checked exact (segments
    // that start at a chunk start are exact).  vS / vE: this segment's start / end vector; vIn: the vector a
    // re-decode starts from (left neighbour's end vector).
    uint32_t verified = 1u;
    if (split)
        for (int q = 1; q < kWaves; q++)
            if (seg_bound(sw, q).a == 0) verified |= 1u << q;
    float vS = 0.0f, vE = 0.0f, vIn = 0.0f;
    uint32_t fdone = 0;  // blocks of the segment's earlier runs (fairness progress)
    for (int pass = 0;; pass++) {
    const bool runs = piece < 0 || pass == 0 || !((verified >> piece) & 1u);
    if (runs) {
    for (int run = 0; run < (pass == 0 ? nrun : 1); run++) {  // a re-decode pass re-runs the first run only
    // the words of this run: [s0, s0 + Sw) of its chunk, written from word s0 + E on; Xspec / Xcmp: the
    // group-start blocks of the segment's left / right boundary in this run (-1: none)
    const RunGeo rg = seg_run(sw, b0, b1, run);
    const uint32_t s0 = rg.s0, Sw = rg.words, E = rg.E;
    const int Xspec = rg.Xspec, Xcmp = rg.Xcmp;
    const ChunkRange cr = chunk_range(geo, sw.c0 + (uint32_t)rg.i);
    // local word k = chunk word s0 + k (32-bit words; O_B16 writes each as two 16-bit words)
    const uint64_t wOut = cr.startWord + s0;  // O_B32: output word of local word 0
    const uint64_t start = (uint64_t)cr.startWord * OB + 32ull * s0;  // first stage of the run
    const uint32_t nblk = Sw + 2;
    // a re-decode starts at the piece's boundary block from its left neighbour's latest end vector
    float V = pass == 0 ? __builtin_bit_cast(float, VBASE) : vIn;
    if (pass > 0) vS = V;
    const uint32_t j0 = pass == 0 ? 0u : (uint32_t)Xspec;
    uint32_t kb = 0;
    uint32_t tbn = pass == 0 ? LL::TBS - 3 * (blockIdx.x & 3) : LL::TBS;
    __amdgpu_buffer_rsrc_t rs = tg_rsrc<CH>(in, start + 32ull * j0, availB);
    typename IN::raw_t rA = IN::template load<0>(rs, vo1);               // stage sA of the group
    typename IN::raw_t rB = IN::template load<0>(rs, vo2);               // stage sB

    // Branch-metric table reads, software-pipelined: the entries of stage r are loaded TGD stages
    // ahead; one ds_read_b64 at an even period also carries the entry of the stage 6 later.  The
    // loads are volatile LDS-address-space loads so they stay single ds_read_b64s (2 LDS cycles) in
    // program order -- left alone the compiler merges neighbours into ds_read2_b64 (8 cycles).
    constexpr int TGD = 4;  // 6 or 8 measured the same (profiles/r02/ablate_prefetch.log)
    typedef __attribute__((address_space(3))) const volatile f2v* lptr;
    const __attribute__((address_space(3))) char* tl = (const __attribute__((address_space(3))) char*)tabb;
    f2v vp[96];  // entry pair read for stage r (the even period of a period pair)
    auto issue = [&](auto Rc) {
        constexpr int r = decltype(Rc)::value;  // stage within the group (the group starts at phase 0)
        constexpr int K = r % 6;
        if constexpr ((r / 6) % 2 == 0) {
            vp[r] = *(lptr)(tl + aK[K] + TT::row(r));
        }
    };
    auto block = [&](auto PHc, uint32_t j) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int BB = PH / 2;
        uint32_t word = 0;
        sfor<32>([&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int K = (PH + i) % 6;
            constexpr int Q = (K + 5) % 6;
            constexpr int r = 32 * BB + i;  // stage within the group
            constexpr bool ODD = (r / 6) % 2 == 1;
            constexpr int RP = ODD ? r - 6 : r;  // where this stage's pair was read
            const f2v e = vp[RP];
            const float m = ODD ? e.y : e.x;
            // Q = 0..3: DPP stage (lane xor 1, 2, 7, 8); Q = 4: xor 16 through ds_swizzle; Q = 5: xor 32
            // through ds_bpermute
            if constexpr (INT) {
                // (SOFT16's phase-0 entries differ in the tag sign between the xor-32 partners: no pre form)
                if constexpr (Q <= 3) tg_stage_dpp_i2<Q>(V, m);
                else if constexpr (Q == 4) tg_stage_lds_pre<false, true>(V, m, pa5);
                else tg_stage_lds_i(V, m, tg_partner(V, pa5));
            } else {
                if constexpr (Q <= 3) tg_stage_dpp2<Q>(V, m);
                else if constexpr (Q == 4) tg_stage_lds_pre<false, false>(V, m, pa5);
                else if constexpr (S32) tg_stage_lds_sg(V, m, tg_partner(V, pa5), sg0);
                else tg_stage_lds_pre<true, false>(V, m, pa5);
            }
            if constexpr (r + TGD < 96) issue(std::integral_constant<int, r + TGD>{});
            if constexpr (i % J == J - 1) {
                // field read-out: bits 1..J of the pattern, (2^(S-1) + h) >> 1 = (h + 2^J - 1) / 2, go straight
                // into byte / half g of the block's ring word (SDWA dst_sel: one op for shift and merge), then
                // the field is cleared to 2^(S-1).  At the end of every block (32 stages) the decision-neutral
                // renormalisation by the metric of position 0 follows: readfirstlane (1 wait state after the
                // clear), the offset on the scalar unit, one vector subtract.  s_sub_u32 writes SCC: the
                // statements with VD_TG_RN declare it clobbered (without that, a compiler that keeps a branch
                // condition in SCC across them decodes wrong words: profiles/r02/scc_clobber_check.log).
                constexpr int g = (i % 32) / J;
                uint32_t sr;
#define VD_TG_RO(SEL, UNUSED) "v_lshrrev_b32_sdwa %[w], 1, %[V] dst_sel:" SEL " dst_unused:" UNUSED             \
                              " src0_sel:DWORD src1_sel:DWORD\n\tv_bitop3_b32 %[V], %[V], %[fnm], %[fhf] bitop3:0xea"
#define VD_TG_RN "\n\ts_nop 0\n\tv_readfirstlane_b32 %[sr], %[V]\n\ts_sub_u32 %[sr], %[sr], %[vb]\n\tv_subrev_u32 %[V], %[sr], %[V]"
#define VD_TG_IN [fnm] "v"(fnm), [fhf] "s"(fhf), [vb] "n"(VBASE)  // fhf on the constant bus: one VGPR fewer
                if constexpr (J == 8 && g == 0)
                    asm(VD_TG_RO("BYTE_0", "UNUSED_PAD") : [V] "+{v60}"(V), [w] "=&v"(word) : VD_TG_IN);
                else if constexpr (J == 8 && g == 1)
                    asm(VD_TG_RO("BYTE_1", "UNUSED_PRESERVE") : [V] "+{v60}"(V), [w] "+v"(word) : VD_TG_IN);
                else if constexpr (J == 8 && g == 2)
                    asm(VD_TG_RO("BYTE_2", "UNUSED_PRESERVE") : [V] "+{v60}"(V), [w] "+v"(word) : VD_TG_IN);
                else if constexpr (J == 8)
                    asm(VD_TG_RO("BYTE_3", "UNUSED_PRESERVE") VD_TG_RN : [V] "+{v60}"(V), [w] "+v"(word), [sr] "=&s"(sr) : VD_TG_IN : "scc");
                else if constexpr (g == 0)
                    asm(VD_TG_RO("WORD_0", "UNUSED_PAD") : [V] "+{v60}"(V), [w] "=&v"(word) : VD_TG_IN);
                else
                    asm(VD_TG_RO("WORD_1", "UNUSED_PRESERVE") VD_TG_RN : [V] "+{v60}"(V), [w] "+v"(word), [sr] "=&s"(sr) : VD_TG_IN : "scc");
#undef VD_TG_IN
#undef VD_TG_RN
#undef VD_TG_RO
            }
        });
        // ring word of position p: byte (J=8) / half (J=16) g = the J path bits of the survivor that
        // ends at p at the end of history field g of this block, stage 8g+j (16g+j) at bit j of it;
        // the bits mark the tie-winning candidate, i.e. the take-bit except where the own one wins (F16)
        if constexpr (CORE == F16) word = ~word;
        wave_sync();
        if (j >= 1) ring[(j - 1 - kb) * 64 + pos] = word;
        if (j >= 2 && (j - 1 - kb == tbn || j == nblk - 1)) {
            wave_sync();
            const uint32_t nw = j - 1 - kb;
            if ((uint32_t)lane < nw && kb + lane >= E) {
                const uint32_t k = kb + (uint32_t)lane;
                // with TBS a multiple of 3 (12: the fp32 cores' label-region table) every batch starts at a
                // multiple of 3 (batches of TBS - 3 (blockIdx.x & 3) or TBS words), so word k's phase follows
                // from the lane; otherwise (SOFT16: 11) from k.  The M_B32 kernels have no VGPR to keep the
                // lane's constants in (64 at 8 waves per SIMD) and compute them here.
                const TbC tc = LL::TBS % 3 == 0 && CORE != B32 ? tb_unpack<CORE == B32>(tbk) : tb_direct<J, CORE == B32>((int)k);
                uint32_t w;
                if constexpr (J == 8) {
                    const uint32_t sft[3] = {tc.off[0] - 2u, tc.off[1] - 2u, tc.off[2] - 2u};
                    const uint32_t m5[3] = {tc.m50, tc.m50 >> 2, tc.m50 >> 4};  // (traceback_word_tg's m5)
                    w = tg8_traceback<CORE == B32>(ringl + 256u * (uint32_t)lane, sft, m5);
                } else {
                    w = traceback_word_tg<J, CORE == B32>((const char*)ring, (uint32_t)(lane + 1) * 256u, tc);
                }
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[wOut + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + cr.startWord;
                    const uint32_t kc = s0 + k;
                    o[2 * kc] = (uint16_t)(w >> 16);
                    if (2 * kc + 1 < cr.words) o[2 * kc + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            wave_sync();
            ring[pos] = word;  // block j becomes slot 0 of the next batch
            kb = j - 1;
            tbn = LL::TBS;
        }
        return j + 1 < nblk;
    };
    // the four entries of a stage from its (A, B) = (BM[3], BM[2]): E[L] = BM[L]*2^S + tag, one per label
    // region (INT phase-0 stages also the +tag entries of the ALT area); part 0: the entries of stage sA
    // (all lanes), part 1: of stage sB (lanes 0..31)
    auto put_row = [&](auto PT, auto A, auto B, int K) {  // A, B: ints, or floats (IN::FAB)
        constexpr int part = decltype(PT)::value;
        const float tg0 = part ? tg0B : tg0A;
        if constexpr (INT) {
            // the tag of the entry's own class: -2^j (the int32 core: exchanged wins ties)
            const int a = A * (1 << S), b = B * (1 << S), tag = -(int)tg0;
            auto f = [](int x) { return __builtin_bit_cast(float, x); };
            lds_write_addtid4<256 * part, TT::REGION>(tabl, f(-a - tag), f(-b - tag), f(b - tag), f(a - tag));
            if (K == 0)  // phase-0 lanes: the +tag entries (ALT), at dword ALT + index + 2L
                lds_write_addtid4<TT::ALT_OFF + 256 * part, 8>(tabl, f(-a + tag), f(-b + tag), f(b + tag), f(a + tag));
            return;
        }
        constexpr float SC = (float)(1 << S);
        const float af = (float)A, bf = (float)B;
        const float E0 = __builtin_fmaf(af, -SC, tg0), E1 = __builtin_fmaf(bf, -SC, tg0);
        const float E2 = __builtin_fmaf(bf, SC, tg0), E3 = __builtin_fmaf(af, SC, tg0);
        lds_write_addtid4<256 * part, TgTabL::REGION>(tabl, E0, E1, E2, E3);
    };
    // S01: entries from the two soft values (six FMAs) instead of (A, B) = (s0 + s1, s0 - s1) (two integer
    // ops, two converts, four FMAs); fp32 cores
    constexpr bool S01 = HasS01<IN>::value && !INT;
    auto put_row_s01 = [&](auto PT, float s0, float s1) {
        constexpr int part = decltype(PT)::value;
        const float tg0 = part ? tg0B : tg0A;
        constexpr float SC = (float)(1 << S);
        const float X = __builtin_fmaf(s0, SC, tg0), Y = __builtin_fmaf(s0, -SC, tg0);
        lds_write_addtid4<256 * part, TgTabL::REGION>(tabl, __builtin_fmaf(s1, -SC, Y), __builtin_fmaf(s1, SC, Y),
                                                      __builtin_fmaf(s1, -SC, X), __builtin_fmaf(s1, SC, X));
    };
    const int r6a = sA % 6, r6b = sB % 6;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    for (uint32_t j = j0;; j += 3) {
        // group head: the table from the inputs loaded one group ago, the next group's loads, then the
        // fairness board (its load returns during this group; nothing here waits on it)
        if constexpr (S01) {
            float s0, s1;
            IN::s01(rA, s0, s1);
            put_row_s01(P0{}, s0, s1);
            if (lane < 32) {
                IN::s01(rB, s0, s1);
                put_row_s01(P1{}, s0, s1);
            }
        } else {
            using ab_t = std::conditional_t<IN::FAB, float, int>;
            auto ab = [&](const typename IN::raw_t& raw, int l, ab_t& A, ab_t& B) {
                if constexpr (IN::FAB) IN::abf(raw, l, A, B, geo.scale);
                else IN::ab(raw, l, A, B, geo.scale);
            };
            ab_t A, B;
            ab(rA, sA, A, B);
            put_row(P0{}, A, B, r6a);
            if (lane < 32) {
                ab(rB, sB, A, B);
                put_row(P1{}, A, B, r6b);
            }
        }
        {  // the next group's input words
            rs = tg_rsrc<CH>(in, start + 32ull * (j + 3), availB);
            rA = IN::template load<0>(rs, vo1);
            rB = IN::template load<0>(rs, vo2);
        }
        // every other group head (6 blocks): 0.7 % faster than every head, every third is 1 % slower
        // (profiles/r02/benchab_fair.log)
        if ((j / 3) % 2 == 0) fair.group((fdone + j) * fscale, 3u * fscale, lane);
        if (split && pass == 0 && (int)j == Xspec) vS = V;
        if (split && (int)j == Xcmp) vE = V;
        wave_sync();
        sfor<TGD>([&](auto X) { issue(X); });
        if (!block(std::integral_constant<int, 0>{}, j)) break;
        if (!block(std::integral_constant<int, 2>{}, j + 1)) break;
        if (!block(std::integral_constant<int, 4>{}, j + 2)) break;
        wave_sync();
    }
    fdone += nblk - j0;
    }  // run
    if (split) {  // publish the segment's vectors in this wave's table LDS (dead after the run)
        wave_sync();
        float* pub = (float*)tabb;
        pub[lane] = vS;
        pub[64 + lane] = vE;
    }
    }  // runs
    if (piece < 0) break;
    // split workgroup: evaluate the boundary checks (every wave the same), then re-decode what failed
    __syncthreads();
    auto vec = [&](int q, int which) {  // segment q's start (0) / end (1) vector, this lane's entry
        return __builtin_bit_cast(uint32_t, ((const float*)(lds + q * LL::WAVE + LL::TAB_OFF))[64 * which + lane]);
    };
    for (int q = 1; q < kWaves; q++)
        if (!((verified >> q) & 1u) && ((verified >> (q - 1)) & 1u) && __ballot(vec(q, 0) != vec(q - 1, 1)) == 0)
            verified |= 1u << q;
    if (verified == (1u << kWaves) - 1u) break;
    if (!((verified >> piece) & 1u)) {
        vIn = __builtin_bit_cast(float, vec(piece - 1, 1));
        if (lane == 0 && geo.stats) atomicAdd(geo.stats, 1u);
    }
    __syncthreads();  // the next pass overwrites the published vectors read above
    }  // pass
    fair.end(lane);
    if (geo.check) {  // guard words intact?  count the ones that are not
        wave_sync();
        const bool bad = lane < 3 * kGuardWords && wlds[LL::guard(lane)] != kGuardPattern;
        const uint32_t nbad = (uint32_t)__builtin_popcountll(__ballot(bad));
        if (lane == 0 && nbad) atomicAdd(geo.check, nbad);
    }
}

}  // namespace vd
