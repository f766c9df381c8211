// vd_kernel_pk.h -- vd_decode_pk<CH, CORE, OB, SPL>: HARD, SOFT4, SOFT8 or FP32 input, two trellis chains per
// wave, one in each 16-bit half of the lane's metric word: two chunks (batched launches) or two parts of one
// chunk (SPL: single-batch split launches, below).  Same decode as vd_decode_tg<CH, CORE, OB> word for word
// (reference viterbi_core, src/viterbi/viterbi.cu:144-207; tie rules viterbiACS.cuh:113-157,216-256; the
// int16x2 idea of selfPM/pairPM<M_B16>, viterbiACS.cuh:113-119,216-220).
//
// Why it is exact.  R stages after a renormalisation (position 0's metric subtracted from every lane) every
// metric lies within [-D, D + (R-1) BMmax] of position 0's: the largest never decreases, grows by at most
// BMmax per stage, and every metric is within D of it.  A candidate's metric part is a metric plus a branch
// metric, so within [-(D + BMmax), D + R BMmax] units of 2^S, and the history field (tags included) adds
// [0, 2^S).  With V = BASE + metric * 2^S + field (vd_decode_tg's INT tagged scheme, J-stage fields, S = J + 1)
// that range sits inside an unsigned 16-bit half (tests/test_metric_range.py::test_packed_halves_fit):
//   HARD   BMmax 1, D 12, J 8, S 9, R 96 (once per group), BASE 7680: values in [1024, 63488);
//   SOFT4 / FP32   BMmax 16, D 192, J 4, S 5, R 32, BASE 8192: values in [1536, 30752);
//   SOFT8  BMmax 256, D 2816, J 2, S 3, R 8, BASE 25600: values in [1024, 64520).
// SOFT8's D: two labels differing in one output bit differ by 2|s| <= 256, and PM[T1] - PM[T2] is at most the
// BM difference along the two 6-stage paths into T1 and T2 from T1's survivor origin, i.e. 256 times the
// Hamming weight of the first six output pairs of the code driven by T1 ^ T2 from the zero state, at most 11
// for (0171, 0133): D = 2816 instead of (K-1)(BMmax - BMmin) = 3072, which would not fit 2-stage fields.
// Two chunks' metrics VA, VB sit in one 32-bit word V = VB * 2^16 + VA, and a table entry holds both chunks'
// entries as the integer m = EB * 2^16 + EA (signed halves).  32-bit integer addition is a ring homomorphism:
// V + m = (VB + EB) * 2^16 + (VA + EA) exactly, and the word's halves ARE VA + EA and VB + EB whenever both
// lie in [0, 2^16) -- which the bound guarantees for every sum the kernel forms.
//
// So one v_add_u32 / v_sub_u32 adds for both chunks, v_pk_max_u16 takes both maxima, and the DPP exchange
// rides on the subtraction (v_sub_u32_dpp: the partner's V minus the shared entry).  A DPP stage is
// v_add_u32 + v_sub_u32_dpp + v_pk_max_u16 for two chunk-states, an LDS-exchange stage v_sub_u32 +
// v_add_u32 + v_pk_max_u16 with one crossbar round trip for both chunks; renormalisation is readfirstlane /
// s_sub / v_subrev (or v_xad) on the whole word (again a homomorphism).
//
// Batched: the two chunks of a wave are consecutive chunks 2w, 2w+1 of the launch (the same batch: 6400 is
// even); they decode in lockstep over the longer one's blocks, each emitting only its own words.  LDS per wave
// (PkLds): [ring | guard | label-region table with the +tag area (TgTabLT<true>) | guard | guard]; 6 ring slots
// of 512 B (both chunks) in a wave's 5,120 B at 8 waves per SIMD, 7 in 5,632 B at 7 (batched SOFT8 and FP32,
// split launches), so a traceback batch traces 5 (6) words per chunk, both chunks' words in one pass (lanes
// 0..4 (0..5) chunk A, lanes 32.. chunk B).
//
// Read-out.  Every field clear is (V & ~field) | base as one v_bitop3_b32 (2 cycles; v_and_or_b32 takes 4,
// profiles/r05/ubench12.log).
//  * J = 8 (HARD): x = V >> 1 puts each half's take-bits in bytes 0 and 2; an odd field's x and the even
//    field's before it become ring word g / 2 = [B odd, A odd, B even, A even] by one v_perm_b32.
//  * J = 4 (SOFT4 / FP32): nibble g of the ring word; field pairs are gathered as c = (V >> 1) of the even
//    field and (V << 3) of the odd one selected into the high nibbles (v_bitop3_b32; chunk A's two fields in
//    byte 0, chunk B's in byte 2), and at the block end four v_perm_b32 turn the four pair words into the two
//    ring words.
//  * J = 2 (SOFT8): after a field F = 4 + h is odd, its take-bits d = bits 1, 2.  x = V & 0x00060006 (both
//    halves, v_and_b32), V = (V & ~7) | 4 per half (v_bitop3_b32) puts F back to 4; every fourth field instead
//    V = (V ^ x) + VBASE - 0x00010001 - (V of position 0 & ~7 in each half) (v_xad_u32, the constant on the
//    scalar unit) clears and renormalises at once; v_lshl_or_b32 collects d into bits 2g of two pair words
//    (fields 0..7 and 8..15; chunk A low, chunk B high half) that are the block's two ring words as they stand.
// Tracebacks (2-cycle VALU ops but a multiply and a perm per field; the per-pass phase constants rotated by
// one v_perm_b32): pk8_traceback (HARD), pk4_traceback (SOFT4 / FP32), pk2_traceback (SOFT8: position space.
// The ring is indexed by p' = rotl6(p, 1), where the two stages of a field (t0 even, t0 + 1) flip position bits
// q' = t0 % 6 and t0 % 6 + 1 (never wrapping).  Tracing back is then position arithmetic: from p' = 0 (state
// 0) at a block end, each field back is p' ^= d << (t0 % 6), and the field's two decoded bits are bits
// t0 % 6, t0 % 6 + 1 of the new p' (the stored bit of an M_B32 phase-0 stage in the upper position half, an
// own-won tag, is complemented once per block so that every stored bit is a take-bit).  A lane keeps its LDS
// read address A = slot | 4 p', so a step is one ds_read_u8_d16_hi at a constant offset and three 2-cycle
// VALU ops: 32 dependent steps per word; tools/pk2_model.py replays the scheme against the reference).
#pragma once
#include "vd_kernel_tg.h"

namespace vd {

// packed stages: V pinned to v60 like the other kernels
template <int Q>
__device__ __forceinline__ void pk_stage_dpp(uint32_t& V, uint32_t m)
{
    uint32_t a, b;
#define VD_PK_DPP(CTRL)                                                                                      \
    asm("v_add_u32 %1, %0, %3\n\ts_nop 0\n\tv_sub_u32_dpp %2, %0, %3 " CTRL " row_mask:0xf bank_mask:0xf\n\t" \
        "v_pk_max_u16 %0, %1, %2"                                                                            \
        : "+{v60}"(V), "=&v"(a), "=&v"(b) : "v"(m))
    if constexpr (Q == 0) VD_PK_DPP("quad_perm:[1,0,3,2]");
    else if constexpr (Q == 1) VD_PK_DPP("quad_perm:[2,3,0,1]");
    else if constexpr (Q == 2) VD_PK_DPP("row_half_mirror");
    else VD_PK_DPP("row_ror:8");
#undef VD_PK_DPP
}
// LDS exchange, subtraction before the exchange (the partners share label and tag); SWZ: the ds_swizzle
// bitmask-mode pattern of the lane xor (0x401F: xor 16), 0: ds_bpermute (xor 32)
template <int SWZ>
__device__ __forceinline__ void pk_stage_lds_pre(uint32_t& V, uint32_t m, int paddr)
{
    uint32_t a, b;
    asm("v_sub_u32 %0, %1, %2" : "=v"(b) : "v"(V), "v"(m));
    const uint32_t bp = SWZ == 0 ? (uint32_t)__builtin_amdgcn_ds_bpermute(paddr, (int)b)
                                 : (uint32_t)__builtin_amdgcn_ds_swizzle((int)b, SWZ);
    asm("v_add_u32 %0, %1, %2" : "=v"(a) : "v"(V), "v"(m));
    asm("v_pk_max_u16 %0, %1, %2" : "={v60}"(V) : "v"(a), "v"(bp));
}
// LDS exchange of V itself (M_B32's phase-0 stage: the partners' tag signs differ)
__device__ __forceinline__ void pk_stage_lds_post(uint32_t& V, uint32_t m, int paddr)
{
    const uint32_t vp = (uint32_t)__builtin_amdgcn_ds_bpermute(paddr, (int)V);
    uint32_t a, b;
    asm("v_add_u32 %1, %0, %3\n\tv_sub_u32 %2, %4, %3\n\tv_pk_max_u16 %0, %1, %2"
        : "+{v60}"(V), "=&v"(a), "=&v"(b) : "v"(m), "v"(vp));
}

// metric format per input (CH >= kLlr: float channel values quantised in the table build as for the base
// format, vd_kernel_tg.h TgInLlr): history field length J, scale 2^S, base of a half, stages between
// renormalisations RN
template <int CH>
struct PkFmt {
    static constexpr int B = CH & 7;
    static constexpr bool P2 = B == SOFT8;  // 2-stage fields, position-space ring (header)
    static constexpr int J = B == HARD ? 8 : P2 ? 2 : 4;
    static constexpr int S = J + 1;
    static constexpr uint32_t BASE = B == HARD ? 7680u : P2 ? 25600u : 8192u;
    static constexpr int RN = B == HARD ? 96 : P2 ? 8 : 32;
    static_assert(B == HARD || B == SOFT4 || B == SOFT8 || B == FP32, "int16 halves hold HARD, SOFT4, SOFT8 and FP32 metrics");
};

// LDS layout of a wave (words), for NW resident workgroups (waves per SIMD) per CU.  The ring leads (its slots
// are 256-B aligned for the OR / XOR addressing of the tracebacks): [ring | guard | table | guard | guard], a
// slot = two words per position (HARD: fields 0, 1 and 2, 3, chunk A in the even, chunk B in the odd bytes;
// SOFT8: fields 0..7 and 8..15, chunk A in the low, chunk B in the high half; SOFT4 / FP32: chunk A's nibbles
// of fields 0..7, then chunk B's, 256 B apart)
template <int NW = 8>
struct PkLds {
    static constexpr int GW = kGuardWords;
    static constexpr int TAB = TgTabLT<true>::BYTES / 4;
    static constexpr int LDSW = 163840 / 4 / (NW * kWaves);                // a wave's share
    static constexpr int TBS = (LDSW - 3 * GW - TAB) / 128 - 1;            // words per traceback batch and chunk
    static constexpr int RING = (TBS + 1) * 64;                            // words per chunk
    static constexpr int TAB_OFF = 2 * RING + GW, RING_OFF = 0;
    static constexpr int WAVE = (3 * GW + TAB + 2 * RING + 63) / 64 * 64;
    static __device__ __forceinline__ int guard(int i) { return 2 * RING + (i < GW ? i : TAB + i); }
};
static_assert(PkLds<8>::TBS == 5 && kWaves * PkLds<8>::WAVE * 4 <= 20480 && PkLds<8>::WAVE % 64 == 0,
              "8 workgroups of 4 waves per CU, ring slots 256-B aligned");
static_assert(PkLds<7>::TBS == 6 && 7 * kWaves * PkLds<7>::WAVE * 4 <= 163840 && PkLds<7>::WAVE % 64 == 0,
              "split launches: 7 workgroups of 4 waves per CU");

// SOFT8 traceback of one word (header "Ring and traceback"): A = the lane's emit slot (block k + 1; the
// convergence block k + 2 is the next slot, +512 B) | 2 for chunk B's half; z[r] = 2 + the position bit of the
// first stage of convergence-block field g (g % 3 = r); the emit block's field g has z[(g + 2) % 3].
template <int CORE>
__device__ __forceinline__ uint32_t pk2_traceback(uint32_t A, const uint32_t (&z)[3], const uint32_t (&zm)[3], uint32_t rho,
                                                  uint32_t mlo)
{
    uint32_t nat = 0, B = 0;
    // a step: the byte holding field g loaded into bits 16..23 (ds_read_u8_d16_hi: its pair at 16 + 2 (g % 4)),
    // shifted right onto the lane's position bits z (v_sub_u32 + v_lshrrev_b32) and XORed in under the mask
    // zm = 3 << z (v_bitop3_b32): 6 cycles of 2-cycle ops where v_bfe / v_lshlrev / v_xor took 10
    auto step = [&](auto EMc, auto Gc) {
        constexpr bool EM = decltype(EMc)::value;
        constexpr int g = decltype(Gc)::value;
        constexpr int off = (EM ? 0 : 512) + 256 * (g / 8) + (g % 8) / 4;
        constexpr int r = EM ? (g + 2) % 3 : g % 3;
        // (one statement: the compiler would otherwise hoist the 12 shift amounts of a pass into registers)
        uint32_t t;
        asm volatile("ds_read_u8_d16_hi %[b], %[a] offset:%[o]\n\tv_sub_u32 %[t], %[k], %[z]\n\ts_waitcnt lgkmcnt(0)\n\t"
                     "v_lshrrev_b32 %[t], %[t], %[b]\n\tv_bitop3_b32 %[a], %[a], %[t], %[m] bitop3:0x78"  // A ^ (t & zm)
                     : [a] "+v"(A), [b] "+v"(B), [t] "=&v"(t)
                     : [o] "n"(off), [k] "n"(16 + 2 * (g % 4)), [z] "v"(z[r]), [m] "v"(zm[r]) : "memory");
        // emit block: after fields 3m + 3, 3m + 2, 3m + 1 (m = 4 .. 0) the address bits 2..7 hold their three
        // decoded pairs (each field sets the pair at its own z, and the z cycle has period 3); snapshot them
        // into bits 6m + 2 .. 6m + 7; field 0's pair goes to bits 0, 1
        if constexpr (EM && g % 3 == 1) nat |= (A & 0xFCu) << (2 * g - 2);
        if constexpr (EM && g == 0) nat |= __builtin_amdgcn_ubfe(A, z[r], 2);
    };
    sfor<16>([&](auto I) { step(std::false_type{}, std::integral_constant<int, 15 - decltype(I)::value>{}); });
    sfor<16>([&](auto I) { step(std::true_type{}, std::integral_constant<int, 15 - decltype(I)::value>{}); });
    // each 6-bit snapshot holds fields 3m + 1, 3m + 2, 3m + 3 at bits rho, rho + 2, rho + 4 (mod 6): rotate every
    // group right by rho (mlo: the groups' low 6 - rho bits) so that field g's pair lands at bits 2g, 2g + 1
    const uint32_t grp = nat & ~3u;
    nat = (nat & 3u) | ((grp >> rho) & mlo) | ((grp << (6u - rho)) & ~mlo);  // v_bfi_b32
    return __builtin_bitreverse32(nat);  // word bit i <-> stage 63+32k-i
}

// HARD traceback of one word (header "HARD ring"): vd_decode_tg's field recursion (traceback_word_tg, J = 8) on
// the ring-first layout.  base = the lane's emit slot | 1 for chunk B's bytes; sft[c] = tb_direct's off[c] - 2,
// so (TX >> sft) & 0xFC is 4 times the position of the state (TX = T * 260: T in bits 2..7 and 8..13).
template <int CORE>
__device__ __forceinline__ uint32_t pk8_traceback(uint32_t base, const uint32_t (&sft)[3], const uint32_t (&m5)[3])
{
    constexpr bool FIX5 = CORE == B32;
    uint32_t TX = 0, nat = 0;
    // a field: the address by v_lshrrev + v_bitop3 ((t & 0xFC) | base), the byte by ds_read_u8 at a constant
    // offset, Y = W ^ TX with the stride-6 fold Y ^= (Y >> 6) & 3 (v_xor, v_lshrrev, v_bitop3), M_B32's raw
    // phase-0 bits back in (v_bitop3 select), the next TX = (Y & 63) * 260, the byte into nat (v_perm):
    // 2-cycle ops but the multiply and the perm, where vd_decode_tg's form (v_bfe, v_lshl_add, v_bfe,
    // v_bfi, v_lshl_or) takes 4 cycles each
    auto step = [&](auto EMc, auto Gc) {
        constexpr bool EM = decltype(EMc)::value;
        constexpr int g = decltype(Gc)::value;
        constexpr int BO = EM ? 0 : 2;
        constexpr int c = (BO + 8 * g + 7) % 6;
        constexpr int off = (EM ? 0 : 512) + 256 * (g / 2) + 2 * (g % 2);
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

// SOFT4 / FP32 traceback of one word (4-stage fields, nibble g of the ring word; vd_decode_tg's J < 6 recursion:
// the field's decoded bits are Y = W ^ (T >> 2), the state at the field start ((T << 4) | Y) & 63).  TX = T * 260
// (T in bits 2..7 and 8..13): the address is ((TX >> sft) & 0xFC) | base as for HARD, and TX >> 4 holds both
// T >> 2 (bits 0..3) and T's low two bits at bits 4, 5, so Y = ((TX >> 4) ^ W) & 15 and the next state
// ((TX >> 4) & 0x30) | Y are one v_bitop3_b32 each.  base = the lane's emit slot + 256 for chunk B.
template <int CORE>
__device__ __forceinline__ uint32_t pk4_traceback(uint32_t base, const uint32_t (&sft)[3], const uint32_t (&m5)[3])
{
    constexpr bool FIX5 = CORE == B32;
    uint32_t TX = 0, nat = 0;
    auto step = [&](auto EMc, auto Gc) {
        constexpr bool EM = decltype(EMc)::value;
        constexpr int g = decltype(Gc)::value;
        constexpr int BO = EM ? 0 : 2;
        constexpr int c = (BO + 4 * g + 3) % 6;
        constexpr int off = (EM ? 0 : 512) + g / 2;
        const uint32_t A = __builtin_amdgcn_bitop3_b32(TX >> (sft[c / 2] & 31u), 0xFCu, base, 0xEA);
        uint32_t W = *(const __attribute__((address_space(3))) uint8_t*)(uintptr_t)(A + off);
        if constexpr (g % 2) W >>= 4;
        const uint32_t T4 = TX >> 4;
        uint32_t Y = __builtin_amdgcn_bitop3_b32(W, T4, 15u, 0x28);  // (W ^ T4) & 15
        if constexpr (FIX5) Y = __builtin_amdgcn_bitop3_b32(m5[((BO + 4 * g) % 6) / 2], W, Y, 0xCA);
        if constexpr (!(EM && g == 0)) TX = __mul24(__builtin_amdgcn_bitop3_b32(T4, 0x30u, Y, 0xEA), 260u);
        if constexpr (EM) nat |= Y << (4 * g);
    };
    sfor<8>([&](auto I) { step(std::false_type{}, std::integral_constant<int, 7 - decltype(I)::value>{}); });
    sfor<8>([&](auto I) { step(std::true_type{}, std::integral_constant<int, 7 - decltype(I)::value>{}); });
    return __builtin_bitreverse32(nat);  // word bit i <-> stage 63+32k-i
}

// Split single-batch launches (SPL).  A chunk of W words is cut into P parts at words cut(1) .. cut(P-1),
// multiples of 3 blocks; part p emits words [cut(p), cut(p+1)).  Part 0 decodes from the chunk start (equal
// metrics, as the chunk itself); part p >= 1 starts kPkWarm blocks before block cut(p) from equal metrics.
// Every origin is a multiple of 3 blocks, so the two halves of a wave see the same stage phases, table
// rows and tags in lockstep.  A wave decodes parts 2q (half A) and 2q+1 (half B).  Part p's metric vector
// at the end of chunk block cut(p)-1 (its start vector) and part p-1's at the same block (its end vector)
// are kept (renormalised; one VGPR holds two halves); equal vectors mean equal decisions from block cut(p)
// on (the recursion and the tie rules depend on metric differences only), so part p's words are exact.
// After each pass every part whose start vector differs from its left neighbour's end vector is decoded
// again from block cut(p) with that end vector; after pass k parts 0 .. k are exact, so the passes end
// (at most P; the result never depends on timing).
//  * Most chunks: one chunk per wave, P = 2 (the check is within the wave).
//  * The last nchunks mod 4 NCU chunks (tail workgroups, Geom::tailWG): one chunk per workgroup of 4 waves,
//    P = 8, so every SIMD gets 6 whole-chunk waves and one short one instead of 7 whole-chunk waves on a
//    quarter of the SIMDs; the end vectors cross waves through LDS after a workgroup barrier.
// Early stop.  A re-decode only has to run until its metric vector equals, at some group end s after the cut,
// the vector of the run whose words currently stand after s: equal vectors mean equal decisions from block
// s + 1 on, so it emits the words whose traceback windows reach back to block s or earlier (local words < s)
// and stops after block s + 1.  The vectors to compare with come from one of two places:
//  * replay (one half re-decodes for the first time, the other is idle: every re-decode of a whole-chunk
//    wave): both halves
//    restart 6 blocks before the cut from equal metrics, the idle half replaying the speculative run
//    exactly (same inputs, same arithmetic per half), the re-decoding half with the correct vector put in
//    at the cut; the two halves are compared at every group end after the cut;
//  * checkpoints (otherwise: tail workgroups only): every run of a part p >= 1 keeps its vectors
//    at the kPkChk group ends after its cut (chunk blocks cut(p) - 1 + 3m, m = 1 .. kPkChk) in registers.
// On uniformly random input 78 % of 6-block warm-ups converge, 96.5 % after one more group, 99.5 % after
// two, all 400 samples within 7 (tools/study/spec_convergence.py); at 0 dB 95 % at the cut, the rest one
// group later.
constexpr int kPkWarm = 6;
constexpr int kPkChk = 2;
__host__ __device__ constexpr uint32_t pk_cut(uint32_t p, uint32_t P, uint32_t W)
{
    // kPkWarm + 3 * round(p (W - kPkWarm) / (3 P)) for 0 < p < P (the parts' first blocks minus the warm-up
    // are multiples of 3 blocks)
    return p == 0 ? 0u : p >= P ? W : (uint32_t)kPkWarm + 3u * ((2u * p * (W - (uint32_t)kPkWarm) + 3u * P) / (6u * P));
}

// NW: waves per SIMD the LDS layout is cut for.  7 for split launches (7 workgroups per CU hold every wave
// of a single batch, so a wave's 5,632 B leave room for 6 words per traceback pass instead of 5: 1.4-1.6 %
// faster, profiles/r05/split_fairness_ab.log) and for batched SOFT8 and FP32 (their heavier stages hide
// latency with 7 waves, and the passes come 5/6 as often: 0.5-0.7 % faster against a repeated 8-wave control,
// profiles/r05/ablate_nw7.log); 8 for batched HARD and SOFT4 (HARD loses 0.6-1.6 % at 7).
template <int CH, int CORE, int OB = 32, bool SPL = false, int NW = (SPL || PkFmt<CH>::P2 || (CH & 7) == FP32) ? 7 : 8>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(SPL ? 7 : NW))) void vd_decode_pk(const void* __restrict__ in_all, void* __restrict__ out_all, Geom geo)
{
    constexpr bool P2 = PkFmt<CH>::P2;
    constexpr int J = PkFmt<CH>::J, S = PkFmt<CH>::S;
    using IN = TgIn<CH>;
    using TT = TgTabLT<true>;
    using LL = PkLds<NW>;
    constexpr bool ALT = CORE == B32;  // M_B32: the upper position half takes the +tag entries at phase 0
    __shared__ __attribute__((aligned(256))) uint32_t lds[kWaves * LL::WAVE];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pos = tg_pos(lane);
    const int ridx = P2 ? ((pos << 1) | (pos >> 5)) & 63 : pos;  // ring index (P2: p' = rotl6(p, 1))
    uint32_t* const wlds = lds + wv * LL::WAVE;
    char* const tabb = (char*)(wlds + LL::TAB_OFF);
    uint32_t* const ringA = wlds + LL::RING_OFF;
    // batched: chunks 2w, 2w+1 of the launch (batch b: launch chunks b * nchunks ..; nchunks is even);
    // SPL: chunk w, both halves; tail workgroups: one chunk, wave q its parts 2q, 2q+1
    const bool tail = SPL && blockIdx.x >= geo.tailWG;
    const uint32_t gc = !SPL ? 2u * (blockIdx.x * kWaves + (uint32_t)wv)
                             : tail ? geo.tailWG * kWaves + (blockIdx.x - geo.tailWG) : blockIdx.x * kWaves + (uint32_t)wv;
    const uint32_t batch = SPL ? 0u : gc / geo.nchunks;
    const uint32_t cA = gc - batch * geo.nchunks;
    const void* const in = (const char*)in_all + batch * geo.inStride;
    char* const out = (char*)out_all + batch * geo.outStride;
    const ChunkRange crA = chunk_range(geo, cA), crB = SPL ? crA : chunk_range(geo, cA + 1);
    if (crA.words == 0 && crB.words == 0) return;
    if (geo.check && lane < 3 * kGuardWords) wlds[LL::guard(lane)] = kGuardPattern;

    // per-lane LDS byte offsets of this position's entries per phase (vd_decode_tg's INT table)
    const bool upper5 = (pos >> 5) & 1;
    int aK[6];
    constexpr int LSTR = TT::REGION;
    sfor<6>([&](auto KK) {
        constexpr int K = decltype(KK)::value;
        aK[K] = LSTR * own_label(pos, K);
    });
    if constexpr (ALT) aK[0] = upper5 ? TT::ALT_OFF + 8 * own_label(pos, 0) : aK[0];
    // P2, M_B32: the upper position half's phase-0 bits are own-won tags; complemented at the block end
    const uint32_t up5m = upper5 ? ~0u : 0u;
    const int pa5 = 4 * (lane ^ 32);
    // table-build roles (as vd_decode_tg): lane l builds table index l (stage sA), lanes 0..31 also 64 + l (sB)
    const int sA = TgTabL::stage(lane), sB = TgTabL::stage(64 + (lane & 31));
    const int tagA = 1 << (sA % J), tagB = 1 << (sB % J);
    // entry tag of the row's own class, both halves: tg0 * 65537 (M_FP16: own wins ties, +2^j; else -2^j)
    const int32_t tg0A = (CORE == F16 ? tagA : -tagA) * 65537, tg0B = (CORE == F16 ? tagB : -tagB) * 65537;
    const uint32_t tabl = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)tabb;
    constexpr uint32_t BASE = PkFmt<CH>::BASE;
    constexpr uint32_t VB1 = BASE + (1u << (S - 1));  // a half with metric 0 and a cleared field
    constexpr uint32_t VBASE = VB1 * 65537u;
    // field clear: (V & FNM) | FHF, both halves
    constexpr uint32_t FNM = (0xFFFFu << S & 0xFFFFu) * 65537u, FHF = (1u << (S - 1)) * 65537u;
    Fair fair;
    fair.begin(batch + 1 < geo.nbatch ? nullptr : geo.fair, lane);
    const uint64_t availB = IN::bytes(geo.availStages);
    const uint32_t vo1 = IN::voff(sA), vo2 = IN::voff(sB);
    // 32-bit words traced per chunk (O_B16: each written as two 16-bit words, vd_decode_tg's policy)
    const uint32_t WA = OB == 32 ? crA.words : (crA.words + 1) / 2, WB = OB == 32 ? crB.words : (crB.words + 1) / 2;
    // the halves' jobs: origin = first chunk block of the decode, and the local words k it emits,
    // kmin <= k < kmax, as chunk words origin + k (local word k is traced from local blocks k + 1 and k + 2);
    // SPL: the local blocks whose end vectors are kept (start ss, end se; ~0u: none)
    const uint64_t stA = crA.startWord * (uint64_t)OB, stB = crB.startWord * (uint64_t)OB;
    const uint32_t P = tail ? 2u * kWaves : 2u, pA = tail ? 2u * (uint32_t)wv : 0u, pB = pA + 1u;
    uint32_t oA = 0, oB = 0, kminA = 0, kmaxA = WA, kminB = 0, kmaxB = WB;
    uint32_t ssA = ~0u, seA = ~0u, ssB = ~0u, seB = ~0u;
    // SPL early stop: local block of checkpoint 1 per half (~0u: none) and whether this run compares there;
    // replay mode: 1 = half A re-decodes (B replays), 2 = half B re-decodes (A replays); its vector at the cut
    // is its kept start vector (A: sv2 low, B: sv1 high)
    uint32_t ckA = ~0u, ckB = ~0u;
    bool rdA = false, rdB = false;
    uint32_t rpl = 0;
    if constexpr (SPL) {
        const uint32_t cA0 = pk_cut(pA, P, WA), cA1 = pk_cut(pA + 1u, P, WA), cB1 = pk_cut(pB + 1u, P, WA);
        oA = pA ? cA0 - kPkWarm : 0u;
        kminA = pA ? kPkWarm : 0u;
        kmaxA = cA1 - oA;
        ssA = pA ? kminA - 1u : ~0u;
        seA = kmaxA - 1u;
        oB = cA1 - kPkWarm;
        kminB = kPkWarm;
        kmaxB = cB1 - oB;
        ssB = kminB - 1u;
        seB = pB + 1u < P ? kmaxB - 1u : ~0u;
        ckA = pA ? kminA + 2u : ~0u;
        ckB = kminB + 2u;
    }
    uint64_t startA = stA + 32ull * oA, startB = stB + 32ull * oB;
    uint32_t nblk = (kmaxA > kmaxB ? kmaxA : kmaxB) + 2;
    uint32_t V = VBASE;
    // SPL: kept vectors, one per half: sv1 = (A's end, B's start), sv2 = (A's start, B's end) (low, high);
    // cpv[m]: the halves' vectors at checkpoint m + 1
    uint32_t sv1 = 0, sv2 = 0;
    uint32_t cpv[kPkChk > 0 ? kPkChk : 1] = {};
    uint32_t kb = 0;
    uint32_t tbn = LL::TBS - (blockIdx.x & 3u) % LL::TBS;  // staggered first traceback batches
    __amdgpu_buffer_rsrc_t rsA = tg_rsrc<CH>(in, startA, availB), rsB = tg_rsrc<CH>(in, startB, availB);
    typename IN::raw_t rAA = IN::template load<0>(rsA, vo1), rBA = IN::template load<0>(rsA, vo2);
    typename IN::raw_t rAB = IN::template load<0>(rsB, vo1), rBB = IN::template load<0>(rsB, vo2);
    // traceback roles: lanes 0..31 trace half A's words, 32..63 half B's
    const bool tbB = lane >= 32;
    const uint32_t tbl = (uint32_t)(lane & 31);
    const uint64_t tbStart = tbB ? crB.startWord : crA.startWord;
    const uint32_t tbWords = tbB ? crB.words : crA.words;
    // RF: the lane's emit-slot LDS address (chunk B: the odd bytes (HARD) / the high half of each word (SOFT8) /
    // the slot's second 64 words (SOFT4, FP32))
    const uint32_t tbA2 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(const char*)ringA +
                          512u * tbl + (tbB ? (P2 ? 2u : J == 8 ? 1u : 256u) : 0u);
    // RF: the lane's phase constants for kb = 0 in bytes 0..2 of two words; a pass rotates them by kb % 3 (one
    // v_perm_b32 each with a wave-uniform selector) instead of deriving them from k % 3 per lane.
    //  HARD, q = (k + 1) % 3 (tb_direct): sft = off - 2 = (5, 3, 1) and M_B32's phase-0 masks (0x41, 0x10, 0x04)
    //  (low bytes of m50 >> 0, 2, 4), rotated left by q;  SOFT8, u = (k + 2) % 3: z = (2, 4, 6) rotated left by u
    auto rot3 = [](uint32_t w, uint32_t r) {
        return __builtin_amdgcn_perm(w, w, r == 0u ? 0x03020100u : r == 1u ? 0x03000201u : 0x03010002u);
    };
    const uint32_t q0 = (tbl + (P2 ? 2u : 1u)) % 3u;
    // (SOFT4 / FP32: tb_direct<6> offsets, (5, 3, 1) rotated by q, are the shifts themselves: TX = T * 260)
    const uint32_t phA = rot3(P2 ? 0x00060402u : 0x00010305u, q0), phB = P2 ? 0u : rot3(0x00041041u, q0);

    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const volatile u2v* lptr;
    const __attribute__((address_space(3))) char* tl = (const __attribute__((address_space(3))) char*)tabb;
    constexpr int TGD = 4;  // table reads ahead
    u2v vp[96];
    auto issue = [&](auto Rc) {
        constexpr int r = decltype(Rc)::value;
        constexpr int K = r % 6;
        if constexpr ((r / 6) % 2 == 0) vp[r] = *(lptr)(tl + aK[K] + TT::row(r));
    };
    auto block = [&](auto PHc, uint32_t j) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int BB = PH / 2;
        uint32_t wA = 0, wB = 0;
        uint32_t cw[4];  // J = 4: field-pair words; J = 2, 8: the two ring words
        uint32_t xe;     // J = 8: the even field's take-bits
        (void)cw;
        (void)xe;
        sfor<32>([&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int K = (PH + i) % 6;
            constexpr int Q = (K + 5) % 6;
            constexpr int r = 32 * BB + i;
            constexpr bool ODD = (r / 6) % 2 == 1;
            constexpr int RP = ODD ? r - 6 : r;
            const uint32_t m = ODD ? vp[RP].y : vp[RP].x;
            // (the xor-8 and xor-7 stages through ds_swizzle too, 8 cycles of VALU instead of 10: +0.6 % / +5.5 %
            // per HARD batch, the LDS pipe being the other busy resource: profiles/r05/abx_lds_exchanges.log)
            if constexpr (Q <= 3) pk_stage_dpp<Q>(V, m);
            else if constexpr (Q == 4) pk_stage_lds_pre<0x401F>(V, m, pa5);
            else if constexpr (ALT) pk_stage_lds_post(V, m, pa5);
            else pk_stage_lds_pre<0>(V, m, pa5);
            if constexpr (r + TGD < 96) issue(std::integral_constant<int, r + TGD>{});
            if constexpr (i % J == J - 1) {
                // field read-out, both chunks, then both fields cleared; renormalisation on the whole word
                // (vd_decode_tg) every RN stages
                constexpr int g = (i % 32) / J;
                uint32_t sr;
#define VD_PK_RN "\n\ts_nop 0\n\tv_readfirstlane_b32 %[sr], %[V]\n\ts_sub_u32 %[sr], %[sr], %[vb]\n\tv_subrev_u32 %[V], %[sr], %[V]"
#define VD_PK_IN [fnm] "v"(FNM), [fhf] "s"(FHF), [vb] "n"(VBASE)
                if constexpr (J == 2) {
                    // x = both take-bit pairs; V = (V ^ x) + 0x00030003 (F odd: back to 4), every fourth field
                    // + the renormalisation, VBASE - 0x00010001 - (position 0's V & ~7 per half) (header)
                    constexpr int h = g % 8;
                    uint32_t x;
                    if constexpr (i % PkFmt<CH>::RN == PkFmt<CH>::RN - 1)
                        asm("v_and_b32 %[x], 0x60006, %[V]\n\ts_nop 0\n\tv_readfirstlane_b32 %[sr], %[V]\n\t"
                            "s_and_b32 %[sr], %[sr], 0xfff8fff8\n\ts_sub_u32 %[sr], %[vb], %[sr]\n\t"
                            "v_xad_u32 %[V], %[V], %[x], %[sr]"
                            : [V] "+{v60}"(V), [x] "=&v"(x), [sr] "=&s"(sr) : [vb] "n"(VBASE - 0x10001u) : "scc");
                    else  // the clear as (V & ~7) | 4 per half: v_bitop3_b32 (2 cycles; v_xad_u32 takes 4)
                        asm("v_and_b32 %[x], 0x60006, %[V]\n\tv_bitop3_b32 %[V], %[V], %[m], %[c] bitop3:0xea"
                            : [V] "+{v60}"(V), [x] "=&v"(x) : [m] "v"(0xFFF8FFF8u), [c] "s"(0x40004u));
                    // one v_lshl_or_b32 per field (left to itself the compiler paired fields as two shifts
                    // and a v_or3_b32: 1.5 ops per field)
                    if constexpr (h == 0) cw[g / 8] = x >> 1;
                    else asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(cw[g / 8]) : "v"(x), "n"(2 * h - 1));
                } else if constexpr (J == 8) {
                    // x = V >> 1: each half's take-bits (bits 1..8) in bytes 0 and 2; an odd field's x and the
                    // even field's before it become ring word g / 2 = [B odd, A odd, B even, A even] by one
                    // v_perm_b32 (2 + 2 + 2 cycles per field for both chunks, where two SDWA shifts took 8)
#define VD_PK_RO8E "v_lshrrev_b32 %[x], 1, %[V]\n\tv_bitop3_b32 %[V], %[V], %[fnm], %[fhf] bitop3:0xea"
#define VD_PK_RO8O                                                                                    \
    "v_lshrrev_b32 %[t], 1, %[V]\n\tv_bitop3_b32 %[V], %[V], %[fnm], %[fhf] bitop3:0xea\n\t"           \
    "v_perm_b32 %[c], %[t], %[x], %[sel]"
                    uint32_t t;
                    uint32_t& x8 = xe;  // (named: asm operands alone do not capture)
                    uint32_t& c8 = cw[g / 2];
                    if constexpr (g % 2 == 0)
                        asm(VD_PK_RO8E : [V] "+{v60}"(V), [x] "=&v"(x8) : VD_PK_IN);
                    else if constexpr (g == 1)
                        asm(VD_PK_RO8O : [V] "+{v60}"(V), [t] "=&v"(t), [c] "=v"(c8) : [x] "v"(x8), [sel] "s"(0x06040200u), VD_PK_IN);
                    else if constexpr (PH != 4)  // (RN = 96: the renormalisation ends the group's last block)
                        asm(VD_PK_RO8O : [V] "+{v60}"(V), [t] "=&v"(t), [c] "=v"(c8) : [x] "v"(x8), [sel] "s"(0x06040200u), VD_PK_IN);
                    else
                        asm(VD_PK_RO8O VD_PK_RN
                            : [V] "+{v60}"(V), [t] "=&v"(t), [c] "=v"(c8), [sr] "=&s"(sr)
                            : [x] "v"(x8), [sel] "s"(0x06040200u), VD_PK_IN : "scc");
#undef VD_PK_RO8E
#undef VD_PK_RO8O
                } else {
                    // bits 1..4 of each half: the even field's as V >> 1, the odd field's (V << 3) into the
                    // high nibbles of the pair word (chunk A byte 0, chunk B byte 2) by a v_bitop3_b32 select
                    constexpr uint32_t HN = 0x00F000F0u;
#define VD_PK_RO4E "v_lshrrev_b32 %[c], 1, %[V]\n\tv_bitop3_b32 %[V], %[V], %[fnm], %[fhf] bitop3:0xea"
#define VD_PK_RO4O "v_lshlrev_b32 %[t], 3, %[V]\n\tv_bitop3_b32 %[V], %[V], %[fnm], %[fhf] bitop3:0xea\n\tv_bitop3_b32 %[c], %[hn], %[t], %[c] bitop3:0xca"
                    uint32_t t;
                    if constexpr (g % 2 == 0)
                        asm(VD_PK_RO4E : [V] "+{v60}"(V), [c] "=&v"(cw[g / 2]) : VD_PK_IN);
                    else if constexpr (g < 7)
                        asm(VD_PK_RO4O : [V] "+{v60}"(V), [c] "+v"(cw[g / 2]), [t] "=&v"(t) : VD_PK_IN, [hn] "s"(HN));
                    else
                        asm(VD_PK_RO4O VD_PK_RN
                            : [V] "+{v60}"(V), [c] "+v"(cw[g / 2]), [t] "=&v"(t), [sr] "=&s"(sr) : VD_PK_IN, [hn] "s"(HN)
                            : "scc");
#undef VD_PK_RO4E
#undef VD_PK_RO4O
                }
#undef VD_PK_IN
#undef VD_PK_RN
            }
        });
        if constexpr (J == 4) {
            // pair words c0..c3 -> ring words: A = bytes 0 of c0..c3, B = bytes 2
            const uint32_t p01 = __builtin_amdgcn_perm(cw[1], cw[0], 0x06020400u);
            const uint32_t p23 = __builtin_amdgcn_perm(cw[3], cw[2], 0x06020400u);
            wA = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
            wB = __builtin_amdgcn_perm(p23, p01, 0x07060302u);
        }
        if constexpr (J == 8) {
            wA = cw[0];
            wB = cw[1];
        }
        if constexpr (J == 2) {
            // the ring words are cw[0], cw[1]; M_B32: complement the upper half's phase-0 bits (fields g with
            // (PH + 2g) % 6 == 0: bit 0 of their pair, both chunks)
            if constexpr (ALT) {
                constexpr uint32_t F0 = (PH == 0 ? 0x1041u : PH == 2 ? 0x0410u : 0x4104u) * 65537u;  // g 0..7
                constexpr uint32_t F1 = (PH == 0 ? 0x4104u : PH == 2 ? 0x1041u : 0x0410u) * 65537u;  // g 8..15
                cw[0] ^= up5m & F0;
                cw[1] ^= up5m & F1;
            }
            wA = cw[0];
            wB = cw[1];
        }
        if constexpr (CORE == F16) {
            wA = ~wA;
            wB = ~wB;
        }
        if constexpr (SPL) {  // kept vectors (block ends: renormalised, fields cleared)
            // (VD_RARE: a real branch -- left alone the compiler turns these rare wave-uniform updates into
            // v_cndmask selects executed at every block end, about 18 cycles each at 8 waves per SIMD)
#define VD_RARE asm volatile("")
            if (j == seA) { VD_RARE; sv1 = __builtin_amdgcn_perm(sv1, V, 0x07060100u); }  // low half from V
            if (j == ssB) { VD_RARE; sv1 = __builtin_amdgcn_perm(V, sv1, 0x07060100u); }  // high half from V
            if (j == ssA) { VD_RARE; sv2 = __builtin_amdgcn_perm(sv2, V, 0x07060100u); }
            if (j == seB) { VD_RARE; sv2 = __builtin_amdgcn_perm(V, sv2, 0x07060100u); }
            if constexpr (PH == 4) {  // checkpoints are group ends (header "Early stop")
                bool stop = false;
                if (rpl) {
                    if (j == kPkWarm - 1u) {  // the cut: the re-decoding half takes the correct vector
                        VD_RARE;
                        if (rpl == 1u) V = __builtin_amdgcn_perm(V, sv2, 0x07060100u);
                        else V = __builtin_amdgcn_perm(sv1, V, 0x07060100u);
                    } else if (j > kPkWarm - 1u && __builtin_amdgcn_ballot_w64((V & 0xFFFFu) != (V >> 16)) == 0) {
                        if (rpl == 1u) kmaxA = kmaxA < j ? kmaxA : j;
                        else kmaxB = kmaxB < j ? kmaxB : j;
                        stop = true;
                    }
                }
                sfor<kPkChk>([&](auto Mc) {
                    constexpr int m = decltype(Mc)::value;
                    if (j == ckA + 3u * m) {
                        VD_RARE;
                        if (rdA && __builtin_amdgcn_ballot_w64((V & 0xFFFFu) != (cpv[m] & 0xFFFFu)) == 0) {
                            kmaxA = kmaxA < j ? kmaxA : j;
                            stop = true;
                        }
                        cpv[m] = __builtin_amdgcn_perm(cpv[m], V, 0x07060100u);
                    }
                    if (j == ckB + 3u * m) {
                        VD_RARE;
                        if (rdB && __builtin_amdgcn_ballot_w64((V >> 16) != (cpv[m] >> 16)) == 0) {
                            kmaxB = kmaxB < j ? kmaxB : j;
                            stop = true;
                        }
                        cpv[m] = __builtin_amdgcn_perm(V, cpv[m], 0x07060100u);
                    }
                });
                // (a half that stopped keeps decoding in lockstep while the other one runs; its further
                // vectors are the converged ones, so keeping them changes nothing)
                if (stop) nblk = (kmaxA > kmaxB ? kmaxA : kmaxB) + 2u;
            }
#undef VD_RARE
        }
        wave_sync();
        if (j >= 1) {
            ringA[(j - 1 - kb) * 128 + ridx] = wA;
            ringA[(j - 1 - kb) * 128 + 64 + ridx] = wB;
        }
        if (j >= 2 && (j - 1 - kb == tbn || j == nblk - 1)) {
            wave_sync();
            const uint32_t nw = j - 1 - kb;
            const uint32_t k = kb + tbl;
            if (tbl < nw && k >= (tbB ? kminB : kminA) && k < (tbB ? kmaxB : kmaxA)) {
                uint32_t w;
                const uint32_t r3 = kb % 3u;  // wave-uniform
                const uint32_t PA = rot3(phA, r3);
                if constexpr (P2) {
                    // the stage phase of the convergence block k + 2: field g of it starts at position bit
                    // 2 ((k + 2 + g) % 3); z[i]: bytes of PA (the shifts read bits 4..0 of their operand), zm =
                    // 3 << z; the emit snapshots are rotated right by rho = 2u per 6-bit group (pk2_traceback),
                    // mlo = their low 6 - rho bits: 0x04104104 (2^(6 - rho) - 1)
                    const uint32_t z[3] = {PA, PA >> 8, PA >> 16};
                    const uint32_t zm[3] = {3u << (z[0] & 31u), 3u << (z[1] & 31u), 3u << (z[2] & 31u)};  // (& 31: the shift v_lshlrev does, no C overflow)
                    const uint32_t rho = (PA & 0xFFu) - 2u;
                    const uint32_t mlo = (0x04104104u << (6u - rho)) - 0x04104104u;
                    w = pk2_traceback<CORE>(tbA2, z, zm, rho, mlo);
                } else if constexpr (J == 8) {
                    // sft[i], m5[i]: bytes of PA, PB (the shifts read bits 4..0; M_B32's select only bits 7..0)
                    const uint32_t PB = rot3(phB, r3);
                    const uint32_t sft[3] = {PA, PA >> 8, PA >> 16};
                    const uint32_t m5[3] = {PB, PB >> 8, PB >> 16};
                    w = pk8_traceback<CORE>(tbA2, sft, m5);
                } else {
                    // (m5 to the field's 4 bits: an even field's byte also holds the odd field's nibble)
                    const uint32_t PB = rot3(phB, r3);
                    const uint32_t sft[3] = {PA, PA >> 8, PA >> 16};
                    const uint32_t m5[3] = {PB & 15u, (PB >> 8) & 15u, (PB >> 16) & 15u};
                    w = pk4_traceback<CORE>(tbA2, sft, m5);
                }
                const uint32_t kc = k + (tbB ? oB : oA);  // chunk word
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[tbStart + kc] = w;
                } else {
                    uint16_t* const o = (uint16_t*)out + tbStart;
                    o[2 * kc] = (uint16_t)(w >> 16);
                    if (2 * kc + 1 < tbWords) o[2 * kc + 1] = (uint16_t)(w & 0xFFFFu);
                }
            }
            wave_sync();
            // block j becomes slot 0 of the next batch
            ringA[ridx] = wA;
            ringA[64 + ridx] = wB;
            kb = j - 1;
            tbn = LL::TBS;
        }
        return j + 1 < nblk;
    };
    // the four entries of a stage for both chunks: E[L] = BM[L] * 2^S + tg0 per half (TgFmt::INT's table),
    // from (A, B) = (BM[3], BM[2]) of each chunk packed as A_A + A_B * 2^16 (signed halves; |.| <= 16 except
    // SOFT8's 256: its entries by shifts, since BM_B * 2^16 leaves __mul24's 24 bits)
    // HARD / SOFT8 words (not the fused-LLR formats): both chunks' inputs merged into one word by v_perm_b32,
    // then (A, B) of both chunks at once in non-negative halves (PK8 below)
    constexpr bool PK8 = CH == HARD || CH == SOFT8;
    // HARD: the 16-bit half of the input word holding the lane's stage (li % 16 < 8: the high half) and the
    // shift that brings its two bits (r0, r1) to bits 1, 0
    const uint32_t hselA = (sA & 15) < 8 ? 0x07060302u : 0x05040100u, hselB = (sB & 15) < 8 ? 0x07060302u : 0x05040100u;
    const uint32_t hshA = 14u - 2u * (uint32_t)(sA & 7), hshB = 14u - 2u * (uint32_t)(sB & 7);
    auto put_row = [&](auto PT, typename IN::raw_t wa, typename IN::raw_t wb, int li, int K) {
        constexpr int part = decltype(PT)::value;
        const int32_t tg = part ? tg0B : tg0A;
        auto f = [](int32_t x) { return __builtin_bit_cast(float, x); };
        int32_t e0, e1, e2, e3;
        if constexpr (CH == HARD) {
            // t: chunk A's (r0, r1) at bits 1, 0, chunk B's at 17, 16; A = r0 + r1 - 1, B = r0 - r1 per half,
            // entries E3 = A 2^9 + tg, E2 = B 2^9 + tg, E0 = 2 tg - E3, E1 = 2 tg - E2 (both chunks: the halves
            // R0, R1 are non-negative, so the 32-bit sums are the packed values m = EB 2^16 + EA)
            const uint32_t t = __builtin_amdgcn_perm(wb, wa, part ? hselB : hselA) >> (part ? hshB : hshA);
            const uint32_t R0 = (t >> 1) & 0x10001u, R1 = t & 0x10001u;
            e3 = (int32_t)(((R0 + R1) << 9) + (uint32_t)tg - 0x02000200u);
            e2 = (int32_t)(((R0 - R1) << 9) + (uint32_t)tg);
            e0 = 2 * tg - e3;
            e1 = 2 * tg - e2;
        } else if constexpr (CH == SOFT8) {
            // X = [s0B, s1B, s0A, s1A] (bytes 3..0); U0, U1 = s0 + 128, s1 + 128 per half (v_bitop3 (x &
            // 0x00FF00FF) ^ 0x00800080): A = U0 + U1 - 256, B = U0 - U1
            const uint32_t X = __builtin_amdgcn_perm(wb, wa, 0x05040100u);
            const uint32_t U1 = __builtin_amdgcn_bitop3_b32(X, 0x00FF00FFu, 0x00800080u, 0x6A);
            const uint32_t U0 = __builtin_amdgcn_bitop3_b32(X >> 8, 0x00FF00FFu, 0x00800080u, 0x6A);
            e3 = (int32_t)(((U0 + U1) << S) + (uint32_t)tg - 0x08000800u);
            e2 = (int32_t)(((U0 - U1) << S) + (uint32_t)tg);
            e0 = 2 * tg - e3;
            e1 = 2 * tg - e2;
        }
        if constexpr (!PK8) {
        int AA, BA, AB, BBv;
        IN::ab(wa, li, AA, BA, geo.scale);
        IN::ab(wb, li, AB, BBv, geo.scale);
        const int32_t pa = AA + AB * 65536, pb = BA + BBv * 65536;
        if constexpr (P2) {
            e3 = (int32_t)((uint32_t)pa << S) + tg;
            e2 = (int32_t)((uint32_t)pb << S) + tg;
            e0 = 2 * tg - e3;
            e1 = 2 * tg - e2;
        } else {
            e3 = __mul24(pa, 1 << S) + tg;
            e2 = __mul24(pb, 1 << S) + tg;
            e0 = __mul24(pa, -(1 << S)) + tg;
            e1 = __mul24(pb, -(1 << S)) + tg;
        }
        }
        lds_write_addtid4<256 * part, TT::REGION>(tabl, f(e0), f(e1), f(e2), f(e3));
        if (ALT && K == 0) {  // phase-0 lanes: the +tag entries E+[L] = BM[L] * 2^S - tg0 (ALT area)
            const int32_t d = -2 * tg;
            lds_write_addtid4<TT::ALT_OFF + 256 * part, 8>(tabl, f(e0 + d), f(e1 + d), f(e2 + d), f(e3 + d));
        }
    };
    const int r6a = sA % 6, r6b = sB % 6;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    for (uint32_t pass = 0;; pass++) {
        for (uint32_t j = 0; nblk; j += 3) {
            put_row(P0{}, rAA, rAB, sA, r6a);
            if (lane < 32) put_row(P1{}, rBA, rBB, sB, r6b);
            {  // the next group's input words
                rsA = tg_rsrc<CH>(in, startA + 32ull * (j + 3), availB);
                rsB = tg_rsrc<CH>(in, startB + 32ull * (j + 3), availB);
                rAA = IN::template load<0>(rsA, vo1);
                rBA = IN::template load<0>(rsA, vo2);
                rAB = IN::template load<0>(rsB, vo1);
                rBB = IN::template load<0>(rsB, vo2);
            }
            // the fairness controller at every group head (every other: SOFT8 split launches 1.4 % slower,
            // profiles/r05/split_fairness_ab.log)
            fair.group(j, 3u, lane);
            wave_sync();
            sfor<TGD>([&](auto X) { issue(X); });
            if (!block(std::integral_constant<int, 0>{}, j)) break;
            if (!block(std::integral_constant<int, 2>{}, j + 1)) break;
            if (!block(std::integral_constant<int, 4>{}, j + 2)) break;
            wave_sync();
        }
        if constexpr (!SPL) break;
        // SPL: the left neighbours' end vectors: B's is A's (sv1 low); A's is the previous wave's B end
        // (tail workgroups, through the waves' table LDS after a barrier)
        uint32_t nb = 0;
        if (tail) {
            __syncthreads();
            wlds[LL::TAB_OFF + lane] = sv2;
            __syncthreads();
            if (wv > 0) nb = lds[(wv - 1) * LL::WAVE + LL::TAB_OFF + lane];
            __syncthreads();
        }
        const bool mA = pA > 0 && __builtin_amdgcn_ballot_w64((sv2 & 0xFFFFu) != (nb >> 16)) != 0;
        const bool mB = __builtin_amdgcn_ballot_w64((sv1 >> 16) != (sv1 & 0xFFFFu)) != 0;
        const bool more = tail ? __syncthreads_or(mA || mB) != 0 : (mA || mB);
        if (!more) break;  // WG-uniform
        if (pass + 1u >= 2u * P) {
            // after P passes no start differs (header), so this cap never binds; if it ever did, the words
            // of the parts still differing would be wrong: count it (geo.stats[1]) so vd_run fails loudly
            if (lane == 0 && geo.stats && (mA || mB)) atomicAdd(geo.stats + 1, 1u);
            break;
        }
        if (lane == 0 && geo.stats && (mA || mB)) atomicAdd(geo.stats, (mA ? 1u : 0u) + (mB ? 1u : 0u));
        // decode again every part whose start vector differs, from block cut(p) with the left end vector;
        // an idle half repeats the other half's job without writing or keeping vectors
        uint32_t vA = 0, vB = 0;
        // (replay only for a part's first re-decode: the run it replays must be the one whose words stand)
        rpl = pass == 0u && mA != mB ? (mA ? 1u : 2u) : 0u;
        if (rpl) {  // replay (header "Early stop"): both halves from 6 blocks before the re-decoding part's cut
            const uint32_t p = mA ? pA : pB;
            const uint32_t o = pk_cut(p, P, WA) - kPkWarm, km = pk_cut(p + 1u, P, WA) - o;
            const uint32_t vin = mA ? nb >> 16 : sv1 & 0xFFFFu;
            oA = oB = o;
            kminA = kmaxA = kminB = kmaxB = 0;
            ssA = seA = ssB = seB = ~0u;
            ckA = ckB = ~0u;  // the re-decoding half keeps its checkpoint vectors (no comparison there)
            rdA = rdB = false;
            if (mA) {
                kminA = kPkWarm;
                kmaxA = km;
                seA = km - 1u;
                ckA = kPkWarm + 2u;
                sv2 = __builtin_amdgcn_perm(sv2, vin, 0x07060100u);  // its start vector
            } else {
                kminB = kPkWarm;
                kmaxB = km;
                seB = pB + 1u < P ? km - 1u : ~0u;
                ckB = kPkWarm + 2u;
                sv1 = __builtin_amdgcn_perm(vin << 16, sv1, 0x07060100u);
            }
            V = VBASE;
            nblk = km + 2u;
        } else {
        rdA = mA;
        rdB = mB;
        ckA = mA ? 2u : ~0u;
        ckB = mB ? 2u : ~0u;
        if (mA) {
            oA = pk_cut(pA, P, WA);
            kminA = 0;
            kmaxA = pk_cut(pA + 1u, P, WA) - oA;
            ssA = ~0u;
            seA = kmaxA - 1u;
            vA = nb >> 16;
            sv2 = __builtin_amdgcn_perm(sv2, vA, 0x07060100u);  // its start vector
        }
        if (mB) {
            oB = pk_cut(pB, P, WA);
            kminB = 0;
            kmaxB = pk_cut(pB + 1u, P, WA) - oB;
            ssB = ~0u;
            seB = pB + 1u < P ? kmaxB - 1u : ~0u;
            vB = sv1 & 0xFFFFu;
            sv1 = __builtin_amdgcn_perm(vB << 16, sv1, 0x07060100u);
        }
        if (!mA) {  // idle A: B's job (or nothing)
            oA = oB;
            kminA = kmaxA = 0;
            ssA = seA = ~0u;
            vA = vB;
        }
        if (!mB) {
            oB = oA;
            kminB = kmaxB = 0;
            ssB = seB = ~0u;
            vB = vA;
        }
        V = vA | vB << 16;
        nblk = mA || mB ? (mA ? kmaxA : kmaxB) + 2u : 0u;
        if (mA && mB && kmaxB > kmaxA) nblk = kmaxB + 2u;
        }
        startA = stA + 32ull * oA;
        startB = stB + 32ull * oB;
        kb = 0;
        tbn = LL::TBS - (blockIdx.x & 3u) % LL::TBS;
        wave_sync();
        rsA = tg_rsrc<CH>(in, startA, availB);
        rsB = tg_rsrc<CH>(in, startB, availB);
        rAA = IN::template load<0>(rsA, vo1);
        rBA = IN::template load<0>(rsA, vo2);
        rAB = IN::template load<0>(rsB, vo1);
        rBB = IN::template load<0>(rsB, vo2);
    }
    fair.end(lane);
    if (geo.check) {
        wave_sync();
        const bool bad = lane < 3 * kGuardWords && wlds[LL::guard(lane)] != kGuardPattern;
        const uint32_t nbad = (uint32_t)__builtin_popcountll(__ballot(bad));
        if (lane == 0 && nbad) atomicAdd(geo.check, nbad);
    }
}

}  // namespace vd
