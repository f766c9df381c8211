// vd_ps_kernel.h -- TOOLS ONLY (timing studies, not in the product).  Round-2 experiment, kept for
// tools/vd_ablate: exact (all GPU parity tests passed with it as the product kernel), but no faster than
// vd_decode_tg in the bench (tg 150.1 / 151.0 Gb/s vs ps 150.0 / 150.2, interleaved, profiles/r02) and
// slower per chunk (balanced 6144-chunk launch 0.1872 vs 0.1841 ms): at 3 waves per SIMD its LDS round
// trips (swizzle, table reads) are exposed.  vd_decode_tg with the xor-32 exchange through ds_bpermute
// took its place.
//
// "paired-state" decode kernel vd_decode_ps (gfx950): the tagged-metric scheme of
// vd_kernel_tg.h (decisions in the low bits of an exact-integer fp32 / int32 metric, bit-field read-out,
// group traceback) with TWO trellis states per lane and two chunks per wave.  Same decode semantics
// (reference src/viterbi/viterbi.cu:144-207, viterbiACS.cuh:113-157,216-256, viterbiTB.cuh:4-21),
// bit-exact for every valid option.
//
// Why.  With one state per lane the xor-32 butterfly (position bit 5) needs a cross-half lane swap:
// v_permlane32_swap_b32 issues at ~3.4 ns per wave per SIMD against ~1.1 for v_add_f32 and ~1.8 for a
// DPP op or v_max (tools/vd_ubench12, profiles/r02/ubench12.log), so the swap stage cost 1.8x a DPP
// stage.  Here lane li of half h holds positions p and p | 32 (p = the 5-bit position of li, same linear
// map as vd_kernel_tg.h on bits 0..4): the bit-5 butterfly is in-lane (two v_pk_fma_f32 and two v_max,
// no data movement), bits 0..3 stay DPP (quad_perm, row_half_mirror, row_ror:8), bit 4 is a ds_swizzle
// xor 16 inside the 32-lane half.  Two independent chains per lane (the two states between in-lane
// stages) also fill the DPP hazard slots without s_nop.
//
// Layout.  Workgroup = kPsWaves waves = kPsSlots chunk slots (slot = 2 * wave + half); lanes 32h..32h+31
// decode slot h of their wave.  Each slot has its own branch-metric table (TgTab layout, per chunk) and
// survivor ring ((kPsTBS + 1) x 64 position words).  A whole-chunk workgroup decodes 8 consecutive
// chunks; in a split launch each remaining chunk is one workgroup of 8 pieces (see "split chunks" in
// vd_kernel_tg.h: same check-and-re-decode protocol, kPsSlots pieces).  LDS per workgroup: 8 x (1,920 +
// 12 x 256) = 39,936 B, so 4 workgroups (16 waves, 32 chunks) fit a CU: 6400 chunks = 25 per CU resident.
#pragma once
#include "../gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h"

namespace vd {

constexpr int kPsWaves = 4;               // waves per workgroup
constexpr int kPsSlots = 2 * kPsWaves;    // chunk slots (wave halves) per workgroup = pieces of a split chunk
constexpr int kPsTBS = 11;                // traceback batch (words) -> ring of 12 slots per chunk
constexpr int kPsVecs = 3 * kPsSlots;     // split chunk: start[q], end[parity 0][q], end[parity 1][q]

__device__ __forceinline__ int ps_start_vec(int q) { return q; }
__device__ __forceinline__ int ps_end_vec(int q, uint32_t par) { return kPsSlots * (1 + (int)par) + q; }
__device__ __forceinline__ uint32_t ps_bound(uint32_t Sc, int q)
{
    const uint32_t k = (uint32_t)q * Sc / kPsSlots;
    return k - (k + 1) % 3;
}
// piece q's frame (as split_geo, kPsSlots pieces)
__device__ __forceinline__ SplitGeo ps_geo(uint32_t Sc, int q)
{
    SplitGeo g;
    const uint32_t kq = q == 0 ? 0 : ps_bound(Sc, q);
    const uint32_t kn = q == kPsSlots - 1 ? Sc : ps_bound(Sc, q + 1);
    g.s0 = q == 0 ? 0 : kq + 1 - kSplitWarm;
    g.words = kn - g.s0;
    g.E = kq - g.s0;
    g.Xspec = q == 0 ? -1 : (int)(kq + 1 - g.s0);
    g.Xcmp = q == kPsSlots - 1 ? -1 : (int)(kn + 1 - g.s0);
    return g;
}

// ---------------------------------------------------------------- two-state stages (inline asm)
// Va lives in v60, Vb in v61 (the pair v[60:61] feeds the in-lane stage's packed FMAs); v62..v65 scratch.
// DPP stage on both states, three-op form; the two chains interleave, so each DPP source is >= 2 VALU
// slots after its write with no s_nop.
template <int Q>
__device__ __forceinline__ void ps_stage_dpp(float& Va, float& Vb, float ma, float mb)
{
#define VD_PS_DPP(CTRL)                                                                                     \
    asm("v_add_f32 v62, %0, %2\n\tv_add_f32 v63, %1, %3\n\t"                                                 \
        "v_sub_f32_dpp v64, %0, %2 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                                  \
        "v_sub_f32_dpp v65, %1, %3 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                                  \
        "v_max_f32 %0, v62, v64\n\tv_max_f32 %1, v63, v65"                                                   \
        : "+{v60}"(Va), "+{v61}"(Vb) : "v"(ma), "v"(mb) : "v62", "v63", "v64", "v65")
    if constexpr (Q == 0) VD_PS_DPP("quad_perm:[1,0,3,2]");
    else if constexpr (Q == 1) VD_PS_DPP("quad_perm:[2,3,0,1]");
    else if constexpr (Q == 2) VD_PS_DPP("row_half_mirror");
    else VD_PS_DPP("row_ror:8");
#undef VD_PS_DPP
}
// int32 patterns (SOFT16): two-op form a = V + m, b = V - m, V' = max(a, partner's b through DPP)
template <int Q>
__device__ __forceinline__ void ps_stage_dpp_i(float& Va, float& Vb, float ma, float mb)
{
#define VD_PS_DPPI(CTRL)                                                                                    \
    asm("v_sub_u32 v64, %0, %2\n\tv_sub_u32 v65, %1, %3\n\tv_add_u32 v62, %0, %2\n\tv_add_u32 v63, %1, %3\n\t" \
        "v_max_i32_dpp %0, v64, v62 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                                 \
        "v_max_i32_dpp %1, v65, v63 " CTRL " row_mask:0xf bank_mask:0xf"                                     \
        : "+{v60}"(Va), "+{v61}"(Vb) : "v"(ma), "v"(mb) : "v62", "v63", "v64", "v65")
    if constexpr (Q == 0) VD_PS_DPPI("quad_perm:[1,0,3,2]");
    else if constexpr (Q == 1) VD_PS_DPPI("quad_perm:[2,3,0,1]");
    else if constexpr (Q == 2) VD_PS_DPPI("row_half_mirror");
    else VD_PS_DPPI("row_ror:8");
#undef VD_PS_DPPI
}
// in-lane stage (position bit 5, stage phase 0): the lane holds both butterfly partners.
//   Va' = max(Va + Ea, Vb - Ea),  Vb' = max(Vb + Eb, Va - Eb)
// with (Ea, Eb) the entries of the shared label: M_B32's pair row (E-, E+) (SEL 2), else the same entry
// twice (SEL 0: the pair's lo, 1: hi -- even / odd period).  One v_pk_fma_f32 forms [Va + Ea, Va - Eb],
// one [Vb - Ea, Vb + Eb] (sx = [1, -1], its halves swapped by op_sel for the second).
template <int SEL>
__device__ __forceinline__ void ps_stage_lane(float& Va, float& Vb, f2v e, f2v sx)
{
#define VD_PS_LANE(OS1, OS2)                                                                                \
    asm("v_pk_fma_f32 v[62:63], %2, %3, v[60:61] " OS1 "\n\t"                                                \
        "v_pk_fma_f32 v[64:65], %2, %3, v[60:61] " OS2 "\n\t"                                                \
        "v_max_f32 %0, v62, v64\n\tv_max_f32 %1, v65, v63"                                                   \
        : "+{v60}"(Va), "+{v61}"(Vb) : "v"(e), "v"(sx) : "v62", "v63", "v64", "v65")
    // OS1: lo = e.(lo|hi) * sx.lo + Va, hi = e.(..) * sx.hi + Va; OS2: lo = e * sx.hi + Vb, hi = e * sx.lo + Vb
    if constexpr (SEL == 0) VD_PS_LANE("op_sel:[0,0,0] op_sel_hi:[0,1,0]", "op_sel:[0,1,1] op_sel_hi:[0,0,1]");
    else if constexpr (SEL == 1) VD_PS_LANE("op_sel:[1,0,0] op_sel_hi:[1,1,0]", "op_sel:[1,1,1] op_sel_hi:[1,0,1]");
    else VD_PS_LANE("op_sel:[0,0,0] op_sel_hi:[1,1,0]", "op_sel:[0,1,1] op_sel_hi:[1,0,1]");
#undef VD_PS_LANE
}
__device__ __forceinline__ void ps_stage_lane_i(float& Va, float& Vb, float ea, float eb)
{
    asm("v_add_u32 v62, %0, %2\n\tv_sub_u32 v64, %1, %2\n\tv_add_u32 v65, %1, %3\n\tv_sub_u32 v63, %0, %3\n\t"
        "v_max_i32 %0, v62, v64\n\tv_max_i32 %1, v65, v63"
        : "+{v60}"(Va), "+{v61}"(Vb) : "v"(ea), "v"(eb) : "v62", "v63", "v64", "v65");
}
// xor-16 stage: the partners' metrics through the LDS crossbar (ds_swizzle inside each 32-lane half)
template <bool INT>
__device__ __forceinline__ void ps_stage_swz(float& Va, float& Vb, float ma, float mb, float pa, float pb)
{
    if constexpr (INT)
        asm("v_add_u32 v62, %0, %2\n\tv_add_u32 v63, %1, %3\n\tv_sub_u32 v64, %4, %2\n\tv_sub_u32 v65, %5, %3\n\t"
            "v_max_i32 %0, v62, v64\n\tv_max_i32 %1, v63, v65"
            : "+{v60}"(Va), "+{v61}"(Vb) : "v"(ma), "v"(mb), "v"(pa), "v"(pb) : "v62", "v63", "v64", "v65");
    else
        asm("v_add_f32 v62, %0, %2\n\tv_add_f32 v63, %1, %3\n\tv_sub_f32 v64, %4, %2\n\tv_sub_f32 v65, %5, %3\n\t"
            "v_max_f32 %0, v62, v64\n\tv_max_f32 %1, v63, v65"
            : "+{v60}"(Va), "+{v61}"(Vb) : "v"(ma), "v"(mb), "v"(pa), "v"(pb) : "v62", "v63", "v64", "v65");
}

// per-slot (wave half) geometry of a pass
struct PsHalf {
    uint64_t wOut;   // output word of frame word 0
    uint32_t Sw;     // frame words (0: slot idle)
    uint32_t E;      // first emitted frame word
    int Xspec, Xcmp; // boundary blocks (split pieces), -1: none
    uint32_t Sc;     // chunk words traced back (32-bit words)
    uint32_t cwords; // chunk output words (bpp units)
    uint64_t cstart; // chunk's first output word
};

// ================================================================ paired-state kernel
template <int CH, int CORE, int OB, int ABL = 0>
__global__ __launch_bounds__(64 * kPsWaves) void vd_decode_ps(const void* __restrict__ in, void* __restrict__ out, Geom geo)
{
    using IN = TgIn<CH>;
    constexpr bool INT = TgFmt<CH>::INT;
    static_assert(!INT || CORE == B32, "int32 patterns: SOFT16 on the int32 core only");
    using TT = TgTab<CORE>;
    constexpr int J = TgFmt<CH>::J, S = TgFmt<CH>::S;
    constexpr int TBS = kPsTBS;
    __shared__ __attribute__((aligned(16))) char tab_all[kPsSlots][TT::BYTES];
    __shared__ __attribute__((aligned(256))) uint32_t ring_all[kPsSlots][(TBS + 1) * 64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, li = lane & 31;
    const int p = tg_pos(li);  // 5-bit position of the lane (bits 0..4); states p and p | 32
    const int slot = 2 * wv + half;
    char* tabb = tab_all[slot];

    // this workgroup's chunks: slots 8w .. 8w+7 (whole), or the 8 pieces of one chunk (split launch)
    const uint32_t nsw = geo.nwhole / kPsSlots;  // whole workgroups of a split launch
    const bool split = OB == 32 && geo.nwhole != 0 && blockIdx.x >= nsw;
    const uint32_t chunk0 = split ? geo.nwhole + (blockIdx.x - nsw) : blockIdx.x * kPsSlots + 2 * wv;
    const ChunkRange crA = chunk_range(geo, chunk0), crB = chunk_range(geo, split ? chunk0 : chunk0 + 1);
    if (crA.words == 0 && crB.words == 0) return;  // never in a split workgroup
    float* const svec = split ? geo.spec + (size_t)(chunk0 - geo.nwhole) * kPsVecs * 64 : nullptr;
    // per-half chunk (uniform per half; selected per lane below)
    auto half_geo = [&](const ChunkRange& cr, int piece, int pass) {
        PsHalf g;
        g.cwords = cr.words;
        g.cstart = cr.startWord;
        g.Sc = OB == 32 ? cr.words : (cr.words + 1) / 2;
        g.Sw = g.Sc;
        g.E = 0;
        g.Xspec = g.Xcmp = -1;
        uint32_t s0 = 0;
        if (piece >= 0) {
            const SplitGeo sg = ps_geo(g.Sc, piece);
            s0 = sg.s0;
            g.Sw = sg.words;
            g.E = sg.E;
            g.Xspec = sg.Xspec;
            g.Xcmp = sg.Xcmp;
        }
        (void)pass;
        g.wOut = cr.startWord + s0;
        if (cr.words == 0) g.Sw = 0;
        return g;
    };

    // table addresses of this lane's two states, per stage phase (row offsets are compile-time)
    int aKa[6], aKb[6];
    sfor<6>([&](auto KK) {
        constexpr int K = decltype(KK)::value;
        aKa[K] = 8 * own_label(p, K);
        aKb[K] = 8 * own_label(p | 32, K);
    });
    const f2v sx = (f2v){1.0f, -1.0f};
    // table build: lane li writes rows li, 32 + li, 64 + li of its slot's group table
    const int rowb0 = TT::row(li), rowb1 = TT::row(32 + li), rowb2 = TT::row(64 + li);
    const float tagv = (float)(1 << (li % J));
    const float tg0 = CORE == F16 ? tagv : -tagv;
    constexpr uint32_t VBASE = (INT ? 0u : 0x4B400000u) + (1u << (S - 1));
    const uint32_t fnm = ~((1u << S) - 1u), fhf = 1u << (S - 1);
    Fair fair;
    if constexpr (!(ABL & 256)) fair.begin(geo.fair, lane);
    const uint64_t availB = IN::bytes(geo.availStages);

    uint32_t verified = 1u, endpar = 0u;  // split workgroups: bit q = piece q (slot q)
    for (int pass = 0;; pass++) {
    // pieces (slots) of this wave that run in this pass
    const int qa = 2 * wv, qb = 2 * wv + 1;
    const bool runA = !split || pass == 0 || !((verified >> qa) & 1u);
    const bool runB = !split || pass == 0 || !((verified >> qb) & 1u);
    if (runA || runB) {
    PsHalf gA = half_geo(crA, split ? qa : -1, pass), gB = half_geo(crB, split ? qb : -1, pass);
    if (!runA) gA.Sw = 0;
    if (!runB) gB.Sw = 0;
    // this lane's half
    const uint32_t Sw = half ? gB.Sw : gA.Sw, E = half ? gB.E : gA.E;
    const uint32_t Sc = half ? gB.Sc : gA.Sc, cwords = half ? gB.cwords : gA.cwords;
    const int Xspec = half ? gB.Xspec : gA.Xspec, Xcmp = half ? gB.Xcmp : gA.Xcmp;
    const uint64_t wOut = half ? gB.wOut : gA.wOut, cstart = half ? gB.cstart : gA.cstart;
    (void)Sc;
    // wave-uniform loop range: the longer running half
    const uint32_t nblk = (gA.Sw > gB.Sw ? gA.Sw : gB.Sw) + 2;
    const uint32_t j0 = pass == 0 ? 0u : (uint32_t)kSplitWarm;  // a re-decode starts at the boundary block
    const uint32_t nblkA = gA.Sw ? gA.Sw + 2 : 0, nblkB = gB.Sw ? gB.Sw + 2 : 0;
    // input: one buffer resource from half A's frame start; half B's lanes add their offset
    const uint64_t startA = gA.wOut * OB, startB = gB.wOut * OB;
    const uint64_t base = startA < startB ? startA : startB;
    const uint32_t hoff = (uint32_t)IN::bytes((half ? startB : startA) - base);
    const uint32_t vo0 = IN::voff(li) + hoff;
    float Va = __builtin_bit_cast(float, VBASE), Vb = Va;
    if (pass > 0 && Sw) {  // re-decode of piece q >= 1: start from piece q-1's latest end vector
        const int q = slot, pl = q > 0 ? q - 1 : 0;
        const float* v = svec + ps_end_vec(pl, (endpar >> pl) & 1u) * 64;
        Va = v[li];
        Vb = v[32 + li];
        svec[ps_start_vec(q) * 64 + li] = Va;
        svec[ps_start_vec(q) * 64 + 32 + li] = Vb;
    }
    uint32_t kb = 0;
    uint32_t tbn = pass == 0 ? TBS - 3 * (blockIdx.x & 3) : TBS;
    __amdgpu_buffer_rsrc_t rs = tg_rsrc<CH>(in, base + 32ull * j0, availB);
    typename IN::raw_t r0 = IN::template load<0>(rs, vo0);
    typename IN::raw_t r1 = IN::template load<1>(rs, vo0);
    typename IN::raw_t r2 = IN::template load<2>(rs, vo0);

    // branch-metric table reads, TGD stages ahead (see vd_kernel_tg.h); K = 0 (in-lane stage) reads one
    // pair for both states (shared label), every other phase one pair per state
    constexpr int TGD = 4;
    typedef __attribute__((address_space(3))) const volatile f2v* lptr;
    const __attribute__((address_space(3))) char* tl = (const __attribute__((address_space(3))) char*)tabb;
    f2v vpa[96], vpb[96];
    auto issue = [&](auto Rc) {
        constexpr int r = decltype(Rc)::value;
        constexpr int K = r % 6;
        if constexpr (ABL & 2) {  // tools only: no table reads
            vpa[r] = (f2v){(float)aKa[K], 1.0f};
            vpb[r] = (f2v){(float)aKb[K], 1.0f};
        } else if constexpr (TT::pairrow(K) || (r / 6) % 2 == 0) {
            vpa[r] = *(lptr)(tl + aKa[K] + TT::row(r));
            if constexpr (K != 0) vpb[r] = *(lptr)(tl + aKb[K] + TT::row(r));
        }
    };
    auto block = [&](auto PHc, uint32_t j) {
        constexpr int PH = decltype(PHc)::value;
        constexpr int BB = PH / 2;
        uint32_t wa = 0, wb = 0;  // ring words of positions p and p | 32
        sfor<32>([&](auto I) {
            constexpr int i = decltype(I)::value;
            constexpr int K = (PH + i) % 6;
            constexpr int Q = (K + 5) % 6;
            constexpr int r = 32 * BB + i;
            constexpr bool ODD = (r / 6) % 2 == 1;
            constexpr int RP = TT::pairrow(K) ? r : (ODD ? r - 6 : r);
            if constexpr (Q <= 3) {
                const float ma = ODD ? vpa[RP].y : vpa[RP].x, mb = ODD ? vpb[RP].y : vpb[RP].x;
                if constexpr (INT) ps_stage_dpp_i<Q>(Va, Vb, ma, mb);
                else ps_stage_dpp<Q>(Va, Vb, ma, mb);
            } else if constexpr (Q == 4) {
                const float pa = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, Va), 0x401F));
                const float pb = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, Vb), 0x401F));
                const float ma = ODD ? vpa[RP].y : vpa[RP].x, mb = ODD ? vpb[RP].y : vpb[RP].x;
                ps_stage_swz<INT>(Va, Vb, ma, mb, pa, pb);
            } else {  // Q == 5: in-lane
                if constexpr (INT) ps_stage_lane_i(Va, Vb, vpa[RP].x, vpa[RP].y);
                else ps_stage_lane<TT::pairrow(K) ? 2 : (ODD ? 1 : 0)>(Va, Vb, vpa[RP], sx);
            }
            if constexpr (r + TGD < 96) issue(std::integral_constant<int, r + TGD>{});
            if constexpr (i % J == J - 1 && !(ABL & 4)) {
                // field read-out of both states into byte / half g of their ring words, field clear; every
                // 16 stages the renormalisation by position 0 of each half's chunk: lane 0 (32) of the
                // half broadcast to the half by row_newbcast:0 + row_bcast:15 (rows 1 and 3)
                constexpr int g = (i % 32) / J;
#define VD_PS_RO(SEL, UNUSED)                                                                                \
    "v_lshrrev_b32_sdwa %[wa], 1, %[Va] dst_sel:" SEL " dst_unused:" UNUSED " src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_lshrrev_b32_sdwa %[wb], 1, %[Vb] dst_sel:" SEL " dst_unused:" UNUSED " src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_and_or_b32 %[Va], %[Va], %[fnm], %[fhf]\n\tv_and_or_b32 %[Vb], %[Vb], %[fnm], %[fhf]"
#define VD_PS_RN                                                                                             \
    "\n\ts_nop 1\n\tv_mov_b32_dpp %[rr], %[Va] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t"       \
    "v_mov_b32_dpp %[rr], %[rr] row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"                                  \
    "v_subrev_u32 %[rr], %[vb], %[rr]\n\tv_sub_u32 %[Va], %[Va], %[rr]\n\tv_sub_u32 %[Vb], %[Vb], %[rr]"
#define VD_PS_IN [fnm] "v"(fnm), [fhf] "v"(fhf), [vb] "v"(VBASE)
                float rr;
                if constexpr (J == 8 && g == 0)
                    asm(VD_PS_RO("BYTE_0", "UNUSED_PAD") : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "=&v"(wa), [wb] "=&v"(wb) : VD_PS_IN);
                else if constexpr (J == 8 && g == 1)
                    asm(VD_PS_RO("BYTE_1", "UNUSED_PRESERVE") VD_PS_RN
                        : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "+v"(wa), [wb] "+v"(wb), [rr] "=&v"(rr) : VD_PS_IN);
                else if constexpr (J == 8 && g == 2)
                    asm(VD_PS_RO("BYTE_2", "UNUSED_PRESERVE") : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "+v"(wa), [wb] "+v"(wb) : VD_PS_IN);
                else if constexpr (J == 8)
                    asm(VD_PS_RO("BYTE_3", "UNUSED_PRESERVE") VD_PS_RN
                        : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "+v"(wa), [wb] "+v"(wb), [rr] "=&v"(rr) : VD_PS_IN);
                else if constexpr (g == 0)
                    asm(VD_PS_RO("WORD_0", "UNUSED_PAD") VD_PS_RN
                        : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "=&v"(wa), [wb] "=&v"(wb), [rr] "=&v"(rr) : VD_PS_IN);
                else
                    asm(VD_PS_RO("WORD_1", "UNUSED_PRESERVE") VD_PS_RN
                        : [Va] "+{v60}"(Va), [Vb] "+{v61}"(Vb), [wa] "+v"(wa), [wb] "+v"(wb), [rr] "=&v"(rr) : VD_PS_IN);
#undef VD_PS_IN
#undef VD_PS_RN
#undef VD_PS_RO
            }
        });
        if constexpr (CORE == F16) {
            wa = ~wa;
            wb = ~wb;
        }
        uint32_t* ring = ring_all[slot];
        wave_sync();
        if (j >= 1) {
            ring[(j - 1 - kb) * 64 + p] = wa;
            ring[(j - 1 - kb) * 64 + 32 + p] = wb;
        }
        if (j >= 2 && (j - 1 - kb == tbn || j == nblk - 1 || j == nblkA - 1 || j == nblkB - 1)) {
            wave_sync();
            const uint32_t nw = j - 1 - kb;
            const uint32_t k = kb + (uint32_t)li;
            if (!(ABL & 1) && (uint32_t)li < nw && k >= E && k < Sw) {
                const uint32_t Q0 = (uint32_t)((li + 1) * 256);
                const uint32_t w = traceback_word_tg<J, CORE == B32>((const char*)ring, Q0, k);
                if constexpr (OB == 32) {
                    ((uint32_t*)out)[wOut + k] = w;
                } else {
                    uint16_t* o = (uint16_t*)out + cstart;
                    o[2 * k] = (uint16_t)(w >> 16);
                    if (2 * k + 1 < cwords) o[2 * k + 1] = (uint16_t)(w & 0xFFFF);
                }
            }
            wave_sync();
            ring[p] = wa;  // block j becomes slot 0 of the next batch
            ring[32 + p] = wb;
            kb = j - 1;
            tbn = TBS;
        }
        return j + 1 < nblk;
    };
    // one group's three table rows per lane
    auto put_row = [&](int rb, int A, int B, int K) {
        if constexpr (INT) {
            uint32_t* e = (uint32_t*)(tabb + rb);
            const int a = A * (1 << S), b = B * (1 << S), tag = 1 << (li % J);
            e[0] = (uint32_t)(-a - tag);
            e[2] = (uint32_t)(-b - tag);
            e[4] = (uint32_t)(b - tag);
            e[6] = (uint32_t)(a - tag);
            if (K == 0) {
                e[1] = (uint32_t)(-a + tag);
                e[3] = (uint32_t)(-b + tag);
                e[5] = (uint32_t)(b + tag);
                e[7] = (uint32_t)(a + tag);
            }
            return;
        }
        constexpr float SC = (float)(1 << S);
        const float af = (float)A, bf = (float)B;
        float* e = (float*)(tabb + rb);
        e[0] = __builtin_fmaf(af, -SC, tg0);
        e[2] = __builtin_fmaf(bf, -SC, tg0);
        e[4] = __builtin_fmaf(bf, SC, tg0);
        e[6] = __builtin_fmaf(af, SC, tg0);
        if constexpr (CORE == B32) {
            if (K == 0) {
                e[1] = __builtin_fmaf(af, -SC, tagv);
                e[3] = __builtin_fmaf(bf, -SC, tagv);
                e[5] = __builtin_fmaf(bf, SC, tagv);
                e[7] = __builtin_fmaf(af, SC, tagv);
            }
        }
    };
    const int r6a = li % 6, r6b = (li + 32) % 6, r6c = (li + 64) % 6;
    for (uint32_t j = j0;; j += 3) {
        if constexpr (!(ABL & 8)) {  // ABL 8 (tools only): no table build
            int A, B;
            IN::ab(r0, li, A, B, geo.scale);
            put_row(rowb0, A, B, r6a);
            IN::ab(r1, li, A, B, geo.scale);
            put_row(rowb1, A, B, r6b);
            IN::ab(r2, li, A, B, geo.scale);
            put_row(rowb2, A, B, r6c);
        }
        if constexpr (!(ABL & 16)) {  // ABL 16 (tools only): no input loads
            rs = tg_rsrc<CH>(in, base + 32ull * (j + 3), availB);
            r0 = IN::template load<0>(rs, vo0);
            r1 = IN::template load<1>(rs, vo0);
            r2 = IN::template load<2>(rs, vo0);
        }
        if constexpr (!(ABL & 256)) fair.group(j, lane);
        if (split) {  // boundary vectors of this lane's piece (positions li and 32 + li)
            if (pass == 0 && (int)j == Xspec) {
                svec[ps_start_vec(slot) * 64 + li] = Va;
                svec[ps_start_vec(slot) * 64 + 32 + li] = Vb;
            }
            if ((int)j == Xcmp && Sw) {
                svec[ps_end_vec(slot, (uint32_t)pass & 1u) * 64 + li] = Va;
                svec[ps_end_vec(slot, (uint32_t)pass & 1u) * 64 + 32 + li] = Vb;
            }
        }
        wave_sync();
        sfor<TGD>([&](auto X) { issue(X); });
        if (!block(std::integral_constant<int, 0>{}, j)) break;
        if (!block(std::integral_constant<int, 2>{}, j + 1)) break;
        if (!block(std::integral_constant<int, 4>{}, j + 2)) break;
        wave_sync();
    }
    }  // runs
    if (!split) break;
    // split workgroup: evaluate the boundary checks (every wave the same), then re-decode what failed
    const uint32_t all = (1u << kPsSlots) - 1u;
    const uint32_t ran = pass == 0 ? all : ~verified & all;
    endpar = (endpar & ~ran) | ((pass & 1) ? ran : 0u);
    __syncthreads();
    for (int q = 1; q < kPsSlots; q++)
        if (!((verified >> q) & 1u) && ((verified >> (q - 1)) & 1u) &&
            split_vec_eq(svec, ps_start_vec(q), ps_end_vec(q - 1, (endpar >> (q - 1)) & 1u), lane))
            verified |= 1u << q;
    if (verified == all) break;
    if (lane == 0 && geo.stats) {
        const uint32_t mine = ~verified & (3u << (2 * wv));
        if (mine) atomicAdd(geo.stats, (uint32_t)__builtin_popcount(mine));
    }
    __syncthreads();  // the next pass overwrites vectors read above
    }  // pass
    if constexpr (!(ABL & 256)) fair.end(lane);
}

}  // namespace vd
