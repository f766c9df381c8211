// vd_kernels.h -- device code of the MI355X (gfx950) Viterbi decoder.
//
// Hot path of the reference (alireza-md93/GPU-Accelerated-Viterbi-Decoder): the fused
// branch-metric + add-compare-select + traceback kernel `viterbi_core` (src/viterbi/viterbi.cu:144-207,
// viterbiBM.cuh, viterbiACS.cuh, viterbiTB.cuh), re-designed for CDNA4 wave64.  Not a translation:
//
//  * State layout.  A wave64 lane holds ONE trellis state (the reference: a warp32 lane holds two).
//    Position p holds, after stage t, the state rotr6(p, t%6); under that rotation the radix-2 butterfly
//    of every stage pairs positions p and p^(1<<q), q = (t%6+5)%6, and a linear position -> lane map
//    turns four of the six butterfly distances into DPP controls fused into the ACS max (quad_perm,
//    row_half_mirror, row_ror:8); xor-16 and xor-32 go through ds_swizzle / ds_bpermute.
//  * Metric cores.  Two kernels, the same mapping and decisions.  vd_decode_tg (vd_kernel_tg.h): one chunk
//    per wave, the metric an exact integer in fp32 (SOFT16: int32 patterns); the metric type only selects
//    the tie rule.  vd_decode_pk (vd_kernel_pk.h): HARD, SOFT4, SOFT8 and FP32 input, two chunks (batched
//    launches) or two parts of one chunk (split single launches) per wave, one in each exact-integer
//    16-bit half of the metric word (v_add_u32, v_sub_u32_dpp, v_pk_max_u16 per stage for both).
//  * Survivors.  Tagged ACS: each stage's decision rides in the low bits of the path metric, so the max
//    itself does the register exchange within a history field (16, 8, 4 or 2 stages by format); the
//    fields' bits go into the block's survivor ring in LDS.  Output words are traced back lane-parallel,
//    one dependent LDS read per field, in POSITION space.
//  * Branch metrics.  Per 96-stage group, every lane builds table rows (the four label entries of one
//    stage) into LDS; every stage each lane reads its own transition's entry (one ds_read_b64 serves
//    two stages of the same phase).
// This file holds the shared pieces (geometry, chunk partition, fairness controller).
//
// Decode semantics (bit-exact with the reference for every valid option): see DESIGN.md and
// oracle/vd_oracle.c.  Tie rules, in own/exchanged terms: M_B16 -> exchanged wins, M_FP16 -> own
// wins, M_B32 -> exchanged wins except at t%6==0 where the odd predecessor wins (upper positions keep own).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

namespace vd {

enum Ch : int { HARD = 0, SOFT4 = 1, SOFT8 = 2, SOFT16 = 3, FP32 = 4 };
enum Core : int { B32 = 0, B16 = 1, F16 = 2 };

constexpr int kChunks = 6400;  // reference blocksNum_total = 16*400 (viterbi.cu:19)

struct Geom {
    uint64_t packNum;      // output words of bpp bits (getMessageLen / bpp)
    uint64_t availStages;  // stages readable from the input buffer
    uint32_t nchunks;
    uint32_t* fair;        // per-SIMD progress board (kFairBoardWords, empty at rest) or null
    float scale;           // LLR input (channel ids 8 + base): SoftDecisionPacker scale, else unused
    // segment launch (vd_kernel_tg.h "segment launches"): workgroup g decodes chunks [seg[g], seg[g+1]) as
    // kWaves segments (their boundary vectors stay in the workgroup's LDS); null = one chunk per wave
    const uint32_t* seg = nullptr;
    uint32_t segWarm = 6;        // warm-up blocks of a segment that starts inside a chunk (a multiple of 3)
    // [0]: count of segments / parts re-decoded; [1]: split waves that reached the re-decode pass cap with
    // a part still differing (never expected; vd_run fails when it is non-zero); or null
    uint32_t* stats = nullptr;
    // LDS guard check (tests): non-null = write guard words around every wave's table and ring and count
    // the ones found overwritten at kernel exit into *check
    uint32_t* check = nullptr;
    // several independent batches of the same size in one launch (never split): batch b decodes
    // in + b * inStride bytes into out + b * outStride bytes; chunk c of the launch = chunk c % nchunks
    // of batch c / nchunks
    uint32_t nbatch = 1;
    uint64_t inStride = 0, outStride = 0;
    // vd_decode_pk split launches: workgroups from tailWG on decode one chunk each (chunk 4 tailWG + g -
    // tailWG) with their 4 waves (vd_kernel_pk.h "split"); ~0u = none
    uint32_t tailWG = ~0u;
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


// Workgroups of kWaves waves (one chunk each): gfx950 admits a bounded number of workgroups per CU, so
// single-wave workgroups could not keep all 6400 chunks resident at once.  The waves of a whole-chunk
// workgroup never synchronise with each other (only the pieces of a split chunk do, vd_kernel_tg.h);
// LDS is partitioned per wave and wave_sync() only orders the wave's own LDS traffic (LDS instructions
// of one wave execute in order).
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
// stamps).  At every other 3-block group head each wave posts its progress to its own board word and sets
// its issue priority from its lag behind the mean of the SIMD's waves, read at the previous call.
// Progress is in blocks started, or, when the waves of a launch differ in length (segment launches,
// vd_kernel_tg.h), the fraction started scaled to 2^20, so that waves of unequal work end together.
// Posting is a plain store and reading one 64-byte load (16 lanes): both stay in the XCD's L2 (all
// waves of a SIMD are on one XCD), so the board adds no HBM or fabric traffic -- a returning atomic per
// group went past the L2 and cost 11 MB of writes per launch (profiles/r02).
struct Fair {
    uint32_t* mine = nullptr;   // this wave's word
    uint32_t* simd = nullptr;   // the SIMD's kFairWaves words
    __amdgpu_buffer_rsrc_t rs;  // ... as a buffer resource (SGPRs: the per-lane read needs one offset VGPR)
    uint32_t seen = kFairEmpty; // lane l < kFairWaves: word l as read at the previous group head
    uint32_t last = kFairEmpty; // this wave's value posted at the previous call

    __device__ __forceinline__ void begin(uint32_t* board, int lane)
    {
        if (!board) return;
        const uint32_t wid = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) & (kFairWaves - 1);
        simd = board + (size_t)simd_slot() * kFairWaves;
        mine = simd + wid;
        rs = __builtin_amdgcn_make_buffer_rsrc(simd, (short)0, (int)(kFairWaves * 4), 0x00020000);
        if (lane == 0) __hip_atomic_store(mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    // group head: now = progress so far, unit3 = the progress of 3 blocks (the priority step); both in the
    // same units for all waves of the launch (uniform values)
    __device__ __forceinline__ void group(uint32_t now, uint32_t unit3, int lane)
    {
        if (!mine) return;
        if (last != kFairEmpty) {
            // (no selects: v_cndmask issues in about 18 cycles at 8 waves per SIMD.)  Lanes 0..15 read the 16
            // words; an empty slot (kFairEmpty = ~0; posted values stay below 2^31) adds 0
            const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(seen != kFairEmpty) & ((1ull << kFairWaves) - 1ull));
            uint32_t x = seen & ~(uint32_t)((int32_t)seen >> 31);
            // sum of the 16 words: row_shr 1, 2, 4, 8 (lanes past the row edge add 0); lane 15 holds it
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
            x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
            const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
            // (own - mean) * n; own = the value posted at the previous call, which the read saw.  32-bit
            // scalar arithmetic (n <= 16, values < 2^26): 64-bit compares would run on the VALU.
            const int32_t d = (int32_t)last * (int32_t)n - (int32_t)sum, n3 = (int32_t)unit3 * (int32_t)n;
            if (d <= -n3) __builtin_amdgcn_s_setprio(3);
            else if (d <= 0) __builtin_amdgcn_s_setprio(2);
            else if (d <= n3) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (lane == 0) __hip_atomic_store(mine, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        last = now;
        // (glc: past the CU's L1, as the relaxed atomic load it replaces)
        seen = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(lane & (kFairWaves - 1)) * 4u, 0, 1);
    }
    __device__ __forceinline__ void end(int lane)
    {
        if (mine && lane == 0) __hip_atomic_store(mine, kFairEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};
}  // namespace vd
