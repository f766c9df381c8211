// vd_capi.hip -- C-ABI runtime of the MI355X Viterbi decoder (see include/vd_capi.h).
//
// Replaces the reference's ViterbiCUDA<options> implementation (src/viterbi/viterbi.cu:10-139,210-262):
// decoder objects own reusable device buffers and a stream; vd_run is the blocking host-to-host
// call with kernel-only event timing like the reference; vd_run_device is the allocation-free,
// sync-free device path; vd_run_batches shards independent batches over the devices of a node.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <chrono>

#include "../../include/vd_capi.h"
#include "vd_kernels.h"
#include "vd_kernel_tg.h"
#include "vd_kernel_pk.h"
#include "vd_pack.h"
#include "vd_mt.h"
#include "vd_mtjump.h"
#include "vd_segplan.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define VD_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(e_ == hipErrorOutOfMemory ? VD_ERR_NOMEM : VD_ERR_DEVICE,            \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                  \
    } while (0)

int ch_of(int o) { return o & 0xF; }
int met_of(int o) { return (o >> 4) & 0xF; }
int out_of(int o) { return (o >> 8) & 0xF; }
int comp_of(int o) { return (o >> 12) & 0xF; }
int bpp_of(int o) { return out_of(o) == 1 ? 16 : 32; }

bool valid(int o)
{
    if (o & ~0xFFFF) return false;
    int ch = ch_of(o), me = met_of(o), out = out_of(o), cm = comp_of(o);
    if (ch > 4 || me > 2 || out > 1 || cm > 1) return false;
    // OptionsValid (viterbi.h:22-41)
    if (ch == 2 && me == 2) return false;
    if (ch == 3 && me == 2) return false;
    if (ch == 3 && me == 1) return false;
    if (me == 2 && cm == 1) return false;
    return true;
}

size_t input_size(int o, size_t n)
{
    switch (ch_of(o)) {
    case 0: return (n + 7) / 8;
    case 1: return (n + 1) / 2;
    case 2: return n;
    case 3: return n * 2;
    case 4: return n * 4;
    }
    return 0;
}
size_t message_len(int o, size_t n)
{
    if (n / 2 < 64) return 0;  // the reference underflows here (size_t); rejected instead
    size_t bpp = (size_t)bpp_of(o);
    return (n / 2 - 64) / bpp * bpp;
}
// stages whose channel data lies in whole 32-bit words of the caller's buffer
uint64_t avail_stages(int o, size_t n)
{
    size_t words = input_size(o, n) / 4;
    uint64_t per = 0;
    switch (ch_of(o)) {
    case 0: per = words * 16; break;
    case 1: per = words * 4; break;
    case 2: per = words * 2; break;
    case 3: per = words; break;
    case 4: per = words / 2; break;
    }
    uint64_t half = n / 2;
    return per < half ? per : half;
}

using launch_fn = void (*)(const void*, void*, vd::Geom, unsigned, hipStream_t);

// workgroups of a launch without a segment table: one chunk per wave
unsigned tg_grid(const vd::Geom& g)
{
    return (unsigned)(((uint64_t)g.nchunks * g.nbatch + vd::kWaves - 1) / vd::kWaves);
}

// one kernel per format (SOFT16 on int32 patterns, TgFmt::INT); CH >= kLlr: float channel values
// quantised in the table build (fused SoftDecisionPacker)
template <int CH, int CORE, int OB>
void launch_t(const void* in, void* out, vd::Geom g, unsigned grid, hipStream_t s)
{
    hipLaunchKernelGGL((vd::vd_decode_tg<CH, CORE, OB>), dim3(grid), dim3(64 * vd::kWaves), 0, s, in, out, g);
}

template <int CH, int CORE>
launch_fn pick_ob(int ob)
{
    return ob == 1 ? &launch_t<CH, CORE, 16> : &launch_t<CH, CORE, 32>;
}

// batched HARD / SOFT4 / FP32 launches: two chunks per wave in int16 halves (vd_kernel_pk.h)
// (SPL: single-batch launches, one chunk per wave in both halves, vd_kernel_pk.h "split")
template <int CH, int CORE, int OB, bool SPL>
void launch_pk(const void* in, void* out, vd::Geom g, unsigned grid, hipStream_t s)
{
    hipLaunchKernelGGL((vd::vd_decode_pk<CH, CORE, OB, SPL>), dim3(grid), dim3(64 * vd::kWaves), 0, s, in, out, g);
}
template <int CH, int OB, bool SPL>
launch_fn pick_pk_core(int me)
{
    return me == 0 ? &launch_pk<CH, 0, OB, SPL> : me == 1 ? &launch_pk<CH, 1, OB, SPL> : &launch_pk<CH, 2, OB, SPL>;
}
template <int CH, bool SPL>
launch_fn pick_pk_ob(int o)
{
    return out_of(o) == 1 ? pick_pk_core<CH, 16, SPL>(met_of(o)) : pick_pk_core<CH, 32, SPL>(met_of(o));
}
template <bool SPL, int L>
launch_fn pick_pk_ch(int o)
{
    switch (ch_of(o)) {
    case 0: return pick_pk_ob<L + vd::HARD, SPL>(o);
    case 1: return pick_pk_ob<L + vd::SOFT4, SPL>(o);
    // (SOFT8 single batches: the split kernel is 9 % faster than vd_decode_tg's segment launch on codewords
    // and, with the early-stop re-decodes, 18 % slower on noise-only input: DESIGN.md 4.3)
    case 2:
        return out_of(o) == 1 ? (met_of(o) == 0 ? &launch_pk<L + vd::SOFT8, 0, 16, SPL> : &launch_pk<L + vd::SOFT8, 1, 16, SPL>)
                              : (met_of(o) == 0 ? &launch_pk<L + vd::SOFT8, 0, 32, SPL> : &launch_pk<L + vd::SOFT8, 1, 32, SPL>);
    case 4: return pick_pk_ob<L + vd::FP32, SPL>(o);
    }
    return nullptr;
}
template <bool SPL>
launch_fn pick_pk(int o, bool llr)
{
    return llr ? pick_pk_ch<SPL, vd::kLlr>(o) : pick_pk_ch<SPL, 0>(o);
}
template <int L>
launch_fn pick_ch(int o)
{
    const int ch = ch_of(o), me = met_of(o), ob = out_of(o);
    switch (ch) {
    case 0: return me == 0 ? pick_ob<L + 0, 0>(ob) : me == 1 ? pick_ob<L + 0, 1>(ob) : pick_ob<L + 0, 2>(ob);
    case 1: return me == 0 ? pick_ob<L + 1, 0>(ob) : me == 1 ? pick_ob<L + 1, 1>(ob) : pick_ob<L + 1, 2>(ob);
    case 2: return me == 0 ? pick_ob<L + 2, 0>(ob) : pick_ob<L + 2, 1>(ob);
    case 3: return pick_ob<L + 3, 0>(ob);
    case 4: return me == 0 ? pick_ob<L + 4, 0>(ob) : me == 1 ? pick_ob<L + 4, 1>(ob) : pick_ob<L + 4, 2>(ob);
    }
    return nullptr;
}
launch_fn pick(int o, bool llr)
{
    return llr ? pick_ch<vd::kLlr>(o) : pick_ch<0>(o);
}

// CORE names the option's tie rule.  vd_decode_tg computes on the fp32 exact-integer tagged core (SOFT16:
// int32 patterns); vd_decode_pk (HARD / SOFT4 / SOFT8 / FP32) on exact-integer tagged int16 halves, two
// chunks per lane; none on fp16 arithmetic
const char* kname(int o)
{
    static const char* names[5][3] = {
        {"vd_decode_pk<HARD,B32> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<HARD,B32> (single batches with chunks under 64 words); M_B32 tie rule",
         "vd_decode_pk<HARD,B16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<HARD,B16> (single batches with chunks under 64 words); M_B16 tie rule",
         "vd_decode_pk<HARD,F16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<HARD,F16> (single batches with chunks under 64 words); M_FP16 tie rule"},
        {"vd_decode_pk<SOFT4,B32> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<SOFT4,B32> (single batches with chunks under 64 words); M_B32 tie rule",
         "vd_decode_pk<SOFT4,B16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<SOFT4,B16> (single batches with chunks under 64 words); M_B16 tie rule",
         "vd_decode_pk<SOFT4,F16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<SOFT4,F16> (single batches with chunks under 64 words); M_FP16 tie rule"},
        {"vd_decode_pk<SOFT8,B32> (int16 halves, 2-stage fields: batched, two chunks per lane; single batch, one "
         "chunk cut in two) / vd_decode_tg<SOFT8,B32> (single batches with chunks under 64 words); M_B32 tie rule",
         "vd_decode_pk<SOFT8,B16> (int16 halves, 2-stage fields: batched, two chunks per lane; single batch, one "
         "chunk cut in two) / vd_decode_tg<SOFT8,B16> (single batches with chunks under 64 words); M_B16 tie rule",
         "-"},
        {"vd_decode_tg<SOFT16,B32> (int32 tagged patterns, M_B32 tie rule)", "-", "-"},
        {"vd_decode_pk<FP32,B32> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<FP32,B32> (single batches with chunks under 64 words); M_B32 tie rule",
         "vd_decode_pk<FP32,B16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<FP32,B16> (single batches with chunks under 64 words); M_B16 tie rule",
         "vd_decode_pk<FP32,F16> (int16 halves: batched, two chunks per lane; single batch, one chunk cut in two) / "
         "vd_decode_tg<FP32,F16> (single batches with chunks under 64 words); M_FP16 tie rule"},
    };
    if (!valid(o)) return "-";
    return names[ch_of(o)][met_of(o)];
}

}  // namespace

// Device address of page-locked, device-mapped host memory (vd_host_alloc / hipHostMalloc /
// hipHostRegister), or null for pageable memory.  Kernels then read inputs from / write decoded words
// to such buffers directly over PCIe (zero-copy), with no staging copies at all.
static void* mapped_host(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

struct DeviceState;
struct vd_decoder {
    int options = 0;
    int device = 0;
    void* in_d = nullptr;
    void* out_d = nullptr;
    void* llr_d = nullptr;  // vd_run_llr's float input buffer
    size_t cap_in = 0, cap_out = 0, cap_llr = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // vd_run_stream: a second buffer set and the copy-in / copy-out streams of the 3-stage pipeline
    void* in2_d = nullptr;
    void* out2_d = nullptr;
    size_t cap2_in = 0, cap2_out = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    DeviceState* ds = nullptr;  // the device's board / segment tables (looked up once, vd_create)
    int split = 1;              // segment launches: 0 none (VD_NO_SPLIT=1), 1 pieces, 2 thirds, 3 sevenths (VD_SPLIT=...)
    int pk = 1;                 // HARD/SOFT4/FP32 launches on vd_decode_pk (VD_NO_PK=1: on vd_decode_tg)
    int pksplit = 1;            // their single-batch launches split on vd_decode_pk (VD_PK_SPLIT=0: tg segments)
    int pktail = 1;             // ... with the tail chunks in 4-wave workgroups (VD_PK_TAIL=0: one chunk per wave)
    uint32_t* check = nullptr;  // LDS guard violation counter (vd_set_guard_check), null = off
};

static int ensure_capacity(vd_decoder* d, size_t inBytes, size_t outBytes)
{
    if (inBytes > d->cap_in) {
        if (d->in_d) (void)hipFree(d->in_d);
        d->in_d = nullptr;
        d->cap_in = 0;
        VD_HIP(hipMalloc(&d->in_d, inBytes));
        d->cap_in = inBytes;
    }
    if (outBytes > d->cap_out) {
        if (d->out_d) (void)hipFree(d->out_d);
        d->out_d = nullptr;
        d->cap_out = 0;
        VD_HIP(hipMalloc(&d->out_d, outBytes));
        d->cap_out = outBytes;
    }
    return VD_OK;
}

// Per-device state shared by every decoder and stream on a device, allocated once per device:
//  * the progress board of the decode kernels' fairness controller (vd_kernels.h Fair, Geom::fair),
//    every word kFairEmpty at rest (the kernels free their slots); concurrent launches sharing it only
//    perturb issue priorities;
//  * the segment tables of segment launches (read only; vd_kernel_tg.h "segment launches");
//  * the re-decode counter of segment and split launches (vd_split_redecodes) and the split launches'
//    pass-cap counter (vd_split_cap_exits: waves that stopped re-decoding at the cap with a part still
//    differing; never expected, and vd_run / vd_run_stream fail when it is non-zero).
// Segment launches keep their boundary vectors in LDS, so launches on any number of streams share no
// scratch.  A decoder looks the state up once (vd_create), not per launch.
struct SegTable {
    uint32_t* d = nullptr;  // first chunk of each workgroup, then the chunk count
    unsigned nwg = 0;
};
struct DeviceState {
    uint32_t* board = nullptr;
    int nsimd = 0;
    uint32_t* stats = nullptr;
    SegTable pieces, thirds, sevenths;
};
static DeviceState* device_state(int device)
{
    static std::mutex mu;
    static std::vector<DeviceState*> st;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)st.size() <= device) st.resize(device + 1, nullptr);
    if (!st[device]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
            return nullptr;
        DeviceState* x = new DeviceState;
        x->nsimd = 4 * cus;
        bool ok = hipMalloc(&x->board, vd::kFairBoardWords * 4) == hipSuccess &&
                  hipMemset(x->board, 0xFF, vd::kFairBoardWords * 4) == hipSuccess &&
                  hipMalloc(&x->stats, 8) == hipSuccess && hipMemset(x->stats, 0, 8) == hipSuccess;
        for (int th = 0; th < 3 && ok; th++) {
            const std::vector<uint32_t> t = vd::seg_table(x->nsimd, th);
            if (t.empty()) continue;
            SegTable& T = th == vd::kSegSevenths ? x->sevenths : th == vd::kSegThirds ? x->thirds : x->pieces;
            ok = hipMalloc(&T.d, t.size() * 4) == hipSuccess &&
                 hipMemcpy(T.d, t.data(), t.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
            T.nwg = (unsigned)(t.size() - 1);
        }
        if (!ok || hipDeviceSynchronize() != hipSuccess) {
            delete x;
            return nullptr;
        }
        st[device] = x;
    }
    return st[device];
}
// Segment launch when the chunks are long enough and the device has a table; returns the grid
static unsigned plan_split(vd::Geom& g, int options, const DeviceState* x, int mode)
{
    const uint64_t words32 = out_of(options) != 0 ? g.packNum / 2 : g.packNum;  // O_B16: 16-bit words
    if (mode == 0 || g.nchunks != (uint32_t)vd::kChunks || words32 / g.nchunks < (uint64_t)vd::kSplitMinWords)
        return tg_grid(g);
    const SegTable& T = mode == 2 && x->thirds.d ? x->thirds : mode == 3 && x->sevenths.d ? x->sevenths : x->pieces;
    if (!T.d) return tg_grid(g);
    g.seg = T.d;
    g.stats = x->stats;
    return T.nwg;
}

// Which kernel and launch form a decode takes (launch_decode and vd_decoder_kernel_name share it):
// batched launches of HARD/SOFT4/SOFT8/FP32 on vd_decode_pk (two chunks per wave); single batches of
// HARD/SOFT4/SOFT8/FP32 with chunks of >= kSplitMinWords words on vd_decode_pk's split kernel; the rest on
// vd_decode_tg (segment launch when plan_split finds a table, else one chunk per wave).
enum class Form { PkBatched, PkSplit, Tg };
static Form plan_form(const vd_decoder* d, uint64_t packNum, uint32_t nbatch, bool llr)
{
    const int options = d->options;
    if (nbatch > 1 && d->pk && vd::kChunks % (2 * vd::kWaves) == 0 && pick_pk<false>(options, llr)) return Form::PkBatched;
    const uint64_t w32 = out_of(options) != 0 ? packNum / 2 : packNum;
    const bool splitok = nbatch == 1 && d->pk && d->pksplit && d->split && vd::kChunks % vd::kWaves == 0 &&
                         w32 / vd::kChunks >= (uint64_t)vd::kSplitMinWords;
    if (splitok && pick_pk<true>(options, llr)) return Form::PkSplit;
    return Form::Tg;
}

// llr: in_d holds inputNum float channel values, quantised in the kernel (scale = packer scale).
// nbatch > 1: batch b at in_d + b * inStride, out_d + b * outStride, all in one launch (never split).
static int launch_decode(const vd_decoder* d, const void* in_d, void* out_d, size_t inputNum, hipStream_t s,
                         bool llr = false, float scale = 1.0f, uint32_t nbatch = 1, uint64_t inStride = 0,
                         uint64_t outStride = 0)
{
    const int options = d->options;
    launch_fn f = pick(options, llr);
    if (!f) return fail(VD_ERR_OPTIONS, "invalid options");
    size_t msg = message_len(options, inputNum);
    vd::Geom g;
    g.packNum = msg / (size_t)bpp_of(options);
    g.availStages = llr ? inputNum / 2 : avail_stages(options, inputNum);
    g.nchunks = vd::kChunks;
    g.scale = scale;
    if (g.packNum == 0) return VD_OK;
    // the launch goes to the stream's device (the null stream: the current device); the board and the
    // guard counter belong to the decoder's device
    int sdev = -1;
    if (s) VD_HIP(hipStreamGetDevice(s, &sdev));
    else VD_HIP(hipGetDevice(&sdev));
    if (sdev != d->device)
        return fail(VD_ERR_ARG, "stream on device " + std::to_string(sdev) + ", decoder on device " +
                                    std::to_string(d->device));
    g.fair = d->ds->board;
    g.check = d->check;
    g.nbatch = nbatch;
    g.inStride = inStride;
    g.outStride = outStride;
    const Form form = plan_form(d, g.packNum, nbatch, llr);
    if (form == Form::PkBatched) {  // two chunks per wave: nchunks * nbatch / 8 workgroups
        pick_pk<false>(options, llr)(in_d, out_d, g, (unsigned)((uint64_t)g.nchunks * nbatch / (2 * vd::kWaves)), s);
        VD_HIP(hipGetLastError());
        return VD_OK;
    }
    if (form == Form::PkSplit) {  // single batch: one chunk per wave, cut in two halves (nchunks / 4 workgroups)
        g.stats = d->ds->stats;
        // the last nchunks mod (SIMDs) chunks one per workgroup of 4 waves (8 parts each): with 6400 chunks
        // on 1024 SIMDs every SIMD then runs 6 whole-chunk waves and one short one (vd_kernel_pk.h "split")
        const uint32_t per = (uint32_t)d->ds->nsimd, tailc = per ? g.nchunks % per : 0u;
        unsigned grid = g.nchunks / vd::kWaves;
        if (d->pktail && tailc) {
            g.tailWG = (g.nchunks - tailc) / vd::kWaves;
            grid = g.tailWG + tailc;
        }
        pick_pk<true>(options, llr)(in_d, out_d, g, grid, s);
        VD_HIP(hipGetLastError());
        return VD_OK;
    }
    const unsigned grid = nbatch == 1 ? plan_split(g, options, d->ds, d->split) : tg_grid(g);
    f(in_d, out_d, g, grid, s);
    VD_HIP(hipGetLastError());
    return VD_OK;
}

extern "C" {

int vd_options_valid(int options) { return valid(options) ? 1 : 0; }
size_t vd_input_size(int options, size_t n) { return input_size(options, n); }
size_t vd_message_len(int options, size_t n) { return message_len(options, n); }
size_t vd_output_size(int options, size_t n) { return message_len(options, n) / 8; }
int vd_num_chunks(void) { return vd::kChunks; }

int vd_split_redecodes(int device, uint64_t* count)
{
    if (!count) return fail(VD_ERR_ARG, "null argument");
    DeviceState* x = device_state(device);
    if (!x) return fail(VD_ERR_DEVICE, "per-device decode state unavailable");
    uint32_t v = 0;
    VD_HIP(hipMemcpy(&v, x->stats, 4, hipMemcpyDeviceToHost));
    *count = v;
    return VD_OK;
}
int vd_split_cap_exits(int device, uint64_t* count)
{
    if (!count) return fail(VD_ERR_ARG, "null argument");
    DeviceState* x = device_state(device);
    if (!x) return fail(VD_ERR_DEVICE, "per-device decode state unavailable");
    uint32_t v = 0;
    VD_HIP(hipMemcpy(&v, x->stats + 1, 4, hipMemcpyDeviceToHost));
    *count = v;
    return VD_OK;
}
const char* vd_last_error(void) { return g_err.c_str(); }
const char* vd_kernel_name(int options) { return kname(options); }

const char* vd_decoder_kernel_name(vd_decoder* d, size_t inputNum, int nbatch, int llr)
{
    static thread_local std::string name;
    if (!d || nbatch < 1) return "-";
    static const char* chs[5] = {"HARD", "SOFT4", "SOFT8", "SOFT16", "FP32"};
    static const char* cores[3] = {"B32", "B16", "F16"};
    const int o = d->options;
    const uint64_t packNum = message_len(o, inputNum) / (size_t)bpp_of(o);
    if (packNum == 0) return "-";  // launch_decode launches nothing
    const std::string args = std::string(llr ? "LLR+" : "") + chs[ch_of(o)] + "," + cores[met_of(o)] + "," +
                             (out_of(o) ? "O16" : "O32") + ">";
    vd::Geom g;
    g.packNum = packNum;
    g.nchunks = vd::kChunks;
    switch (plan_form(d, packNum, (uint32_t)nbatch, llr != 0)) {
    case Form::PkBatched: name = "vd_decode_pk<" + args + " batched: two chunks per wave, int16 halves"; break;
    case Form::PkSplit: name = "vd_decode_pk<" + args + " split: one chunk per wave cut in two, int16 halves"; break;
    default:
        if (nbatch == 1) (void)plan_split(g, o, d->ds, d->split);
        name = "vd_decode_tg<" + args + (g.seg ? " segment launch: one chunk or piece per wave, fp32 tagged core"
                                               : " one chunk per wave, fp32 tagged core");
        if (ch_of(o) == 3) name.replace(name.find("fp32 tagged core"), 16, "int32 tagged patterns");
    }
    return name.c_str();
}

int vd_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int vd_create(int options, size_t preallocInputNum, int device, vd_decoder** out)
{
    if (!out) return fail(VD_ERR_ARG, "null output handle");
    *out = nullptr;
    if (!valid(options)) return fail(VD_ERR_OPTIONS, "options disabled by OptionsValid");
    int ndev = 0;
    VD_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(VD_ERR_ARG, "device index out of range");
    VD_HIP(hipSetDevice(device));
    vd_decoder* d = new vd_decoder();
    d->options = options;
    d->device = device;
    d->ds = device_state(device);
    if (!d->ds) {
        delete d;
        return fail(VD_ERR_NOMEM, "per-device decode state allocation failed");
    }
    const char* nosplit = std::getenv("VD_NO_SPLIT");
    const char* smode = std::getenv("VD_SPLIT");
    d->split = nosplit && nosplit[0] == '1' ? 0 : smode && !strcmp(smode, "thirds") ? 2 : smode && !strcmp(smode, "sevenths") ? 3 : 1;
    const char* nopk = std::getenv("VD_NO_PK");
    d->pk = nopk && nopk[0] == '1' ? 0 : 1;
    const char* pks = std::getenv("VD_PK_SPLIT");
    d->pksplit = pks && pks[0] == '0' ? 0 : 1;
    const char* pkt = std::getenv("VD_PK_TAIL");
    d->pktail = pkt && pkt[0] == '0' ? 0 : 1;
    const char* chk = std::getenv("VD_CHECK");
    if (chk && chk[0] == '1') {
        int rc = vd_set_guard_check(d, 1);
        if (rc != VD_OK) { vd_destroy(d); return rc; }
    }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&d->ev0) != hipSuccess || hipEventCreate(&d->ev1) != hipSuccess) {
        vd_destroy(d);
        return fail(VD_ERR_DEVICE, "stream/event creation failed");
    }
    if (preallocInputNum) {
        int rc = ensure_capacity(d, input_size(options, preallocInputNum),
                                 message_len(options, preallocInputNum) / 8 + 16);
        if (rc != VD_OK) { vd_destroy(d); return rc; }
    }
    *out = d;
    return VD_OK;
}

int vd_destroy(vd_decoder* d)
{
    if (!d) return VD_OK;
    (void)hipSetDevice(d->device);
    if (d->in_d) (void)hipFree(d->in_d);
    if (d->out_d) (void)hipFree(d->out_d);
    if (d->llr_d) (void)hipFree(d->llr_d);
    if (d->in2_d) (void)hipFree(d->in2_d);
    if (d->out2_d) (void)hipFree(d->out2_d);
    if (d->s_in) (void)hipStreamDestroy(d->s_in);
    if (d->s_out) (void)hipStreamDestroy(d->s_out);
    if (d->ev0) (void)hipEventDestroy(d->ev0);
    if (d->ev1) (void)hipEventDestroy(d->ev1);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    if (d->check) (void)hipFree(d->check);
    delete d;
    return VD_OK;
}

// vd_run / vd_run_stream (blocking): a single-batch split launch whose re-decode passes hit their cap with a part
// still differing (vd_kernel_pk.h "Split"; never expected) fails the call instead of returning wrong words
static int check_split_cap(const vd_decoder* d, size_t inputNum, bool llr = false)
{
    const uint64_t packNum = message_len(d->options, inputNum) / (size_t)bpp_of(d->options);
    if (packNum == 0 || plan_form(d, packNum, 1, llr) != Form::PkSplit) return VD_OK;
    uint32_t v = 0;
    VD_HIP(hipMemcpy(&v, d->ds->stats + 1, 4, hipMemcpyDeviceToHost));
    if (v)
        return fail(VD_ERR_DEVICE, "split launch reached its re-decode pass cap with a part still differing (" +
                                       std::to_string(v) + " waves on this device so far): decoded words may be wrong");
    return VD_OK;
}

int vd_run(vd_decoder* d, const void* input_h, void* output_h, size_t inputNum, float* kernel_ms)
{
    if (!d || !input_h || !output_h) return fail(VD_ERR_ARG, "null argument");
    const size_t inB = input_size(d->options, inputNum), outB = message_len(d->options, inputNum) / 8;
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    VD_HIP(hipSetDevice(d->device));
    void* zin = mapped_host(input_h);
    void* zout = zin ? mapped_host(output_h) : nullptr;
    if (zin && zout) {  // pinned host buffers: zero-copy decode (kernel_ms then includes the PCIe traffic)
        VD_HIP(hipEventRecord(d->ev0, d->stream));
        int rc = launch_decode(d, zin, zout, inputNum, d->stream);
        if (rc != VD_OK) return rc;
        VD_HIP(hipEventRecord(d->ev1, d->stream));
        VD_HIP(hipStreamSynchronize(d->stream));
        if (kernel_ms) VD_HIP(hipEventElapsedTime(kernel_ms, d->ev0, d->ev1));
        return check_split_cap(d, inputNum);
    }
    int rc = ensure_capacity(d, inB, outB + 16);
    if (rc != VD_OK) return rc;
    VD_HIP(hipMemcpyAsync(d->in_d, input_h, inB, hipMemcpyHostToDevice, d->stream));
    VD_HIP(hipEventRecord(d->ev0, d->stream));
    rc = launch_decode(d, d->in_d, d->out_d, inputNum, d->stream);
    if (rc != VD_OK) return rc;
    VD_HIP(hipEventRecord(d->ev1, d->stream));
    VD_HIP(hipMemcpyAsync(output_h, d->out_d, outB, hipMemcpyDeviceToHost, d->stream));
    VD_HIP(hipStreamSynchronize(d->stream));
    if (kernel_ms) VD_HIP(hipEventElapsedTime(kernel_ms, d->ev0, d->ev1));
    return check_split_cap(d, inputNum);
}

int vd_set_guard_check(vd_decoder* d, int enable)
{
    if (!d) return fail(VD_ERR_ARG, "null argument");
    VD_HIP(hipSetDevice(d->device));
    if (!enable) {
        if (d->check) VD_HIP(hipDeviceSynchronize());
        if (d->check) (void)hipFree(d->check);
        d->check = nullptr;
        return VD_OK;
    }
    // kernels still in flight on the decoder's or a caller's (non-blocking) stream may add to the counter:
    // let them finish before the reset
    if (d->check) VD_HIP(hipDeviceSynchronize());
    else VD_HIP(hipMalloc(&d->check, 4));
    VD_HIP(hipMemset(d->check, 0, 4));
    VD_HIP(hipDeviceSynchronize());
    return VD_OK;
}

int vd_guard_violations(vd_decoder* d, uint64_t* count)
{
    if (!d || !count) return fail(VD_ERR_ARG, "null argument");
    if (!d->check) return fail(VD_ERR_ARG, "guard check not enabled (vd_set_guard_check)");
    VD_HIP(hipSetDevice(d->device));
    VD_HIP(hipDeviceSynchronize());
    uint32_t v = 0;
    VD_HIP(hipMemcpy(&v, d->check, 4, hipMemcpyDeviceToHost));
    *count = v;
    return VD_OK;
}

int vd_run_device(vd_decoder* d, const void* input_d, void* output_d, size_t inputNum, void* stream)
{
    if (!d || !input_d || !output_d) return fail(VD_ERR_ARG, "null argument");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    return launch_decode(d, input_d, output_d, inputNum, (hipStream_t)stream);
}

int vd_run_device_batch(vd_decoder* d, const void* input_d, size_t input_stride, void* output_d, size_t output_stride,
                        size_t inputNum, int nbatch, void* stream)
{
    if (!d || !input_d || !output_d) return fail(VD_ERR_ARG, "null argument");
    if (nbatch < 1) return fail(VD_ERR_ARG, "nbatch must be >= 1");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    if (nbatch > 1 && output_stride < message_len(d->options, inputNum) / 8)
        return fail(VD_ERR_ARG, "output_stride smaller than the output size: batches would overlap");
    // input_stride: any (0 = every batch decodes the same input); inputs are only read, so overlapping
    // windows (e.g. sliding) are valid
    if ((uint64_t)vd::kChunks * (uint64_t)nbatch > 0xFFFFFFFFull) return fail(VD_ERR_ARG, "nbatch too large");
    if ((input_stride | output_stride) & 3) return fail(VD_ERR_ARG, "strides must be multiples of 4 bytes");
    if (nbatch == 1) return launch_decode(d, input_d, output_d, inputNum, (hipStream_t)stream);
    return launch_decode(d, input_d, output_d, inputNum, (hipStream_t)stream, false, 1.0f, (uint32_t)nbatch, input_stride,
                         output_stride);
}

static int launch_pack(int options, const float* llr_d, size_t inputNum, float scale, void* packed_d, hipStream_t s)
{
    if (((uintptr_t)llr_d & 15) != 0) return fail(VD_ERR_ARG, "llr buffer must be 16-byte aligned");
    const int ch = ch_of(options);
    const int per = ch == 0 ? 32 : ch == 1 ? 8 : ch == 2 ? 4 : ch == 3 ? 2 : 1;
    const uint64_t nw = (inputNum + per - 1) / per;
    if (nw == 0) return VD_OK;
    const dim3 blk(256), grd((unsigned)((nw + 255) / 256));
    switch (ch) {
    case 0: hipLaunchKernelGGL(vd::pack_llr<0>, grd, blk, 0, s, llr_d, (uint64_t)inputNum, scale, packed_d); break;
    case 1: hipLaunchKernelGGL(vd::pack_llr<1>, grd, blk, 0, s, llr_d, (uint64_t)inputNum, scale, packed_d); break;
    case 2: hipLaunchKernelGGL(vd::pack_llr<2>, grd, blk, 0, s, llr_d, (uint64_t)inputNum, scale, packed_d); break;
    case 3: hipLaunchKernelGGL(vd::pack_llr<3>, grd, blk, 0, s, llr_d, (uint64_t)inputNum, scale, packed_d); break;
    case 4: hipLaunchKernelGGL(vd::pack_llr<4>, grd, blk, 0, s, llr_d, (uint64_t)inputNum, scale, packed_d); break;
    }
    VD_HIP(hipGetLastError());
    return VD_OK;
}

int vd_pack_device(int options, const float* llr_d, size_t inputNum, float scale, void* packed_d, void* stream)
{
    if (!valid(options)) return fail(VD_ERR_OPTIONS, "options disabled by OptionsValid");
    if (!llr_d || !packed_d) return fail(VD_ERR_ARG, "null argument");
    return launch_pack(options, llr_d, inputNum, scale, packed_d, (hipStream_t)stream);
}

int vd_run_device_llr(vd_decoder* d, const float* llr_d, void* output_d, size_t inputNum, float scale, void* stream)
{
    if (!d || !llr_d || !output_d) return fail(VD_ERR_ARG, "null argument");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    return launch_decode(d, llr_d, output_d, inputNum, (hipStream_t)stream, true, scale);
}

int vd_run_device_llr_batch(vd_decoder* d, const float* llr_d, size_t llr_stride, void* output_d, size_t output_stride,
                            size_t inputNum, float scale, int nbatch, void* stream)
{
    if (!d || !llr_d || !output_d) return fail(VD_ERR_ARG, "null argument");
    if (nbatch < 1) return fail(VD_ERR_ARG, "nbatch must be >= 1");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    if (nbatch > 1 && output_stride < message_len(d->options, inputNum) / 8)
        return fail(VD_ERR_ARG, "output_stride smaller than the output size: batches would overlap");
    if ((uint64_t)vd::kChunks * (uint64_t)nbatch > 0xFFFFFFFFull) return fail(VD_ERR_ARG, "nbatch too large");
    if ((llr_stride & 15) || (output_stride & 3)) return fail(VD_ERR_ARG, "llr_stride % 16 or output_stride % 4 != 0");
    if (nbatch == 1) return launch_decode(d, llr_d, output_d, inputNum, (hipStream_t)stream, true, scale);
    return launch_decode(d, llr_d, output_d, inputNum, (hipStream_t)stream, true, scale, (uint32_t)nbatch, llr_stride,
                         output_stride);
}

int vd_run_llr(vd_decoder* d, const float* llr_h, void* output_h, size_t inputNum, float scale, float* kernel_ms)
{
    if (!d || !llr_h || !output_h) return fail(VD_ERR_ARG, "null argument");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    const size_t inB = inputNum * sizeof(float), outB = message_len(d->options, inputNum) / 8;
    VD_HIP(hipSetDevice(d->device));
    if (inB > d->cap_llr) {
        if (d->llr_d) (void)hipFree(d->llr_d);
        d->llr_d = nullptr;
        d->cap_llr = 0;
        VD_HIP(hipMalloc(&d->llr_d, inB));
        d->cap_llr = inB;
    }
    int rc = ensure_capacity(d, 0, outB + 16);
    if (rc != VD_OK) return rc;
    VD_HIP(hipMemcpyAsync(d->llr_d, llr_h, inB, hipMemcpyHostToDevice, d->stream));
    VD_HIP(hipEventRecord(d->ev0, d->stream));
    rc = vd_run_device_llr(d, (const float*)d->llr_d, d->out_d, inputNum, scale, d->stream);
    if (rc != VD_OK) return rc;
    VD_HIP(hipEventRecord(d->ev1, d->stream));
    VD_HIP(hipMemcpyAsync(output_h, d->out_d, outB, hipMemcpyDeviceToHost, d->stream));
    VD_HIP(hipStreamSynchronize(d->stream));
    if (kernel_ms) VD_HIP(hipEventElapsedTime(kernel_ms, d->ev0, d->ev1));
    return check_split_cap(d, inputNum, true);
}

void* vd_host_alloc(size_t bytes)
{
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        fail(VD_ERR_NOMEM, "pinned host allocation failed");
        return nullptr;
    }
    return p;
}

int vd_host_free(void* p)
{
    if (p) VD_HIP(hipHostFree(p));
    return VD_OK;
}

// Three-stage pipeline over independent batches on one device: H2D of batch b+1 (stream s_in),
// decode of batch b (the decoder's stream), D2H of batch b-1 (s_out), two device buffer sets.
// Host buffers at full PCIe rate when pinned (vd_host_alloc); pageable ones work, staged by HIP.
int vd_run_stream(vd_decoder* d, const void* const* input_h, void* const* output_h, int nbatches, size_t inputNum,
                  float* wall_ms)
{
    if (!d || !input_h || !output_h || nbatches < 0) return fail(VD_ERR_ARG, "bad arguments");
    if (message_len(d->options, inputNum) == 0) return fail(VD_ERR_ARG, "inputNum too small");
    const size_t inB = input_size(d->options, inputNum), outB = message_len(d->options, inputNum) / 8;
    VD_HIP(hipSetDevice(d->device));
    // all buffers pinned: the kernels stream them over PCIe themselves, back to back on one stream
    bool zc = true;
    for (int b = 0; b < nbatches && zc; b++) zc = mapped_host(input_h[b]) && mapped_host(output_h[b]);
    if (zc) {
        auto t0 = std::chrono::steady_clock::now();
        for (int b = 0; b < nbatches; b++) {
            int rc = launch_decode(d, mapped_host(input_h[b]), mapped_host(output_h[b]), inputNum, d->stream);
            if (rc != VD_OK) return rc;
        }
        VD_HIP(hipStreamSynchronize(d->stream));
        if (wall_ms)
            *wall_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return nbatches > 0 ? check_split_cap(d, inputNum) : VD_OK;
    }
    int rc = ensure_capacity(d, inB, outB + 16);
    if (rc != VD_OK) return rc;
    if (inB > d->cap2_in) {
        if (d->in2_d) (void)hipFree(d->in2_d);
        d->in2_d = nullptr;
        d->cap2_in = 0;
        VD_HIP(hipMalloc(&d->in2_d, inB));
        d->cap2_in = inB;
    }
    if (outB + 16 > d->cap2_out) {
        if (d->out2_d) (void)hipFree(d->out2_d);
        d->out2_d = nullptr;
        d->cap2_out = 0;
        VD_HIP(hipMalloc(&d->out2_d, outB + 16));
        d->cap2_out = outB + 16;
    }
    if (!d->s_in) VD_HIP(hipStreamCreateWithFlags(&d->s_in, hipStreamNonBlocking));
    if (!d->s_out) VD_HIP(hipStreamCreateWithFlags(&d->s_out, hipStreamNonBlocking));
    void* ins[2] = {d->in_d, d->in2_d};
    void* outs[2] = {d->out_d, d->out2_d};
    // per buffer set: input landed, decode done (input free, output ready), output drained
    hipEvent_t landed[2], decoded[2], drained[2];
    for (int k = 0; k < 2; k++) {
        VD_HIP(hipEventCreateWithFlags(&landed[k], hipEventDisableTiming));
        VD_HIP(hipEventCreateWithFlags(&decoded[k], hipEventDisableTiming));
        VD_HIP(hipEventCreateWithFlags(&drained[k], hipEventDisableTiming));
    }
    // Submission order matters: the runtime runs the copies of a device in submission order, so the
    // H2D of batch b+1 is enqueued BEFORE the D2H of batch b (it then overlaps decode b).
    auto h2d = [&](int b) -> int {
        const int k = b & 1;
        if (b >= 2 && hipStreamWaitEvent(d->s_in, decoded[k], 0) != hipSuccess) return fail(VD_ERR_DEVICE, "wait");
        if (hipMemcpyAsync(ins[k], input_h[b], inB, hipMemcpyHostToDevice, d->s_in) != hipSuccess ||
            hipEventRecord(landed[k], d->s_in) != hipSuccess)
            return fail(VD_ERR_DEVICE, "H2D enqueue failed");
        return VD_OK;
    };
    auto t0 = std::chrono::steady_clock::now();
    rc = nbatches > 0 ? h2d(0) : VD_OK;
    for (int b = 0; b < nbatches && rc == VD_OK; b++) {
        const int k = b & 1;
        if (hipStreamWaitEvent(d->stream, landed[k], 0) != hipSuccess ||
            (b >= 2 && hipStreamWaitEvent(d->stream, drained[k], 0) != hipSuccess)) {
            rc = fail(VD_ERR_DEVICE, "pipeline enqueue failed");
            break;
        }
        rc = launch_decode(d, ins[k], outs[k], inputNum, d->stream);
        if (rc != VD_OK) break;
        if (hipEventRecord(decoded[k], d->stream) != hipSuccess) { rc = fail(VD_ERR_DEVICE, "record"); break; }
        if (b + 1 < nbatches && (rc = h2d(b + 1)) != VD_OK) break;
        if (hipStreamWaitEvent(d->s_out, decoded[k], 0) != hipSuccess ||
            hipMemcpyAsync(output_h[b], outs[k], outB, hipMemcpyDeviceToHost, d->s_out) != hipSuccess ||
            hipEventRecord(drained[k], d->s_out) != hipSuccess) {
            rc = fail(VD_ERR_DEVICE, "pipeline enqueue failed");
            break;
        }
    }
    const hipError_t e1 = hipStreamSynchronize(d->s_out), e2 = hipStreamSynchronize(d->stream),
                     e3 = hipStreamSynchronize(d->s_in);
    auto t1 = std::chrono::steady_clock::now();
    for (int k = 0; k < 2; k++) {
        (void)hipEventDestroy(landed[k]);
        (void)hipEventDestroy(decoded[k]);
        (void)hipEventDestroy(drained[k]);
    }
    if (rc != VD_OK) return rc;
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) return fail(VD_ERR_DEVICE, "pipeline failed");
    if (wall_ms) *wall_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    return nbatches > 0 ? check_split_cap(d, inputNum) : VD_OK;
}

int vd_run_batches(int options, const void* const* input_h, void* const* output_h, size_t inputNum,
                   int nbatches, const int* devices, int ndev, float* wall_ms)
{
    if (!valid(options)) return fail(VD_ERR_OPTIONS, "options disabled by OptionsValid");
    if (!input_h || !output_h || !devices || ndev <= 0 || nbatches < 0) return fail(VD_ERR_ARG, "bad arguments");
    std::vector<vd_decoder*> decs(ndev, nullptr);
    for (int i = 0; i < ndev; i++) {
        int rc = vd_create(options, inputNum, devices[i], &decs[i]);
        if (rc != VD_OK) {
            for (auto* x : decs) vd_destroy(x);
            return rc;
        }
    }
    std::vector<int> rcs(ndev, VD_OK);
    std::vector<std::string> errs(ndev);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int i = 0; i < ndev; i++) {
        th.emplace_back([&, i]() {
            for (int b = i; b < nbatches; b += ndev) {
                int rc = vd_run(decs[i], input_h[b], output_h[b], inputNum, nullptr);
                if (rc != VD_OK) { rcs[i] = rc; errs[i] = g_err; return; }
            }
        });
    }
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    for (auto* x : decs) vd_destroy(x);
    for (int i = 0; i < ndev; i++)
        if (rcs[i] != VD_OK) return fail(rcs[i], errs[i]);
    if (wall_ms) *wall_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    return VD_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- reference-exact channel source
namespace {
constexpr uint64_t kMtL = 65536;  // engine outputs per parallel segment
constexpr int kMtR = 8;           // radix of the jump tree
constexpr int kMtLevels = 6;      // jump polynomials for trees of up to R^6 = 262144 segments (2^34 outputs)
int mt_levels(uint64_t T)
{
    int k = 0;
    for (uint64_t p = 1; p < T; p *= kMtR) k++;
    return k;
}
// segment-start states of std::mt19937(seed) for T segments of kMtL outputs: st[m] = the state after
// m * kMtL outputs.  Jump tree, top level first: every state at a multiple of R^(k+1) generates its
// raw words (mt_xseq), then the R-1 children at +c R^k are XOR-accumulated from them (mt_jump).
// jump polynomials on the current device (uploaded once per device, kept for the process)
int mt_polys_device(const uint32_t** out)
{
    static std::mutex mu;
    static std::vector<uint32_t*> per_dev;
    int dev = 0;
    VD_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1, nullptr);
    if (!per_dev[dev]) {
        const std::vector<uint32_t>* polys;
        try {
            polys = &vd::mtj::jump_polys(kMtL, kMtR, kMtLevels);
        } catch (const std::exception& e) {
            return fail(VD_ERR_DEVICE, std::string("mt19937 jump polynomials: ") + e.what());
        }
        uint32_t* p = nullptr;
        VD_HIP(hipMalloc(&p, polys->size() * 4));
        VD_HIP(hipMemcpy(p, polys->data(), polys->size() * 4, hipMemcpyHostToDevice));
        per_dev[dev] = p;
    }
    *out = per_dev[dev];
    return VD_OK;
}
int mt_states(uint32_t seed, uint64_t T, uint32_t* st, uint32_t* xs, hipStream_t s)
{
    using namespace vd::mt;
    VD_HIP(hipMemsetAsync(st, 0, T * kN * 4, s));
    hipLaunchKernelGGL(mt_seed, dim3(1), dim3(64), 0, s, seed, st);
    VD_HIP(hipGetLastError());
    const int levels = mt_levels(T);
    if (!levels) return VD_OK;
    if (levels > kMtLevels) return fail(VD_ERR_ARG, "mt19937 stream longer than the jump tree");
    const uint32_t* polys_d = nullptr;  // level k's polynomials do not depend on the tree depth
    int rc = mt_polys_device(&polys_d);
    if (rc) return rc;
    uint64_t step = 1;
    for (int k = 0; k < levels; k++) step *= kMtR;  // R^levels
    for (int k = levels - 1; k >= 0; k--) {
        const uint64_t dstStep = step / kMtR, nsrc = (T + step - 1) / step;
        hipLaunchKernelGGL(mt_xseq, dim3((unsigned)nsrc), dim3(kThreads), 0, s, st, (uint32_t)step, xs);
        VD_HIP(hipGetLastError());
        // slice width: enough workgroups (>= ~4096) on narrow levels, 64 poly words at most
        const uint64_t jumps = nsrc * (kMtR - 1);
        int sw = (int)std::min<uint64_t>(kSliceWords, std::max<uint64_t>(4, jumps * kQW / 4096));
        const unsigned nsl = (unsigned)((kQW + sw - 1) / sw);
        hipLaunchKernelGGL(mt_jump, dim3((unsigned)nsrc, kMtR - 1, nsl), dim3(64), 0, s, xs,
                           polys_d + (size_t)k * (kMtR - 1) * kQW, (uint32_t)step, (uint32_t)dstStep, (uint32_t)T, sw, st);
        VD_HIP(hipGetLastError());
        step = dstStep;
    }
    return VD_OK;
}
struct DevBuf {  // stream-ordered scratch
    void* p = nullptr;
    hipStream_t s;
    explicit DevBuf(hipStream_t s_) : s(s_) {}
    hipError_t alloc(size_t n) { return hipMallocAsync(&p, n ? n : 4, s); }
    ~DevBuf() { if (p) (void)hipFreeAsync(p, s); }
};
}  // namespace

extern "C" {

int vd_channel_device(size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed, uint8_t* bits_d, float* values_d,
                      void* stream)
{
    using namespace vd::mt;
    if (!bits_d || !values_d) return fail(VD_ERR_ARG, "null argument");
    if (N == 0) return VD_OK;
    if (N > (1ull << 30)) return fail(VD_ERR_ARG, "N above 2^30 bits");
    hipStream_t s = (hipStream_t)stream;
    const float sigma = (float)std::pow(10, -snr / 5.0);  // AddNoise(pow(10, -snr/5.0)), main.cpp:135
    const uint64_t nval = 2 * (uint64_t)N;
    // message bits
    const uint64_t Tb = (N + kMtL - 1) / kMtL;
    const uint64_t attempts = std::isinf(sigma) ? 0 : (uint64_t)(1.30 * (double)N) + 4096;  // E = 4/pi N
    const uint64_t Tn = (2 * attempts + kMtL - 1) / kMtL;
    const uint64_t Tmax = std::max(Tb, Tn);
    const uint64_t nxs = (Tmax + kMtR - 1) / kMtR;
    DevBuf stb(s), stn(s), xs(s), cnt(s);
    VD_HIP(stb.alloc(Tb * kN * 4));
    VD_HIP(xs.alloc(nxs * kNX * 4));
    int rc = mt_states(bitSeed, Tb, (uint32_t*)stb.p, (uint32_t*)xs.p, s);
    if (rc) return rc;
    hipLaunchKernelGGL(mt_bits, dim3((unsigned)Tb), dim3(kThreads), 0, s, (const uint32_t*)stb.p, kMtL, (uint64_t)N, bits_d);
    VD_HIP(hipGetLastError());
    if (std::isinf(sigma)) {  // AddNoise's stddev = +inf branch (viterbiDF.h:79-85)
        hipLaunchKernelGGL(mt_add_base<false>, dim3((unsigned)((nval + 1023) / 1024)), dim3(256), 0, s,
                           (const uint8_t*)bits_d, nval, values_d);
        VD_HIP(hipGetLastError());
        return VD_OK;
    }
    VD_HIP(stn.alloc(Tn * kN * 4));
    VD_HIP(cnt.alloc((Tn + 1) * 4));
    rc = mt_states(noiseSeed, Tn, (uint32_t*)stn.p, (uint32_t*)xs.p, s);
    if (rc) return rc;
    uint32_t* counts = (uint32_t*)cnt.p;
    hipLaunchKernelGGL(mt_noise<0>, dim3((unsigned)Tn), dim3(kThreads), 0, s, (const uint32_t*)stn.p, kMtL, counts,
                       nval, sigma, values_d);
    VD_HIP(hipGetLastError());
    hipLaunchKernelGGL(scan_counts, dim3(1), dim3(1024), 0, s, counts, (uint32_t)Tn);
    VD_HIP(hipGetLastError());
    hipLaunchKernelGGL(mt_noise<1>, dim3((unsigned)Tn), dim3(kThreads), 0, s, (const uint32_t*)stn.p, kMtL, counts,
                       nval, sigma, values_d);
    VD_HIP(hipGetLastError());
    hipLaunchKernelGGL(mt_add_base<true>, dim3((unsigned)((nval + 1023) / 1024)), dim3(256), 0, s,
                       (const uint8_t*)bits_d, nval, values_d);
    VD_HIP(hipGetLastError());
    uint32_t total = 0;
    VD_HIP(hipMemcpyAsync(&total, counts + Tn, 4, hipMemcpyDeviceToHost, s));
    VD_HIP(hipStreamSynchronize(s));
    if (total < N) return fail(VD_ERR_DEVICE, "polar method: too few accepted pairs generated");
    return VD_OK;
}

int vd_simulate_device(int options, size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed, uint8_t* bits_d,
                       void* packed_d, void* stream)
{
    if (!valid(options)) return fail(VD_ERR_OPTIONS, "options disabled by OptionsValid");
    if (!packed_d || N % 16) return fail(VD_ERR_ARG, "null argument or N not a multiple of 16");
    hipStream_t s = (hipStream_t)stream;
    DevBuf bb(s), vb(s);
    if (!bits_d) {
        VD_HIP(bb.alloc(N));
        bits_d = (uint8_t*)bb.p;
    }
    VD_HIP(vb.alloc(2 * N * sizeof(float)));
    int rc = vd_channel_device(N, snr, bitSeed, noiseSeed, bits_d, (float*)vb.p, stream);
    if (rc) return rc;
    return launch_pack(options, (const float*)vb.p, 2 * N, 40000.0f, packed_d, s);  // SoftDecisionPacker(type, 40000)
}

}  // extern "C"

