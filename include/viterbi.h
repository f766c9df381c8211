/*
 * viterbi.h -- header-only drop-in for the reference decoder class ViterbiCUDA<options>
 * (alireza-md93/GPU-Accelerated-Viterbi-Decoder, src/viterbi/viterbi.h:1-152), implemented over the
 * C-ABI in vd_capi.h (libvitdec.so: HIP kernels for MI355X / gfx950).
 *
 * Same option enums and bit layout (viterbi.h:7-20), same OptionsValid filter (:22-41), same
 * static constexpr members callers read (constLen, polyn1, polyn2, extraL, extraR, bitsPerPack,
 * encDataPerPack, ... :50-87), same types (encPack_t, decPack_t, metric_t), same constructors and
 * run()/getInputSize()/getMessageLen()/getOutputSize() (:126-134).  No CUDA/HIP types appear here:
 * metric_t for M_FP16 is an opaque 16-bit value (vd_half_t).
 *
 * Behaviour differences a caller can observe, all deliberate:
 *   - device buffers are reused across run() calls instead of allocated/freed per call, and the
 *     pre-allocating constructor really pre-allocates (the reference leaks, viterbi.cu:31-36);
 *   - the device is vd_create's `device` argument (VITDEC_DEVICE env, default 0) rather than a
 *     hard-coded 0 (viterbi.cu:134);
 *   - O_B16 output is race-free (each chunk writes only its own words; DESIGN.md "O_B16").
 * Errors keep the reference convention: message on stderr, then exit(EXIT_FAILURE)
 * (gpuerrors.h:8-17).
 */
#ifndef VITDEC_VITERBI_H
#define VITDEC_VITERBI_H

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "vd_capi.h"

constexpr int CHANNEL_SHIFT = 0;
constexpr int METRIC_SHIFT = 4;
constexpr int DECODE_SHIFT = 8;
constexpr int COMP_SHIFT = 12;
constexpr int CHANNEL_MASK = 0xf << CHANNEL_SHIFT;
constexpr int METRIC_MASK = 0xf << METRIC_SHIFT;
constexpr int DECODE_MASK = 0xf << DECODE_SHIFT;
constexpr int COMP_MASK = 0xf << COMP_SHIFT;

enum ChannelIn { HARD = 0x0, SOFT4 = 0x1, SOFT8 = 0x2, SOFT16 = 0x3, FP32 = 0x4 };
enum Metric { M_B32 = 0x00, M_B16 = 0x10, M_FP16 = 0x20 };
enum DecodeOut { O_B32 = 0x000, O_B16 = 0x100 };
enum CompMode { REG = 0x0000, DPX = 0x1000 };

/* opaque IEEE binary16 storage type standing in for CUDA's __half */
struct vd_half_t {
    uint16_t bits;
};

template <int options>
struct OptionsValid {
    static constexpr int ch = options & CHANNEL_MASK;
    static constexpr int me = options & METRIC_MASK;
    static constexpr int cm = options & COMP_MASK;
    static constexpr bool value = !((ch == SOFT8 && me == M_FP16) || (ch == SOFT16 && me == M_FP16) ||
                                    (ch == SOFT16 && me == M_B16) || (me == M_FP16 && cm == DPX));
};

template <int options = 0, bool enable = OptionsValid<options>::value>
class ViterbiCUDA;

/* constexpr description of an option combination (usable for disabled combinations too) */
template <int options>
class ViterbiCUDA<options, false> {
public:
    static constexpr ChannelIn inputType = static_cast<ChannelIn>(options & CHANNEL_MASK);
    static constexpr Metric metricType = static_cast<Metric>(options & METRIC_MASK);
    static constexpr DecodeOut outputType = static_cast<DecodeOut>(options & DECODE_MASK);
    static constexpr CompMode compMode = static_cast<CompMode>(options & COMP_MASK);

    using metric_t = std::conditional_t<metricType == M_B16, int16_t,
                     std::conditional_t<metricType == M_B32, int32_t, vd_half_t>>;
    using decPack_t = std::conditional_t<outputType == O_B16, uint16_t, uint32_t>;
    using encPack_t = std::conditional_t<inputType == FP32, float, int32_t>;

    static constexpr int constLen = 7;
    static constexpr int polyn1 = 0171;
    static constexpr int polyn2 = 0133;

    // both overloads of the reference (viterbi.h:65-66)
    static constexpr int roundup(int a, int b) { return a <= 0 ? 0 : (a + b - 1) / b * b; }
    static constexpr size_t roundup(size_t a, size_t b) { return a == 0 ? 0 : (a + b - 1) / b * b; }
    static constexpr int bitsPerMetric = metricType == M_B16 ? 16 : metricType == M_B32 ? 32 : 11;
    static constexpr int bitsPerPack = outputType == O_B16 ? 16 : 32;
    static constexpr int extraL_raw = 32;
    static constexpr int extraR_raw = 32;
    static constexpr int slideSize_raw = 32;
    static constexpr int extraL = roundup(extraL_raw, bitsPerPack) - (constLen - 1);
    static constexpr int extraR = roundup(extraR_raw, bitsPerPack) + (constLen - 1);
    static constexpr int slideSize = roundup(slideSize_raw, bitsPerPack);
    static constexpr int forwardLen = extraL + slideSize + extraR;
    static constexpr int bmMemWidth = 32;
    static constexpr int blockDimY = 2;
    static constexpr int FPprecision = 4;
    static constexpr int encDataPerPack = inputType == HARD ? 32 : inputType == SOFT4 ? 8
                                        : inputType == SOFT8 ? 4 : inputType == SOFT16 ? 2 : 1;
    static constexpr int encDataWidth = inputType == HARD ? 1 : inputType == SOFT4 ? 4
                                      : inputType == SOFT8 ? 8 : inputType == SOFT16 ? 16 : FPprecision;
};

template <int options>
class ViterbiCUDA<options, true> : public ViterbiCUDA<options, false> {
    using Base = ViterbiCUDA<options, false>;

public:
    using typename Base::decPack_t;
    using typename Base::encPack_t;
    using typename Base::metric_t;

    ViterbiCUDA() { create(0); }
    explicit ViterbiCUDA(size_t inputNum) { create(inputNum); }
    ~ViterbiCUDA() { vd_destroy(h_); }
    ViterbiCUDA(const ViterbiCUDA&) = delete;
    ViterbiCUDA& operator=(const ViterbiCUDA&) = delete;

    /* decode inputNum encoded values (viterbi.cu:210-238); kernelTime = decode-kernel ms */
    void run(encPack_t* input_h, decPack_t* output_h, size_t inputNum, float* kernelTime = nullptr)
    {
        check(vd_run(h_, input_h, output_h, inputNum, kernelTime), "run");
    }
    /* device-resident variant: pointers on this decoder's device, stream = hipStream_t or nullptr */
    void runDevice(const encPack_t* input_d, decPack_t* output_d, size_t inputNum, void* stream = nullptr)
    {
        check(vd_run_device(h_, input_d, output_d, inputNum, stream), "runDevice");
    }
    /* nbatch independent batches in one launch (strides in bytes; input stride 0 = the same input) */
    void runDeviceBatch(const encPack_t* input_d, size_t inputStride, decPack_t* output_d, size_t outputStride,
                        size_t inputNum, int nbatch, void* stream = nullptr)
    {
        check(vd_run_device_batch(h_, input_d, inputStride, output_d, outputStride, inputNum, nbatch, stream),
              "runDeviceBatch");
    }

    size_t getInputSize(size_t inputNum) { return vd_input_size(options, inputNum); }
    size_t getMessageLen(size_t inputNum) { return vd_message_len(options, inputNum); }
    size_t getOutputSize(size_t inputNum) { return vd_output_size(options, inputNum); }

private:
    vd_decoder* h_ = nullptr;

    static int device_from_env()
    {
        const char* e = std::getenv("VITDEC_DEVICE");
        return e ? std::atoi(e) : 0;
    }
    void create(size_t inputNum) { check(vd_create(options, inputNum, device_from_env(), &h_), "create"); }
    static void check(int rc, const char* what)
    {
        if (rc != VD_OK) {
            std::fprintf(stderr, "vitdec %s failed (%d): %s\n", what, rc, vd_last_error());
            std::exit(EXIT_FAILURE);
        }
    }
};

#endif /* VITDEC_VITERBI_H */
