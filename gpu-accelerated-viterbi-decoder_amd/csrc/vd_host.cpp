// vd_host.cpp -- host-side harness entry points of the C-ABI (product side).
//
// vd_simulate_host runs the reference's simulation chain with the C++ standard library generators
// the reference uses (RandBitGen, ConvolutionalEncoder, AddNoise, SoftDecisionPacker:
// src/viterbiDF.h:20-167, seeded as in src/main.cpp:131-137), streaming so a 32M-bit message needs
// no 256 MB float staging vector.  vd_count_errors is the BER loop of src/main.cpp:151-171.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>

#include "../../include/vd_capi.h"

namespace {
constexpr int kExtraL = 26;  // roundup(32, bpp) - (K-1) (viterbi.h:73)

inline uint32_t parity(uint32_t v) { return (uint32_t)__builtin_popcount(v) & 1u; }

inline uint32_t quant(int ch, float v)
{
    switch (ch) {
    case 0: return v > 0.0f ? 1u : 0u;
    case 1: { int q = (int)std::lrintf(v); if (q < -8) q = -8; if (q > 7) q = 7; return (uint32_t)q & 0xFu; }
    case 2: { int q = (int)std::lrintf(v); if (q < -128) q = -128; if (q > 127) q = 127; return (uint32_t)q & 0xFFu; }
    case 3: { long q = std::lrintf(v); if (q < -32768) q = -32768; if (q > 32767) q = 32767; return (uint32_t)q & 0xFFFFu; }
    }
    return 0;
}
}  // namespace

extern "C" int vd_simulate_host(int options, size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed,
                                uint8_t* bits, void* packed)
{
    if (!vd_options_valid(options) || !bits || !packed || N % 16) return VD_ERR_ARG;
    const int ch = options & 0xF;
    std::mt19937 rb(bitSeed);
    std::uniform_int_distribution<int> ud(0, 1);
    for (size_t i = 0; i < N; i++) bits[i] = ud(rb) ? 1 : 0;

    const float stddev = (float)std::pow(10, -snr / 5.0);
    std::mt19937 rn(noiseSeed);
    std::normal_distribution<float> nd(0.0f, stddev);
    const float scale = 40000.0f;
    int packLen = 0, per = 0;
    switch (ch) {
    case 0: packLen = 1; per = 32; break;
    case 1: packLen = 4; per = 8; break;
    case 2: packLen = 8; per = 4; break;
    case 3: packLen = 16; per = 2; break;
    default: break;
    }
    uint32_t buf = 0, acc = 0;
    int nacc = 0;
    size_t wi = 0;
    uint32_t* pw = (uint32_t*)packed;
    float* pf = (float*)packed;
    for (size_t i = 0; i < N; i++) {
        buf >>= 1;
        buf |= (uint32_t)bits[i] << 6;
        const uint32_t o[2] = {parity(buf & 0171u), parity(buf & 0133u)};
        for (int j = 0; j < 2; j++) {
            float base = o[j] ? 1.0f : -1.0f;
            float v = base + nd(rn);
            if (ch == 4) { pf[2 * i + j] = v * scale; continue; }
            acc = (acc << packLen) | quant(ch, v * scale);
            if (++nacc == per) { pw[wi++] = acc; acc = 0; nacc = 0; }
        }
    }
    return VD_OK;
}

extern "C" long long vd_count_errors(int options, const uint8_t* bits, size_t N, const void* decoded, size_t decodedBytes)
{
    const int bpp = ((options >> 8) & 0xF) == 1 ? 16 : 32;
    const size_t nbits = decodedBytes * 8;
    long long ben = 0;
    for (size_t i = 0; i < nbits; i++) {
        int b;
        if (bpp == 32) b = (int)((((const uint32_t*)decoded)[i / 32] >> (31 - i % 32)) & 1u);
        else b = (int)((((const uint16_t*)decoded)[i / 16] >> (15 - i % 16)) & 1u);
        if (i + kExtraL >= N || b != bits[i + kExtraL]) ben++;
    }
    return ben;
}
