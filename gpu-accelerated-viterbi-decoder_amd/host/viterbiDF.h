// viterbiDF.h -- simulation elements around the decoder (host side).
// Interface-compatible with the reference's src/viterbiDF.h:20-209 (RandBitGen, ConvolutionalEncoder,
// AddNoise, SoftDecisionPacker, ViterbiDecoder<options>) with identical numerics (std::mt19937 +
// uniform_int_distribution<int>(0,1) bits, std::normal_distribution<float> noise, lrintf quantiser,
// MSB-first packing), so a given seed pair reproduces the reference's BER.  The decoder element
// calls the MI355X decode through include/viterbi.h -> vd_capi.h.
#pragma once

#include <cmath>
#include <cstdint>
#include <iomanip>
#include <limits>
#include <random>
#include <sstream>
#include <vector>

#include "dataflow.h"
#include "viterbi.h"

enum class Bit : uint8_t { OFF = 0, ON = 1 };
using Bits = std::vector<Bit>;
using soft_t = int32_t;
using Soft = std::vector<soft_t>;
using Reals = std::vector<float>;

class RandBitGen : public ComputeElement {
public:
    RandBitGen(size_t n, unsigned seed = 0) : n_(n), rng_(seed) {}
    std::any process(const OptData&) override
    {
        std::uniform_int_distribution<int> coin(0, 1);
        Bits b(n_);
        for (auto& x : b) x = coin(rng_) ? Bit::ON : Bit::OFF;
        return b;
    }

private:
    size_t n_;
    std::mt19937 rng_;
};

// rate-1/2 feed-forward encoder; out0 from p0 first (reference viterbiDF.h:36-63)
class ConvolutionalEncoder : public ComputeElement {
public:
    ConvolutionalEncoder(int constLen, uint32_t p0, uint32_t p1) : k_(constLen), p0_(p0), p1_(p1) {}
    std::any process(const OptData& in) override
    {
        if (!in) throw std::runtime_error("ConvolutionalEncoder expects input bits");
        const Bits& src = std::any_cast<const Bits&>(*in);
        Bits out(2 * src.size());
        uint32_t reg = 0;
        for (size_t i = 0; i < src.size(); i++) {
            reg = (reg >> 1) | ((uint32_t)(src[i] == Bit::ON) << (k_ - 1));
            out[2 * i] = __builtin_parity(reg & p0_) ? Bit::ON : Bit::OFF;
            out[2 * i + 1] = __builtin_parity(reg & p1_) ? Bit::ON : Bit::OFF;
        }
        return out;
    }

private:
    int k_;
    uint32_t p0_, p1_;
};

// BPSK (+1 for a one) plus N(0, stddev^2); stddev = +inf means noiseless (viterbiDF.h:66-95)
class AddNoise : public ComputeElement {
public:
    AddNoise(float stddev = std::numeric_limits<float>::infinity(), unsigned seed = 0) : sd_(stddev), seed_(seed) {}
    std::any process(const OptData& in) override
    {
        if (!in) throw std::runtime_error("AddNoise expects input bits");
        const Bits& src = std::any_cast<const Bits&>(*in);
        Reals out(src.size());
        const bool noiseless = sd_ == std::numeric_limits<float>::infinity();
        std::mt19937 rng(seed_);
        std::normal_distribution<float> gauss(0.0f, sd_);
        for (size_t i = 0; i < src.size(); i++) {
            const float s = src[i] == Bit::ON ? 1.0f : -1.0f;
            out[i] = noiseless ? s : s + gauss(rng);
        }
        return out;
    }

private:
    float sd_;
    unsigned seed_;
};

// quantise-and-pack into int32 words, first value in the most significant field (viterbiDF.h:98-167)
class SoftDecisionPacker : public ComputeElement {
public:
    SoftDecisionPacker(ChannelIn cfg, float scale = 1.0f) : cfg_(cfg), scale_(scale) {}
    std::any process(const OptData& in) override
    {
        if (!in) throw std::runtime_error("SoftDecisionPacker expects input reals");
        const Reals& src = std::any_cast<const Reals&>(*in);
        if (cfg_ == FP32) {
            Reals out(src.size());
            for (size_t i = 0; i < src.size(); i++) out[i] = scale_ == 1.0f ? src[i] : src[i] * scale_;
            return out;
        }
        const int width = cfg_ == HARD ? 1 : cfg_ == SOFT4 ? 4 : cfg_ == SOFT8 ? 8 : 16;
        const int per = 32 / width;
        Soft out(src.size() / per);
        for (size_t w = 0; w < out.size(); w++) {
            uint32_t acc = 0;
            for (int j = 0; j < per; j++) acc = (acc << width) | quant(src[w * per + j] * scale_);
            out[w] = (soft_t)acc;
        }
        return out;
    }

private:
    ChannelIn cfg_;
    float scale_;
    uint32_t quant(float v) const
    {
        if (cfg_ == HARD) return v > 0.0f ? 1u : 0u;
        const long lo = cfg_ == SOFT4 ? -8 : cfg_ == SOFT8 ? -128 : -32768;
        const long hi = -lo - 1;
        const uint32_t mask = cfg_ == SOFT4 ? 0xFu : cfg_ == SOFT8 ? 0xFFu : 0xFFFFu;
        // SOFT4/SOFT8 narrow lrintf's long to int BEFORE saturating, SOFT16 saturates the long
        // (reference viterbiDF.h:108,114 vs :120): |v| >= 2^31 quantises differently
        long q = std::lrintf(v);
        if (cfg_ != SOFT16) q = (long)(int)q;
        q = q < lo ? lo : (q > hi ? hi : q);
        return (uint32_t)q & mask;
    }
};

template <int options>
struct ViterbiDecoder : ComputeElement {
    using Dec = ViterbiCUDA<options>;
    using decPack_t = typename Dec::decPack_t;
    using decVec_t = std::vector<decPack_t>;
    using encPack_t = typename Dec::encPack_t;
    static constexpr int bitsPerPack = Dec::bitsPerPack;
    static constexpr int encDataPerPack = Dec::encDataPerPack;

    ViterbiDecoder() : dec_(new Dec()) {}
    ViterbiDecoder(int inputNum) : dec_(new Dec((size_t)inputNum)) {}

    std::any process(const OptData& in) override
    {
        if (!in) throw std::runtime_error("ViterbiDecoder expects packed input");
        std::vector<encPack_t> enc = std::any_cast<std::vector<encPack_t>>(*in);
        const size_t n = enc.size() * encDataPerPack;
        decVec_t out(dec_->getOutputSize(n) / sizeof(decPack_t));
        float ms = 0.0f;
        dec_->run(enc.data(), out.data(), n, &ms);
        setStatus("GPU kernel time", ms);
        return out;
    }
    std::string getStatusString(const std::string& key) const override
    {
        if (key != "GPU kernel time") return ComputeElement::getStatusString(key);
        const float ms = std::any_cast<float>(getStatus(key));
        std::ostringstream os;
        os << std::fixed << std::setprecision(3);
        if (ms < 1.0f) os << ms * 1000.0f << " us";
        else if (ms < 1000.0f) os << ms << " ms";
        else os << ms / 1000.0f << " s";
        return os.str();
    }

private:
    std::unique_ptr<Dec> dec_;
};
