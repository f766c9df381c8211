// main.cpp -- reference-compatible CLI: random bits -> K=7 R=1/2 encoder -> BPSK+AWGN -> quantiser
// -> MI355X Viterbi decode -> bit-error count.  Same flags and output line as the reference's
// src/main.cpp:174-264 (-n -s -i -m -o -c -v -h; "Final results -> BEN: x   BER: y"), plus
//   --seed B,N   fix the bit and noise seeds (the reference draws both from std::random_device)
//   --device D   HIP device (also VITDEC_DEVICE)
#include <cstdlib>
#include <iostream>
#include <random>
#include <string>

#include "viterbiDF.h"

namespace {

struct Args {
    int messageLen = 32000000;
    float snr = 15.0f;
    int options = 0;
    bool verbose = false;
    bool seeded = false;
    unsigned bitSeed = 0, noiseSeed = 0;
};

[[noreturn]] void usage_exit(const char* prog, int code)
{
    std::cout << "Usage: " << prog << " [options]\n"
              << "Options:\n"
              << "  -n, --num <integer>      Set the message length.\n"
              << "  -s, --snr <float>        Set the Signal-to-Noise Ratio (SNR).\n"
              << "  -i, --input <type>       Set the input channel type (HARD|h, SOFT4|s4, SOFT8|s8, SOFT16|s16, FP32|f).\n"
              << "  -m, --metric <type>      Set the metric type (b16, b32, f16).\n"
              << "  -o, --output <type>      Set the output type (b16, b32).\n"
              << "  -c, --compMode <type>    Set the computation mode (REG|reg, DPX|dpx).\n"
              << "  -v, --verbose            Enable verbose output.\n"
              << "      --seed <b>,<n>       Fix the bit and noise seeds.\n"
              << "      --device <d>         HIP device index.\n"
              << "  -h, --help               Display this help message.\n";
    std::exit(code);
}

[[noreturn]] void bad(const std::string& msg)
{
    std::cerr << "Error: " << msg << std::endl;
    std::exit(1);
}

Args parse(int argc, char** argv)
{
    Args a;
    for (int i = 1; i < argc; i++) {
        const std::string s = argv[i];
        const bool hasv = i + 1 < argc;
        auto val = [&]() { return std::string(argv[++i]); };
        if (s == "-h" || s == "--help") usage_exit(argv[0], 0);
        else if ((s == "-n" || s == "--num") && hasv) {
            try { a.messageLen = std::stoi(val()); } catch (...) { bad("Invalid argument for " + s + ". Please provide an integer."); }
        } else if ((s == "-s" || s == "--snr") && hasv) {
            try { a.snr = std::stof(val()); } catch (...) { bad("Invalid argument for " + s + ". Please provide a float."); }
        } else if ((s == "-m" || s == "--metric") && hasv) {
            const std::string v = val();
            if (v == "b16") a.options |= M_B16;
            else if (v == "b32") a.options |= M_B32;
            else if (v == "f16") a.options |= M_FP16;
            else bad("Invalid metric type for " + s + ".");
        } else if ((s == "-i" || s == "--input") && hasv) {
            const std::string v = val();
            if (v == "HARD" || v == "h") a.options |= HARD;
            else if (v == "SOFT4" || v == "s4") a.options |= SOFT4;
            else if (v == "SOFT8" || v == "s8") a.options |= SOFT8;
            else if (v == "SOFT16" || v == "s16") a.options |= SOFT16;
            else if (v == "FP32" || v == "f") a.options |= FP32;
            else bad("Invalid input channel type for " + s + ".");
        } else if ((s == "-o" || s == "--output") && hasv) {
            const std::string v = val();
            if (v == "b16") a.options |= O_B16;
            else if (v == "b32") a.options |= O_B32;
            else bad("Invalid output type for " + s + ".");
        } else if ((s == "-c" || s == "--compMode") && hasv) {
            const std::string v = val();
            if (v == "REG" || v == "reg") a.options |= REG;
            else if (v == "DPX" || v == "dpx") a.options |= DPX;
            else bad("Invalid computation mode for " + s + ".");
        } else if (s == "--seed" && hasv) {
            const std::string v = val();
            const size_t c = v.find(',');
            if (c == std::string::npos) bad("--seed expects <bits>,<noise>");
            a.bitSeed = (unsigned)std::stoul(v.substr(0, c));
            a.noiseSeed = (unsigned)std::stoul(v.substr(c + 1));
            a.seeded = true;
        } else if (s == "--device" && hasv) {
            setenv("VITDEC_DEVICE", val().c_str(), 1);
        } else if (s == "-v" || s == "--verbose") {
            a.verbose = true;
        } else {
            bad("Unknown or incomplete argument: " + s);
        }
    }
    return a;
}

template <int options>
long long runPipeline(const Args& a)
{
    using V = ViterbiCUDA<options>;
    std::random_device rd;
    const unsigned bitSeed = a.seeded ? a.bitSeed : rd();
    const unsigned noiseSeed = a.seeded ? a.noiseSeed : rd();
    RandBitGen src((size_t)a.messageLen, bitSeed);
    ConvolutionalEncoder enc(V::constLen, V::polyn1, V::polyn2);
    AddNoise noise((float)std::pow(10, -a.snr / 5.0), noiseSeed);
    SoftDecisionPacker pack(V::inputType, 40000.0f);
    ViterbiDecoder<options> dec;

    Pipeline pipe = src.probe() | enc | noise | pack | dec;
    PipelineResult res = pipe.run();
    if (a.verbose) {
        std::cout << std::endl;
        pipe.printStatus();
        std::cout << std::endl;
    }
    using decVec_t = typename ViterbiDecoder<options>::decVec_t;
    const decVec_t& out = std::any_cast<const decVec_t&>(res.final_output);
    const Bits& bits = std::any_cast<const Bits&>(res.probed_outputs[0]);
    constexpr int bpp = V::bitsPerPack;
    long long ben = 0;
    for (size_t i = 0; i < out.size() * bpp; i++) {
        const bool d = (out[i / bpp] >> (bpp - 1 - i % bpp)) & 1u;
        const bool g = bits[i + V::extraL] == Bit::ON;
        ben += d != g;
    }
    return ben;
}

// runtime options -> template instantiation (the 42 valid combinations)
template <int I>
long long dispatch(const Args& a)
{
    if constexpr (I < 0x2000) {
        if constexpr ((I & 0xF) <= FP32 && ((I >> 4) & 0xF) <= 2 && ((I >> 8) & 0xF) <= 1 && OptionsValid<I>::value) {
            if (a.options == I) return runPipeline<I>(a);
        }
        constexpr int next = (I & 0xF) < FP32 ? I + 1
                           : ((I >> 4) & 0xF) < 2 ? (I & ~0xF) + 0x10
                           : ((I >> 8) & 0xF) < 1 ? (I & ~0xFF) + 0x100
                           : (I & ~0xFFF) + 0x1000;
        return dispatch<next>(a);
    } else {
        return -1;
    }
}

}  // namespace

int main(int argc, char** argv)
{
    const Args a = parse(argc, argv);
    const int ch = a.options & CHANNEL_MASK, me = a.options & METRIC_MASK, cm = a.options & COMP_MASK;
    if (me == M_B16 && ch == SOFT16) { std::cerr << "Error: 16-bit metric does not support 16-bit soft decision input." << std::endl; return -1; }
    if (me == M_FP16 && ch == SOFT16) { std::cerr << "Error: fp16 metric does not support 16-bit soft decision input." << std::endl; return -1; }
    if (me == M_FP16 && ch == SOFT8) { std::cerr << "Error: fp16 metric does not support 8-bit soft decision input." << std::endl; return -1; }
    if (me == M_FP16 && cm == DPX) { std::cerr << "Error: fp16 metric does not support DPX computation mode." << std::endl; return -1; }

    if (a.verbose) {
        static const char* in_names[] = {"Hard Decision", "4-bit Soft Decision", "8-bit Soft Decision",
                                         "16-bit Soft Decision", "32-bit Floating Point"};
        std::cout << "Message Length: " << a.messageLen << std::endl;
        std::cout << "SNR: " << a.snr << " dB" << std::endl;
        std::cout << "Input Channel Type: " << (ch <= FP32 ? in_names[ch] : "Unknown Type") << std::endl;
        std::cout << "Metric Type: " << (me == M_B16 ? "16-bit" : me == M_B32 ? "32-bit" : "FP16") << std::endl;
        std::cout << "Output Type: " << ((a.options & DECODE_MASK) == O_B16 ? "16-bit" : "32-bit") << std::endl;
        std::cout << "Computation Mode: " << (cm == REG ? "Regular" : "DPX") << std::endl << std::endl;
    }
    const long long ben = dispatch<0>(a);
    if (ben < 0) { std::cerr << "Error: unsupported option combination." << std::endl; return -1; }
    std::cout << "Pipeline executed." << std::endl;
    std::cout << "Final results -> BEN: " << ben << "   BER: " << (double)ben / a.messageLen << std::endl;
    return 0;
}
