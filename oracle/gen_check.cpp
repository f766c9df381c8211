// gen_check.cpp -- TEST INFRASTRUCTURE ONLY (oracle side).
// Draws from the C++ standard library generators the reference harness uses
// (std::mt19937 + uniform_int_distribution<int>(0,1), viterbiDF.h:20-33, and
// std::normal_distribution<float>, viterbiDF.h:66-95) so tests can pin the explicit
// restatement in vd_oracle.c against this container's libstdc++.
#include <random>
#include <cstdint>
#include <cstddef>
extern "C" void vo_std_bits(uint32_t seed, size_t n, uint8_t* bits) {
    std::mt19937 rng(seed);
    std::uniform_int_distribution<int> d(0, 1);
    for (size_t i = 0; i < n; i++) bits[i] = (uint8_t)d(rng);
}
extern "C" void vo_std_normals(uint32_t seed, float stddev, size_t n, float* out) {
    std::mt19937 rng(seed);
    std::normal_distribution<float> d(0.0f, stddev);
    for (size_t i = 0; i < n; i++) out[i] = d(rng);
}
