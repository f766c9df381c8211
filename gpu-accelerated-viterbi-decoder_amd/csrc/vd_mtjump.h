// vd_mtjump.h -- jump-ahead for the reference harness's std::mt19937 streams (host side).
//
// The reference draws its message bits and its channel noise from two std::mt19937 engines
// (RandBitGen, AddNoise: src/viterbiDF.h:20-33,66-95, seeded src/main.cpp:131-137).  To generate
// those exact streams on the GPU, the output sequence is cut into segments of L outputs that are
// generated in parallel; the engine state at each segment start comes from the GF(2) jump-ahead
// x^(m L) mod P(x), P the characteristic polynomial of the mt19937 transition (degree 19937).
//
// State convention: a state is 624 raw (untempered) words x_n .. x_{n+623} of the sequence
// x_{k+624} = x_{k+397} ^ twist(x_k, x_{k+1}), with x_0 .. x_623 the seeded array; it is
// std::mt19937's internal array at index 624 after n outputs, and output n is temper(x_{n+624}).
// Jumping by a polynomial q(x) = sum q_i x^i: state'_j = XOR over i with q_i = 1 of x_{i+j}.
#pragma once
#include <cstdint>
#include <vector>

namespace vd {
namespace mtj {

constexpr int kN = 624;        // state words
constexpr int kMexp = 19937;   // degree of P
constexpr int kQW = 624;       // 32-bit words of a reduced polynomial (bits 0 .. 19936)
constexpr int kNX = 20592;     // raw words x_0 .. x_{kNX-1} a jump reads (33 blocks of 624 >= 19937 + 623)

// coefficient bits (kQW u32 words each) of x^(c * L * R^k) mod P, c = 1 .. R-1, k = 0 .. levels-1,
// stored [k][c-1][kQW]; computed once per (L, R, levels) and cached (thread-safe)
const std::vector<uint32_t>& jump_polys(uint64_t L, int R, int levels);

// seeded state (std::mt19937(seed) before its first output)
void seed_state(uint32_t seed, uint32_t st[kN]);
// the state after n more outputs (host jump, for tests and checks)
void jump_state(uint32_t st[kN], uint64_t n);
// next 624 outputs of a state, advancing it (tests)
void next_block(uint32_t st[kN], uint32_t out[kN]);

}  // namespace mtj
}  // namespace vd
