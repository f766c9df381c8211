// vd_mtjump.cpp -- GF(2) polynomial arithmetic for mt19937 jump-ahead (see vd_mtjump.h).
//
// P(x) comes from Berlekamp-Massey on 2 * 19937 output bits of the engine (the transition is linear
// over GF(2) and P is irreducible of degree 19937, so the minimal polynomial of any output-bit
// sequence is P itself).  Polynomials are bit vectors, bit i = coefficient of x^i.
#include "vd_mtjump.h"

#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <tuple>

namespace vd {
namespace mtj {
namespace {

constexpr int W = (kMexp + 64) / 64;  // 312 u64 words hold degrees 0 .. 19967 (P has degree 19937)
using Poly = std::vector<uint64_t>;

inline uint32_t temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    return y ^ (y >> 18);
}
// one twist of a std::mt19937 array (the raw sequence advances by 624 words)
void twist(uint32_t* mt)
{
    for (int i = 0; i < kN; i++) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % kN] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
}

inline int getbit(const Poly& a, size_t i) { return (int)((a[i >> 6] >> (i & 63)) & 1u); }
inline void flipbit(Poly& a, size_t i) { a[i >> 6] ^= 1ull << (i & 63); }

// P(x) by Berlekamp-Massey over the low bit of the outputs of std::mt19937(5489)
Poly make_charpoly()
{
    const size_t n = 2 * (size_t)kMexp;
    const size_t nw = n / 64 + 2;
    Poly R(nw + 1, 0);  // reversed sequence: R bit t = s[n-1-t]
    {
        uint32_t st[kN], out[kN];
        seed_state(5489u, st);
        size_t k = 0;
        while (k < n) {
            next_block(st, out);
            for (int i = 0; i < kN && k < n; i++, k++)
                if (out[i] & 1u) flipbit(R, n - 1 - k);
        }
    }
    auto window = [&](size_t off, size_t w) -> uint64_t {  // bits off + 64w .. +63 of R
        const size_t b = off + 64 * w, q = b >> 6, r = b & 63;
        uint64_t v = q < R.size() ? R[q] >> r : 0;
        if (r && q + 1 < R.size()) v |= R[q + 1] << (64 - r);
        return v;
    };
    Poly C(nw, 0), B(nw, 0), T;
    C[0] = B[0] = 1;
    size_t L = 0, m = 1;
    for (size_t N = 0; N < n; N++) {
        // discrepancy s[N] + sum_{i=1..L} c_i s[N-i] = parity of C & (R >> (n-1-N)) over bits 0..L
        const size_t off = n - 1 - N;
        uint64_t acc = 0;
        for (size_t w = 0; w <= L / 64; w++) acc ^= C[w] & window(off, w);
        if (!(__builtin_popcountll(acc) & 1)) {
            m++;
            continue;
        }
        const size_t ws = m >> 6, bs = m & 63, top = (L + m) / 64 + 2;
        if (2 * L <= N) T = C;
        for (size_t w = 0; w + ws < nw && w < top; w++) {  // C ^= B << m
            C[w + ws] ^= B[w] << bs;
            if (bs && w + ws + 1 < nw) C[w + ws + 1] ^= B[w] >> (64 - bs);
        }
        if (2 * L <= N) {
            L = N + 1 - L;
            B = T;
            m = 1;
        } else {
            m++;
        }
    }
    if (L != (size_t)kMexp) throw std::runtime_error("mt19937 characteristic polynomial: unexpected degree");
    Poly P(W, 0);  // P(x) = x^L C(1/x)
    for (size_t k = 0; k <= L; k++)
        if (getbit(C, L - k)) flipbit(P, k);
    return P;
}

const Poly& charpoly()
{
    static Poly P;
    static std::once_flag once;
    std::call_once(once, [] { P = make_charpoly(); });
    return P;
}

// r (2W words, degree < 2 * kMexp) mod P, in place; returns the low W words
Poly reduce(Poly r)
{
    const Poly& P = charpoly();
    for (size_t d = 2 * W * 64 - 1; d >= (size_t)kMexp; d--) {
        if (!getbit(r, d)) continue;
        const size_t s = d - kMexp, ws = s >> 6, bs = s & 63;
        for (int i = 0; i < W; i++) {
            r[ws + i] ^= P[i] << bs;
            if (bs && ws + i + 1 < r.size()) r[ws + i + 1] ^= P[i] >> (64 - bs);
        }
    }
    r.resize(W);
    return r;
}
Poly sqrmod(const Poly& a)
{
    static uint16_t spread[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int b = 0; b < 256; b++) {
            uint16_t v = 0;
            for (int i = 0; i < 8; i++) v |= (uint16_t)(((b >> i) & 1) << (2 * i));
            spread[b] = v;
        }
    });
    Poly r(2 * W, 0);
    for (int w = 0; w < W; w++) {
        const uint64_t x = a[w];
        uint64_t lo = 0, hi = 0;
        for (int k = 0; k < 4; k++) {
            lo |= (uint64_t)spread[(x >> (8 * k)) & 0xFF] << (16 * k);
            hi |= (uint64_t)spread[(x >> (32 + 8 * k)) & 0xFF] << (16 * k);
        }
        r[2 * w] = lo;
        r[2 * w + 1] = hi;
    }
    return reduce(std::move(r));
}
Poly mulmod(const Poly& a, const Poly& b)
{
    Poly r(2 * W, 0);
    for (size_t i = 0; i < (size_t)W * 64; i++) {
        if (!getbit(a, i)) continue;
        const size_t ws = i >> 6, bs = i & 63;
        for (int w = 0; w < W; w++) {
            r[ws + w] ^= b[w] << bs;
            if (bs) r[ws + w + 1] ^= b[w] >> (64 - bs);
        }
    }
    return reduce(std::move(r));
}
// x * a mod P
Poly mulx(const Poly& a)
{
    Poly r(W, 0);
    for (int w = W - 1; w >= 0; w--) r[w] = (a[w] << 1) | (w ? a[w - 1] >> 63 : 0);
    if (getbit(r, kMexp)) {
        const Poly& P = charpoly();
        for (int w = 0; w < W; w++) r[w] ^= P[w];
    }
    return r;
}
// x^n mod P
Poly xpow(uint64_t n)
{
    Poly t(W, 0);
    t[0] = 1;
    for (int b = 63; b >= 0; b--) {
        t = sqrmod(t);
        if ((n >> b) & 1u) t = mulx(t);
    }
    return t;
}
void to_words(const Poly& p, uint32_t* q)
{
    for (int i = 0; i < kQW; i++) q[i] = (uint32_t)(p[i / 2] >> (32 * (i % 2)));
}
// state' = q(A) state: the XOR of the windows x_{i .. i+623} over the set coefficients q_i
void apply(uint32_t st[kN], const uint32_t* q)
{
    std::vector<uint32_t> x(kNX);
    uint32_t mt[kN];
    std::memcpy(mt, st, sizeof mt);
    for (int b = 0; b * kN < kNX; b++) {
        std::memcpy(&x[(size_t)b * kN], mt, sizeof mt);
        twist(mt);
    }
    uint32_t r[kN] = {0};
    for (int i = 0; i < kMexp; i++)
        if ((q[i >> 5] >> (i & 31)) & 1u)
            for (int j = 0; j < kN; j++) r[j] ^= x[(size_t)i + j];
    std::memcpy(st, r, sizeof r);
}

}  // namespace

void seed_state(uint32_t seed, uint32_t st[kN])
{
    st[0] = seed;
    for (int i = 1; i < kN; i++) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
}
void next_block(uint32_t st[kN], uint32_t out[kN])
{
    twist(st);
    for (int i = 0; i < kN; i++) out[i] = temper(st[i]);
}
void jump_state(uint32_t st[kN], uint64_t n)
{
    std::vector<uint32_t> q(kQW);
    to_words(xpow(n), q.data());
    apply(st, q.data());
}

const std::vector<uint32_t>& jump_polys(uint64_t L, int R, int levels)
{
    static std::mutex mu;
    static std::map<std::tuple<uint64_t, int, int>, std::vector<uint32_t>> cache;
    if (R < 2 || (R & (R - 1)) || levels < 0) throw std::invalid_argument("jump_polys: R must be a power of two");
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(L, R, levels);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    std::vector<uint32_t> out((size_t)levels * (R - 1) * kQW);
    Poly D = xpow(L);  // x^(L R^k)
    for (int k = 0; k < levels; k++) {
        if (k > 0)
            for (int c = 1; c < R; c <<= 1) D = sqrmod(D);  // D^R, R a power of two
        std::vector<Poly> Q(R);
        Q[1] = D;
        for (int c = 2; c < R; c++) Q[c] = (c % 2 == 0) ? sqrmod(Q[c / 2]) : mulmod(Q[c - 1], D);
        for (int c = 1; c < R; c++) to_words(Q[c], &out[((size_t)k * (R - 1) + (c - 1)) * kQW]);
    }
    return cache.emplace(key, std::move(out)).first->second;
}

}  // namespace mtj
}  // namespace vd

// C-ABI test hook (declared in include/vd_capi.h): the engine state after n outputs, host jump-ahead
extern "C" int vd_mt_state_after(uint32_t seed, uint64_t n, uint32_t* state624)
{
    if (!state624) return -1;
    try {
        vd::mtj::seed_state(seed, state624);
        if (n) vd::mtj::jump_state(state624, n);
    } catch (...) {
        return -2;
    }
    return 0;
}
