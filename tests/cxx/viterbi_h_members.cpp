// Compile-time check of include/viterbi.h against the reference's own uses of ViterbiCUDA<options>'s
// static members and types (src/main.cpp:121-128,137; src/viterbiDF.h:176-180) and the constants of
// src/viterbi/viterbi.h:50-87, for every valid option.  Built with g++ by tests/test_cli.py; nothing runs.
#include <cstdint>
#include <type_traits>
#include "viterbi.h"

template <int options>
constexpr bool check()
{
    using V = ViterbiCUDA<options>;
    // main.cpp:121-128,137
    static_assert(V::constLen == 7 && V::polyn1 == 0171 && V::polyn2 == 0133);
    static_assert(V::extraL == V::roundup(32, V::bitsPerPack) - 6 && V::extraR == V::roundup(32, V::bitsPerPack) + 6);
    static_assert(V::inputType == static_cast<ChannelIn>(options & 0xF));
    // viterbiDF.h:176-180
    static_assert(std::is_same_v<typename V::decPack_t, std::conditional_t<(options & 0xF00) == 0x100, uint16_t, uint32_t>>);
    static_assert(std::is_same_v<typename V::encPack_t, std::conditional_t<(options & 0xF) == 4, float, int32_t>>);
    static_assert(V::bitsPerPack == ((options & 0xF00) == 0x100 ? 16 : 32));
    static_assert(V::encDataPerPack * V::encDataWidth == 32 || (options & 0xF) == 4);
    // both roundup overloads (viterbi.h:65-66), as constant expressions
    static_assert(V::roundup(33, 32) == 64 && V::roundup(0, 16) == 0 && V::roundup(-5, 16) == 0);
    static_assert(V::roundup(size_t(33), size_t(32)) == size_t(64) && V::roundup(size_t(0), size_t(8)) == 0);
    static_assert(std::is_same_v<decltype(V::roundup(size_t(1), size_t(1))), size_t>);
    static_assert(V::forwardLen == V::extraL + V::slideSize + V::extraR && V::slideSize == V::roundup(32, V::bitsPerPack));
    return true;
}

#define CH(o) (check<(o)>() && check<(o) | 0x100>())
static_assert(CH(0x00) && CH(0x10) && CH(0x20) && CH(0x01) && CH(0x11) && CH(0x21) && CH(0x02) && CH(0x12));
static_assert(CH(0x03) && CH(0x04) && CH(0x14) && CH(0x24) && CH(0x1000) && CH(0x1012));
static_assert(!OptionsValid<0x22>::value && !OptionsValid<0x13>::value && !OptionsValid<0x1020>::value);

int main() { return 0; }
