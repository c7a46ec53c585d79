// Exhaustive host check (CPU test infrastructure, tests/test_csa.py): the
// carry-save counter's threshold Csa<NL>::ge<K, TH> (ba_device.hpp, the
// majorities of ba.py:159-195 in bit-sliced form) equals popcount >= TH for
// every input pattern of K <= 16 inputs and every threshold.
#include "ba_device.hpp"
#include <cstdio>
using namespace ba;
template <int K, int NL>
int check() {
    int bad = 0;
    for (uint32_t m = 0; m < (1u << K); ++m) {
        Csa<NL, uint32_t> c;
        static_for_h<0, K>([&](auto i) { c.template add<i()>((m >> i()) & 1u ? 1u : 0u); });
        const int pc = __builtin_popcount(m);
        static_for_h<0, K + 2>([&](auto th) {
            const uint32_t g = c.template ge<K, th()>() & 1u;
            if (g != (pc >= th() ? 1u : 0u)) ++bad;
        });
    }
    return bad;
}
int main() {
    int bad = 0;
    bad += check<1, 1>(); bad += check<2, 2>(); bad += check<3, 2>(); bad += check<4, 3>();
    bad += check<5, 3>(); bad += check<6, 3>(); bad += check<7, 3>(); bad += check<8, 4>();
    bad += check<9, 4>(); bad += check<10, 4>(); bad += check<11, 4>(); bad += check<12, 4>();
    bad += check<13, 4>(); bad += check<14, 4>(); bad += check<15, 4>(); bad += check<16, 5>();
    printf("bad=%d\n", bad);
    return bad != 0;
}
