// Host check of the carry-save column counter (ba_device.hpp Csa) against
// popcount: for every input count K <= 16 and threshold T, ge<K, T>() must
// select exactly the lanes whose count of set inputs is >= T.  Built with
// hipcc as host code by tests/test_lib.py (no device needed).
#include <cstdio>
#include <random>

#include "../../byzantine-agreement_amd/csrc/ba_device.hpp"

using namespace ba;

template <int B, int E, typename F>
void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

template <int K>
int check(std::mt19937_64& rng) {
    constexpr int NL = K < 2 ? 1 : (K < 4 ? 2 : (K < 8 ? 3 : (K < 16 ? 4 : 5)));
    int bad = 0;
    for (int rep = 0; rep < 200; ++rep) {
        uint64_t x[K + 1];
        for (int i = 0; i < K; ++i) x[i] = rng() & rng();  // vary the density
        if (rep & 1)
            for (int i = 0; i < K; ++i) x[i] |= rng();
        Csa<NL> c;
        sfor<0, K>([&](auto i) { c.template add<i()>(x[i()]); });
        sfor<0, K + 2>([&](auto t) {
            const uint64_t got = c.template ge<K, t()>();
            uint64_t want = 0;
            for (int lane = 0; lane < 64; ++lane) {
                int cnt = 0;
                for (int i = 0; i < K; ++i) cnt += (x[i] >> lane) & 1;
                if (cnt >= t()) want |= 1ull << lane;
            }
            if (got != want) {
                ++bad;
                if (bad < 5) printf("K=%d T=%d mismatch\n", K, t());
            }
        });
    }
    return bad;
}

int main() {
    std::mt19937_64 rng(12345);
    int bad = 0;
    sfor<1, 17>([&](auto k) { bad += check<k()>(rng); });
    printf("csa_check %s (%d mismatches)\n", bad ? "FAILED" : "ok", bad);
    return bad ? 1 : 0;
}
