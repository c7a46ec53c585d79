// ba_mt.cpp -- ba.py's coin source, replayed in C++ (host only, no device).
//
// ba.py draws every lie from CPython's global Mersenne Twister:
// random.randint(0, 1) == 0 -> "attack" (ba.py:45 relay, ba.py:269 commander).
// randint(0, 1) is _randbelow(2): take the top 2 bits of one MT19937 output
// word and retry while they are >= 2 (CPython 3.10 Lib/random.py:239-249), so
// a coin costs one word with bit 31 clear and its value is bit 30 (0 =
// attack).  random.seed(int) keys the generator with init_by_array over the
// little-endian 32-bit limbs of |seed| (one zero limb for seed 0).
//
// The canonical per-round draw order (SURVEY.md §8a lie row) is: the
// commander's coins for lieutenants 1..n-1 if it is faulty, then every
// lieutenant r = 1..n-1 in id order polls, in port order, the commander (only
// when its primary_port is stale, ba.py:171) and every other lieutenant j; a
// faulty answerer draws.  ba_om1_coin_count gives that count; the table
// layout is the one BA_LIE_TABLE consumes (bit c of row t = coin c).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/ba.h"

namespace {

constexpr int kN = 624, kM = 397;

void init_genrand(ba_mt* g, uint32_t s) {
    g->state[0] = s;
    for (int i = 1; i < kN; ++i)
        g->state[i] = 1812433253u * (g->state[i - 1] ^ (g->state[i - 1] >> 30)) + (uint32_t)i;
    g->index = kN;
}

void init_by_array(ba_mt* g, const uint32_t* key, int len) {
    init_genrand(g, 19650218u);
    uint32_t* mt = g->state;
    int i = 1, j = 0;
    for (int k = kN > len ? kN : len; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        ++i;
        ++j;
        if (i >= kN) {
            mt[0] = mt[kN - 1];
            i = 1;
        }
        if (j >= len) j = 0;
    }
    for (int k = kN - 1; k; --k) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        ++i;
        if (i >= kN) {
            mt[0] = mt[kN - 1];
            i = 1;
        }
    }
    mt[0] = 0x80000000u;
    g->index = kN;
}

void twist(ba_mt* g) {
    uint32_t* mt = g->state;
    for (int i = 0; i < kN; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % kN] & 0x7fffffffu);
        mt[i] = mt[(i + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->index = 0;
}

inline uint32_t next32(ba_mt* g) {
    if (g->index >= (uint32_t)kN) twist(g);
    uint32_t y = g->state[g->index++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// one random.randint(0, 1) draw; returns 1 for "attack" (the draw was 0)
inline uint32_t coin(ba_mt* g) {
    for (;;) {
        const uint32_t r = next32(g) >> 30;
        if (r < 2) return r == 0;
    }
}

inline uint32_t live_mask(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

}  // namespace

extern "C" void ba_mt_seed(ba_mt* g, uint64_t seed) {
    if (!g) return;
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    init_by_array(g, key, key[1] ? 2 : 1);
}

extern "C" uint32_t ba_mt_next32(ba_mt* g) { return g ? next32(g) : 0u; }

extern "C" uint32_t ba_om1_coin_count(uint32_t n, uint32_t m, uint32_t faulty_mask,
                                      uint32_t poll_commander) {
    if (n < 1 || n > BA_MAX_GENERALS) return 0;
    const uint32_t all = live_mask(n), fm = faulty_mask & all, pm = poll_commander & all & ~1u;
    const uint32_t L = n - 1;
    uint32_t c = (fm & 1u) ? L : 0u;  // ba.py:263-273 commander send
    if (m == 0) return c;
    const uint32_t flt = __builtin_popcount(fm & ~1u);
    for (uint32_t r = 1; r < n; ++r) {  // ba.py:169-186, receiver-major
        c += flt - ((fm >> r) & 1u);
        if (((pm >> r) & 1u) && (fm & 1u)) ++c;
    }
    return c;
}

extern "C" int ba_mt_draw_coins(ba_mt* g, uint32_t count, uint32_t* packed, uint32_t words) {
    if (!g || (count && !packed)) return BA_EINVAL;
    if ((uint64_t)words * 32 < count) return BA_EINVAL;
    memset(packed, 0, (size_t)words * sizeof(uint32_t));
    for (uint32_t c = 0; c < count; ++c)
        if (coin(g)) packed[c >> 5] |= 1u << (c & 31);
    return BA_OK;
}

extern "C" int ba_mt_table(uint32_t n, uint32_t m, uint64_t batch, const uint64_t* seeds,
                           const uint32_t* faulty_mask, const uint32_t* poll_commander,
                           uint32_t stride, uint32_t* table, uint32_t* next_word, int threads) {
    if (n < 1 || n > BA_MAX_GENERALS) return BA_EINVAL;
    if (batch && (!seeds || !faulty_mask || !table)) return BA_EINVAL;
    const uint64_t L = n - 1;
    if ((uint64_t)stride * 32 < L + L * L) return BA_EINVAL;
    unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if ((uint64_t)nt > batch / 64 + 1) nt = (unsigned)(batch / 64 + 1);
    auto work = [&](uint64_t b, uint64_t e) {
        ba_mt g;
        for (uint64_t t = b; t < e; ++t) {
            ba_mt_seed(&g, seeds[t]);
            const uint32_t cnt =
                ba_om1_coin_count(n, m, faulty_mask[t], poll_commander ? poll_commander[t] : 0u);
            ba_mt_draw_coins(&g, cnt, table + t * stride, stride);
            if (next_word) next_word[t] = next32(&g);
        }
    };
    if (nt == 1) {
        work(0, batch);
        return BA_OK;
    }
    std::vector<std::thread> pool;
    const uint64_t per = (batch + nt - 1) / nt;
    for (unsigned i = 0; i < nt; ++i) {
        const uint64_t b = i * per, e = std::min<uint64_t>(batch, b + per);
        if (b < e) pool.emplace_back(work, b, e);
    }
    for (auto& th : pool) th.join();
    return BA_OK;
}
