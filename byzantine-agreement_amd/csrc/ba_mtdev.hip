// ba_mtdev.hip -- ba.py's coin source on the device (ba_mt_table_device): for
// every trial t, random.seed(seeds[t]) and then one ba.py round's coins in the
// canonical draw order (ba.py:45 relay lies, ba.py:269 commander lies), packed
// into row t of the BA_LIE_TABLE coin table -- the same rows ba_mt_table
// (ba_mt.cpp, host threads) writes, which the ba.py fixtures pin.
//
// CPython's Mersenne Twister (ba_mt.cpp restates it): random.seed(int) is
// init_by_array over the seed's 32-bit limbs -- init_genrand(19650218), one
// sweep of 624 key steps, one of 623 mixing steps -- and every output word
// comes from the twisted state.  One thread per trial:
//  * the 624-word initial state init_genrand(19650218) is the same for every
//    seed: a compile-time table in constant memory, read at the same index by
//    every lane of a wave (a broadcast);
//  * the key sweep is a recurrence over i whose values the mixing sweep needs
//    again, index by index: it is run once to its end (to get mt[623] and the
//    wrap step's mt[1]) and once more in lockstep with the mixing sweep, so
//    nothing of it is stored;
//  * the mixed state goes to HBM once, i-major ([624][T]: every step of a wave
//    is one coalesced 256-B access), and the outputs twist it lazily in place,
//    in index order -- exactly CPython's twist, for as many outputs (and twists)
//    as the round draws;
//  * a coin is the first output whose top two bits are < 2 (randint(0, 1) =
//    _randbelow(2)), bit 30 = 0 meaning "attack".
#include "ba_leaf.hpp"  // static_for

namespace ba {

namespace {

constexpr int kMtN = 624, kMtM = 397;

struct MtInitTable {
    uint32_t v[kMtN];
    constexpr MtInitTable() : v() {
        v[0] = 19650218u;
        for (int i = 1; i < kMtN; ++i) v[i] = 1812433253u * (v[i - 1] ^ (v[i - 1] >> 30)) + (uint32_t)i;
    }
};
__constant__ MtInitTable kMtInit = MtInitTable();

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// ba_om1_coin_count (ba_mt.cpp), per trial
__device__ __forceinline__ uint32_t om1_coins(uint32_t n, uint32_t m, uint32_t fm, uint32_t pm) {
    const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    fm &= all;
    pm &= all & ~1u;
    const uint32_t L = n - 1;
    uint32_t c = (fm & 1u) ? L : 0u;  // ba.py:263-273 commander send
    if (m == 0) return c;
    const uint32_t flt = (uint32_t)__popc(fm & ~1u);
    for (uint32_t r = 1; r < n; ++r) {  // ba.py:169-186, receiver-major
        c += flt - ((fm >> r) & 1u);
        if (((pm >> r) & 1u) && (fm & 1u)) ++c;
    }
    return c;
}

__global__ __launch_bounds__(256) void k_mt_table(uint32_t n, uint32_t m, uint64_t T,
                                                  const uint64_t* __restrict__ seeds,
                                                  const uint32_t* __restrict__ faulty,
                                                  const uint32_t* __restrict__ poll, uint32_t stride,
                                                  uint32_t* __restrict__ table,
                                                  uint32_t* __restrict__ next_word,
                                                  uint32_t* __restrict__ st) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    // random.seed(seed): key = the 32-bit limbs of |seed| (one zero limb for 0)
    const uint64_t seed = seeds[t];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const bool two = k1 != 0;
    // key sweep step at index i adds key[j] + j, j = (i - 1) % len
    const uint32_t add_even = k0, add_odd = two ? k1 + 1u : k0;
    // 1. the key sweep to its end: p1 = mt[1] after its first step, a = mt[623]
    uint32_t a = kMtInit.v[0], p1 = 0;
    for (int i = 1; i < kMtN; ++i) {
        a = (kMtInit.v[i] ^ ((a ^ (a >> 30)) * 1664525u)) + (((i - 1) & 1) ? add_odd : add_even);
        if (i == 1) p1 = a;
    }
    // its 624th step wraps to i = 1 (mt[0] = mt[623], j = 623 % len)
    const uint32_t p1w = (p1 ^ ((a ^ (a >> 30)) * 1664525u)) + add_odd;
    // 2. the mixing sweep, i = 2 .. 623, with the key sweep's mt[i] recomputed
    //    alongside; then its wrap step for mt[1], and mt[0] = 0x80000000
    uint32_t c1 = p1, c2 = p1w;
    for (int i = 2; i < kMtN; ++i) {
        c1 = (kMtInit.v[i] ^ ((c1 ^ (c1 >> 30)) * 1664525u)) + (((i - 1) & 1) ? add_odd : add_even);
        c2 = (c1 ^ ((c2 ^ (c2 >> 30)) * 1566083941u)) - (uint32_t)i;
        st[(uint64_t)i * T + t] = c2;
    }
    st[T + t] = (p1w ^ ((c2 ^ (c2 >> 30)) * 1566083941u)) - 1u;
    st[t] = 0x80000000u;
    // 3. the round's coins from lazily twisted outputs (CPython's twist is an
    //    in-place sweep in index order: new[i] reads mt[i], mt[i+1], mt[i+397],
    //    the last two already new where they wrapped -- so is this), in blocks
    //    of kBlk outputs: the 2*kBlk+1 state words a block reads are loaded
    //    together (each output's source lies 227 or more positions behind any
    //    output of its own block), the lanes of a wave at the same positions
    //    (coalesced), for as long as any lane still draws
    constexpr uint32_t kBlk = 16;
    const uint32_t cnt = om1_coins(n, m, faulty[t], poll ? poll[t] : 0u);
    uint32_t* row = table + t * stride;
    const bool want_next = next_word != nullptr;
    uint32_t pos = 0, c = 0, word = 0;
    bool done = !want_next && cnt == 0;
    while (__any(!done)) {
        if (!done) {
            uint32_t cur[kBlk + 1], far[kBlk];
            static_for<0, kBlk + 1>([&](auto k) {
                uint32_t i = pos + k();
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                cur[k()] = st[(uint64_t)i * T + t];
            });
            static_for<0, kBlk>([&](auto k) {
                uint32_t i = pos + k() + kMtM;
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                far[k()] = st[(uint64_t)i * T + t];
            });
            static_for<0, kBlk>([&](auto k) {
                uint32_t i = pos + k();
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                const uint32_t y = (cur[k()] & 0x80000000u) | (cur[k() + 1] & 0x7fffffffu);
                const uint32_t v = far[k()] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
                st[(uint64_t)i * T + t] = v;
                const uint32_t out = mt_temper(v);
                if (c < cnt) {
                    const uint32_t r = out >> 30;  // randint(0, 1): top two bits, retried >= 2
                    if (r < 2) {
                        word |= (r == 0 ? 1u : 0u) << (c & 31);  // == 0: "attack"
                        if ((c & 31) == 31) {
                            row[c >> 5] = word;
                            word = 0;
                        }
                        ++c;
                        if (c == cnt && !want_next) done = true;
                    }
                } else if (!done) {  // the word after the round: getrandbits(32)
                    next_word[t] = out;
                    done = true;
                }
            });
            pos += kBlk;
            pos = pos >= (uint32_t)kMtN ? pos - kMtN : pos;
        }
    }
    if (cnt & 31) row[cnt >> 5] = word;
    for (uint32_t wi = (cnt + 31) >> 5; wi < stride; ++wi) row[wi] = 0;  // the row's unused words
}

}  // namespace

// state words per trial (the chunk's scratch: [624][T] uint32)
uint64_t mt_table_state_bytes_per_trial() { return (uint64_t)kMtN * sizeof(uint32_t); }

hipError_t launch_mt_table(uint32_t n, uint32_t m, uint64_t T, const uint64_t* seeds,
                           const uint32_t* faulty, const uint32_t* poll, uint32_t stride,
                           uint32_t* table, uint32_t* next_word, uint32_t* state, hipStream_t s,
                           Prof* prof) {
    ProfScope ps(prof, "k_mt_table", s);
    const uint64_t blocks = (T + 255) / 256;
    hipLaunchKernelGGL(k_mt_table, dim3((uint32_t)blocks), dim3(256), 0, s, n, m, T, seeds, faulty,
                       poll, stride, table, next_word, state);
    return hipGetLastError();
}

}  // namespace ba
