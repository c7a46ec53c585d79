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
//    is one coalesced 256-B access) -- only the positions the round's outputs
//    will read (a window sized per wave, k_mt_table) -- and the outputs twist it
//    lazily in place, in index order -- exactly CPython's twist, for as many
//    outputs (and twists) as the round draws;
//  * a coin is the first output whose top two bits are < 2 (randint(0, 1) =
//    _randbelow(2)), bit 30 = 0 meaning "attack".
#include "ba_leaf.hpp"  // static_for

namespace ba {

namespace {

constexpr int kMtN = 624, kMtM = 397;
#ifndef BA_MT_BLK
#define BA_MT_BLK 8
#endif
#ifndef BA_MT_TPL
#define BA_MT_TPL 2
#endif
constexpr uint32_t kMtDrawBlk = BA_MT_BLK;  // outputs twisted per block of loads (mt_draw)

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

// Draw the round's coins (and the next word) from the state stored at the
// slots `slot(i)` maps state positions to, twisting lazily in place: output k
// reads positions k, k+1 and k+397 (mod 624; a position below k+397-624 is
// already new, as in CPython's in-place twist).  `lim` = the number of outputs
// the stored positions allow (a window), or 0 for the full state (any number,
// second twists included: positions wrap).  Returns false if the lane needed
// more than `lim` outputs (it then starts over on the full state).
template <typename Slot>
__device__ __forceinline__ bool mt_draw(uint32_t* __restrict__ st, uint64_t T, uint64_t t, Slot slot,
                                        uint32_t lim, uint32_t cnt, bool want_next, uint32_t* row,
                                        uint32_t* __restrict__ next_word) {
    constexpr uint32_t kBlk = kMtDrawBlk;
    uint32_t pos = 0, c = 0, word = 0;
    bool done = !want_next && cnt == 0, ok = true;
    while (__any(!done)) {
        if (!done && lim != 0 && pos >= lim) {  // the window is used up: the slow path
            done = true;
            ok = false;
        }
        if (!done) {
            // every lane still drawing is at the same position: row addresses
            // are wave-uniform (scalar), the lane's column its offset
            const uint32_t upos = (uint32_t)__builtin_amdgcn_readfirstlane((int)pos);
            uint32_t* col = st + t;
            auto at = [&](uint32_t i) { return col + (uint64_t)slot(i) * T; };
            uint32_t cur[kBlk + 1], far[kBlk];
            static_for<0, kBlk + 1>([&](auto k) {
                uint32_t i = upos + k();
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                cur[k()] = *at(i);
            });
            static_for<0, kBlk>([&](auto k) {
                uint32_t i = upos + k() + kMtM;
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                far[k()] = *at(i);
            });
            static_for<0, kBlk>([&](auto k) {
                uint32_t i = upos + k();
                i = i >= (uint32_t)kMtN ? i - kMtN : i;
                const uint32_t y = (cur[k()] & 0x80000000u) | (cur[k() + 1] & 0x7fffffffu);
                const uint32_t v = far[k()] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
                // in place, where a later output reads it (its k + 397 wraps here)
                if (lim == 0 || i + (kMtN - kMtM) < lim) *at(i) = v;
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
    if (ok && (cnt & 31)) row[cnt >> 5] = word;
    return ok;
}

// CPython init_by_array's two recurrences (key sweep, mixing sweep)
__device__ __forceinline__ uint32_t mt_key_step(uint32_t init_i, uint32_t a, uint32_t add) {
    return (init_i ^ ((a ^ (a >> 30)) * 1664525u)) + add;
}
__device__ __forceinline__ uint32_t mt_mix_step(uint32_t c1, uint32_t c2, uint32_t i) {
    return (c1 ^ ((c2 ^ (c2 >> 30)) * 1566083941u)) - i;
}

// Mixing-sweep steps i in [i0, i1) (uniform bounds) of J trials at once (J
// independent recurrence chains per lane: the sweep is a chain of dependent
// multiplies, so its issue rate is the chains in flight), each with the key
// sweep's mt[i] recomputed alongside; STORE: mt[i] to *p[j], the pointers
// advancing one row (R words) per step.  Unrolled so the constant table's
// scalar loads go out in groups.
template <int J, bool STORE>
__device__ __forceinline__ void mt_mix_range(uint32_t i0, uint32_t i1, uint32_t (&c1)[J], uint32_t (&c2)[J],
                                             const uint32_t (&add_even)[J], const uint32_t (&add_odd)[J],
                                             uint32_t* (&p)[J], uint64_t R) {
#pragma unroll 4
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t init = kMtInit.v[i];
        const bool odd = ((i - 1) & 1) != 0;
        static_for<0, J>([&](auto j) {
            c1[j()] = mt_key_step(init, c1[j()], odd ? add_odd[j()] : add_even[j()]);
            c2[j()] = mt_mix_step(c1[j()], c2[j()], i);
            if constexpr (STORE) {
                *p[j()] = c2[j()];
                p[j()] += R;
            }
        });
    }
}

// random.seed(seed[j])'s state (init_by_array, CPython) for J trials: rows
// 2..lo_end-1 hold positions 2..lo_end-1 and rows lo_end.. positions 397..
// 397+hi-1 (rows of R words from col[j] = the trial's column), rows 1 and 0
// positions 1 and 0 -- every trial of the wave the same rows (whole-wave
// stores: storing only each trial's own positions, a store of some lanes,
// measured 1.6x slower at n=10: partial lines).  lo_end = 624, hi = 0: the
// full state, row = position.  The
// key sweep is a recurrence over i whose values the mixing sweep needs again,
// index by index: it is run once to its end (for mt[623] and the wrap step's
// mt[1]) and once more in lockstep with the mixing sweep, so nothing of it is
// stored.
template <int J>
__device__ __forceinline__ void mt_seed(uint32_t* const (&col)[J], uint64_t R, const uint64_t (&seed)[J],
                                        uint32_t lo_end, uint32_t hi) {
    uint32_t add_even[J], add_odd[J], p1[J], a[J];
    static_for<0, J>([&](auto j) {
        // random.seed(seed): key = the 32-bit limbs of |seed| (one zero limb for 0);
        // key sweep step at index i adds key[k] + k, k = (i - 1) % len
        const uint32_t k0 = (uint32_t)seed[j()], k1 = (uint32_t)(seed[j()] >> 32);
        add_even[j()] = k0;
        add_odd[j()] = k1 != 0 ? k1 + 1u : k0;
        // 1. the key sweep to its end: p1 = mt[1] after its first step, a = mt[623]
        p1[j()] = mt_key_step(kMtInit.v[1], kMtInit.v[0], add_even[j()]);
        a[j()] = p1[j()];
    });
#pragma unroll 4
    for (uint32_t i = 2; i < (uint32_t)kMtN; ++i) {
        const uint32_t init = kMtInit.v[i];
        const bool odd = ((i - 1) & 1) != 0;
        static_for<0, J>([&](auto j) { a[j()] = mt_key_step(init, a[j()], odd ? add_odd[j()] : add_even[j()]); });
    }
    // its 624th step wraps to i = 1 (mt[0] = mt[623], k = 623 % len)
    uint32_t c1[J], c2[J], p1w[J];
    uint32_t* p[J];
    static_for<0, J>([&](auto j) {
        p1w[j()] = (p1[j()] ^ ((a[j()] ^ (a[j()] >> 30)) * 1664525u)) + add_odd[j()];
        c1[j()] = p1[j()];
        c2[j()] = p1w[j()];
        p[j()] = col[j()] + 2 * R;
    });
    // 2. the mixing sweep, i = 2 .. 623; then its wrap step for mt[1], and
    //    mt[0] = 0x80000000
    if (hi == 0) {  // the full state
        mt_mix_range<J, true>(2u, (uint32_t)kMtN, c1, c2, add_even, add_odd, p, R);
    } else {
        mt_mix_range<J, true>(2u, lo_end, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, false>(lo_end, (uint32_t)kMtM, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, true>((uint32_t)kMtM, (uint32_t)kMtM + hi, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, false>((uint32_t)kMtM + hi, (uint32_t)kMtN, c1, c2, add_even, add_odd, p, R);
    }
    static_for<0, J>([&](auto j) {
        col[j()][R] = (p1w[j()] ^ ((c2[j()] ^ (c2[j()] >> 30)) * 1566083941u)) - 1u;
        col[j()][0] = 0x80000000u;
    });
}

// kMtTrialsPerLane trials per thread, the block's 256 threads owning 512
// consecutive trials: trial t_j = block * 512 + j * 256 + thread, so every
// store of a wave is one coalesced 256-B row segment.  The state goes to HBM
// [slot][R] (R = the chunk rounded up to whole blocks: a block's trials past
// the chunk's end run on zero inputs into padding columns, branch-free), but
// only the positions the round's outputs read (round 6: the whole 624-word
// state was written, 2.5 KB per trial, and the kernel was bound by those
// writes): a round of D <= 227 outputs reads positions 0..D and 397..397+D-1,
// and a few more past 227 (the in-place twist reads its own new words there).
// Each wave sizes its window from its trials' coin counts (om1_coins): Wv = max
// over the wave of 2.5 cnt + 16 (+1 for the next word; a coin takes 2 outputs
// on average, so that is > 4 sigma of retries), rounded to the draw block.  A
// trial that still needs more outputs starts over on its full 624-word state
// (positions = slots), as does every trial of a wave whose window would not
// fit below position 397.
constexpr int kMtTrialsPerLane = BA_MT_TPL, kMtBlock = 256;

__global__ __launch_bounds__(kMtBlock) void k_mt_table(uint32_t n, uint32_t m, uint64_t T, uint64_t R,
                                                       const uint64_t* __restrict__ seeds,
                                                       const uint32_t* __restrict__ faulty,
                                                       const uint32_t* __restrict__ poll, uint32_t stride,
                                                       uint32_t* __restrict__ table,
                                                       uint32_t* __restrict__ next_word,
                                                       uint32_t* __restrict__ st) {
    constexpr int J = kMtTrialsPerLane;
    constexpr uint32_t kBlk = kMtDrawBlk, kFar = kMtN - kMtM;  // 227 outputs before a wrap
    const bool want_next = next_word != nullptr;
    uint64_t t[J], seed[J];
    uint32_t cnt[J], need = 0;
    bool live[J];
    uint32_t* col[J];
    static_for<0, J>([&](auto j) {
        t[j()] = (uint64_t)blockIdx.x * (kMtBlock * J) + j() * kMtBlock + threadIdx.x;
        live[j()] = t[j()] < T;
        cnt[j()] = live[j()] ? om1_coins(n, m, faulty[t[j()]], poll ? poll[t[j()]] : 0u) : 0u;
        seed[j()] = live[j()] ? seeds[t[j()]] : 0ull;
        col[j()] = st + t[j()];  // t < R: padding columns for the dead trials
        // the outputs this trial's window holds (whole draw blocks)
        const uint32_t nj = live[j()] && (cnt[j()] != 0 || want_next)
                                ? 2u * cnt[j()] + cnt[j()] / 2u + 16u + (want_next ? 1u : 0u) : 0u;
        need = max(need, (nj + kBlk - 1) / kBlk * kBlk);
    });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) need = max(need, (uint32_t)__shfl_xor((int)need, off, 64));
    // the wave-uniform window (outputs)
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)need);
    bool ok[J];
    static_for<0, J>([&](auto j) { ok[j()] = true; });
    if (wv == 0) {
        // no trial of the wave draws: random.seed's state is never read
    } else if (wv < (uint32_t)kMtM) {
        // window: positions 0..wv at rows 0..wv, 397..397+min(wv,227)-1 after them
        // (outputs past 227 read positions <= wv back as new)
        const uint32_t hi = wv < kFar ? wv : kFar;
        mt_seed<J>(col, R, seed, wv + 1, hi);
        auto slot = [wv](uint32_t i) { return i <= wv ? i : wv + 1u + (i - (uint32_t)kMtM); };
        static_for<0, J>([&](auto j) {
            if (live[j()])
                ok[j()] = mt_draw(st, R, t[j()], slot, wv, cnt[j()], want_next, table + t[j()] * stride,
                                  next_word);
        });
    } else {
        static_for<0, J>([&](auto j) { ok[j()] = false; });
    }
    static_for<0, J>([&](auto j) {
        if (!live[j()]) return;
        uint32_t* row = table + t[j()] * stride;
        if (!ok[j()]) {  // the full state: every position at its own row, any number of outputs
            uint32_t* const c1[1] = {col[j()]};
            const uint64_t s1[1] = {seed[j()]};
            mt_seed<1>(c1, R, s1, (uint32_t)kMtN, 0u);
            (void)mt_draw(st, R, t[j()], [](uint32_t i) { return i; }, 0u, cnt[j()], want_next, row, next_word);
        }
        for (uint32_t wi = (cnt[j()] + 31) >> 5; wi < stride; ++wi) row[wi] = 0;  // the row's unused words
    });
}

}  // namespace

// the chunk's scratch: [624][R] uint32, R = the chunk's trials rounded up to
// whole blocks of kMtTrialsPerLane * kMtBlock
uint64_t mt_table_state_bytes_per_trial() { return (uint64_t)kMtN * sizeof(uint32_t); }
uint64_t mt_table_state_rows(uint64_t T) {
    constexpr uint64_t b = (uint64_t)kMtTrialsPerLane * kMtBlock;
    return (T + b - 1) / b * b;
}

hipError_t launch_mt_table(uint32_t n, uint32_t m, uint64_t T, const uint64_t* seeds,
                           const uint32_t* faulty, const uint32_t* poll, uint32_t stride,
                           uint32_t* table, uint32_t* next_word, uint32_t* state, hipStream_t s,
                           Prof* prof) {
    ProfScope ps(prof, "k_mt_table", s);
    const uint64_t R = mt_table_state_rows(T);
    const uint64_t blocks = R / ((uint64_t)kMtTrialsPerLane * kMtBlock);
    hipLaunchKernelGGL(k_mt_table, dim3((uint32_t)blocks), dim3(kMtBlock), 0, s, n, m, T, R, seeds, faulty,
                       poll, stride, table, next_word, state);
    return hipGetLastError();
}

}  // namespace ba
