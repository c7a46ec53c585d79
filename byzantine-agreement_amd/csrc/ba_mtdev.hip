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
//    outputs (and twists) as the round draws; a window of <= 227 outputs is
//    drawn inside the mixing sweep itself (MtStream), positions 397.. never
//    stored;
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
#ifndef BA_MT_SORT
#define BA_MT_SORT 1  // 0: lab A/B, trials in index order over the waves
#endif
#ifndef BA_MT_STREAM
#define BA_MT_STREAM 1  // 0: lab A/B, every window drawn after the sweep (mt_draw)
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

// Draw the round's coins (and the next word) of trial t from the state stored
// in column `col` (rows of T words) at the slots `slot(i)` maps state positions to, twisting lazily in place: output k
// reads positions k, k+1 and k+397 (mod 624; a position below k+397-624 is
// already new, as in CPython's in-place twist).  `lim` = the number of outputs
// the stored positions allow (a window), or 0 for the full state (any number,
// second twists included: positions wrap).  Returns false if the lane needed
// more than `lim` outputs (it then starts over on the full state).
template <typename Slot>
__device__ __forceinline__ bool mt_draw(uint32_t* __restrict__ col, uint64_t T, uint64_t t, Slot slot,
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
// (c1 ^ ((c2 ^ (c2 >> 30)) * 1566083941)) - i with -i (wave-uniform) an SGPR
// operand: the xor and the add are one v_xad_u32, where the compiler folded
// -i's constant part into a v_add3_u32 after a separate v_xor_b32 (one VALU op
// more per step; n=4 tables 0.29 -> 0.28 ms per 1M trials)
__device__ __forceinline__ uint32_t mt_mix_step_s(uint32_t c1, uint32_t c2, uint32_t i) {
    const uint32_t prod = (c2 ^ (c2 >> 30)) * 1566083941u;
    uint32_t r;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(c1), "v"(prod), "s"(0u - i));
    return r;
}

// Mixing-sweep steps i in [i0, i1) (uniform bounds) of J trials at once (J
// independent recurrence chains per lane: the sweep is a chain of dependent
// multiplies, so its issue rate is the chains in flight), each with the key
// sweep's mt[i] recomputed alongside; STORE: mt[i] to *p[j], the pointers
// advancing one row (R words) per step.  Unrolled by hand, four steps from an
// even i (the key's limb parity a compile-time choice, the constant table's
// scalar loads in groups): the xad asm is convergent, which keeps the compiler
// from unrolling a loop with a run-time trip count itself.
template <int J, bool STORE, bool ODD>
__device__ __forceinline__ void mt_mix_one(uint32_t init, uint32_t i, uint32_t (&c1)[J], uint32_t (&c2)[J],
                                           const uint32_t (&add_even)[J], const uint32_t (&add_odd)[J],
                                           uint32_t* (&p)[J], uint64_t R) {
    static_for<0, J>([&](auto j) {
        // key sweep step at index i adds key[k] + k, k = (i - 1) % 2: ODD = (i - 1) odd
        c1[j()] = mt_key_step(init, c1[j()], ODD ? add_odd[j()] : add_even[j()]);
        c2[j()] = mt_mix_step_s(c1[j()], c2[j()], i);
        if constexpr (STORE) {
            *p[j()] = c2[j()];
            p[j()] += R;
        }
    });
}
template <int J, bool STORE>
__device__ __forceinline__ void mt_mix_range(uint32_t i0, uint32_t i1, uint32_t (&c1)[J], uint32_t (&c2)[J],
                                             const uint32_t (&add_even)[J], const uint32_t (&add_odd)[J],
                                             uint32_t* (&p)[J], uint64_t R) {
    uint32_t i = i0;
    if (i < i1 && (i & 1u)) {  // to an even i
        mt_mix_one<J, STORE, false>(kMtInit.v[i], i, c1, c2, add_even, add_odd, p, R);
        ++i;
    }
    for (; i + 4 <= i1; i += 4) {
        mt_mix_one<J, STORE, true>(kMtInit.v[i], i, c1, c2, add_even, add_odd, p, R);
        mt_mix_one<J, STORE, false>(kMtInit.v[i + 1], i + 1, c1, c2, add_even, add_odd, p, R);
        mt_mix_one<J, STORE, true>(kMtInit.v[i + 2], i + 2, c1, c2, add_even, add_odd, p, R);
        mt_mix_one<J, STORE, false>(kMtInit.v[i + 3], i + 3, c1, c2, add_even, add_odd, p, R);
    }
    for (; i < i1; ++i) {
        if (i & 1u) mt_mix_one<J, STORE, false>(kMtInit.v[i], i, c1, c2, add_even, add_odd, p, R);
        else mt_mix_one<J, STORE, true>(kMtInit.v[i], i, c1, c2, add_even, add_odd, p, R);
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
// 1. of init_by_array: the key sweep to its end; leaves the mixing sweep's start
// (c1 = the key sweep's mt[1] before the wrap, c2 = mt[1] after it) and p1w.
template <int J>
__device__ __forceinline__ void mt_key_sweep(const uint64_t (&seed)[J], uint32_t (&add_even)[J],
                                             uint32_t (&add_odd)[J], uint32_t (&c1)[J], uint32_t (&c2)[J],
                                             uint32_t (&p1w)[J]) {
    uint32_t p1[J], a[J];
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
    static_for<0, J>([&](auto j) {
        p1w[j()] = (p1[j()] ^ ((a[j()] ^ (a[j()] >> 30)) * 1664525u)) + add_odd[j()];
        c1[j()] = p1[j()];
        c2[j()] = p1w[j()];
    });
}
// the mixing sweep's wrap step: the final mt[1]
__device__ __forceinline__ uint32_t mt_wrap(uint32_t p1w, uint32_t c2) {
    return (p1w ^ ((c2 ^ (c2 >> 30)) * 1566083941u)) - 1u;
}

template <int J>
__device__ __forceinline__ void mt_seed(uint32_t* const (&col)[J], uint64_t R, const uint64_t (&seed)[J],
                                        uint32_t lo_end, uint32_t hi) {
    uint32_t add_even[J], add_odd[J], c1[J], c2[J], p1w[J];
    mt_key_sweep<J>(seed, add_even, add_odd, c1, c2, p1w);
    uint32_t* p[J];
    static_for<0, J>([&](auto j) { p[j()] = col[j()] + 2 * R; });
    // 2. the mixing sweep, i = 2 .. 623; then its wrap step for mt[1], and
    //    mt[0] = 0x80000000
    if (hi == 0) {  // the full state
        uint32_t end = kMtN;
        asm("" : "+s"(end));  // a run-time trip count: not unrolled 155 times over
        mt_mix_range<J, true>(2u, end, c1, c2, add_even, add_odd, p, R);
    } else {
        mt_mix_range<J, true>(2u, lo_end, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, false>(lo_end, (uint32_t)kMtM, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, true>((uint32_t)kMtM, (uint32_t)kMtM + hi, c1, c2, add_even, add_odd, p, R);
        mt_mix_range<J, false>((uint32_t)kMtM + hi, (uint32_t)kMtN, c1, c2, add_even, add_odd, p, R);
    }
    static_for<0, J>([&](auto j) {
        col[j()][R] = mt_wrap(p1w[j()], c2[j()]);
        col[j()][0] = 0x80000000u;
    });
}

// ---------------------------------------------------------------------------
// Streamed window (a wave whose window is Wv <= 227 outputs): output k >= 2
// reads post-seed positions k, k+1 and 397+k, and the mixing sweep produces
// 397+k after k and k+1 -- so the output is drawn right there, in the sweep,
// from the one word it produces and the two stored ones.  Only positions
// 2..Wv go to HBM (once, read back once); 397.. are never stored and no
// separate draw pass runs.  Outputs 0 and 1 read position 1, which the sweep's
// wrap step writes last: they are drawn after it, from mt[397], mt[398] and
// mt[2] kept in registers, and the coins of outputs 2.. -- counted from coin 0
// meanwhile -- move up by the coins that 0 and 1 turn out to give (0, 1 or 2).
// The word after the round is the output right after the cnt-th coin: caught
// for each of the three possible offsets (cand[d]: right after coin cnt - d of
// outputs 2..).  A trial whose window runs out starts over on the full state.
struct MtStream {
    uint32_t cnt;          // the round's coins
    uint32_t c2;           // coins taken from outputs 2.. (at most cnt)
    uint32_t word;         // coin bits of the current row word
    uint32_t cand0, cand1, cand2, cap;  // cand[d] and which were caught (bit d)
    uint32_t prev;         // post-seed mt[k] for the next output k
    uint32_t far0, far1;   // post-seed mt[397], mt[398]
    uint32_t m2, o2;       // post-seed mt[2]; output 2
    uint32_t inc;          // the previous output was a coin counted into c2 (0/1)
};

__device__ __forceinline__ bool mt_stream_done(const MtStream& s, bool want) {
    // conservative (as if outputs 0 and 1 gave no coin): every coin, and the
    // word after the last one, whatever 0 and 1 give
    return s.c2 >= s.cnt && (!want || s.cnt == 0 || (s.cap & 1u));
}

// output k (>= 2) of the round: `far` = post-seed mt[397 + k] (just produced),
// `nxt` = post-seed mt[k + 1]
__device__ __forceinline__ void mt_stream_out(MtStream& s, uint32_t far, uint32_t nxt, uint32_t k, uint32_t* row) {
    const uint32_t y = (s.prev & 0x80000000u) | (nxt & 0x7fffffffu);
    const uint32_t out = mt_temper(far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    s.prev = nxt;
    if (k == 2) s.o2 = out;
    // (branches: a branch-free form of the two ifs measured 1-3% slower)
    if (s.inc) {  // the first output after coin c2 of outputs 2..: c2 = cnt - d
        const uint32_t d = s.cnt - s.c2;
        if (d == 0) {
            s.cand0 = out;
            s.cap |= 1u;
        } else if (d == 1) {
            s.cand1 = out;
            s.cap |= 2u;
        } else if (d == 2) {
            s.cand2 = out;
            s.cap |= 4u;
        }
    }
    const uint32_t r = out >> 30;  // randint(0, 1): top two bits, retried >= 2
    s.inc = (r < 2u && s.c2 < s.cnt) ? 1u : 0u;
    if (s.inc) {
        s.word |= (r == 0u ? 1u : 0u) << (s.c2 & 31u);  // == 0: "attack"
        ++s.c2;
        if ((s.c2 & 31u) == 0u) {
            row[(s.c2 >> 5) - 1u] = s.word;
            s.word = 0;
        }
    }
}

// Mixing-sweep steps [i0, i1) (i0 odd) drawing output i - 397 of every trial
// while any trial of the wave still needs outputs (groups of four steps, the
// next four post-seed words of each trial loaded at the group's start).
template <int J>
__device__ __forceinline__ void mt_stream_range(uint32_t i0, uint32_t i1, uint32_t (&c1)[J], uint32_t (&c2)[J],
                                                const uint32_t (&add_even)[J], const uint32_t (&add_odd)[J],
                                                MtStream (&S)[J], uint32_t* const (&col)[J], uint64_t R,
                                                uint32_t* const (&row)[J], bool want) {
    uint32_t* nop[J];  // mt_mix_one's store pointers (STORE = false: unused)
    static_for<0, J>([&](auto j) { nop[j()] = nullptr; });
    auto need = [&]() {
        bool nd = false;
        static_for<0, J>([&](auto j) { nd = nd || !mt_stream_done(S[j()], want); });
        return __any(nd) != 0;
    };
    auto draw = [&](uint32_t k, const uint32_t (&nx)[J]) {
        static_for<0, J>([&](auto j) { mt_stream_out(S[j()], c2[j()], nx[j()], k, row[j()]); });
    };
    auto load4 = [&](uint32_t k, uint32_t (&nx)[4][J]) {
        static_for<0, 4>([&](auto q) {
            static_for<0, J>([&](auto j) { nx[q()][j()] = col[j()][(uint64_t)(k + 1 + q()) * R]; });
        });
    };
    uint32_t i = i0;
    // (loading the next group's words a group ahead measured 3-8% slower: 112
    // VGPRs, r06v)
    for (; i + 4 <= i1; i += 4) {
        const uint32_t k = i - (uint32_t)kMtM;
        if (need()) {
            uint32_t nx[4][J];
            load4(k, nx);
            mt_mix_one<J, false, false>(kMtInit.v[i], i, c1, c2, add_even, add_odd, nop, R);
            draw(k, nx[0]);
            mt_mix_one<J, false, true>(kMtInit.v[i + 1], i + 1, c1, c2, add_even, add_odd, nop, R);
            draw(k + 1, nx[1]);
            mt_mix_one<J, false, false>(kMtInit.v[i + 2], i + 2, c1, c2, add_even, add_odd, nop, R);
            draw(k + 2, nx[2]);
            mt_mix_one<J, false, true>(kMtInit.v[i + 3], i + 3, c1, c2, add_even, add_odd, nop, R);
            draw(k + 3, nx[3]);
        } else {
            mt_mix_one<J, false, false>(kMtInit.v[i], i, c1, c2, add_even, add_odd, nop, R);
            mt_mix_one<J, false, true>(kMtInit.v[i + 1], i + 1, c1, c2, add_even, add_odd, nop, R);
            mt_mix_one<J, false, false>(kMtInit.v[i + 2], i + 2, c1, c2, add_even, add_odd, nop, R);
            mt_mix_one<J, false, true>(kMtInit.v[i + 3], i + 3, c1, c2, add_even, add_odd, nop, R);
        }
    }
    for (; i < i1; ++i) {
        if (i & 1u) mt_mix_one<J, false, false>(kMtInit.v[i], i, c1, c2, add_even, add_odd, nop, R);
        else mt_mix_one<J, false, true>(kMtInit.v[i], i, c1, c2, add_even, add_odd, nop, R);
        if (need()) {
            const uint32_t k = i - (uint32_t)kMtM;
            uint32_t nx[J];
            static_for<0, J>([&](auto j) { nx[j()] = col[j()][(uint64_t)(k + 1) * R]; });
            draw(k, nx);
        }
    }
}

// random.seed(seed[j]) and the round's draws over a streamed window of wv
// outputs (16 <= wv <= 227): positions 2..wv stored at rows 2..wv.  Leaves each
// trial's final mt[1] in mt1[j]; mt_stream_finish completes the row.
template <int J>
__device__ __forceinline__ void mt_seed_stream(uint32_t* const (&col)[J], uint64_t R, const uint64_t (&seed)[J],
                                               uint32_t wv, MtStream (&S)[J], uint32_t* const (&row)[J],
                                               bool want, uint32_t (&mt1)[J]) {
    uint32_t add_even[J], add_odd[J], c1[J], c2[J], p1w[J];
    mt_key_sweep<J>(seed, add_even, add_odd, c1, c2, p1w);
    uint32_t* p[J];
    static_for<0, J>([&](auto j) { p[j()] = col[j()] + 2 * R; });
    mt_mix_range<J, true>(2u, wv + 1u, c1, c2, add_even, add_odd, p, R);          // rows 2..wv
    mt_mix_range<J, false>(wv + 1u, (uint32_t)kMtM, c1, c2, add_even, add_odd, p, R);
    // 397 and 398 feed outputs 0 and 1 (after the wrap)
    mt_mix_one<J, false, false>(kMtInit.v[kMtM], (uint32_t)kMtM, c1, c2, add_even, add_odd, p, R);
    static_for<0, J>([&](auto j) { S[j()].far0 = c2[j()]; });
    mt_mix_one<J, false, true>(kMtInit.v[kMtM + 1], (uint32_t)kMtM + 1, c1, c2, add_even, add_odd, p, R);
    static_for<0, J>([&](auto j) {
        S[j()].far1 = c2[j()];
        S[j()].m2 = S[j()].prev = col[j()][2 * R];
    });
    mt_stream_range<J>((uint32_t)kMtM + 2, (uint32_t)kMtM + wv, c1, c2, add_even, add_odd, S, col, R, row, want);
    mt_mix_range<J, false>((uint32_t)kMtM + wv, (uint32_t)kMtN, c1, c2, add_even, add_odd, p, R);
    static_for<0, J>([&](auto j) { mt1[j()] = mt_wrap(p1w[j()], c2[j()]); });
}

// Outputs 0 and 1, then the row: the coins of outputs 2.. move up by a01 (the
// coins of 0 and 1) behind them, bits from cnt on cleared; the word after the
// round.  Returns false if the window held too few outputs.
__device__ __forceinline__ bool mt_stream_finish(const MtStream& s, uint32_t mt1, bool want, uint32_t* row,
                                                 uint32_t* __restrict__ next_word, uint64_t t) {
    const uint32_t y0 = 0x80000000u | (mt1 & 0x7fffffffu);  // post-seed mt[0] = 0x80000000
    const uint32_t o0 = mt_temper(s.far0 ^ (y0 >> 1) ^ ((y0 & 1u) ? 0x9908b0dfu : 0u));
    const uint32_t y1 = (mt1 & 0x80000000u) | (s.m2 & 0x7fffffffu);
    const uint32_t o1 = mt_temper(s.far1 ^ (y1 >> 1) ^ ((y1 & 1u) ? 0x9908b0dfu : 0u));
    const bool acc0 = (o0 >> 30) < 2u, acc1 = (o1 >> 30) < 2u;
    uint32_t pre = 0, a01 = 0;
    if (acc0) {
        pre = (o0 >> 30) == 0u ? 1u : 0u;
        a01 = 1;
    }
    if (acc1) {
        pre |= ((o1 >> 30) == 0u ? 1u : 0u) << a01;
        ++a01;
    }
    if (a01 + s.c2 < s.cnt) return false;
    uint32_t nw = 0;
    if (want) {
        if (s.cnt == 0) {
            nw = o0;
        } else if (s.cnt <= a01) {  // coin cnt is output 0 (cnt = 1, acc0) or output 1
            nw = (s.cnt == 1 && acc0) ? o1 : s.o2;
        } else {
            if (!((s.cap >> a01) & 1u)) return false;
            // masks, not a select of the three fields (which became a load from a
            // selected address: the lanes' states in scratch memory)
            nw = (s.cand0 & (0u - (a01 == 0 ? 1u : 0u))) | (s.cand1 & (0u - (a01 == 1 ? 1u : 0u))) |
                 (s.cand2 & (0u - (a01 == 2 ? 1u : 0u)));
        }
    }
    if (s.cnt != 0) {
        if (s.c2 & 31u) row[s.c2 >> 5] = s.word;
        if (a01 != 0) {
            const uint32_t nsrc = (s.c2 + 31u) >> 5, ndst = (s.cnt + 31u) >> 5;
            uint32_t carry = pre;
            for (uint32_t w = 0; w < ndst; ++w) {
                const uint32_t src = w < nsrc ? row[w] : 0u;
                row[w] = (src << a01) | carry;
                carry = src >> (32u - a01);
            }
        }
        if (s.cnt & 31u) row[s.cnt >> 5] &= (1u << (s.cnt & 31u)) - 1u;
    }
    if (want) next_word[t] = nw;
    return true;
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
// on average, so that is > 4 sigma of retries), rounded to the draw block.
// Wv <= 227 (every wave up to n = 10 at m = 1): the streamed window
// (mt_seed_stream), rows 2..Wv only.  227 < Wv < 397: rows 0..Wv and
// 397..623, drawn after the sweep (mt_draw).  A trial that still needs more
// outputs starts over on its full 624-word state (positions = slots), as does
// every trial of a wave whose window would not fit below position 397.
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
    const uint64_t base = (uint64_t)blockIdx.x * (kMtBlock * J);
    if constexpr (BA_MT_SORT) {
        // The block's trials go to its waves in order of coin count (a bitonic
        // sort of (cnt, index) keys in LDS): a wave's window -- its largest trial's
        // -- then fits its trials, where in index order nearly every wave held
        // a trial near the block's largest count, and a wave of trials that draw
        // nothing skips random.seed altogether (n=4: 0.26 -> 0.21 ms per 1M
        // trials; n=10 the same).  Trial t_j's scratch column is its sorted
        // position (the wave's stores stay one 256-B segment).
        constexpr uint32_t NK = kMtBlock * J;
        __shared__ uint32_t key[NK];
        static_for<0, J>([&](auto j) {
            const uint32_t li = j() * kMtBlock + threadIdx.x;
            const uint64_t tt = base + li;
            const uint32_t c = tt < T ? om1_coins(n, m, faulty[tt], poll ? poll[tt] : 0u) : 0u;
            key[li] = c << 10 | li;  // c < 2^22 (n <= 32)
        });
        __syncthreads();
        for (uint32_t k = 2; k <= NK; k <<= 1) {
            for (uint32_t h = k >> 1; h > 0; h >>= 1) {
                for (uint32_t q = threadIdx.x; q < NK / 2; q += kMtBlock) {
                    const uint32_t i = 2 * h * (q / h) + q % h;
                    const uint32_t a = key[i], b = key[i + h];
                    if ((a > b) == ((i & k) == 0)) {
                        key[i] = b;
                        key[i + h] = a;
                    }
                }
                __syncthreads();
            }
        }
        // (wave w taking sorted quarter (w + block) mod 4 instead measured the same)
        const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
        static_for<0, J>([&](auto j) {
            const uint32_t p = wave * (64u * J) + j() * 64u + lane, kk = key[p];
            t[j()] = base + (kk & 1023u);
            cnt[j()] = kk >> 10;
            col[j()] = st + base + p;
        });
    } else {
        static_for<0, J>([&](auto j) {
            t[j()] = base + j() * kMtBlock + threadIdx.x;
            cnt[j()] = t[j()] < T ? om1_coins(n, m, faulty[t[j()]], poll ? poll[t[j()]] : 0u) : 0u;
            col[j()] = st + t[j()];
        });
    }
    static_for<0, J>([&](auto j) {
        live[j()] = t[j()] < T;
        seed[j()] = live[j()] ? seeds[t[j()]] : 0ull;
        // (columns < R: padding columns for the dead trials)
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
    } else if (BA_MT_STREAM && wv <= kFar) {
        // streamed window: outputs 2..wv-1 drawn in the mixing sweep
        MtStream S[J];
        uint32_t* row[J];
        static_for<0, J>([&](auto j) {
            S[j()].cnt = cnt[j()];
            S[j()].c2 = S[j()].word = S[j()].cap = S[j()].inc = 0;
            S[j()].cand0 = S[j()].cand1 = S[j()].cand2 = S[j()].o2 = 0;
            row[j()] = table + t[j()] * stride;  // written only for a trial that takes coins
        });
        uint32_t mt1[J];
        mt_seed_stream<J>(col, R, seed, wv, S, row, want_next, mt1);
        static_for<0, J>([&](auto j) {
            if (live[j()]) ok[j()] = mt_stream_finish(S[j()], mt1[j()], want_next, row[j()], next_word, t[j()]);
        });
    } else if (wv < (uint32_t)kMtM) {
        // window: positions 0..wv at rows 0..wv, 397..397+min(wv,227)-1 after them
        // (outputs past 227 read positions <= wv back as new)
        const uint32_t hi = wv < kFar ? wv : kFar;
        mt_seed<J>(col, R, seed, wv + 1, hi);
        auto slot = [wv](uint32_t i) { return i <= wv ? i : wv + 1u + (i - (uint32_t)kMtM); };
        static_for<0, J>([&](auto j) {
            if (live[j()])
                ok[j()] = mt_draw(col[j()], R, t[j()], slot, wv, cnt[j()], want_next, table + t[j()] * stride,
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
            (void)mt_draw(col[j()], R, t[j()], [](uint32_t i) { return i; }, 0u, cnt[j()], want_next, row,
                          next_word);
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
