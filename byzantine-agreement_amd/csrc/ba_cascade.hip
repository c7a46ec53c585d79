// ba_cascade.hip -- the LEVELS tree in ONE launch (gfx950): k_cascade<N, ME>.
//
// The multi-launch LEVELS pipeline for an OM(me) tree (n=16, m=5: k_input,
// k_relay_top, k_leaf_up, k_majority, k_tail) spends a third of a 1024-instance
// call in short latency-bound launches and their gaps.  Here
// every majority level above the leaf blocks is taken by whichever wave
// finishes the LAST input of it -- a fan-in cascade inside the launch, no grid
// barrier and no waiting anywhere:
//
//   unit (word w, level-Q slot rho; Q = me-3), G = S+1 lanes, one leaf block
//   each (the leaf-up kernel's unit, ba_fused.hip k_leaf_up):
//     inputs   the block bit-slices the trials of its words into LDS once
//     chain    L_0 .. L_{me-2} of the lane's slot sr = rho.x, relayed from the
//              commander down (one Philox pair per level, ba.py:42-57, 257-285)
//     leaf     relay levels me-1, me and the leaf majorities (leaf_block<S>)
//     up       R_{me-2}[rho.x] = maj(L_{me-2}[rho.x], R_{me-1}[rho.a.x] : a != x)
//   then arrives at the counter of rho's parent sigma.  The arrival that
//   completes sigma's children runs step q = Q for sigma:
//     R_q[sigma.r] = maj(L_q[sigma.r], R_{q+1}[sigma.j.r] : j != r)
//   (ba.py:159-195 generalised, inner tie -> non-attack), arrives at sigma's
//   parent, and so on up to q = 0: the root majorities (tie -> undefined) and
//   the quorum epilogue of the word (ba.py:197-255, wave_epilogue).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): results are
// stored write-through (sc1: relaxed agent-scope atomic stores), the storing
// wave drains vmcnt, then ONE lane per unit adds to the parent's counter (agent
// scope); the wave whose add returns the last count reads the children with
// sc1 loads only (L2-served, never L1).  The children of one parent sit on
// 128-B lines of their own (each sigma's child block is padded to whole lines,
// casc_pad), so no line a reader pulls into its XCD's L2 is ever shared with a
// hand-off still being written.  Counters sit on 128-B lines of their own; the
// last arriver resets its counter, so the buffer is zero between calls (zeroed
// once when the ctx allocates it).
//
// CHECK (test builds, BA_CASC_CHECK=1|2): every R store also stores a tag of
// the call's epoch (sc1, parallel array), every child load also loads its tag,
// and mismatches are counted into counter slot BA_C_CHECK_MISMATCH; =2 makes
// the first unit of the launch store a stale tag (the detector must fire once).
//
// Range mode (a.h = 1 or 2; the subtree split, ba_split_votes_device): the
// units are the level-Q slots below the h-hop subtrees [ub, ue); the step at
// level h writes its majorities to the vote array and the fan-in stops there.
//
// Bit-identical to the LEVELS pipeline: same lie keying (level, global slot
// pair, global word), same majorities and epilogue.
//
// The carry-save thresholds here use the resolve-then-compare form: the level-bit
// form (Csa::ge_from, the WAVE kernels' default) took k_cascade<16,5> from 126
// to 142 VGPRs (4 -> 3 waves per SIMD) for ~1% fewer instructions.
#define BA_CSA_GE_RESOLVE 1
#include "ba_wave.hpp"
#include "../../include/ba.h"  // BA_C_CHECK_MISMATCH

namespace ba {

// Lab builds only (tools/casc_stamps.sh compiles this file with
// -DBA_CASC_STAMPS into a separate library): every wave of the units launch
// records s_memtime at its phase boundaries, its HW_ID / XCC_ID and
// s_memrealtime at entry and exit, read back by ba_lab_casc_stamps_read.  The
// product build compiles none of it.
#ifdef BA_CASC_STAMPS
constexpr uint32_t kStampWaves = 1u << 16, kStampWords = 12;
extern "C" __device__ unsigned long long ba_lab_casc_stamps[kStampWaves][kStampWords];
__device__ unsigned long long ba_lab_casc_stamps[kStampWaves][kStampWords];
#define CASC_STAMP(i) (st_[i] = __builtin_amdgcn_s_memtime())
// k_cascade_mtop's wave 0 (and the root step it may take): one row per block
extern "C" __device__ unsigned long long ba_lab_mtop_stamps[kStampWaves][16];
__device__ unsigned long long ba_lab_mtop_stamps[kStampWaves][16];
#define CASC_MSTAMP(i)                                                                   \
    do {                                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kStampWaves)                         \
            ba_lab_mtop_stamps[blockIdx.x][i] = (i) >= 14 ? __builtin_amdgcn_s_memrealtime() \
                                                          : __builtin_amdgcn_s_memtime(); \
    } while (0)
#define CASC_MVAL(i, v)                                                                  \
    do {                                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kStampWaves) ba_lab_mtop_stamps[blockIdx.x][i] = (v); \
    } while (0)
#else
#define CASC_STAMP(i) ((void)0)
#define CASC_MSTAMP(i) ((void)0)
#define CASC_MVAL(i, v) ((void)0)
#endif

constexpr int kCascMaxLevels = 8;
constexpr uint32_t kCascCounterStride = 32;  // uint32 per counter: one 128-B line each
// waves per block (one-wave blocks, so that a wave taking fan-in steps holds
// only its own slot, measured no faster: 70.6 vs 69.9 us, n=16 m=5 x 1024)
constexpr uint32_t kCascWaves = 4;

struct CascArgs {
    uint64_t seed;
    GenSpec gs;
    uint64_t first_trial;  // global index of the chunk's trial 0
    uint64_t ntrials;      // trials of this chunk
    uint32_t W;            // words of this chunk
    uint32_t units;        // W * rr
    uint32_t rr;           // units (level-Q slots) per word: |L_Q|, or the range's share
    uint32_t rho0;         // first level-Q slot of the range (0: whole tree)
    const uint32_t* faulty;  // chunk-relative (GIVEN), or nullptr
    const uint8_t* order;
    const uint8_t* sender;   // Geometry::sender
    uint32_t snd_off[kCascMaxLevels];
    const uint64_t* members;  // level me-2 leaf-block member ids, 5 bits each
    uint64_t* R[kCascMaxLevels];    // R_k, k = 1..me-2: [W][groups][casc_pad] (casc_addr)
    uint64_t* tag[kCascMaxLevels];  // CHECK: the same layout, epoch tags
    uint64_t epoch;                 // CHECK: this launch's tag
    uint32_t inject;                // CHECK: 1 = unit 0 stores a stale tag (detector test)
    uint64_t wait_ticks;            // bound of every granule poll (s_memrealtime ticks, 100 MHz)
    uint32_t* cnt;                // counters [..] x kCascCounterStride
    uint32_t cnt_off[kCascMaxLevels];  // level k (0..Q-1) counters of word w at cnt_off[k] + w*|L_k|;
                                       // cnt_off[Q]: the word's root counter at cnt_off[Q] + w
    uint32_t h;           // range mode: the vote level (1 or 2); 0 = whole tree
    uint32_t ub;          // range mode: first h-hop subtree of the range
    uint32_t ue;          // range mode: one past the last
    uint32_t s0b, s0n;    // k_cascade_mtop: its level-(me-5) slots per word, [s0b, s0b + s0n)
    uint32_t nub;         // CO launches: blocks [0, nub) run units, the rest the fan-in
    uint64_t* votes;      // range mode: [(u - ub)(L - h) + c][W]
    const uint64_t* vin;  // root mode: every unit's votes, [level-h slot][W]
    uint64_t* decisions;  // chunk-relative
    uint8_t* outcome;
    uint64_t* counters;   // nullptr in range mode
    Sink sk;
};

// |L_k| = P(L, k+1)
constexpr uint32_t casc_sz(int L, int k) {
    uint32_t p = 1;
    for (int i = 0; i <= k; ++i) p *= (uint32_t)(L - i);
    return p;
}
// R_k (k >= 1) is stored in groups: the children of one level k-1 slot's
// children, i.e. one step's whole input block (L-k+1)(L-k) words (k = 1: the
// word's root step), each group padded to whole 128-B lines.
constexpr uint32_t casc_grp(int L, int k) { return (uint32_t)((L - k + 1) * (L - k)); }
constexpr uint32_t casc_pad(int L, int k) { return (casc_grp(L, k) + 15u) & ~15u; }
constexpr uint32_t casc_ngrp(int L, int k) { return k >= 2 ? casc_sz(L, k - 2) : 1u; }
// R_1 (the hand-off into the roots) is stored as granules: two 8-byte {value
// half, epoch tag} words per value (casc_put / casc_kids), so its level takes
// twice the words
// (and in CO launches so is R_{me-2}, the units' hand-off: `gran`)
constexpr uint64_t casc_level_words(int L, int k, bool gran = false) {
    return (uint64_t)casc_ngrp(L, k) * casc_pad(L, k) * (k == 1 || gran ? 2u : 1u);
}

template <int N, int ME>
struct Casc {
    static constexpr int L = N - 1, S = N - ME, G = S + 1, GP = G + 1, GPW = 64 / G;
    static constexpr int Q = ME - 3, NIN = N + 3;
    static constexpr uint32_t sz(int k) { return casc_sz(L, k); }
    // word w's level-k slot x (k >= 1) in R_k / tag_k
    template <int k>
    static __device__ __forceinline__ uint64_t addr(uint32_t w, uint32_t x) {
        constexpr uint32_t gk = casc_grp(L, k);
        const uint32_t grp = x / gk;
        return ((uint64_t)w * casc_ngrp(L, k) + grp) * casc_pad(L, k) + (x - grp * gk);
    }
    static constexpr int tr_words = GPW * G * GP;  // per wave: [unit][receiver][sender] transpose
    // fewest units per word: a range of one h-hop subtree with h = Q (L - Q
    // level-Q slots), or the whole |L_Q| at Q = 0
    static constexpr uint32_t rr_min = Q >= 1 ? (uint32_t)(L - Q) : casc_sz(L, Q);
    // words a block's 4 * GPW units can span, and their input planes
    static constexpr uint32_t nw_max = (kCascWaves * GPW + rr_min - 1) / rr_min + 1;
    static constexpr uint32_t planes_words = (nw_max * NIN + 1u) & ~1u;
};

// The units' lane layout: one lane per level-(me-2) slot, or two (LAT: latency
// mode, leaf_half), G slots per unit, GPW units per wave.
template <int N, int ME, bool LAT>
struct CascU {
    using C = Casc<N, ME>;
    static constexpr int LPS = LAT ? 2 : 1, GL = C::G * LPS, GPW = 64 / GL;
    static constexpr int tr_words = GPW * C::G * C::GP;
    static constexpr uint32_t nw_max = (kCascWaves * GPW + C::rr_min - 1) / C::rr_min + 1;
    static constexpr uint32_t planes_words = (nw_max * C::NIN + 1u) & ~1u;
};

// CHECK: the tag stored beside every R word of one launch
__device__ __forceinline__ uint64_t casc_tag(uint64_t epoch) { return epoch | (~epoch << 32); }

__device__ __forceinline__ uint64_t sel64(uint64_t f, uint64_t a, uint64_t b) { return (f & a) | (~f & b); }

// the lie word of level-k slot x of trial word gw: half x%2 of Philox pair x/2
__device__ __forceinline__ uint64_t lie_word(uint64_t seed, uint32_t k, uint32_t x, uint64_t gw) {
    uint64_t l0, l1;
    lie_pair(seed, k, x >> 1, gw, l0, l1);
    return (x & 1u) ? l1 : l0;
}

// ---------------------------------------------------------------------------
// Latency mode: one leaf block on TWO lanes (lanes 2x, 2x+1 of a unit), for
// batches too small to fill the chip, where a lane's chain of S(S-1)/2 Philox
// calls in a row is the units' time.  Lane h = 1 works in MIRRORED labels:
// member a is its member S-1-a.  Mirroring maps slot e = a(S-1) + c of the
// block to E-1-e (E = S(S-1)), so Philox pair q to NPAIR-1-q with the two
// halves swapped, and receiver b to S-1-b.  Both lanes then run ONE compile-time
// schedule in their own labels (SIMD code cannot branch per lane): rows
// 0..M-1 (M = (S-1)/2) whole, row M's first floor(NPR/2) pairs (NPR = pairs
// per row), and for odd NPR row M's middle pair, whose first local half only
// each lane counts (lane 0: actual receiver M-1, lane 1: M+1).  Lane 0 covers
// actual rows 0..M-1, lane 1 rows S-1..M+1, row M is shared: every pair once,
// the middle pair on both lanes (one call of S(S-1)/2 extra per lane pair).
// Counts are partial per receiver; each lane adds its partner's count of the
// same actual receiver (its own index S-1-b, one DPP swap per word) and takes
// the majority: RL[b] = R of local receiver b, on both lanes.  S odd only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t swap_pair64(uint64_t v) {
    return (uint64_t)swap_pair((uint32_t)(v >> 32)) << 32 | swap_pair((uint32_t)v);
}

struct LeafHalf {
    // step k of a lane's schedule -> local (row i, pair cp); half 1 used unless mid
    static constexpr int rows(int S) { return (S - 1) / 2; }
    static constexpr int npr(int S) { return (S - 1) / 2; }
    static constexpr int steps(int S) {
        return rows(S) * npr(S) + npr(S) / 2 + (npr(S) % 2 == 1 ? 1 : 0);
    }
    static constexpr int row(int S, int k) {
        return k < rows(S) * npr(S) ? k / npr(S) : rows(S);
    }
    static constexpr int cp(int S, int k) {
        return k < rows(S) * npr(S) ? k % npr(S) : k - rows(S) * npr(S);
    }
    static constexpr bool mid(int S, int k) { return npr(S) % 2 == 1 && k == steps(S) - 1; }
    static constexpr int recv(int S, int k, int h) {
        const int c = 2 * cp(S, k) + h, i = row(S, k);
        return c + (c >= i ? 1 : 0);
    }
    // adds receiver b's counter holds before step k half h (slot 0: its diag)
    static constexpr int before(int S, int b, int k, int h) {
        int n = 1;
        for (int u = 0; u <= k; ++u)
            for (int hh = 0; hh < 2; ++hh) {
                if (u == k && hh >= h) return n;
                if (hh == 1 && mid(S, u)) continue;
                if (recv(S, u, hh) == b) ++n;
            }
        return n;
    }
    static constexpr int total(int S, int b) { return before(S, b, steps(S), 0); }
    static constexpr int max_total(int S) {
        int m = 0;
        for (int b = 0; b < S; ++b) m = total(S, b) > m ? total(S, b) : m;
        return m;
    }
};

template <int NB>
__device__ __forceinline__ uint64_t ge_bits(const uint64_t (&s)[NB], int th) {
    // s (binary digits) >= th, MSB first
    uint64_t gt = 0, eq = ~0ull;
#pragma unroll
    for (int i = NB - 1; i >= 0; --i) {
        if ((th >> i) & 1) {
            eq &= s[i];
        } else {
            gt |= eq & s[i];
            eq &= ~s[i];
        }
    }
    return gt | eq;
}

template <int S>
__device__ __forceinline__ void leaf_half(uint32_t me, uint64_t seed, uint64_t gw, uint32_t sr, uint32_t h,
                                          const uint64_t (&diagL)[S], const uint64_t (&FmL)[S],
                                          uint64_t (&RL)[S]) {
    static_assert(S % 2 == 1 && S >= 3, "leaf_half: odd S");
    using LH = LeafHalf;
    constexpr int NPAIR = S * (S - 1) / 2, NST = LH::steps(S);
    constexpr int NL = planes_c(LH::max_total(S));
    constexpr int PG = NST % 4 == 0 ? 4 : (NST % 3 == 0 ? 3 : 4);
    Csa<NL> cnt[S];
    const uint64_t dmask = h ? 0ull : ~0ull;  // each receiver's own value: lane 0 counts it
    static_for<0, S>([&](auto b) { cnt[b()].template add<0>(diagL[b()] & dmask); });
    const uint32_t base = sr * (uint32_t)NPAIR + (h ? (uint32_t)(NPAIR - 1) : 0u);
    static_for<0, (NST + PG - 1) / PG>([&](auto grp) {
        constexpr int k0 = grp() * PG, ng = NST - k0 < PG ? NST - k0 : PG;
        P4 c[ng];
        static_for<0, ng>([&](auto g) {
            constexpr uint32_t kp = (uint32_t)(LH::row(S, k0 + g()) * ((S - 1) / 2) + LH::cp(S, k0 + g()));
            uint32_t cx = h ? base - kp : base + kp;
            asm("" : "+v"(cx));
            c[g()] = P4{cx, me, (uint32_t)gw, (uint32_t)(gw >> 32)};
        });
        philox10_n<ng>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        static_for<0, ng>([&](auto g) {
            constexpr int k = k0 + g(), i = LH::row(S, k);
            const uint64_t w0 = (uint64_t)c[g()].y << 32 | c[g()].x, w1 = (uint64_t)c[g()].w << 32 | c[g()].z;
            static_for<0, 2>([&](auto hh) {
                if constexpr (!(hh() == 1 && LH::mid(S, k))) {
                    constexpr int b = LH::recv(S, k, hh());
                    constexpr int K = LH::before(S, b, k, hh());
                    const uint64_t lw = (hh() == 0) == (h == 0) ? w0 : w1;  // lane 1: halves swapped
                    cnt[b].template add<K>((FmL[i] & lw) | (~FmL[i] & diagL[i]));
                }
            });
        });
    });
    // full counts: mine of local b plus the partner's of the same actual receiver
    static_for<0, S>([&](auto b) {
        constexpr int KM = LH::total(S, b()), KP = LH::total(S, S - 1 - b());
        uint64_t rm[NL], rp[NL], s[NL + 1];
        cnt[b()].template resolve<0, KM, false>(rm, 0);
        cnt[S - 1 - b()].template resolve<0, KP, false>(rp, 0);
        uint64_t cy = 0;
        static_for<0, NL>([&](auto l) {
            const uint64_t p = swap_pair64(rp[l()]);
            s[l()] = rm[l()] ^ p ^ cy;
            cy = (rm[l()] & p) | (cy & (rm[l()] ^ p));
        });
        s[NL] = cy;
        RL[b()] = ge_bits<NL + 1>(s, S / 2 + 1);  // S inputs, strict majority
    });
}

// L_K[x] (level-K slot x) of the word whose planes are `in`: the relay chain
// from the commander (L_0 = commander's coin or order, ba.py:263-285), each
// level relayed by the last general of the slot above (ba.py:42-57).
template <int N, int K>
__device__ __forceinline__ uint64_t chain_value(const CascArgs& a, const uint64_t* in, uint32_t x,
                                                uint64_t gw) {
    constexpr int L = N - 1;
    uint32_t anc[K + 1];
    anc[K] = x;
    static_for<0, K>([&](auto i) {
        constexpr int k = K - 1 - i();
        anc[k] = anc[k + 1] / (uint32_t)(L - (k + 1));
    });
    uint64_t v = in[N];  // OB
    static_for<0, K + 1>([&](auto k) {
        uint32_t snd = 0;  // level 0: the commander relays
        if constexpr (k() > 0) snd = a.sender[a.snd_off[k() - 1] + anc[k() - 1]];
        v = sel64(in[snd], lie_word(a.seed, k(), anc[k()], gw), v);
    });
    return v;
}

// Lieutenant indices j[0..K] of the path of level-K slot x (lexicographic rank
// over (K+1)-permutations of the L lieutenants): digit k is the rank of j[k]
// among the lieutenants not in j[0..k-1], picked by one compare-increment per
// earlier pick against the picks kept sorted (srt, ascending).
template <int L, int K>
__device__ __forceinline__ void unrank_path(uint32_t x, uint32_t (&j)[K + 1], uint32_t (&srt)[K + 1]) {
    uint32_t c[K + 1];
    static_for<0, K>([&](auto i) {
        constexpr int k = K - i();
        c[k] = x % (uint32_t)(L - k);
        x /= (uint32_t)(L - k);
    });
    c[0] = x;
    static_for<0, K + 1>([&](auto k) {
        uint32_t pos = c[k()];
        static_for<0, k()>([&](auto i) { pos += srt[i()] <= pos ? 1u : 0u; });
        j[k()] = pos;
        uint32_t v = pos;  // sorted insert
        static_for<0, k()>([&](auto i) {
            const uint32_t lo = srt[i()] < v ? srt[i()] : v, hi = srt[i()] < v ? v : srt[i()];
            srt[i()] = lo;
            v = hi;
        });
        srt[k()] = v;
    });
}

// Relay values of NS consecutive level-KS slots base..base+NS-1 below the
// level-(KS-1) slot `s` (or below the commander at KS = 0), one per lane of a
// group of NL lanes (lane t < NS: slot base + t), drawn cooperatively: the
// distinct Philox pairs -- the pairs of the NS slots and one pair per ancestor
// level of s -- are spread over the group's lanes (call c on lane c % NL) and
// exchanged through the group's LDS `xch` (>= 2 * (NPR + KS) words)
// (relay_draw: no input planes needed), then every lane relays the chain down
// from the commander (relay_apply, ba.py:257-285, 42-57).  path: the
// lieutenants of s (j[0..KS-1]); inactive lanes draw but never write; every
// lane of the wave must call both.
template <int N, int KS, int NS>
struct RelayPlan {
    static constexpr int L = N - 1, NPR = NS / 2 + 1, CALLS = NPR + KS;
    uint32_t anc[KS > 0 ? KS : 1];
    uint32_t p0;
    __device__ __forceinline__ RelayPlan(uint32_t s, uint32_t base) : p0(base >> 1) {
        if constexpr (KS > 0) {
            anc[KS - 1] = s;
            static_for<0, KS - 1>([&](auto i) {
                constexpr int k = KS - 2 - i();
                anc[k] = anc[k + 1] / (uint32_t)(L - (k + 1));
            });
        }
    }
};

template <int N, int KS, int NS, int NL>
__device__ __forceinline__ void relay_draw(const CascArgs& a, const RelayPlan<N, KS, NS>& rp,
                                           uint64_t* xch, uint32_t t, bool active, uint64_t gw) {
    using RP = RelayPlan<N, KS, NS>;
    constexpr int ROUNDS = (RP::CALLS + NL - 1) / NL;
    static_for<0, ROUNDS>([&](auto rd) {
        const uint32_t c = t + (uint32_t)(rd() * NL);  // this lane's call
        uint32_t lvl = KS, pair = rp.p0 + c;
        static_for<0, KS>([&](auto k) {
            if (c == (uint32_t)(RP::NPR + k())) {
                lvl = k();
                pair = rp.anc[k()] >> 1;
            }
        });
        uint64_t l0, l1;
        lie_pair(a.seed, lvl, pair, gw, l0, l1);
        if (active && c < (uint32_t)RP::CALLS) {
            xch[2 * c] = l0;
            xch[2 * c + 1] = l1;
        }
    });
}

template <int N, int KS, int NS>
__device__ __forceinline__ uint64_t relay_apply(const RelayPlan<N, KS, NS>& rp, const uint64_t* in,
                                                const uint64_t* xch, uint32_t t, uint32_t base,
                                                const uint32_t* path) {
    using RP = RelayPlan<N, KS, NS>;
    uint64_t v = in[N];  // OB: the commander's order
    static_for<0, KS>([&](auto k) {
        uint32_t snd = 0;  // level 0: the commander relays
        if constexpr (k() > 0) snd = path[k() - 1] + 1;
        v = sel64(in[snd], xch[2 * (RP::NPR + k()) + (rp.anc[k()] & 1u)], v);
    });
    const uint32_t x = base + (t < (uint32_t)NS ? t : 0u);
    uint32_t snd = 0;
    if constexpr (KS > 0) snd = path[KS - 1] + 1;
    return sel64(in[snd], xch[2 * ((x >> 1) - rp.p0) + (x & 1u)], v);
}

template <int N, int KS, int NS, int NL>
__device__ __forceinline__ uint64_t relay_slots(const CascArgs& a, const uint64_t* in, uint64_t* xch,
                                                uint32_t t, bool active, uint32_t s, uint32_t base,
                                                const uint32_t* path, uint64_t gw) {
    const RelayPlan<N, KS, NS> rp(s, base);
    relay_draw<N, KS, NS, NL>(a, rp, xch, t, active, gw);
    __builtin_amdgcn_wave_barrier();
    const uint64_t r = relay_apply<N, KS, NS>(rp, in, xch, t, base, path);
    __builtin_amdgcn_wave_barrier();  // xch is reused by the caller
    return r;
}

// No agent-scope acquire before the children are read: it would invalidate
// this CU's L1 and nothing else (MI355X_MICROARCH.md, fence table), and every
// child load is an sc1 load, which bypasses L1; with the child blocks padded to
// lines of their own no L2 holds a line of a hand-off before its reader loads
// it.  Measured cost of the acquire (round 4's A/B build): +4.1 us per
// 1024-instance n=16 m=5 call, +1.3 us per single instance
// (profiles/r04a_acquire_ab.log).

// R_1 granules (MI355X_MICROARCH.md's R2 form, cdna_hip_programming.md
// Guideline 16): each 32-bit half of an R_1 word travels with the launch's
// 32-bit tag in ONE aligned 8-byte sc1 store, so the data is its own flag: the
// producer does not drain before its arrival, and the consumer (the step that
// completes the word's root counter) re-reads every granule until all carry
// the tag -- bounded: the stores were issued before the arrivals that let the
// consumer in.  The consumer then zeroes the granules it read, so a replayed
// launch (a captured graph repeats its epoch argument) never sees an old tag;
// the tag is never 0.
// Every poll of a granule is bounded in time (s_memrealtime, 100 MHz): 2 s in
// the product -- long enough that a launch descheduled by another process's
// work is not taken for a lost hand-off -- and 200 ms in the check build, whose
// stale-tag injection waits out the bound once per launch.  A granule still
// stale at the bound (never in a correct run) is counted into slot 14.
// The bound is a launch argument (CascArgs::wait_ticks): kCascWaitTicks, or
// kCascWaitTicksCheck in the check build; BA_TEST_GRANULE_TICKS (tests only)
// shrinks it so a launch times out.  A timed-out launch's results are invalid,
// and every host entry point that reads the counters back returns BA_EDEVICE
// for it (ba_api.cpp handoff_lost, ba_multi.cpp finish_job).
constexpr uint64_t kCascWaitTicks = 200000000ull, kCascWaitTicksCheck = 20000000ull;
__device__ __forceinline__ uint32_t casc_gtag(uint64_t epoch) { return ((uint32_t)epoch << 1) | 1u; }

// A relay value computed ahead of its step (CO fan-in blocks), or none.
struct Pre {
    bool on = false;
    uint64_t v = 0;
};

// R store of one hand-off word (+ its tag in CHECK builds): write-through;
// level 1 as two granules
template <int N, int ME, int k, bool CHECK>
__device__ __forceinline__ void casc_put(const CascArgs& a, uint32_t w, uint32_t x, uint64_t v,
                                         bool stale = false) {
    const uint64_t i = Casc<N, ME>::template addr<k>(w, x);
    if constexpr (k == 1) {
        const uint64_t tag = (uint64_t)casc_gtag(stale ? a.epoch - 1 : a.epoch) << 32;
        store_sc1(a.R[1] + 2 * i, tag | (uint32_t)v);
        store_sc1(a.R[1] + 2 * i + 1, tag | (uint32_t)(v >> 32));
    } else {
        store_sc1(a.R[k] + i, v);
        if constexpr (CHECK) store_sc1(a.tag[k] + i, casc_tag(stale ? a.epoch - 1 : a.epoch));
    }
}

// Step q for sigma (level q-1 slot s; q = 0: the word's roots), run by one
// whole wave, lane r = receiver index among the K = L - q lieutenants not in
// sigma.  in: the word's input planes (LDS); scr: the wave's LDS scratch.
// mm: CHECK builds' per-lane count of child tags that were not this launch's.
// VIN: the children are rows of the gathered vote array a.vin (the root pass of
// the subtree split: written by an earlier launch / RCCL, plain loads), not a
// hand-off of this launch.
// The children of sigma at step q: R_{q+1}[sigma.j.r], j != r -- child
// c = r - (r > j) of level-q slot s*K + j (sigma's child block: one padded
// group of R_{q+1}), or the vote rows (VIN).  Issued before the relay of
// L_q[sigma.r], so its Philox work covers their latency.
template <int N, int ME, int q, bool CHECK, bool VIN>
__device__ __forceinline__ void casc_kids(const CascArgs& a, uint32_t lane, uint32_t w, uint32_t s,
                                          uint64_t (&cv)[N - 1 - q - 1], uint32_t& mm) {
    using C = Casc<N, ME>;
    constexpr int L = C::L, K = L - q;
    const bool act = lane < (uint32_t)K;
    const uint32_t r = act ? lane : 0u;
    static_assert(q > 0 || VIN, "the roots read R_1 granules: casc_root_step");
    static_for<0, K - 1>([&](auto jj) {
        const uint32_t j = (uint32_t)jj() + ((uint32_t)jj() >= r ? 1u : 0u);
        const uint32_t x = (s * (uint32_t)K + j) * (uint32_t)(K - 1) + r - (r > j ? 1u : 0u);
        if constexpr (VIN) {  // vote row = level-(q+1) slot, W words per row
            cv[jj()] = act ? a.vin[(uint64_t)x * a.W + w] : 0ull;
        } else {
            const uint64_t i = C::template addr<q + 1>(w, x);
            cv[jj()] = act ? load_sc1(a.R[q + 1] + i) : 0ull;
            if constexpr (CHECK) {
                if (act && load_sc1(a.tag[q + 1] + i) != casc_tag(a.epoch)) ++mm;
            }
        }
    });
}

template <int N, int ME, int q, bool CHECK, bool VIN = false>
__device__ __forceinline__ void casc_step(const CascArgs& a, const uint64_t* in, uint64_t* scr,
                                          uint32_t lane, uint32_t w, uint32_t s, uint64_t gw,
                                          TrialCounts& tc, uint32_t& mm, Pre l0 = Pre{});

// The word's per-lane run counts of a one-word epilogue (wave_epilogue, W = 1:
// only lanes 0..7, one byte of trials each, hold counts) to lane c = counter c:
// an 8-lane sum by DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror: three
// VALU adds per counter, where 64-lane __shfl_xor sums took six LDS permutes in a
// row -- ~1 us on the tail of a one-instance call), then lane 0's totals spread.
__device__ __forceinline__ uint64_t word_counts_to_lanes(const TrialCounts& tw, uint32_t lane) {
    uint64_t mine = 0;
#pragma unroll
    for (int c = 0; c < C_NUM; ++c) {
        uint32_t x = tw.v[c];
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
        if (lane == (uint32_t)c) mine = tot;
    }
    return mine;
}

// The roots of word w from L_0 (lq) and the level-1 results cv: strict
// majority attacks, a tie is undefined (ba.py:188-195); the quorum epilogue
// (ba.py:197-255) and the word's counts into the counter sink.
template <int N, int ME>
__device__ __forceinline__ void casc_roots(const CascArgs& a, const uint64_t* in, uint64_t* scr,
                                           uint32_t lane, uint32_t w, uint64_t lq,
                                           const uint64_t (&cv)[N - 2]) {
    using C = Casc<N, ME>;
    constexpr int L = C::L, K = L, NIN = C::NIN;
    const bool act = lane < (uint32_t)K;
    const uint32_t r = act ? lane : 0u;
    Csa<planes_c(K)> cnt;
    cnt.template add<0>(lq);
    static_for<0, K - 1>([&](auto jj) { cnt.template add<jj() + 1>(cv[jj()]); });
    const uint64_t att = cnt.template ge<K, K / 2 + 1>();
    const uint64_t tie = (K % 2 == 0) ? (cnt.template ge<K, K / 2>() & ~att) : 0ull;
    // the epilogue overwrites bytes of its input planes: a private copy
    if (lane < (uint32_t)NIN) scr[lane] = in[lane];
    if (act) {
        scr[NIN + r] = att;
        scr[NIN + L + r] = tie;
    }
    __builtin_amdgcn_wave_barrier();
    TrialCounts tw;
    wave_epilogue<N, 1, (uint32_t)ME, 0>(scr, scr + NIN, lane, w, a.ntrials, a.decisions, a.outcome, tw);
    __builtin_amdgcn_wave_barrier();
    CASC_MSTAMP(10);
    // the word's counts, straight into the sink: every word's root step runs
    // exactly once per launch, so the word is the sink's unit and no block
    // barrier is needed to combine waves (a wave exits as soon as it is done)
    const uint64_t mine = word_counts_to_lanes(tw, lane);
    if (a.counters) sink_counters(lane, mine, w, a.W, a.counters, a.sk);
    CASC_MSTAMP(11);
}

// The root step of word w in a launch that handed R_1 off (the last arrival at
// the word's root counter): the R_1 granules' loads go out first, L_0 is relayed
// while they land, then every granule's tag is checked -- re-read (bounded)
// until all are this launch's -- and the granules are zeroed for the next launch
// (each has exactly one reader: receiver r of its slot).
template <int N, int ME, bool CHECK>
__device__ __forceinline__ void casc_root_step(const CascArgs& a, const uint64_t* in, uint64_t* scr,
                                               uint32_t lane, uint32_t w, uint64_t gw, uint32_t& mm,
                                               Pre l0 = Pre{}) {
    using C = Casc<N, ME>;
    constexpr int L = C::L, K = L;
    const bool act = lane < (uint32_t)K;
    const uint32_t r = act ? lane : 0u;
    const uint32_t tag = casc_gtag(a.epoch);
    uint64_t* gp[K - 1];
    uint64_t g0[K - 1], g1[K - 1];
    static_for<0, K - 1>([&](auto jj) {
        const uint32_t j = (uint32_t)jj() + ((uint32_t)jj() >= r ? 1u : 0u);
        gp[jj()] = a.R[1] + 2 * C::template addr<1>(w, j * (uint32_t)(K - 1) + r - (r > j ? 1u : 0u));
        g0[jj()] = act ? load_sc1(gp[jj()]) : 0ull;
        g1[jj()] = act ? load_sc1(gp[jj()] + 1) : 0ull;
    });
    uint32_t path[1];
    // l0: L_0 relayed ahead (a CO fan-in block does it while it waits)
    const uint64_t lq = l0.on ? l0.v : relay_slots<N, 0, K, 64>(a, in, scr, lane, true, 0u, 0u, path, gw);
    CASC_MSTAMP(9);
    auto fresh = [&]() {
        bool ok = true;
        static_for<0, K - 1>([&](auto jj) {
            ok &= !act || ((uint32_t)(g0[jj()] >> 32) == tag && (uint32_t)(g1[jj()] >> 32) == tag);
        });
        return ok;
    };
    bool ok = fresh();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (!__all(ok) && __builtin_amdgcn_s_memrealtime() - t0 <= a.wait_ticks) {  // wave-uniform
        __builtin_amdgcn_s_sleep(1);
        static_for<0, K - 1>([&](auto jj) {
            g0[jj()] = act ? load_sc1(gp[jj()]) : 0ull;
            g1[jj()] = act ? load_sc1(gp[jj()] + 1) : 0ull;
        });
        ok = fresh();
    }
    // a granule still stale at the bound: never in a correct run.  Counted into
    // slot 14 (BA_C_CHECK_MISMATCH) so tests see it -- per stale lane in CHECK
    // builds (their stale-tag injection expects exactly one), once per wave
    // otherwise
    if constexpr (CHECK) {
        mm += ok ? 0u : 1u;
    } else {
        if (!__all(ok) && lane == 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), 1ull);
    }
    uint64_t cv[K - 1];
    static_for<0, K - 1>([&](auto jj) {
        cv[jj()] = (g1[jj()] << 32) | (uint32_t)g0[jj()];
        if (act) {
            store_sc1(gp[jj()], 0ull);
            store_sc1(gp[jj()] + 1, 0ull);
        }
    });
    casc_roots<N, ME>(a, in, scr, lane, w, lq, cv);
}

// Step q for sigma with its children cv already loaded: relay L_q[sigma.r],
// majority, then store + arrive (q > 0) or roots + epilogue (q = 0).
// lqp / l0 (CO fan-in blocks): L_q[sigma.lane] / L_0[lane] relayed ahead, while
// the block waited for the units.
template <int N, int ME, int q, bool CHECK>
__device__ __forceinline__ void casc_finish(const CascArgs& a, const uint64_t* in, uint64_t* scr,
                                            uint32_t lane, uint32_t w, uint32_t s, uint64_t gw,
                                            const uint64_t (&cv)[N - 1 - q - 1], TrialCounts& tc,
                                            uint32_t& mm, Pre lqp = Pre{}, Pre l0 = Pre{}) {
    using C = Casc<N, ME>;
    constexpr int L = C::L, K = L - q;
    const bool act = lane < (uint32_t)K;
    const uint32_t r = act ? lane : 0u;
    // L_q[sigma.r], sigma's path unranked (no tables)
    uint32_t path[q > 0 ? q : 1], srt[q > 0 ? q : 1];
    if constexpr (q > 0) unrank_path<L, q - 1>(s, path, srt);
    const uint64_t lq = lqp.on ? lqp.v
                               : relay_slots<N, q, K, 64>(a, in, scr, lane, true, s, s * (uint32_t)K, path, gw);
    CASC_MSTAMP(q == 0 ? 9 : 5);
    Csa<planes_c(K)> cnt;
    cnt.template add<0>(lq);
    static_for<0, K - 1>([&](auto jj) { cnt.template add<jj() + 1>(cv[jj()]); });
    if constexpr (q > 0) {
        const uint64_t rq = cnt.template ge<K, K / 2 + 1>();  // inner tie -> non-attack
        if (a.h == (uint32_t)q) {  // range mode: sigma's majorities are votes, the fan-in stops
            if (act) a.votes[((uint64_t)(s - a.ub) * K + r) * a.W + w] = rq;
            return;
        }
        if (act) casc_put<N, ME, q, CHECK>(a, w, s * (uint32_t)K + r, rq);
        CASC_MSTAMP(6);
        if constexpr (q != 1) drain_stores();  // R_1: granules, no drain before the arrival
        CASC_MSTAMP(7);
        // arrive at sigma's parent (level q-2), or at the word's root counter
        constexpr uint32_t up_fan = (uint32_t)(L - (q - 1));  // children of a level q-2 slot
        const uint32_t ps = s / up_fan;
        bool last_;
        if (q == 1 && a.nub != 0) {
            // a CO launch: no arrival -- the word's s0 = 0 block takes the roots,
            // polling the other blocks' R_1 granules (casc_root_step) as they land
            last_ = s == 0;
        } else {
            uint32_t* c;
            if constexpr (q - 1 >= 1)
                c = a.cnt + (uint64_t)(a.cnt_off[q - 2] + w * C::sz(q - 2) + ps) * kCascCounterStride;
            else
                c = a.cnt + (uint64_t)(a.cnt_off[C::Q] + w) * kCascCounterStride;
            last_ = arrive_last(c, up_fan, lane);
        }
        CASC_MSTAMP(8);
        if (last_) {
            casc_step<N, ME, q - 1, CHECK>(a, in, scr, lane, w, ps, gw, tc, mm, q == 1 ? l0 : Pre{});
        }
    } else {
        casc_roots<N, ME>(a, in, scr, lane, w, lq, cv);
        (void)tc;
        (void)l0;
    }
}


template <int N, int ME, int q, bool CHECK, bool VIN>
__device__ __forceinline__ void casc_step(const CascArgs& a, const uint64_t* in, uint64_t* scr,
                                          uint32_t lane, uint32_t w, uint32_t s, uint64_t gw,
                                          TrialCounts& tc, uint32_t& mm, Pre l0) {
    if constexpr (q == 0 && !VIN) {  // the word's roots from the R_1 granules
        (void)s;
        (void)tc;
        casc_root_step<N, ME, CHECK>(a, in, scr, lane, w, gw, mm, l0);
    } else {
        (void)l0;
        uint64_t cv[N - 1 - q - 1];
        casc_kids<N, ME, q, CHECK, VIN>(a, lane, w, s, cv, mm);
        casc_finish<N, ME, q, CHECK>(a, in, scr, lane, w, s, gw, cv, tc, mm);
    }
}

// The fan-in block's shape (k_cascade_mtop, and the fan-in blocks of a CO
// launch): one block per (word, level-(Q-2) slot s0), step Q for its NG sigmas.
template <int N, int ME>
struct CascMtop {
    using C = Casc<N, ME>;
    static constexpr int L = C::L, Q = C::Q, K = L - Q;  // step Q: K receivers per sigma
    static constexpr int NG = L - (Q - 1);                // sigmas per block (children of s0)
    static constexpr int GW = 64 / K;                     // sigma groups per wave
    static constexpr int NWV = (NG + GW - 1) / GW;        // waves per block
    static constexpr uint32_t PB = Q >= 2 ? C::sz(Q - 2) : 1u;  // blocks per word
    static constexpr int XW = 2 * RelayPlan<N, (Q >= 1 ? Q : 1), K>::CALLS;  // relay words per group
    // LDS words of one fan-in block: planes, relay exchange, R_Q of the sigmas, step scratch
    static constexpr uint32_t oXCH = (C::NIN + 1) & ~1, oRV = oXCH + NWV * GW * XW,
                              oSCR = oRV + ((NG * K + 1) & ~1), oXQ1 = oSCR + 64,
                              oX0 = oXQ1 + 2 * RelayPlan<N, (Q >= 1 ? Q - 1 : 0), NG>::CALLS,
                              words = oX0 + 2 * RelayPlan<N, 0, L>::CALLS;
};

// CO launches: one launch holds the units AND the fan-in blocks (blocks
// [nub, nub + W * PB)), so the units -> fan-in hop is no kernel boundary.  A
// fan-in block is k_cascade_mtop's, except that it starts while the units run:
// it draws its relays (and the later steps' Philox pairs) and slices its word's
// inputs at once, then each wave polls its sigmas' children R_{me-2} -- granules,
// {value half, epoch tag} in one 8-B sc1 store (MI355X_MICROARCH.md's R2 form),
// so the units neither drain nor count -- until every lane's carry this launch's
// tag, and zeroes them for the next launch (each granule has one reader).  The
// poll is bounded (a.wait_ticks of s_memrealtime; a granule still stale then is
// counted into BA_C_CHECK_MISMATCH, which the host turns into BA_EDEVICE).
// Forward progress rests on two things:
//  - in-order dispatch of one launch's blocks: the units blocks (which wait for
//    nothing) hold their slots before any fan-in block of the launch is placed;
//  - at me = 5 (PB > 1) the word's s0 = 0 fan-in block also polls the R_1
//    granules of its siblings s0 = 1..PB-1, which have HIGHER block indices: they
//    must find slots while s0 = 0 spins.  The host bounds the polling blocks of
//    all CO launches in flight on a device (ba_api.cpp co_admit: at most half
//    the chip's block slots), so slots stay free for them; past the bound a
//    call takes the two-launch cascade.

template <int N, int ME, bool CHECK>
__device__ __forceinline__ void casc_co_top(const CascArgs& a, uint64_t* lds, uint32_t bid) {
    using C = Casc<N, ME>;
    using M = CascMtop<N, ME>;
    constexpr int L = M::L, Q = M::Q, K = M::K, NG = M::NG, GW = M::GW;
    static_assert(Q >= 1 && M::NWV <= (int)kCascWaves, "CO fan-in: me >= 4, <= 4 waves");
    uint64_t* planes = lds + 0;
    uint64_t* xch = lds + M::oXCH;
    uint64_t* rv = lds + M::oRV;
    uint64_t* scr = lds + M::oSCR;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t w = bid / M::PB, s0 = bid - w * M::PB;
    const uint64_t gw = (a.first_trial >> 6) + w;
    const uint32_t g = lane / (uint32_t)K, r = lane - g * (uint32_t)K;
    const uint32_t j = wv * (uint32_t)GW + g;  // sigma = child j of s0
    const bool act = g < (uint32_t)GW && j < (uint32_t)NG;
    const uint32_t sg = s0 * (uint32_t)NG + (act ? j : 0u);
    TrialCounts tc;
    uint32_t mm = 0;
    if (wv == 0) {
        CASC_MSTAMP(14);
        CASC_MSTAMP(0);
    }
    // 1. everything that needs no unit: step Q's relay draws, the word's inputs
    const RelayPlan<N, Q, K> rp(sg, sg * (uint32_t)K);
    uint64_t* xg = xch + (act ? (wv * (uint32_t)GW + g) * (uint32_t)M::XW : 0u);
    relay_draw<N, Q, K, K>(a, rp, xg, r, act, gw);
    if (wv == 0) wave_inputs<N, 1, 0>(planes, lane, w, a.seed, a.gs, a.first_trial, a.ntrials, a.faulty, a.order);
    //    and the later steps' draws: L_{Q-1}[s0.*] (step Q-1) and L_0 (the
    //    roots, should this block's arrival be the word's last), off the chain
    //    that starts when the units are in
    if (wv == kCascWaves - 1) {
        relay_draw<N, Q - 1, NG, 64>(a, RelayPlan<N, Q - 1, NG>(s0, s0 * (uint32_t)NG), lds + M::oXQ1, lane,
                                     true, gw);
        if constexpr (Q - 1 > 0)
            relay_draw<N, 0, L, 64>(a, RelayPlan<N, 0, L>(0u, 0u), lds + M::oX0, lane, true, gw);
    }
    if (wv == 0) CASC_MSTAMP(1);
    __syncthreads();  // the planes (wave 0) and the later steps' draws (wave 3) are in LDS
    //    every relay value the block's steps need, while the units still run:
    //    L_Q[sigma.r] per group lane; wave 0 also L_{Q-1}[s0.lane] and L_0[lane]
    uint64_t lqQ = 0;
    if (act) {
        uint32_t path[Q], srt[Q];
        unrank_path<L, Q - 1>(sg, path, srt);
        lqQ = relay_apply<N, Q, K>(rp, planes, xg, r, sg * (uint32_t)K, path);
    }
    Pre p1, p0;
    if (wv == 0) {
        uint32_t path1[Q > 1 ? Q - 1 : 1], srt1[Q > 1 ? Q - 1 : 1];
        if constexpr (Q > 1) unrank_path<L, Q - 2>(s0, path1, srt1);
        p1.on = true;
        p1.v = relay_apply<N, Q - 1, NG>(RelayPlan<N, Q - 1, NG>(s0, s0 * (uint32_t)NG), planes, lds + M::oXQ1,
                                         lane, s0 * (uint32_t)NG, path1);
        if constexpr (Q > 1) {
            uint32_t path0[1];
            p0.on = true;
            p0.v = relay_apply<N, 0, L>(RelayPlan<N, 0, L>(0u, 0u), planes, lds + M::oX0, lane, 0u, path0);
        }
    }
    // 2. the children R_{Q+1}[sigma.jc.r], jc != r: granules, polled by each wave
    //    until all of its lanes' carry this launch's tag (the data is its own
    //    flag: no counter, no drain on the units' side), s_memrealtime-bounded
    const uint32_t tag = casc_gtag(a.epoch);
    uint64_t* gp[K - 1];
    uint64_t g0[K - 1], g1[K - 1];
    static_for<0, K - 1>([&](auto jj) {
        const uint32_t jc = (uint32_t)jj() + ((uint32_t)jj() >= r ? 1u : 0u);
        const uint32_t x = (sg * (uint32_t)K + jc) * (uint32_t)(K - 1) + r - (r > jc ? 1u : 0u);
        gp[jj()] = a.R[Q + 1] + 2 * C::template addr<Q + 1>(w, act ? x : 0u);
    });
    auto load_all = [&]() {
        static_for<0, K - 1>([&](auto jj) {
            g0[jj()] = act ? load_sc1(gp[jj()]) : 0ull;
            g1[jj()] = act ? load_sc1(gp[jj()] + 1) : 0ull;
        });
    };
    auto fresh = [&]() {
        bool ok = true;
        static_for<0, K - 1>([&](auto jj) {
            ok &= !act || ((uint32_t)(g0[jj()] >> 32) == tag && (uint32_t)(g1[jj()] >> 32) == tag);
        });
        return ok;
    };
    if (wv == 0) CASC_MSTAMP(2);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t polls = 0;
    load_all();
    bool ok = fresh();
    while (!__all(ok)) {  // wave-uniform
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.wait_ticks) break;
        __builtin_amdgcn_s_sleep(2);
        load_all();
        ok = fresh();
        ++polls;
    }
    if (wv == 0) {
        CASC_MVAL(12, __builtin_amdgcn_s_memrealtime());
        CASC_MVAL(13, (unsigned long long)polls);
    }
    (void)polls;
    if constexpr (CHECK) {
        mm += ok ? 0u : 1u;
    } else {
        if (!__all(ok) && lane == 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), 1ull);
    }
    uint64_t cv[K - 1];
    static_for<0, K - 1>([&](auto jj) {
        cv[jj()] = (g1[jj()] << 32) | (uint32_t)g0[jj()];
        if (act) {
            store_sc1(gp[jj()], 0ull);
            store_sc1(gp[jj()] + 1, 0ull);
        }
    });
    if (wv == 0) CASC_MSTAMP(3);
    // 4. step Q for the sigmas into LDS, then step Q-1 for s0 (k_cascade_mtop)
    if (act) {
        Csa<planes_c(K)> cnt;
        cnt.template add<0>(lqQ);
        static_for<0, K - 1>([&](auto jj) { cnt.template add<jj() + 1>(cv[jj()]); });
        rv[j * (uint32_t)K + r] = cnt.template ge<K, K / 2 + 1>();  // inner tie -> non-attack
    }
    __syncthreads();
    if (wv == 0) {
        CASC_MSTAMP(4);
        const uint32_t r1 = lane < (uint32_t)NG ? lane : 0u;
        uint64_t cv1[NG - 1];
        static_for<0, NG - 1>([&](auto jj) {
            const uint32_t j1 = (uint32_t)jj() + ((uint32_t)jj() >= r1 ? 1u : 0u);
            cv1[jj()] = rv[j1 * (uint32_t)K + r1 - (r1 > j1 ? 1u : 0u)];
        });
        casc_finish<N, ME, Q - 1, CHECK>(a, planes, scr, lane, w, s0, gw, cv1, tc, mm, p1, p0);
        CASC_MSTAMP(15);
    }
    if constexpr (CHECK) {
        uint32_t t = mm;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if (lane == 0 && t != 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), (unsigned long long)t);
    }
}

// One block = 4 * GPW consecutive units (their words: <= nw_max, sliced into
// LDS once).  Per wave:
//   1. every Philox draw that needs no input: the level me-1 diagonal lies of
//      the lane's leaf block and the unit's relay-chain lies (relay_draw) --
//      the slicing waves' input loads land meanwhile
//   2. inputs bit-sliced (one wave per word), block barrier
//   3. relay chain, leaf block, R_{me-2}[rho.x] = maj over the unit's
//      transpose, stored write-through
//   4. drain, one arrival per unit; a completed parent's steps run at once
// (A persistent, software-pipelined variant that deferred every drain and
// arrival by one block-iteration measured slower: 97.6 vs 74.6 us for n=16,
// m=5 at 1024 instances, at 207 VGPRs = 2 waves per SIMD.)
// DIAG: 2 = units only, no fan-in (the first launch of the two-launch mode,
// k_cascade_top does the fan-in; alone: the lab's units-only ablation), 4 =
// arrivals but no steps (lab only, tools/casc_lab.py, BA_CASC_DIAG; wrong
// results).  The one-launch product uses 0.
template <int N, int ME, int DIAG = 0, bool CHECK = false, bool LAT = false>
__global__ __launch_bounds__(64 * kCascWaves) void k_cascade(CascArgs a) {
    using C = Casc<N, ME>;
    using U = CascU<N, ME, LAT>;
    constexpr int L = C::L, S = C::S, G = C::G, GP = C::GP, GPW = U::GPW, NIN = C::NIN, Q = C::Q;
    constexpr int GL = U::GL;
    static_assert(!LAT || (DIAG & 2) != 0, "latency mode: units-only launches");
    constexpr bool CO = (DIAG & 8) != 0;  // units + co-resident fan-in blocks (casc_co_top)
    static_assert(!CO || ((DIAG & 2) != 0 && !LAT), "CO: units-only body, normal lanes");
    constexpr int NPD = (S + 1) / 2;
    constexpr uint32_t fan = (uint32_t)(L - Q);  // children of a level Q-1 slot (or of the root)
    using RP = RelayPlan<N, Q + 1, G>;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    if constexpr (CO) {
        if (blockIdx.x >= a.nub) {  // block-uniform
            casc_co_top<N, ME, CHECK>(a, lds, blockIdx.x - a.nub);
            return;
        }
    }
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t RR = a.rr;  // units per word
    const uint32_t u0 = blockIdx.x * kCascWaves * GPW;
    const uint32_t wfirst = u0 / RR, nw = (min(u0 + kCascWaves * GPW, a.units) - 1u) / RR - wfirst + 1u;
    uint64_t* planes = lds;  // [nw][NIN]
    uint64_t* tr = lds + U::planes_words + wv * (uint32_t)U::tr_words;
    const uint64_t gw0 = a.first_trial >> 6;
    TrialCounts tc;
    uint32_t mm = 0;  // CHECK: stale child tags seen by this lane
    const uint32_t g = lane / GL, y = lane - g * GL;  // y: the lane within its unit
    const uint32_t x = LAT ? y >> 1 : y, hh = LAT ? (y & 1u) : 0u;  // slot, half (LAT)
    const uint32_t u = u0 + wv * GPW + g;
    const bool act = g < (uint32_t)GPW && u < a.units;
#ifdef BA_CASC_STAMPS
    unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long rt_in = __builtin_amdgcn_s_memrealtime();
    CASC_STAMP(0);
#endif
    const uint32_t uu = act ? u : u0;
    const uint32_t w = uu / RR, rho = a.rho0 + (uu - w * RR);
    const uint64_t gw = gw0 + w;
    const uint32_t sr = rho * (uint32_t)G + x;  // the lane's level me-2 slot
    const uint32_t gg = act ? g : 0u;
    uint64_t* xch = tr + gg * (G * GP);  // the unit's relay exchange (before its transpose)
    // 0. staged inputs: the loads of this wave's word go out first, so the draws
    //    below hide their latency
    const bool staged = a.gs.faulty_mode == 0 && a.gs.order_mode == 0;
    uint32_t pfm = 0, poc = 0;
    const uint64_t pi = (uint64_t)(wfirst + wv) * 64 + lane;
    const bool pv = staged && wv < nw && pi < a.ntrials;
    if (pv) {
        pfm = a.faulty[pi];
        poc = a.order[pi];
    }
    // 1. input-free draws
    uint64_t lw[2 * NPD], mem = 0;
    const RP rp(rho, rho * (uint32_t)G);
    if (act) {
        mem = a.members[sr];
        if constexpr (LAT) {  // the slot's diagonal pairs split over its two lanes, swapped by DPP
            constexpr int NH = (NPD + 1) / 2;
            uint64_t mine[2 * NH], other[2 * NH];
            lie_pairs<NH>(a.seed, ME - 1, ((sr * (uint32_t)S) >> 1) + hh * (uint32_t)NH, gw, mine);
            static_for<0, 2 * NH>([&](auto i) { other[i()] = swap_pair64(mine[i()]); });
            static_for<0, 2 * NPD>([&](auto k) {
                if constexpr (k() < 2 * NH) lw[k()] = hh ? other[k()] : mine[k()];
                else lw[k()] = hh ? mine[k() - 2 * NH] : other[k() - 2 * NH];
            });
        } else {
            lie_pairs<NPD>(a.seed, ME - 1, (sr * (uint32_t)S) >> 1, gw, lw);
        }
        relay_draw<N, Q + 1, G, GL>(a, rp, xch, y, true, gw);
    }
    CASC_STAMP(1);
    // 2. inputs
    if (staged) {
        if (wv < nw) stage_slice<N>(planes + wv * NIN, lane, pfm, poc, pv);
        for (uint32_t k = wv + kCascWaves; k < nw; k += kCascWaves)  // blocks spanning > 4 words
            wave_inputs<N, 1, 0>(planes + k * NIN, lane, wfirst + k, a.seed, a.gs, a.first_trial,
                                 a.ntrials, a.faulty, a.order);
    } else {
        for (uint32_t k = wv; k < nw; k += kCascWaves)
            wave_inputs<N, 1, 0>(planes + k * NIN, lane, wfirst + k, a.seed, a.gs, a.first_trial,
                                 a.ntrials, a.faulty, a.order);
    }
    CASC_STAMP(2);
    __syncthreads();
    CASC_STAMP(3);
    // 3. the units (the leaf work sits in a divergent branch: as straight-line
    //    code for every lane the compiler's schedule needed 256 VGPRs and spilled)
    const uint64_t* in = planes + (w - wfirst) * NIN;
    if (act) {
        uint32_t path[Q + 2], srt[Q + 2];
        unrank_path<L, Q + 1>(sr, path, srt);
        const uint64_t par = relay_apply<N, Q + 1, G>(rp, in, xch, x, rho * (uint32_t)G, path);
        __builtin_amdgcn_wave_barrier();  // xch becomes the transpose below
        CASC_STAMP(4);
        const uint64_t fs = in[path[Q + 1] + 1];  // level me-1 relayer: the slot's last lieutenant
        const uint64_t oddmask = 0ull - (uint64_t)((sr * (uint32_t)S) & 1u);
        uint64_t diag[S], Fm[S], Rm[S];
        static_for<0, S>([&](auto b) {
            uint64_t lie;
            if constexpr (S % 2 == 1) lie = lw[b()] ^ ((lw[b()] ^ lw[b() + 1]) & oddmask);
            else lie = lw[b()];
            diag[b()] = sel64(fs, lie, par);
            if constexpr (LAT) {  // lane 1: mirrored member labels
                const uint32_t sh = hh ? 5u * (uint32_t)(S - 1 - b()) : 5u * (uint32_t)b();
                Fm[b()] = in[(mem >> sh) & 31u];
            } else {
                Fm[b()] = in[(mem >> (5 * b())) & 31u];
            }
        });
        if constexpr (LAT) {
            uint64_t diagL[S];
            static_for<0, S>([&](auto b) { diagL[b()] = hh ? diag[S - 1 - b()] : diag[b()]; });
            leaf_half<S>(ME, a.seed, gw, sr, hh, diagL, Fm, Rm);  // lane 0: actual labels
        } else {
            leaf_block<S>(ME, a.seed, gw, sr, diag, Fm, Rm);
        }
        CASC_STAMP(5);
        if (hh == 0) {
            uint64_t* t = tr + (gg * G) * GP + x;
            t[x * GP] = par;
            static_for<0, S>([&](auto d) { t[(d() + (d() >= x ? 1u : 0u)) * GP] = Rm[d()]; });
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (act && hh == 0) {
        const uint64_t* col = tr + (gg * G + x) * GP;
        Csa<planes_c(G)> cnt;
        static_for<0, G>([&](auto b) { cnt.template add<b()>(col[b()]); });
        const uint64_t rv = cnt.template ge<G, G / 2 + 1>();
        const bool stale = CHECK && a.inject && u == 0 && x == 0;
        if constexpr (CO) {  // two granules: the fan-in block polls them (no drain, no arrival)
            const uint64_t i = C::template addr<ME - 2>(w, sr);
            const uint64_t tg = (uint64_t)casc_gtag(stale ? a.epoch - 1 : a.epoch) << 32;
            store_sc1(a.R[ME - 2] + 2 * i, tg | (uint32_t)rv);
            store_sc1(a.R[ME - 2] + 2 * i + 1, tg | (uint32_t)(rv >> 32));
        } else {
            casc_put<N, ME, ME - 2, CHECK>(a, w, sr, rv, stale);
        }
    }
    __builtin_amdgcn_wave_barrier();
#ifdef BA_CASC_STAMPS
    CASC_STAMP(6);
    drain_stores();
    CASC_STAMP(7);
    {
        const uint32_t wid = blockIdx.x * kCascWaves + wv;
        if (lane == 0 && wid < kStampWaves) {
            for (int i = 0; i < 8; ++i) ba_lab_casc_stamps[wid][i] = st_[i];
            ba_lab_casc_stamps[wid][8] = rt_in;
            ba_lab_casc_stamps[wid][9] = __builtin_amdgcn_s_memrealtime();
            ba_lab_casc_stamps[wid][10] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) |
                ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)) << 32);
            ba_lab_casc_stamps[wid][11] = (unsigned long long)nw | ((unsigned long long)(act ? 1 : 0) << 32);
        }
    }
#endif
    if constexpr ((DIAG & 2) == 0) {
        if constexpr (ME - 2 != 1) drain_stores();  // R_1 (me = 3): granules, no drain
        // 4. arrivals: one lane per unit at the counter of rho's parent (level
        //    Q-1) or, at Q = 0, of the word
        bool last = false;
        if (act && x == 0) {
            uint32_t* c;
            if constexpr (Q >= 1)
                c = a.cnt + (uint64_t)(a.cnt_off[Q - 1] + w * C::sz(Q - 1) + rho / fan) * kCascCounterStride;
            else
                c = a.cnt + (uint64_t)(a.cnt_off[0] + w) * kCascCounterStride;
            const uint32_t old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = old + 1 == fan;
            if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint64_t lastmask = (DIAG & 4) ? 0ull : __ballot(last);
        while (lastmask) {  // wave-uniform: every lane runs each completed parent's step
            const uint32_t b = (uint32_t)__builtin_ctzll(lastmask);
            lastmask &= lastmask - 1;
            const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)w, (int)b);
            const uint32_t rb = (uint32_t)__builtin_amdgcn_readlane((int)rho, (int)b);
            casc_step<N, ME, Q, CHECK>(a, planes + (wb - wfirst) * NIN, tr, lane, wb,
                                       Q >= 1 ? rb / fan : 0u, gw0 + wb, tc, mm);
        }
    }
    if constexpr (CHECK) {
        uint32_t t = mm;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if (lane == 0 && t != 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), (unsigned long long)t);
    }
    // no end-of-block flush: the root steps put each word's counts into the sink
}

// ---------------------------------------------------------------------------
// k_cascade_top<N, ME, QS, VIN>: the fan-in from level QS up, in ONE launch,
// over children an earlier launch (or RCCL) wrote.  One wave per (word,
// level-(QS-1) slot sigma; QS = 0: the word) slices its word's inputs, relays
// L_QS[sigma.r] and takes step QS (casc_step); the levels above hand off as in
// k_cascade, and each word's root step runs the roots, the quorum epilogue
// (ba.py:159-255) and feeds the counter sink.  No wave waits for another and
// there is no block barrier.
//   VIN = true: the subtree split's root pass -- the children are the gathered
//     vote rows a.vin (QS = h-1).
//   VIN = false: the two-launch cascade -- the children are R_{QS+1} from a
//     units-only k_cascade launch (QS = me-3): the latency-bound steps no
//     longer hold wave slots that the compute-bound units could use.
// ---------------------------------------------------------------------------
template <int N, int ME, int QS, bool VIN, bool CHECK = false>
__global__ __launch_bounds__(64 * kCascWaves) void k_cascade_top(CascArgs a) {
    using C = Casc<N, ME>;
    constexpr int NIN = C::NIN;
    constexpr uint32_t PER = QS >= 1 ? C::sz(QS - 1) : 1u;  // waves per word
    constexpr uint32_t WS = 64;                              // step scratch words per wave
    __shared__ __attribute__((aligned(16))) uint64_t sh[kCascWaves][((NIN + 1) & ~1) + WS];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t u = blockIdx.x * kCascWaves + wv;
    if (u >= a.units) return;  // wave-uniform; no barrier follows
    const uint32_t w = u / PER, sg = u - w * PER;
    uint64_t* planes = sh[wv];
    uint64_t* scr = sh[wv] + ((NIN + 1) & ~1);
    TrialCounts tc;
    uint32_t mm = 0;
    // the children's loads go out first; the word's input loads and slicing and
    // the relay of L_QS then overlap their latency
    uint64_t cv[N - 1 - QS - 1];
    casc_kids<N, ME, QS, CHECK, VIN>(a, lane, w, sg, cv, mm);
    wave_inputs<N, 1, 0>(planes, lane, w, a.seed, a.gs, a.first_trial, a.ntrials, a.faulty, a.order);
    __builtin_amdgcn_wave_barrier();
    casc_finish<N, ME, QS, CHECK>(a, planes, scr, lane, w, sg, (a.first_trial >> 6) + w, cv, tc, mm);
    if constexpr (CHECK) {
        uint32_t t = mm;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if (lane == 0 && t != 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), (unsigned long long)t);
    }
}

// ---------------------------------------------------------------------------
// k_cascade_mtop<N, ME>: the two-launch fan-in with one hand-off fewer.  One
// block per (word, level-(Q-2) slot s0; Q = me-3 = the units' level; Q = 1: the
// word): step Q for EVERY child sigma of s0 at once -- one group of K = L-Q
// lanes per sigma, GW groups per wave, children R_{Q+1} from the units launch,
// each group drawing its own relay (relay_draw over the group's K lanes) -- into
// LDS, one block barrier, then step Q-1 for s0 by wave 0 with its children
// from LDS (casc_finish: relay, majority, then R_{Q-1} stored + the arrival at
// the root counter, the last arriver taking the roots, or at Q = 1 the roots
// and the epilogue directly).  k_cascade_top hands step Q's results to step
// Q-1 through memory (store, drain, returning add, reload); here that hop is
// one barrier.
// ---------------------------------------------------------------------------
template <int N, int ME, bool CHECK = false>
__global__ __launch_bounds__(256) void k_cascade_mtop(CascArgs a) {
    using C = Casc<N, ME>;
    using M = CascMtop<N, ME>;
    constexpr int L = M::L, Q = M::Q, K = M::K, NG = M::NG, GW = M::GW, NIN = C::NIN;
    static_assert(Q >= 1 && M::NWV <= 4, "k_cascade_mtop: me >= 4, <= 4 waves");
    __shared__ __attribute__((aligned(16))) uint64_t planes[(NIN + 1) & ~1];
    __shared__ __attribute__((aligned(16))) uint64_t xch[M::NWV * GW * M::XW];
    __shared__ __attribute__((aligned(16))) uint64_t rv[NG * K];  // R_Q of s0's sigmas
    __shared__ __attribute__((aligned(16))) uint64_t scr[64];      // wave 0's step Q-1 (and roots)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t w = blockIdx.x / a.s0n, s0 = a.s0b + (blockIdx.x - w * a.s0n);
    const uint64_t gw = (a.first_trial >> 6) + w;
    const uint32_t g = lane / (uint32_t)K, r = lane - g * (uint32_t)K;
    const uint32_t j = wv * (uint32_t)GW + g;  // sigma = child j of s0
    const uint32_t sg0 = s0 * (uint32_t)NG + j;
    // range mode at the vote level h = Q: only the range's sigmas
    const bool act = g < (uint32_t)GW && j < (uint32_t)NG && (a.h != (uint32_t)Q || (sg0 >= a.ub && sg0 < a.ue));
    const uint32_t sg = act ? sg0 : s0 * (uint32_t)NG;
    TrialCounts tc;
    uint32_t mm = 0;
    if (wv == 0) {
        CASC_MSTAMP(14);
        CASC_MSTAMP(0);
    }
    // children first; the inputs (wave 0) and the relay draws overlap them
    uint64_t cv[K - 1];
    casc_kids<N, ME, Q, CHECK, false>(a, act ? r : (uint32_t)K, w, sg, cv, mm);
    const RelayPlan<N, Q, K> rp(sg, sg * (uint32_t)K);
    uint64_t* xg = xch + (wv * (uint32_t)GW + (act ? g : 0u)) * (uint32_t)M::XW;
    relay_draw<N, Q, K, K>(a, rp, xg, r, act, gw);
    if (wv == 0) wave_inputs<N, 1, 0>(planes, lane, w, a.seed, a.gs, a.first_trial, a.ntrials, a.faulty, a.order);
    if (wv == 0) CASC_MSTAMP(1);
    __syncthreads();
    if (wv == 0) CASC_MSTAMP(2);
    if (act) {
        uint32_t path[Q], srt[Q];
        unrank_path<L, Q - 1>(sg, path, srt);
        const uint64_t lq = relay_apply<N, Q, K>(rp, planes, xg, r, sg * (uint32_t)K, path);
        Csa<planes_c(K)> cnt;
        cnt.template add<0>(lq);
        static_for<0, K - 1>([&](auto jj) { cnt.template add<jj() + 1>(cv[jj()]); });
        const uint64_t rq = cnt.template ge<K, K / 2 + 1>();  // inner tie -> non-attack
        if (a.h == (uint32_t)Q) a.votes[((uint64_t)(sg - a.ub) * K + r) * a.W + w] = rq;  // range: votes
        else rv[j * (uint32_t)K + r] = rq;
    }
    if (wv == 0) CASC_MSTAMP(3);
    if (a.h == (uint32_t)Q) return;  // block-uniform: the range's fan-in ends at these votes
    __syncthreads();
    if (wv == 0) CASC_MSTAMP(4);
    if (wv == 0) {
        // step Q-1 for s0: receiver r1 = lane < NG, children R_Q[s0.j1.r1], j1 != r1
        const uint32_t r1 = lane < (uint32_t)NG ? lane : 0u;
        uint64_t cv1[NG - 1];
        static_for<0, NG - 1>([&](auto jj) {
            const uint32_t j1 = (uint32_t)jj() + ((uint32_t)jj() >= r1 ? 1u : 0u);
            cv1[jj()] = rv[j1 * (uint32_t)K + r1 - (r1 > j1 ? 1u : 0u)];
        });
        casc_finish<N, ME, Q - 1, CHECK>(a, planes, scr, lane, w, s0, gw, cv1, tc, mm);
        CASC_MSTAMP(15);
    }
    if constexpr (CHECK) {
        uint32_t t = mm;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
        if (lane == 0 && t != 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), (unsigned long long)t);
    }
}

// ---------------------------------------------------------------------------
// k_cascade_wtop<N, ME, QS, VIN>: the same fan-in as k_cascade_top, one BLOCK
// of 1024 threads per word and no hand-off at all: the block relays L_0..L_QS
// of its word into LDS (one Philox pair per item, level by level), takes every
// level-QS majority over children from memory (R_{QS+1} of the units launch,
// or the gathered votes), then every lower level from LDS, block barrier in
// between, and the roots and the quorum epilogue (ba.py:159-255) by wave 0,
// which feeds the counter sink.  k_cascade_top's chain of three hand-offs
// (store, drain, returning add, reload) becomes three block barriers.
// ---------------------------------------------------------------------------
constexpr uint32_t kWtopThreads = 1024;

template <int N, int ME, int QS>
struct CascWtop {
    using C = Casc<N, ME>;
    static constexpr int L = C::L, NIN = C::NIN;
    static constexpr uint32_t oIN = 0, oAU = (NIN + 1) & ~1;
    static constexpr uint32_t oLV = oAU + ((2 * L + 1) & ~1);
    static constexpr uint32_t lv_off(int k) {  // L_k of the word
        uint32_t o = oLV;
        for (int i = 0; i < k; ++i) o += C::sz(i);
        return o;
    }
    static constexpr uint32_t rv_off(int k) {  // R_k of the word, k = 1..QS
        uint32_t o = lv_off(QS + 1);
        for (int i = 1; i < k; ++i) o += C::sz(i);
        return o;
    }
    static constexpr uint32_t words = rv_off(QS + 1);
};

template <int N, int ME, int QS, bool VIN, bool CHECK = false>
__global__ __launch_bounds__(kWtopThreads) void k_cascade_wtop(CascArgs a) {
    using C = Casc<N, ME>;
    using B = CascWtop<N, ME, QS>;
    constexpr int L = C::L;
    constexpr uint32_t T = kWtopThreads;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t w = blockIdx.x;
    const uint64_t gw = (a.first_trial >> 6) + w;
    uint64_t* planes = lds + B::oIN;
    uint64_t* au = lds + B::oAU;
    uint32_t mm = 0;
    if (wv == 0) wave_inputs<N, 1, 0>(planes, lane, w, a.seed, a.gs, a.first_trial, a.ntrials, a.faulty, a.order);
    __syncthreads();
    // relay L_0 .. L_QS (ba.py:257-285, 42-57): level k slot x is relayed by the
    // last general of its parent slot x / (L - k)
    static_for<0, QS + 1>([&](auto k) {
        constexpr uint32_t SK = C::sz(k()), NP = (SK + 1) / 2;
        uint64_t* lv = lds + B::lv_off(k());
        for (uint32_t p = t; p < NP; p += T) {
            uint64_t l[2];
            lie_pair(a.seed, k(), p, gw, l[0], l[1]);
            static_for<0, 2>([&](auto h) {
                const uint32_t x = 2 * p + h();
                if (x < SK) {
                    uint64_t par, f;
                    if constexpr (k() == 0) {
                        par = planes[N];  // OB: the commander's order
                        f = planes[0];
                    } else {
                        const uint32_t px = x / (uint32_t)(L - k());
                        par = lds[B::lv_off(k() - 1) + px];
                        f = planes[a.sender[a.snd_off[k() - 1] + px]];
                    }
                    lv[x] = sel64(f, l[h()], par);
                }
            });
        }
        __syncthreads();
    });
    // majorities, level QS (children from memory) down to the roots (from LDS)
    static_for<0, QS + 1>([&](auto i) {
        constexpr int q = QS - i();
        constexpr int K = L - q;
        constexpr uint32_t SQ = C::sz(q);
        const uint64_t* lq = lds + B::lv_off(q);
        for (uint32_t y = t; y < SQ; y += T) {
            const uint32_t sg = y / (uint32_t)K, r = y - sg * (uint32_t)K;
            uint64_t cv[K - 1];
            static_for<0, K - 1>([&](auto jj) {
                const uint32_t j = (uint32_t)jj() + ((uint32_t)jj() >= r ? 1u : 0u);
                const uint32_t x = (sg * (uint32_t)K + j) * (uint32_t)(K - 1) + r - (r > j ? 1u : 0u);
                if constexpr (q < QS) {
                    cv[jj()] = lds[B::rv_off(q + 1) + x];
                } else if constexpr (VIN) {
                    cv[jj()] = a.vin[(uint64_t)x * a.W + w];
                } else {
                    const uint64_t ix = C::template addr<q + 1>(w, x);
                    cv[jj()] = a.R[q + 1][ix];
                    if constexpr (CHECK) {
                        if (a.tag[q + 1][ix] != casc_tag(a.epoch)) ++mm;
                    }
                }
            });
            Csa<planes_c(K)> cnt;
            cnt.template add<0>(lq[y]);
            static_for<0, K - 1>([&](auto jj) { cnt.template add<jj() + 1>(cv[jj()]); });
            if constexpr (q > 0) {
                lds[B::rv_off(q) + y] = cnt.template ge<K, K / 2 + 1>();  // inner tie -> non-attack
            } else {  // roots: tie -> undefined
                const uint64_t att = cnt.template ge<K, K / 2 + 1>();
                au[r] = att;
                au[L + r] = (K % 2 == 0) ? (cnt.template ge<K, K / 2>() & ~att) : 0ull;
            }
        }
        __syncthreads();
    });
    if constexpr (CHECK) {
        uint32_t v = mm;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0 && v != 0 && a.counters)
            atomicAdd((unsigned long long*)(a.counters + BA_C_CHECK_MISMATCH), (unsigned long long)v);
    }
    if (wv == 0) {
        TrialCounts tw;
        wave_epilogue<N, 1, (uint32_t)ME, 0>(planes, au, lane, w, a.ntrials, a.decisions, a.outcome, tw);
        if (a.counters) sink_counters(lane, word_counts_to_lanes(tw, lane), w, a.W, a.counters, a.sk);
    }
}

template <int N, int ME, int QS, bool VIN, bool CHECK = false>
static hipError_t launch_wtop(const CascArgs& ca, uint32_t W, hipStream_t st) {
    using B = CascWtop<N, ME, QS>;
    hipLaunchKernelGGL((k_cascade_wtop<N, ME, QS, VIN, CHECK>), dim3(W), dim3(kWtopThreads),
                       (size_t)B::words * sizeof(uint64_t), st, ca);
    return hipGetLastError();
}

// Which fan-in kernel: one block per word (k_cascade_wtop) or one wave per
// level-(QS-1) slot with hand-offs (k_cascade_top).  Measured (profiles/r04i):
// the split's root pass (QS <= 1, children = votes) is faster by blocks (batch
// 1: 4.8 vs 5.1 us at h = 1, 5.5 vs 6.8 at h = 2), the two-launch cascade's
// fan-in from level me-3 by waves (n=16 m=5: 66.0 vs 67.2 us per 1024-instance
// call, 18.1 vs 21.2 us per instance: one block per word leaves the chip idle
// at small batches).  BA_CASC_WTOP=1/0 (read per call; A/B) forces one.
static bool use_wtop(bool root_pass) {
    const char* e = getenv("BA_CASC_WTOP");
    if (e) return e[0] != '0';
    return root_pass;
}
// the split's root pass touches neither the scratch nor the fan-in counters
// when it runs as k_cascade_wtop (one block per word, LDS only)
bool cascade_root_pass_uses_scratch() { return !use_wtop(true); }
// The units launch in latency mode (two lanes per leaf block) when its waves
// would occupy at most BA_CASC_LAT_WAVES of the 1,024 SIMDs: there each SIMD
// runs at most one wave and a lane's chain of Philox calls is the launch's time,
// which the mode halves.  Above it (a whole n=16, m=5 instance: 546 waves, or
// 1,365 in latency mode) SIMDs would take two latency-mode waves and the mode
// loses (18.4 vs 16.5 us per instance, profiles/r04m_lat_ab.log).  BA_CASC_LAT=1/0
// (read per call; A/B) forces it on or off where the shape has it.
#ifndef BA_CASC_LAT_WAVES
#define BA_CASC_LAT_WAVES 768
#endif
static bool use_lat(uint32_t units, uint32_t gpw_lat) {
    const char* e = getenv("BA_CASC_LAT");
    if (e) return e[0] != '0';
    return (units + gpw_lat - 1) / gpw_lat <= BA_CASC_LAT_WAVES;
}

// The two-launch fan-in by k_cascade_mtop (one hand-off fewer) or k_cascade_top.
// BA_CASC_MTOP=1/0 (read per call; A/B) forces one.
static bool use_mtop() {
    const char* e = getenv("BA_CASC_MTOP");
    if (e) return e[0] != '0';
    return true;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
#define BA_CASC_SHAPES(X) X(16, 5) X(16, 4) X(16, 3) X(10, 3) X(9, 4) X(8, 5)
// shapes whose subtree split (h <= me-3) runs through the cascade (range and root modes),
// and that have the two-launch mode (me >= 4)
#define BA_CASC_RANGE_SHAPES(X) X(16, 5) X(16, 4) X(9, 4) X(8, 5)
#define BA_CASC_TWO_SHAPES(X) X(16, 5) X(16, 4) X(9, 4) X(8, 5)
// two-launch shapes with the latency mode (odd S = n - me: leaf_half)
#define BA_CASC_LAT_SHAPES(X) X(16, 5) X(9, 4) X(8, 5)
// CHECK builds (tests only): depth 5 at two fan-outs, and a root-only cascade
#define BA_CASC_CHECK_SHAPES(X) X(16, 5) X(8, 5) X(10, 3)

bool cascade_supported(const Geometry& g) {
#define BA_CASC_OK(nn, mm) if (g.n == nn && g.me == mm) return true;
    BA_CASC_SHAPES(BA_CASC_OK)
#undef BA_CASC_OK
    return false;
}

// counters per word (units of kCascCounterStride uint32): every level-k slot,
// k < me-3, plus the word's root counter
uint64_t cascade_counters_per_word(const Geometry& g) {
    uint64_t c = 1;
    for (uint32_t k = 0; k + 3 < g.me; ++k) c += g.S[k];
    return c;
}

// R_1 .. R_{me-2} of one word, each step's child block padded to whole lines
// (co: R_{me-2} as granules, a CO launch's units -> fan-in hand-off)
uint64_t cascade_scratch_words_per_word(const Geometry& g, bool co) {
    uint64_t s = 0;
    for (uint32_t k = 1; k + 2 <= g.me; ++k) s += casc_level_words((int)g.L, (int)k, co && k + 2 == g.me);
    return s;
}

// the subtree split through the cascade: h-hop subtrees need h <= me-3 (the
// vote step is a fan-in step, not the units' own level)
bool cascade_range_supported(const Geometry& g, uint32_t h) {
    bool shape = false;
#define BA_CASC_OK(nn, mm) if (g.n == nn && g.me == mm) shape = true;
    BA_CASC_RANGE_SHAPES(BA_CASC_OK)
#undef BA_CASC_OK
    return shape && (h == 1 || h == 2) && h + 3 <= g.me;
}

// CO launch: the units blocks, then W * PB fan-in blocks (casc_co_top)
template <int N, int ME, bool CHECK = false>
static hipError_t launch_cascade_co(CascArgs& ca, hipStream_t st) {
    using U = CascU<N, ME, false>;
    using M = CascMtop<N, ME>;
    constexpr uint32_t per_block = kCascWaves * U::GPW;
    ca.nub = (ca.units + per_block - 1) / per_block;
    const uint32_t blocks = ca.nub + ca.W * M::PB;
    const uint32_t uw = U::planes_words + kCascWaves * U::tr_words;
    const size_t lds = (size_t)(uw > M::words ? uw : M::words) * sizeof(uint64_t);
    hipLaunchKernelGGL((k_cascade<N, ME, 10, CHECK>), dim3(blocks), dim3(64 * kCascWaves), lds, st, ca);
    return hipGetLastError();
}

template <int N, int ME, int DIAG = 0, bool CHECK = false, bool LAT = false>
static hipError_t launch_cascade_t(CascArgs& ca, hipStream_t st) {
    using U = CascU<N, ME, LAT>;
    constexpr uint32_t per_block = kCascWaves * U::GPW;
    const uint32_t blocks = (ca.units + per_block - 1) / per_block;
    const size_t lds = (size_t)(U::planes_words + kCascWaves * U::tr_words) * sizeof(uint64_t);
    hipLaunchKernelGGL((k_cascade<N, ME, DIAG, CHECK, LAT>), dim3(blocks ? blocks : 1), dim3(64 * kCascWaves),
                       lds, st, ca);
    return hipGetLastError();
}

hipError_t launch_cascade(const RunArgs& a, const Geometry& g, const uint8_t* d_sender,
                          uint64_t* scratch, uint32_t* d_cnt, uint64_t trial0, uint64_t ntrials,
                          const CascJob& job) {
    CascArgs ca{};
    const uint64_t W = (ntrials + 63) / 64;
    ca.seed = a.seed;
    ca.gs = a.gen;
    ca.first_trial = a.first_trial + trial0;
    ca.ntrials = ntrials;
    ca.W = (uint32_t)W;
    const uint64_t RQ = g.S[g.me - 3];
    if (job.h == 0) {
        ca.rr = (uint32_t)RQ;
        ca.rho0 = 0;
    } else {  // level-Q slots below the h-hop subtrees [ub, ue)
        const uint64_t per = RQ / g.S[job.h - 1];
        ca.rr = (uint32_t)((job.ue - job.ub) * per);
        ca.rho0 = (uint32_t)(job.ub * per);
    }
    ca.units = (uint32_t)(W * ca.rr);
    ca.faulty = a.faulty ? a.faulty + trial0 : nullptr;
    ca.order = a.order ? a.order + trial0 : nullptr;
    ca.sender = d_sender;
    for (uint32_t k = 0; k < g.me && k < (uint32_t)kCascMaxLevels; ++k)
        ca.snd_off[k] = (uint32_t)g.sender_off[k];
    ca.members = a.members;
    uint64_t off = 0;
    const uint64_t per_word = cascade_scratch_words_per_word(g, job.co);
    for (uint32_t k = 1; k + 2 <= g.me; ++k) {
        ca.R[k] = scratch + off;
        if (job.check) ca.tag[k] = scratch + W * per_word + off;
        off += W * casc_level_words((int)g.L, (int)k, job.co && k + 2 == g.me);
    }
    ca.epoch = job.epoch & 0xffffffffull;
    ca.inject = job.check == 2 ? 1u : 0u;
    ca.wait_ticks = job.wait_ticks ? job.wait_ticks : job.check ? kCascWaitTicksCheck : kCascWaitTicks;
    ca.cnt = d_cnt;
    uint32_t coff = 0;
    for (uint32_t k = 0; k + 3 < g.me; ++k) {
        ca.cnt_off[k] = coff;
        coff += (uint32_t)(W * g.S[k]);
    }
    ca.cnt_off[g.me - 3] = coff;  // root counters
    ca.h = job.h;
    ca.ub = job.ub;
    ca.ue = job.ue;
    ca.votes = job.votes;
    ca.decisions = a.decisions ? a.decisions + trial0 : nullptr;
    ca.outcome = a.outcome ? a.outcome + trial0 : nullptr;
    ca.counters = job.h ? nullptr : a.counters;
    ca.sk = a.sink;
    if (job.vin && use_wtop(true)) {  // the split's root pass: one block per word
        ca.vin = job.vin;
        ca.h = 0;
        ca.counters = a.counters;
        ProfScope ps(a.prof, "k_cascade_wtop", a.stream);
#define BA_CASC_WROOT_LAUNCH(nn, mm)                                                               \
    if (g.n == nn && g.me == mm)                                                                  \
        return job.root_h == 2 ? launch_wtop<nn, mm, 1, true>(ca, (uint32_t)W, a.stream)          \
                               : launch_wtop<nn, mm, 0, true>(ca, (uint32_t)W, a.stream);
        BA_CASC_RANGE_SHAPES(BA_CASC_WROOT_LAUNCH)
#undef BA_CASC_WROOT_LAUNCH
        return hipErrorInvalidValue;
    }
    if (job.vin) {  // the split's root pass: one wave per (word, level root_h-2 slot)
        ca.vin = job.vin;
        ca.h = 0;
        ca.units = (uint32_t)(W * (job.root_h == 2 ? g.L : 1u));
        ca.counters = a.counters;
        ProfScope ps(a.prof, "k_cascade_top", a.stream);
        const uint32_t blocks = (ca.units + kCascWaves - 1) / kCascWaves;
#define BA_CASC_ROOT_LAUNCH(nn, mm)                                                                    \
    if (g.n == nn && g.me == mm) {                                                                   \
        if (job.root_h == 2)                                                                         \
            hipLaunchKernelGGL((k_cascade_top<nn, mm, 1, true>), dim3(blocks), dim3(64 * kCascWaves), \
                               0, a.stream, ca);                                                     \
        else                                                                                         \
            hipLaunchKernelGGL((k_cascade_top<nn, mm, 0, true>), dim3(blocks), dim3(64 * kCascWaves), \
                               0, a.stream, ca);                                                     \
        return hipGetLastError();                                                                    \
    }
        BA_CASC_RANGE_SHAPES(BA_CASC_ROOT_LAUNCH)
#undef BA_CASC_ROOT_LAUNCH
        return hipErrorInvalidValue;
    }
    if (job.co) {  // one launch: units + co-resident fan-in blocks (whole tree, me >= 4)
        if (job.h != 0 || g.me < 4) return hipErrorInvalidValue;
        ProfScope ps(a.prof, "k_cascade_co", a.stream);
#define BA_CASC_CO_LAUNCH(nn, mm)                                                         \
    if (g.n == nn && g.me == mm)                                                        \
        return job.check ? launch_cascade_co<nn, mm, true>(ca, a.stream)                \
                         : launch_cascade_co<nn, mm>(ca, a.stream);
        BA_CASC_TWO_SHAPES(BA_CASC_CO_LAUNCH)
#undef BA_CASC_CO_LAUNCH
        return hipErrorInvalidValue;
    }
    if (job.two && g.me >= 4 && (job.h == 0 || cascade_range_two_supported(g, job.h))) {
        // two launches: the units (k_cascade, DIAG 2: no fan-in), then the fan-in
        // from level me-3 up (k_cascade_top), one wave per level-(me-4) slot
        {
            bool lat = false;
            uint32_t gpw_lat = 0;
#define BA_CASC_LAT_OK(nn, mm) if (g.n == nn && g.me == mm) gpw_lat = CascU<nn, mm, true>::GPW;
            BA_CASC_LAT_SHAPES(BA_CASC_LAT_OK)
#undef BA_CASC_LAT_OK
            lat = gpw_lat && use_lat(ca.units, gpw_lat);
            ProfScope ps(a.prof, lat ? "k_cascade_units_lat" : "k_cascade_units", a.stream);
            hipError_t e = hipErrorInvalidValue;
#define BA_CASC_UNITS_LAUNCH(nn, mm)                                                         \
    if (g.n == nn && g.me == mm)                                                           \
        e = job.check ? launch_cascade_t<nn, mm, 2, true>(ca, a.stream)                    \
                      : launch_cascade_t<nn, mm, 2>(ca, a.stream);
#define BA_CASC_LAT_LAUNCH(nn, mm)                                                           \
    if (g.n == nn && g.me == mm)                                                           \
        e = job.check ? launch_cascade_t<nn, mm, 2, true, true>(ca, a.stream)              \
                      : launch_cascade_t<nn, mm, 2, false, true>(ca, a.stream);
            if (lat) {
                BA_CASC_LAT_SHAPES(BA_CASC_LAT_LAUNCH)
            } else {
                BA_CASC_TWO_SHAPES(BA_CASC_UNITS_LAUNCH)
            }
#undef BA_CASC_LAT_LAUNCH
#undef BA_CASC_UNITS_LAUNCH
            if (e != hipSuccess) return e;
        }
        CascArgs ct = ca;
        if (use_wtop(false) && job.h == 0) {
            ProfScope ps(a.prof, "k_cascade_wtop", a.stream);
#define BA_CASC_WTOP_LAUNCH(nn, mm)                                                          \
    if (g.n == nn && g.me == mm)                                                           \
        return job.check ? launch_wtop<nn, mm, mm - 3, false, true>(ct, (uint32_t)W, a.stream) \
                         : launch_wtop<nn, mm, mm - 3, false>(ct, (uint32_t)W, a.stream);
            BA_CASC_TWO_SHAPES(BA_CASC_WTOP_LAUNCH)
#undef BA_CASC_WTOP_LAUNCH
            return hipErrorInvalidValue;
        }
        if (use_mtop() || job.h != 0) {  // the range mode's fan-in is k_cascade_mtop's
            ProfScope ps(a.prof, "k_cascade_mtop", a.stream);
#define BA_CASC_MTOP_LAUNCH(nn, mm)                                                                   \
    if (g.n == nn && g.me == mm) {                                                                  \
        using M = CascMtop<nn, mm>;                                                                 \
        if (job.h == 0) {                       /* every level-(me-5) slot */                       \
            ct.s0b = 0;                                                                             \
            ct.s0n = M::PB;                                                                         \
        } else if (job.h + 1 == (uint32_t)M::Q) { /* votes at step Q-1: s0 = the h-hop subtrees */  \
            ct.s0b = job.ub;                                                                        \
            ct.s0n = job.ue - job.ub;                                                               \
        } else {                                /* h = Q: the s0 over the range's sigmas */         \
            ct.s0b = job.ub / (uint32_t)M::NG;                                                      \
            ct.s0n = (job.ue - 1) / (uint32_t)M::NG - ct.s0b + 1;                                   \
        }                                                                                           \
        const dim3 grid((uint32_t)(W * ct.s0n)), blk(64 * M::NWV);                                   \
        if (job.check)                                                                              \
            hipLaunchKernelGGL((k_cascade_mtop<nn, mm, true>), grid, blk, 0, a.stream, ct);          \
        else                                                                                        \
            hipLaunchKernelGGL((k_cascade_mtop<nn, mm>), grid, blk, 0, a.stream, ct);                \
        return hipGetLastError();                                                                   \
    }
            BA_CASC_TWO_SHAPES(BA_CASC_MTOP_LAUNCH)
#undef BA_CASC_MTOP_LAUNCH
            return hipErrorInvalidValue;
        }
        ct.units = (uint32_t)(W * g.S[g.me - 4]);
        ProfScope ps(a.prof, "k_cascade_top", a.stream);
        const uint32_t blocks = (ct.units + kCascWaves - 1) / kCascWaves;
#define BA_CASC_TOP_LAUNCH(nn, mm)                                                                      \
    if (g.n == nn && g.me == mm) {                                                                    \
        if (job.check)                                                                                \
            hipLaunchKernelGGL((k_cascade_top<nn, mm, mm - 3, false, true>), dim3(blocks),              \
                               dim3(64 * kCascWaves), 0, a.stream, ct);                               \
        else                                                                                          \
            hipLaunchKernelGGL((k_cascade_top<nn, mm, mm - 3, false>), dim3(blocks),                    \
                               dim3(64 * kCascWaves), 0, a.stream, ct);                               \
        return hipGetLastError();                                                                     \
    }
        BA_CASC_TWO_SHAPES(BA_CASC_TOP_LAUNCH)
#undef BA_CASC_TOP_LAUNCH
        return hipErrorInvalidValue;
    }
    ProfScope ps(a.prof, "k_cascade", a.stream);
    if (const char* d = getenv("BA_CASC_DIAG")) {  // lab ablations, n=16 m=5 only
        if (g.n == 16 && g.me == 5 && job.h == 0 && !job.check) switch (atoi(d)) {
            case 2: return launch_cascade_t<16, 5, 2>(ca, a.stream);
            case 4: return launch_cascade_t<16, 5, 4>(ca, a.stream);
            default: break;
        }
    }
    if (job.check) {
#define BA_CASC_CHECK_LAUNCH(nn, mm) \
    if (g.n == nn && g.me == mm) return launch_cascade_t<nn, mm, 0, true>(ca, a.stream);
        BA_CASC_CHECK_SHAPES(BA_CASC_CHECK_LAUNCH)
#undef BA_CASC_CHECK_LAUNCH
        return hipErrorInvalidValue;
    }
#define BA_CASC_LAUNCH(nn, mm) \
    if (g.n == nn && g.me == mm) return launch_cascade_t<nn, mm>(ca, a.stream);
    BA_CASC_SHAPES(BA_CASC_LAUNCH)
#undef BA_CASC_LAUNCH
    return hipErrorInvalidValue;
}

// the range mode in two launches (units, then k_cascade_mtop): me >= 4 and the
// vote level h at step me-3 or me-4
bool cascade_range_two_supported(const Geometry& g, uint32_t h) {
    bool shape = false;
#define BA_CASC_OK(nn, mm) if (g.n == nn && g.me == mm) shape = true;
    BA_CASC_TWO_SHAPES(BA_CASC_OK)
#undef BA_CASC_OK
    return shape && cascade_range_supported(g, h) && g.me >= 4 && h + 4 >= g.me && h + 3 <= g.me;
}

#ifdef BA_CASC_STAMPS
extern "C" int ba_lab_casc_stamps_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(ba_lab_casc_stamps), bytes, 0, hipMemcpyDeviceToHost) ==
                   hipSuccess ? 0 : -3;
}
extern "C" int ba_lab_stamps_clear() {
    static unsigned long long zero[kStampWaves][16];
    return hipMemcpyToSymbol(HIP_SYMBOL(ba_lab_mtop_stamps), zero, sizeof zero) == hipSuccess &&
                   hipMemcpyToSymbol(HIP_SYMBOL(ba_lab_casc_stamps), zero,
                                     sizeof(unsigned long long) * kStampWaves * kStampWords) == hipSuccess
               ? 0 : -3;
}
extern "C" int ba_lab_mtop_stamps_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(ba_lab_mtop_stamps), bytes, 0, hipMemcpyDeviceToHost) ==
                   hipSuccess ? 0 : -3;
}
#endif

bool cascade_check_supported(const Geometry& g) {
#define BA_CASC_OK(nn, mm) if (g.n == nn && g.me == mm) return true;
    BA_CASC_CHECK_SHAPES(BA_CASC_OK)
#undef BA_CASC_OK
    return false;
}

}  // namespace ba
