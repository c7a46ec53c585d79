// ba_wave.hpp -- the WAVE engine (gfx950): one wave resolves a task of W
// 64-trial words alone, walking the OM tree one first-hop (k_om3w, effective
// depth 3) or second-level (k_om4w, depth 4) subtree per round; see DESIGN.md.
// Instantiated by ba_wave3.hip / ba_wave4.hip (two translation units, so the
// two kernel families compile in parallel).
#pragma once
#include "ba_leaf.hpp"

namespace ba {

// ---------------------------------------------------------------------------
// WAVE engine, effective depth 3: each wave owns W consecutive trial words and
// resolves them alone (no block barrier anywhere; the 4 waves of a block only
// share the launch).  The tree is walked one first-hop subtree j1 at a time:
// a subtree has C = L-1 level-1 slots (j1, a), i.e. C leaf blocks, so lane
// (w, a), w < W = 64 / C, owns leaf block (j1, a) of word w in every round.
// For n=10 that is 8 words x 8 leaf blocks = all 64 lanes.  Per round:
//   1. L1[j1, a] = F[j1] ? lie : L0[j1]            (the lane's own leaf parent)
//   2. leaf block (j1, a): R2[j1, a, *]             (registers -> LDS, S words)
//   3. lane (w, b = a): R1[j1, b] = maj(L1[j1, b], R2[j1, a', b] : a' != b),
//      added into the bit-sliced root counter of receiver column j2(b)
// R1 is never stored: each root column accumulates as the subtrees finish.
// R2 is stored receiver-major (R2T[w][b][a] = R2[j1, a, b], with the lane's
// own L1[j1, b] on the diagonal a == b), so step 3 counts C contiguous words
// with a compile-time carry-save schedule.
// Lie bits are keyed exactly as in k_fused (level, global slot pair, global
// word), so both kernels give identical results.
// LDS per wave (uint64 words): IN[W][N+3] (F[N] OB OO VAL) | L0[W][L] |
// R2T[W][C][C] | RC[W][L][P] (root counters) ; A/U roots reuse R2T when it fits.
// ---------------------------------------------------------------------------
// Branch-free synthetic inputs for compile-time N: the same draws as
// gen_trial (ba_device.hpp), but every Philox call is issued up front, the
// PK selection steps are predicated and the modes are selects, so the code
// for several trials is one basic block and their chains interleave.  fm / oc
// carry the given values in and the resolved ones out.  Valid for
// min(f, N) <= PK.
template <int N, int PK>
__device__ __forceinline__ void gen_trial_u(uint64_t seed, const GenSpec& g, uint64_t t,
                                            uint32_t& fm, uint32_t& oc) {
    constexpr int CALLS = (2 + PK + 3) / 4;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t u[4 * CALLS];
    static_for<0, CALLS>([&](auto c) {
        const P4 b = philox10(P4{(uint32_t)c(), kGenTag, (uint32_t)t, (uint32_t)(t >> 32)}, k0, k1);
        u[4 * c()] = b.x;
        u[4 * c() + 1] = b.y;
        u[4 * c() + 2] = b.z;
        u[4 * c() + 3] = b.w;
    });
    oc = g.order_mode == 1 ? u[0] >> 31 : (g.order_mode == 2 ? g.order_value : oc);
    const uint32_t fcap = g.f < (uint32_t)N ? g.f : (uint32_t)N;
    const uint32_t nf = g.faulty_mode == 1 ? mulhi_range(u[1], fcap + 1) : fcap;
    // step i takes the j-th (ascending) general not yet chosen: with the
    // chosen ones kept sorted (s[0] < s[1] < ...), that general is j plus the
    // number of chosen positions at or below it, found by one compare-increment
    // per chosen general in ascending order
    constexpr int NP = PK < N ? PK : N;
    uint32_t srt[NP > 0 ? NP : 1];
    uint32_t mask = 0;
    static_for<0, NP>([&](auto i) {
        uint32_t pos = mulhi_range(u[2 + i()], (uint32_t)N - i());
        static_for<0, i()>([&](auto k) { pos += srt[k()] <= pos ? 1u : 0u; });
        const bool take = (uint32_t)i() < nf;
        mask |= take ? (1u << pos) : 0u;
        // insert pos into the sorted list (an untaken step appends N: sorts last)
        uint32_t x = take ? pos : (uint32_t)N;
        static_for<0, i()>([&](auto k) {
            const uint32_t lo = srt[k()] < x ? srt[k()] : x, hi = srt[k()] < x ? x : srt[k()];
            srt[k()] = lo;
            x = hi;
        });
        srt[i()] = x;
    });
    fm = g.faulty_mode != 0 ? mask : fm;
}

// Inputs of words [0, W) of a wave task -> bit-sliced words in LDS
// (in[w*NIN + g] = F[g], then OB, OO, VAL).  PK = 0: the generic gen_trial;
// PK = -1: both inputs given (loads only).
template <int N, int W, int PK>
__device__ __forceinline__ void gen_words(uint64_t* in0, uint32_t lane, uint64_t w0, uint64_t seed,
                                          const GenSpec& gs, uint64_t first_trial, uint64_t batch,
                                          const uint32_t* __restrict__ faulty,
                                          const uint8_t* __restrict__ order) {
    constexpr int NIN = N + 3, G4 = W < 8 ? W : 8;
    static_for<0, (W + G4 - 1) / G4>([&](auto grp) {
        constexpr int wb = grp() * G4, nq = W - wb < G4 ? W - wb : G4;
        uint32_t fm[nq], oc[nq];
        bool valid[nq];
        // given inputs first (uniform branches kept out of the draw code)
        static_for<0, nq>([&](auto q) {
            const uint64_t i = (w0 + wb + q()) * 64 + lane;
            valid[q()] = i < batch;
            fm[q()] = 0;
            oc[q()] = 0;
        });
        if (gs.faulty_mode == 0)
            static_for<0, nq>([&](auto q) {
                if (valid[q()]) fm[q()] = faulty[(w0 + wb + q()) * 64 + lane];
            });
        if (gs.order_mode == 0)
            static_for<0, nq>([&](auto q) {
                if (valid[q()]) oc[q()] = order[(w0 + wb + q()) * 64 + lane];
            });
        static_for<0, nq>([&](auto q) {
            const uint64_t t = first_trial + (w0 + wb + q()) * 64 + lane;
            if constexpr (PK > 0) gen_trial_u<N, PK>(seed, gs, t, fm[q()], oc[q()]);
            else if constexpr (PK == 0) {
                if (valid[q()]) gen_trial(N, seed, gs, t, fm[q()], oc[q()]);
            }
        });
        static_for<0, nq>([&](auto q) {
            uint64_t mine = 0;
            static_for<0, N>([&](auto g) {
                const uint64_t b = __ballot(valid[q()] && ((fm[q()] >> g()) & 1u));
                if (lane == g()) mine = b;
            });
            const uint64_t ob = __ballot(valid[q()] && oc[q()] == 1);
            const uint64_t oo = __ballot(valid[q()] && oc[q()] == 2);
            const uint64_t vv = __ballot(valid[q()]);
            uint64_t* in = in0 + (wb + q()) * NIN;
            if (lane < (uint32_t)N) in[lane] = mine;
            if (lane == 0) {
                in[N] = ob;
                in[N + 1] = oo;
                in[N + 2] = vv;
            }
        });
    });
}

// Staged inputs (both given, e.g. ba_gen_inputs_device buffers) of words
// [0, W) of a wave task -> bit-sliced words in LDS, in0[w*(N+3) + g].  Every
// lane packs its trial's faulty bits, order bits and live bit into one dword
// (bits 0..N-1 F, N OB, N+1 OO, N+2 VAL); plane g is one ballot (an SGPR
// pair) that v_writelane drops into lane g of a VGPR pair (writelane4), and
// lanes g < N+3 store their plane with one LDS write.  Against gen_words<.., -1> (a ballot
// per plane, then a lane-select of every ballot in every lane) this is ~60
// instead of ~140 instructions per word, and it keeps no ballot live across
// words (the old code's SGPRs spilled to VGPR lanes).  All 2W loads are issued
// before the first use.
// Lanes G0..G0+CNT-1 of the VGPR pair (lo, hi) = the uniform 64-bit values
// b[0..CNT) (v_writelane_b32; clang has no writelane builtin here).  The
// ballots that produced b are VALU writes of SGPRs, and v_writelane reads its
// data SGPR early: without wait states between them a GPU run got wrong planes
// (the hazard recognizer cannot see into the asm), so each group of up to 4
// planes pays one s_nop 4 after its ballots.
// BA_WRITELANE_NOP: the wait states in front of each group (tests/test_lib.py
// builds a copy with it empty to prove its code-object check catches that).
#ifndef BA_WRITELANE_NOP
#define BA_WRITELANE_NOP "s_nop 4\n\t"
#endif
template <int G0, int CNT>
__device__ __forceinline__ void writelane4(uint32_t& lo, uint32_t& hi, const uint64_t (&b)[4]) {
    const uint32_t l0 = (uint32_t)b[0], h0 = (uint32_t)(b[0] >> 32), l1 = (uint32_t)b[1],
                   h1 = (uint32_t)(b[1] >> 32), l2 = (uint32_t)b[2], h2 = (uint32_t)(b[2] >> 32),
                   l3 = (uint32_t)b[3], h3 = (uint32_t)(b[3] >> 32);
    if constexpr (CNT == 4)
        asm volatile(BA_WRITELANE_NOP "v_writelane_b32 %0, %2, %10\n\tv_writelane_b32 %1, %3, %10\n\t"
                     "v_writelane_b32 %0, %4, %11\n\tv_writelane_b32 %1, %5, %11\n\t"
                     "v_writelane_b32 %0, %6, %12\n\tv_writelane_b32 %1, %7, %12\n\t"
                     "v_writelane_b32 %0, %8, %13\n\tv_writelane_b32 %1, %9, %13"
                     : "+v"(lo), "+v"(hi)
                     : "s"(l0), "s"(h0), "s"(l1), "s"(h1), "s"(l2), "s"(h2), "s"(l3), "s"(h3),
                       "i"(G0), "i"(G0 + 1), "i"(G0 + 2), "i"(G0 + 3));
    else if constexpr (CNT == 3)
        asm volatile(BA_WRITELANE_NOP "v_writelane_b32 %0, %2, %8\n\tv_writelane_b32 %1, %3, %8\n\t"
                     "v_writelane_b32 %0, %4, %9\n\tv_writelane_b32 %1, %5, %9\n\t"
                     "v_writelane_b32 %0, %6, %10\n\tv_writelane_b32 %1, %7, %10"
                     : "+v"(lo), "+v"(hi)
                     : "s"(l0), "s"(h0), "s"(l1), "s"(h1), "s"(l2), "s"(h2), "i"(G0), "i"(G0 + 1),
                       "i"(G0 + 2));
    else if constexpr (CNT == 2)
        asm volatile(BA_WRITELANE_NOP "v_writelane_b32 %0, %2, %6\n\tv_writelane_b32 %1, %3, %6\n\t"
                     "v_writelane_b32 %0, %4, %7\n\tv_writelane_b32 %1, %5, %7"
                     : "+v"(lo), "+v"(hi)
                     : "s"(l0), "s"(h0), "s"(l1), "s"(h1), "i"(G0), "i"(G0 + 1));
    else
        asm volatile(BA_WRITELANE_NOP "v_writelane_b32 %0, %2, %4\n\tv_writelane_b32 %1, %3, %4"
                     : "+v"(lo), "+v"(hi)
                     : "s"(l0), "s"(h0), "i"(G0));
    (void)l1; (void)h1; (void)l2; (void)h2; (void)l3; (void)h3;
}

// One word's staged inputs (this lane's trial: faulty mask fm, order code oc,
// live v) -> the word's N+3 bit-sliced planes in0[0..N+3): one ballot per
// plane, plane g dropped into lane g by v_writelane.
template <int N>
__device__ __forceinline__ void stage_slice(uint64_t* in0, uint32_t lane, uint32_t fm, uint32_t c,
                                            bool v) {
    constexpr int NIN = N + 3;
    constexpr uint32_t FMASK = N >= 32 ? 0xFFFFFFFFu : ((1u << N) - 1u);
    const uint32_t x = (fm & FMASK) | (c == 1u ? 1u << N : 0u) | (c == 2u ? 2u << N : 0u) |
                       (v ? 4u << N : 0u);
    uint32_t lo = 0, hi = 0;
    static_for<0, (NIN + 3) / 4>([&](auto grp) {
        constexpr int g0 = 4 * grp();
        uint64_t b[4];
        static_for<0, 4>([&](auto j) { b[j()] = g0 + j() < NIN ? __ballot((x >> (g0 + j())) & 1u) : 0ull; });
        writelane4<g0, (NIN - g0 < 4 ? NIN - g0 : 4)>(lo, hi, b);
    });
    if (lane < (uint32_t)NIN) in0[lane] = (uint64_t)hi << 32 | lo;
}

template <int N, int W>
__device__ __forceinline__ void stage_words(uint64_t* in0, uint32_t lane, uint64_t w0, uint64_t batch,
                                            const uint32_t* __restrict__ faulty,
                                            const uint8_t* __restrict__ order) {
    constexpr int NIN = N + 3;
    uint32_t fm[W], oc[W];
    static_for<0, W>([&](auto q) {
        const uint64_t i = (w0 + q()) * 64 + lane;
        const bool v = i < batch;
        fm[q()] = v ? faulty[i] : 0u;
        oc[q()] = v ? (uint32_t)order[i] : 0u;
    });
    static_for<0, W>([&](auto q) {
        stage_slice<N>(in0 + q() * NIN, lane, fm[q()], oc[q()], (w0 + q()) * 64 + lane < batch);
    });
}

// ---------------------------------------------------------------------------
// Pieces shared by the WAVE kernels (one wave resolves a task of W words).
// ---------------------------------------------------------------------------
// Inputs of a task's W words -> bit-sliced words in0[w*(N+3) + g].
template <int N, int W, int DIAG>
__device__ __forceinline__ void wave_inputs(uint64_t* in0, uint32_t lane, uint64_t w0,
                                            uint64_t seed, const GenSpec& gs,
                                            uint64_t first_trial, uint64_t batch,
                                            const uint32_t* __restrict__ faulty,
                                            const uint8_t* __restrict__ order) {
    constexpr int NIN = N + 3;
    const uint32_t pk = gs.faulty_mode == 0 ? 0u : (gs.f < (uint32_t)N ? gs.f : (uint32_t)N);
    if (gs.faulty_mode == 0 && gs.order_mode == 0) {  // staged inputs: loads only
        stage_words<N, W>(in0, lane, w0, batch, faulty, order);
    } else if constexpr ((DIAG & 16) != 0) {  // lab: near-free stand-in inputs
        static_for<0, W>([&](auto wq) {
            const uint64_t h = (w0 + wq() + 1) * 0x9E3779B97F4A7C15ull;
            if (lane < (uint32_t)NIN) in0[wq() * NIN + lane] = lane == N + 2 ? ~0ull : (h >> lane) & (h << 3);
        });
    } else if (pk <= 2) gen_words<N, W, 2>(in0, lane, w0, seed, gs, first_trial, batch, faulty, order);
    else if (pk <= 3) gen_words<N, W, 3>(in0, lane, w0, seed, gs, first_trial, batch, faulty, order);
    else if (pk <= 6) gen_words<N, W, 6>(in0, lane, w0, seed, gs, first_trial, batch, faulty, order);
    else gen_words<N, W, 0>(in0, lane, w0, seed, gs, first_trial, batch, faulty, order);
}

// Level 0 of W words (one Philox per slot pair) into l0[w*L + j], and the
// root counters rc[(w*L + j)*P + q] initialised with it (plane 0 = L0).
template <int N, int W, int P>
__device__ __forceinline__ void wave_level0(const uint64_t* in0, uint64_t* l0, uint64_t* rc,
                                            uint32_t lane, uint64_t seed, uint64_t gw0) {
    constexpr int L = N - 1, NIN = N + 3;
    constexpr uint32_t NP0 = (L + 1) / 2;
    for (uint32_t it = lane; it < (uint32_t)W * NP0; it += 64) {
        const uint32_t w = it / NP0, p = it - w * NP0;
        const uint64_t* in = in0 + w * NIN;
        const uint64_t F0 = in[0], ob = in[N];
        uint64_t lv[2];
        lie_pair(seed, 0, p, gw0 + w, lv[0], lv[1]);
        static_for<0, 2>([&](auto h) {
            const uint32_t j = 2 * p + h();
            if (j < (uint32_t)L) {
                const uint64_t v = (F0 & lv[h()]) | (~F0 & ob);
                l0[w * L + j] = v;
                uint64_t* c = rc + (w * L + j) * P;
                c[0] = v;
                static_for<1, P>([&](auto q) { c[q()] = 0; });
            }
        });
    }
}

// c[0..P) (bit-sliced planes in LDS) += x
template <int P>
__device__ __forceinline__ void planes_add(uint64_t* c, uint64_t x) {
    static_for<0, P>([&](auto q) {
        const uint64_t v = c[q()];
        c[q()] = v ^ x;
        x &= v;
    });
}

// Root majorities of W words from the root counters (L inputs each): strict
// majority attacks, a tie is "undefined" (ba.py:188-195).  au[w*2L + b] = A,
// au[w*2L + L + b] = U.
template <int L, int W, int P>
__device__ __forceinline__ void wave_roots(const uint64_t* rc, uint64_t* au, uint32_t lane) {
    for (uint32_t it = lane; it < (uint32_t)W * L; it += 64) {
        const uint32_t w = it / L, col = it - w * L;
        const uint64_t* c = rc + (w * L + col) * P;
        Count<P> cnt;
        static_for<0, P>([&](auto q) { cnt.c[q()] = c[q()]; });
        const uint64_t att = cnt.ge(L / 2 + 1);
        const uint64_t tie = (L & 1) ? 0ull : (cnt.ge(L / 2) & ~att);
        au[w * 2 * L + col] = att;
        au[w * 2 * L + L + col] = tie;
    }
}

// Quorum epilogue of W words in two phases (ba.py:206-262, restated per trial
// by trial_result in ba_device.hpp, which the oracle test pins):
//  1. lane = (word, byte): the whole decision is bit-sliced over 8 trials of
//     one word -- byte k of every plane -- with compile-time carry-save counts
//     of attacks / non-retreats / faulty generals against the quorum
//     thresholds, ORs and ANDs over the loyal lieutenants for agreement and
//     validity; the run counters are popcounts of the resulting planes masked
//     by the live-trial bits.  The six outcome planes overwrite the word's
//     faulty planes in LDS (byte k each).  Every operation is bitwise, so a
//     word splits into 8 independent byte lanes: 8 words x 8 bytes = one
//     instruction stream for the whole task, where lane = word left 56 of 64
//     lanes idle through ~380 instructions of 64-bit (two-half) operations.
//  2. lane = trial: the 2L decision bits and 6 outcome bits of each word are
//     picked out of the 32-bit half holding this lane (one bfe + one shift-or
//     per bit) and stored.
// Per trial this is ~3x fewer instructions than running trial_result in every
// lane, which needed all 2L+N+3 bits gathered first.
// epilogue_core: plane p of the inputs is in(p) (F[0..N), OB, OO, VAL), root
// planes au(b) (A[0..L), U[0..L)), outcome plane k is written by out(k, v);
// T is the slice type (uint64_t: a whole word; uint32_t: one byte of it).
template <typename T>
__device__ __forceinline__ uint32_t popc_t(T x) {
    if constexpr (sizeof(T) == 8) return (uint32_t)__popcll(x);
    else return (uint32_t)__popc(x);
}

// ME = 0: the effective depth is the runtime me_rt (the LEVELS tail, any tree of
// N generals); it only sets the in-bound flag, taken from the resolved planes.
template <int N, uint32_t ME, typename T, typename In, typename Au, typename Out>
__device__ __forceinline__ void epilogue_core(In in, Au au, Out out, TrialCounts& tc,
                                              uint32_t me_rt = ME) {
    constexpr int L = N - 1, NB = planes_c(N);
    // an odd number of root inputs never ties: no undefined decisions, U == 0
    constexpr bool TIES = L % 2 == 0;
    constexpr int needed = N == 1 ? 1 : (N <= 3 ? N - 1 : 2 * ((N - 1) / 3) + 1);
    constexpr int K0 = L - needed;  // retreat: #(A|U) <= K0 (+1 when the commander retreats)
    const T val = in(N + 2), oo = in(N + 1);
    const T ob = in(N) & ~oo, orr = ~in(N) & ~oo;  // commander attack / retreat
    const T f0 = in(0);
    Csa<NB, T> cA, cX, cF;
    cF.template add<0>(f0);
    T anyA = 0, anyU = 0, anyR = 0, allA = (T)~(T)0, allR = (T)~(T)0;
    uint32_t nU = 0;
    static_for<0, L>([&](auto b) {
        const T a = au(b()), f = in(b() + 1);
        const T u = TIES ? au(L + b()) & ~a : (T)0, x = a | u;
        cA.template add<b()>(a);
        if constexpr (TIES) cX.template add<b()>(x);
        cF.template add<b() + 1>(f);
        anyA |= a & ~f;
        if constexpr (TIES) anyU |= u & ~f;
        anyR |= ~(x | f);
        allA &= a | f;
        allR &= ~x | f;
        if constexpr (TIES) nU += popc_t<T>(u & val);
    });
    // per-trial counts as bit planes: the run totals are plane popcounts
    T rA[NB], rF[NB];
    cA.template resolve<0, L, false>(rA, 0);
    cF.template resolve<0, N, false>(rF, 0);
    uint32_t nA = 0, nf = 0;
    static_for<0, NB>([&](auto i) {
        nA += popc_t<T>(rA[i()] & val) << i();
        nf += popc_t<T>(rF[i()] & val) << i();
    });
    const Csa<NB, T>& cXr = TIES ? cX : cA;
    const T retreat = ~cXr.template ge<L, K0 + 1>() | (orr & ~cXr.template ge<L, K0 + 2>());
    const T attc = cA.template ge<L, needed>() | (ob & cA.template ge<L, needed - 1>());
    const T q1 = ~retreat & attc, q2 = ~retreat & ~attc;
    const T agree = TIES ? ~maj3(anyA, anyU, anyR) : ~(anyA & anyR);
    const T appl = ~f0;
    const T valid = appl & ((ob & allA) | (~ob & allR));
    T inb = (T)0;
    if constexpr (ME > 0) {
        inb = (N > 3 * (int)ME) ? ~cF.template ge<N, (int)ME + 1>() : (T)0;
    } else if ((uint32_t)N > 3 * me_rt) {  // inb = faulty count <= me_rt, from the count planes
        const uint32_t th = me_rt + 1;
        T gt = 0, eq = (T)~(T)0;
        static_for<0, NB>([&](auto j) {
            constexpr int i = NB - 1 - j();
            if ((th >> i) & 1u) eq &= rF[i];
            else {
                gt |= eq & rF[i];
                eq &= ~rF[i];
            }
        });
        inb = (th >> NB) ? (T)~(T)0 : ~(gt | eq);
    }
    tc.v[C_TRIALS] += popc_t<T>(val);
    tc.v[C_AGREE] += popc_t<T>(agree & val);
    tc.v[C_VAPPL] += popc_t<T>(appl & val);
    tc.v[C_VALID] += popc_t<T>(valid & val);
    tc.v[C_QR] += popc_t<T>(retreat & val);
    tc.v[C_QA] += popc_t<T>(q1 & val);
    tc.v[C_QU] += popc_t<T>(q2 & val);
    tc.v[C_UNDEF] += nU;
    tc.v[C_INB] += popc_t<T>(inb & val);
    tc.v[C_VIOL] += popc_t<T>(inb & (~agree | (appl & ~valid)) & val);
    tc.v[C_FTOT] += nf;
    tc.v[C_ATT] += nA;
    out(0, q1);
    out(1, q2);
    out(2, agree);
    out(3, appl);
    out(4, valid);
    out(5, inb);
}

// One byte of one word (trials 8k..8k+7 of the word): inw / au are the word's
// input and root planes in LDS, k the byte.  The outcome bytes overwrite bytes
// k of planes F[0..5] (every lane of the word reads its inputs before any lane
// writes: all reads of a byte come from its own lane, and each lane touches
// only its own byte k).
template <int N, uint32_t ME>
__device__ __forceinline__ void epilogue_byte(uint64_t* inw, const uint64_t* au, uint32_t k,
                                              TrialCounts& tc, uint32_t me_rt = ME) {
    uint8_t* ib = reinterpret_cast<uint8_t*>(inw) + k;
    const uint8_t* ab = reinterpret_cast<const uint8_t*>(au) + k;
    epilogue_core<N, ME, uint32_t>([&](int p) -> uint32_t { return ib[8 * p]; },
                                   [&](int b) -> uint32_t { return ab[8 * b]; },
                                   [&](int o, uint32_t v) { ib[8 * o] = (uint8_t)v; }, tc, me_rt);
}

template <int N, int W, uint32_t ME, int DIAG>
__device__ __forceinline__ void wave_epilogue(uint64_t* in0, const uint64_t* au0,
                                              uint32_t lane, uint64_t w0, uint64_t batch,
                                              uint64_t* __restrict__ decisions,
                                              uint8_t* __restrict__ outcome, TrialCounts& tc,
                                              uint32_t me_rt = ME) {
    constexpr int L = N - 1, NIN = N + 3;
    static_assert(L <= 16, "decision word: 2 bits per lieutenant in the low 32 bits");
    if constexpr ((DIAG & 32) != 0) {  // lab: near-free stand-in epilogue
        static_for<0, W>([&](auto wq) {
            const uint64_t i = (w0 + wq()) * 64 + lane;
            if (i < batch) decisions[i] = au0[wq() * 2 * L + (lane & 15)];
        });
        return;
    }
    for (uint32_t it = lane; it < (uint32_t)W * 8; it += 64)
        epilogue_byte<N, ME>(in0 + (it >> 3) * NIN, au0 + (it >> 3) * 2 * L, it & 7u, tc, me_rt);
    __builtin_amdgcn_wave_barrier();
    const uint32_t half = lane >> 5, sh = lane & 31;
    auto bit = [&](const uint64_t* p) -> uint32_t {
        return __builtin_amdgcn_ubfe(reinterpret_cast<const uint32_t*>(p)[half], sh, 1);
    };
#pragma unroll 2
    for (int w = 0; w < W; ++w) {
        const uint64_t* inw = in0 + w * NIN;
        const uint64_t* au = au0 + w * 2 * L;
        const uint64_t i = (w0 + w) * 64 + lane;
        const uint32_t live = bit(inw + N + 2);  // 0: not a trial of this batch
        uint32_t dec = 0, out = 0;
        static_for<0, L>([&](auto b) {
            dec |= bit(au + b()) << (2 * b());
            if constexpr (L % 2 == 0) dec |= bit(au + L + b()) << (2 * b() + 1);  // ties only at even L
        });
        static_for<0, 6>([&](auto k) { out |= bit(inw + k()) << k(); });
        if (live) {
            if (!(DIAG & 1) && decisions) decisions[i] = dec;
            if (!(DIAG & 2) && outcome) outcome[i] = (uint8_t)out;
        }
    }
}

// Wave sums of one task's run counters added into `mine` (lane c holds
// counter c).  Folding after every task keeps the C_NUM per-lane counters live
// only across the epilogue, not across the task's rounds (12 VGPRs).
__device__ __forceinline__ void wave_fold(const TrialCounts& tc, uint32_t lane, uint64_t& mine) {
#pragma unroll
    for (int c = 0; c < C_NUM; ++c) {
        const uint32_t x = wave_sum_u32(tc.v[c]);
        if (lane == (uint32_t)c) mine += x;
    }
}

// Run counters of the block from the waves' folded sums: the waves combine in
// LDS, then one sink unit per block.  Every wave of the block must call it (it
// contains a block barrier).
__device__ __forceinline__ void wave_flush_folded(uint64_t mine, uint32_t lane, uint32_t wv,
                                                  uint32_t wpb, uint64_t* __restrict__ counters,
                                                  const Sink& sk, bool skip) {
    __shared__ unsigned long long wcnt[kWaveThreads / 64][16];
    if (lane < 16) wcnt[wv][lane] = mine;
    __syncthreads();
    if (wv == 0 && !skip) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < wpb; ++k) tot += lane < 16 ? wcnt[k][lane] : 0;
        sink_counters(lane, tot, blockIdx.x, gridDim.x, counters, sk);
    }
}

// Run counters of the block: wave sums (lane c holds counter c), the waves
// combine in LDS, then one sink unit per block.  Every wave of the block
// must call it (it contains a block barrier).
__device__ __forceinline__ void wave_flush(const TrialCounts& tc, uint32_t lane, uint32_t wv,
                                           uint32_t wpb, uint64_t* __restrict__ counters,
                                           const Sink& sk, bool skip) {
    uint64_t mine = 0;
#pragma unroll
    for (int c = 0; c < C_NUM; ++c) {
        uint32_t x = tc.v[c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if (lane == (uint32_t)c) mine = x;
    }
    __shared__ unsigned long long wcnt[kWaveThreads / 64][16];
    if (lane < 16) wcnt[wv][lane] = mine;
    __syncthreads();
    if (wv == 0 && !skip) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < wpb; ++k) tot += lane < 16 ? wcnt[k][lane] : 0;
        sink_counters(lane, tot, blockIdx.x, gridDim.x, counters, sk);
    }
}

// Issue priority of the two waves sharing a SIMD alternates every round
// (wave slot parity): with equal priority the older wave takes nearly every
// VALU slot and the younger one finishes its task alone.
__device__ __forceinline__ void wave_alternate_priority(uint32_t round) {
    const uint32_t slot = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (3 << 11)) & 1u;
    if (((round + slot) & 1u) != 0) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// ---------------------------------------------------------------------------
// One first-hop round j1 of the depth-3 WAVE kernels (k_om3w; lab: k_om3q): lane
// (lw, la) resolves leaf block (j1, la) of trial word lw, then R1[j1, b] for
// b = la, which it returns (the receiver is lieutenant j2 = la + (la >= j1)).
//   in     the word's input planes F[N] OB OO VAL (LDS)
//   l0j1   L0[j1] of word lw
//   r2t    the wave's R2T scratch [W][C][C+1] (LDS): receiver-major, rows
//          padded to C+1 words so the column reads of step 3 are free of bank
//          conflicts (stride 9 words = 18 banks for n=10: 32 distinct bank pairs)
// Every lane of the wave calls it (it holds a wave barrier); lanes with !act
// return 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ P4 sel_p4(bool c, const P4& a, const P4& b) {
    return P4{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w};
}

// The value of lane ^ 1 (DPP quad_perm [1,0,3,2]: a VALU move, where
// __shfl_xor goes through ds_bpermute and waits out an LDS round trip).
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// Per-lane byte offsets (EROW mode of om3_round): K small offsets packed one
// per byte, fixed per lane for the whole kernel.  Addresses built from them
// inside the round (one byte-select add each) replace K loop-invariant address
// VGPRs that the compiler would otherwise hoist out of the round loop.
template <int K>
struct LaneBytes {
    static constexpr int NB = (K + 7) / 8;
    uint64_t b[NB];
    template <typename F>
    __device__ __forceinline__ explicit LaneBytes(F f) {
        static_for<0, NB>([&](auto k) { b[k()] = 0; });
        static_for<0, K>([&](auto i) { b[i() / 8] |= (uint64_t)(f(i()) & 0xffu) << (8 * (i() % 8)); });
    }
    template <int I>
    __device__ __forceinline__ uint32_t get() const {
        return (uint32_t)(b[I / 8] >> (8 * (I % 8))) & 0xffu;
    }
};

__device__ __forceinline__ void opaque_v(uint64_t& x) { asm volatile("" : "+v"(x)); }

// The two tables of lane (lw, la) in the depth-3 rounds (n <= 14: every
// offset < 256):
//   mem[a] = 8 (a + (a >= la)): member a's word in the E row (below)
//   r2t[d] = 8 (C + 1) (d >= la): member d's R2T row is d + (d >= la); the
//            8 (C + 1) d part is the store's immediate offset
// LDS row paddings of k_om3w (lab A/B only: tools/lds_bank_model.py predicts
// each group's bank conflicts; BA_OM3W_R2T_PAD = 1 keeps the R2T column reads
// conflict-free, BA_OM3W_R1T_PAD = 0 the R1T rows unpadded)
#ifndef BA_OM3W_R2T_PAD
#define BA_OM3W_R2T_PAD 1
#endif
#ifndef BA_OM3W_R1T_PAD
#define BA_OM3W_R1T_PAD 0
#endif
// lab ablations for the bank-conflict attribution (results wrong; never built
// into the product): drop the R2T leaf stores or the R1T store of a round
#ifndef BA_OM3W_LAB_NO_R2T
#define BA_OM3W_LAB_NO_R2T 0
#endif
#ifndef BA_OM3W_LAB_NO_R1T
#define BA_OM3W_LAB_NO_R1T 0
#endif
template <int N>
struct Om3LaneOffsets {
    static constexpr int S = N - 3, CP = N - 2 + BA_OM3W_R2T_PAD;
    LaneBytes<S> mem, r2t;
    __device__ __forceinline__ explicit Om3LaneOffsets(uint32_t la)
        : mem([la](int a) { return 8u * (a + ((uint32_t)a >= la ? 1u : 0u)); }),
          r2t([la](int d) { return (uint32_t)d >= la ? 8u * CP : 0u; }) {}
    // a copy the compiler cannot see through, taken once per round
    __device__ __forceinline__ Om3LaneOffsets round_copy() const {
        Om3LaneOffsets o = *this;
        static_for<0, LaneBytes<S>::NB>([&](auto k) {
            opaque_v(o.mem.b[k()]);
            opaque_v(o.r2t.b[k()]);
        });
        return o;
    }
};

// EROW = true (k_om3w, rounds in order j1 = 0, 1, ...): the members' faulty
// words come from the word's E row (erow: E[lw][0..C], E[C] a spare slot):
// E = the lieutenants other than j1 in rank order, which moves by ONE entry per
// round (E[j1] becomes lieutenant j1's word for round j1 + 1: the lanes with
// la == j1 write it, after this round's reads).  One byte extract + add per
// member instead of two rank compares, selects and shifts.  EROW = false
// (lab k_om3q: rounds in any order) ranks the members from j1 and j2 each round.
template <int N, bool EROW = false>
__device__ __forceinline__ uint64_t om3_round(const uint64_t* in, uint64_t l0j1, uint64_t* r2t_w,
                                              uint32_t lw, uint32_t la, bool act, uint32_t j1,
                                              uint64_t seed, uint64_t gw,
                                              uint64_t* erow = nullptr,
                                              const Om3LaneOffsets<N>* lo_ = nullptr) {
    constexpr int L = N - 1, S = N - 3, C = L - 1, CP = C + BA_OM3W_R2T_PAD;
    constexpr uint32_t ME = 3;
    const uint32_t sr = j1 * C + la;             // level-1 slot (j1, j2)
    const uint32_t j2 = la + (la >= j1);
    Om3LaneOffsets<N> ofs(0u);
    if constexpr (EROW) ofs = lo_->round_copy();
    if (act) {
        // the round's input planes, loaded before the Philox group so their
        // LDS latency hides under it: F[j1] (level-1 sender), F[j2] (level-2
        // sender) and the faulty words of the block's S members
        const uint64_t fj = in[j1 + 1], fs = in[j2 + 1];
        uint64_t Fm[S];
        if constexpr (EROW) {
            const char* eb = (const char*)erow;
            static_for<0, S>([&](auto a) {
                Fm[a()] = *(const uint64_t*)(eb + ofs.mem.template get<a()>());
            });
        } else {
            const uint32_t lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
            static_for<0, S>([&](auto a) {
                const uint32_t ida = a() + (a() >= lo) + (a() + 1 >= hi);  // member a's rank
                Fm[a()] = in[ida + 1];
            });
        }
        // 1. L1[j1, a] (sender j1 relays L0[j1]) and the level-2 diagonal
        //    pairs of leaf block (j1, a): one interleaved Philox group
        const uint32_t x0 = sr * S;
        constexpr int NPD = (S + 1) / 2;
        uint64_t lw2[2 * NPD], lie;
        if constexpr (S % 2 == 1 && C % 2 == 0) {
            // Lanes a, a^1 hold leaf blocks sr even / odd of one word: they
            // share the level-1 pair sr>>1 and one level-2 pair (the even
            // block's last = the odd block's first), 2*NPD distinct calls
            // for the two.  Each lane issues NPD of them and takes the
            // missing one from its partner: the even lane the shared
            // level-2 pair, the odd lane the level-1 pair.
            const bool odd = (sr & 1u) != 0;
            const uint32_t d0 = x0 >> 1;  // first level-2 pair of this block
            P4 pc[NPD];
            static_for<0, NPD>([&](auto qd) {
                const bool l1 = !odd && qd() == NPD - 1;
                pc[qd()] = P4{l1 ? (sr >> 1) : d0 + qd(), l1 ? 1u : 2u, (uint32_t)gw,
                              (uint32_t)(gw >> 32)};
            });
            philox10_n<NPD>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
            // even lane sends its level-1 pair, odd lane its first level-2 pair
            // (component-wise selects: a select of whole P4 values can become a
            // dynamically indexed scratch array)
            const P4 snd = sel_p4(odd, pc[0], pc[NPD - 1]);
            P4 rcv;
            rcv.x = swap_pair(snd.x);
            rcv.y = swap_pair(snd.y);
            rcv.z = swap_pair(snd.z);
            rcv.w = swap_pair(snd.w);
            const P4 p1 = sel_p4(odd, rcv, pc[NPD - 1]);
            static_for<0, NPD>([&](auto qd) {
                const P4 q = qd() == NPD - 1 ? sel_p4(odd, pc[qd()], rcv) : pc[qd()];
                lw2[2 * qd()] = (uint64_t)q.y << 32 | q.x;
                lw2[2 * qd() + 1] = (uint64_t)q.w << 32 | q.z;
            });
            lie = odd ? ((uint64_t)p1.w << 32 | p1.z) : ((uint64_t)p1.y << 32 | p1.x);
        } else {
            P4 pc[NPD + 1];
            static_for<0, NPD>([&](auto qd) {
                pc[qd()] = P4{(x0 >> 1) + qd(), 2u, (uint32_t)gw, (uint32_t)(gw >> 32)};
            });
            pc[NPD] = P4{sr >> 1, 1u, (uint32_t)gw, (uint32_t)(gw >> 32)};
            philox10_n<NPD + 1>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
            static_for<0, NPD>([&](auto qd) {
                lw2[2 * qd()] = (uint64_t)pc[qd()].y << 32 | pc[qd()].x;
                lw2[2 * qd() + 1] = (uint64_t)pc[qd()].w << 32 | pc[qd()].z;
            });
            lie = (sr & 1u) ? ((uint64_t)pc[NPD].w << 32 | pc[NPD].z)
                            : ((uint64_t)pc[NPD].y << 32 | pc[NPD].x);
        }
        const uint64_t par = (fj & lie) | (~fj & l0j1);
        // 2. leaf block (j1, a): level-2 diagonal (sender j2), then S(S-1) leaves
        const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
        uint64_t diag[S];
        static_for<0, S>([&](auto a) {
            uint64_t lie2;
            if constexpr (S % 2 == 1) lie2 = lw2[a()] ^ ((lw2[a()] ^ lw2[a() + 1]) & oddmask);
            else lie2 = lw2[a()];
            diag[a()] = (fs & lie2) | (~fs & par);
        });
        // receiver-major: member d of block a is receiver b = d + (d >= a)
        uint64_t* r2t = r2t_w + lw * C * CP + la;
        char* rb = (char*)r2t;
        leaf_block_emit<S>(ME, seed, gw, sr, diag, Fm, [&](auto d, uint64_t v) {
            if constexpr (BA_OM3W_LAB_NO_R2T) {  // lab ablation (wrong results): PMC attribution only
                asm volatile("" ::"v"(v));
            } else if constexpr (EROW) {
                *(uint64_t*)(rb + ofs.r2t.template get<d()>() + 8 * CP * d()) = v;
            } else {
                r2t[(d() + (d() >= la ? 1u : 0u)) * CP] = v;
            }
        });
        if constexpr (!BA_OM3W_LAB_NO_R2T) r2t[la * CP] = par;
        else asm volatile("" ::"v"(par));
    }
    __builtin_amdgcn_wave_barrier();
    uint64_t r1 = 0;
    if (act) {
        // 3. R1[j1, b], b = la: L1[j1, b] (this lane's own parent) plus
        //    column b of the word's other leaf blocks a' != b
        const uint64_t* col = r2t_w + (lw * C + la) * CP;
        uint64_t cv[C];
        static_for<0, C>([&](auto a) { cv[a()] = col[a()]; });
        // every column read in flight before the first add (left alone, the
        // scheduler waited out each ds_read2 in turn)
        __builtin_amdgcn_sched_barrier(0);
        Csa<planes_c(C)> cnt;
        static_for<0, C>([&](auto a) { cnt.template add<a()>(cv[a()]); });
        r1 = cnt.template ge<C, C / 2 + 1>();  // inner tie -> non-attack
        // E for round j1 + 1: E[j1] = lieutenant j1's word (this round's E reads
        // were issued above, and one wave's LDS operations complete in order);
        // the other lanes store to the row's spare slot E[C], so no branch
        if constexpr (EROW) erow[la == j1 ? la : (uint32_t)C] = in[j1 + 1];
    }
    __builtin_amdgcn_wave_barrier();  // r2t is rewritten by the next round
    return r1;
}

// ---------------------------------------------------------------------------
// k_om3w: effective depth 3 (see the WAVE engine note above)
// ---------------------------------------------------------------------------
template <int N>
struct Om3W {
    static constexpr int L = N - 1, S = N - 3, C = L - 1;
    static constexpr int W = 64 / C;               // trial words per wave task
    static constexpr int BPC = 2;                  // launch cap: blocks per CU
    static constexpr int LANES = W * C;            // lanes busy in the subtree rounds
    static constexpr int NIN = N + 3;
    static constexpr int CP = C + BA_OM3W_R2T_PAD;  // padded R2T row (om3_round)
    static constexpr int LP = L + BA_OM3W_R1T_PAD;  // R1T row
    // IN[W][NIN] | L0[W][L] | R2T[W][C][CP] | R1T[W][L][LP] (root inputs, receiver-major:
    // R1T[w][j2][j1] = R1[j1, j2], L0[j2] on the diagonal) ; A/U roots reuse R2T
    static constexpr int oIN = 0, oL0 = oIN + W * NIN, oR2 = oL0 + W * L, oR1 = oR2 + W * C * CP;
    static constexpr int oE = oR1 + W * L * LP;    // E[W][C + 1] (om3_round EROW mode)
    static constexpr int end0 = oE + W * (C + 1);
    static constexpr bool au_in_r2 = 2 * L <= C * CP;
    static constexpr int oAU = au_in_r2 ? oR2 : end0;
    static constexpr int words = ((au_in_r2 ? end0 : end0 + W * 2 * L) + 1) & ~1;
};

// Level 0 of a task's W words (one Philox per slot pair) into l0[w*L + j] and
// the diagonal r1t[(w*L + j)*L + j] (root column j counts L0[j] as its own input).
template <int N, int W, int LP = N - 1>
__device__ __forceinline__ void level0_r1t(const uint64_t* in0, uint64_t* l0, uint64_t* r1t,
                                           uint32_t lane, uint64_t seed, uint64_t gw0) {
    constexpr int L = N - 1, NIN = N + 3;
    constexpr uint32_t NP0 = (L + 1) / 2;
    for (uint32_t it = lane; it < (uint32_t)W * NP0; it += 64) {
        const uint32_t w = it / NP0, p = it - w * NP0;
        const uint64_t* in = in0 + w * NIN;
        const uint64_t F0 = in[0], ob = in[N];
        uint64_t lv[2];
        lie_pair(seed, 0, p, gw0 + w, lv[0], lv[1]);
        static_for<0, 2>([&](auto h) {
            const uint32_t j = 2 * p + h();
            if (j < (uint32_t)L) {
                const uint64_t v = (F0 & lv[h()]) | (~F0 & ob);
                l0[w * L + j] = v;
                r1t[(w * L + j) * LP + j] = v;
            }
        });
    }
}

// Root majorities of W words from R1T (L contiguous inputs per column, a
// compile-time carry-save count): strict majority attacks, a tie is
// "undefined" (ba.py:188-195; only an even L ties).  au[w*2L + b] = A,
// au[w*2L + L + b] = U.
template <int L, int W, int LP = L>
__device__ __forceinline__ void roots_r1t(const uint64_t* r1t0, uint64_t* au, uint32_t lane) {
    for (uint32_t it = lane; it < (uint32_t)W * L; it += 64) {
        const uint32_t w = it / L, col = it - w * L;
        const uint64_t* r1t = r1t0 + (w * L + col) * LP;
        Csa<planes_c(L)> cnt;
        static_for<0, L>([&](auto j) { cnt.template add<j()>(r1t[j()]); });
        const uint64_t att = cnt.template ge<L, L / 2 + 1>();
        au[w * 2 * L + col] = att;
        if constexpr (L % 2 == 0) au[w * 2 * L + L + col] = cnt.template ge<L, L / 2>() & ~att;
    }
}

// Hand-offs between waves of one launch through L2 (k_cascade): results
// are stored write-through (sc1: relaxed agent-scope atomic stores), drained,
// and announced with one atomic add; the arrival that completes a counter reads
// the others' results with sc1 loads only, after its add returned.  No wave ever
// waits for another.
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void store_sc1(uint64_t* p, uint64_t v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t load_sc1(const uint64_t* p) {
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// One arrival at counter c (lane 0 adds; every lane gets the answer): true on
// the arrival that completes `expect`, which also resets the counter.
__device__ __forceinline__ bool arrive_last(uint32_t* c, uint32_t expect, uint32_t lane) {
    uint32_t old = 0;
    if (lane == 0)
        old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
    const bool last = old + 1 == expect;
    if (last && lane == 0) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // compiler ordering only: no load of the children may move above the add
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return last;
}

// DIAG: lab-only ablation switches (tools/om3_lab.hip); the product uses 0.
// STAGED: both inputs given (ba_gen_inputs_device buffers): the task's inputs
// are loads and ballots only, the draw code is not compiled in.
// Occupancy target: 3 blocks of 4 waves per CU (<= 168 VGPRs, 3 waves/SIMD: a
// second step in flight fills the third slot) for n <= 10; the larger trees
// (172-215 VGPRs) stay at 2 rather than spill.  Round 3, one box's A/B
// (profiles/r03h_ab_vgpr_keys.log): the n=10 kernel at 168 VGPRs (2 spills)
// ran 50.3 us vs 50.4 us at 170, and the two-step bench 2.41-2.44e10 vs
// 2.26-2.31e10.
#ifndef BA_OM3W_MIN_BLOCKS
#define BA_OM3W_MIN_BLOCKS(n) ((n) <= 10 ? 3 : 2)
#endif
template <int N, int DIAG = 0, bool STAGED = false>
__global__ __launch_bounds__(kWaveThreads, BA_OM3W_MIN_BLOCKS(N)) void k_om3w(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk) {
    using G = Om3W<N>;
    constexpr int L = G::L, C = G::C, W = G::W, NIN = G::NIN;
    constexpr uint32_t ME = 3;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6,
                   wpb = blockDim.x >> 6;
    uint64_t* img = lds + (uint64_t)wv * G::words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W;
    uint64_t folded = 0;  // run counters folded per task (wave_fold)
    FUSED_STAMP_INIT();
#ifdef BA_FUSED_STAMPS
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // static task stride: the bench's 1M-trial launch has one task per wave, and
    // the dynamic counter of k_om4w cost this kernel 6 VGPRs (163 -> 169: no
    // third wave per SIMD for a second launch in flight)
    for (uint64_t task = (uint64_t)blockIdx.x * wpb + wv; task < ntasks;
         task += (uint64_t)gridDim.x * wpb) {
        // every lane-derived value is formed per task from the lane index (mbcnt,
        // no VGPR live across tasks): kept live across the task loop, they were
        // the values the register allocator spilled around the prologue
        uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        asm volatile("" : "+v"(lane));
        // this lane's (word, leaf block) in the subtree rounds
        const uint32_t lw_ = lane / C, la = lane - lw_ * C;
        const bool act = lane < (uint32_t)G::LANES;
        const uint32_t lw = act ? lw_ : 0;
        const Om3LaneOffsets<N> lofs(la);
        const uint64_t w0 = task * W;
        const uint64_t gw0 = (first_trial >> 6) + w0;
        if constexpr (STAGED)
            stage_words<N, W>(img + G::oIN, lane, w0, batch, faulty, order);
        else
            wave_inputs<N, W, DIAG>(img + G::oIN, lane, w0, seed, gs, first_trial, batch, faulty, order);
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(0);
        level0_r1t<N, W, G::LP>(img + G::oIN, img + G::oL0, img + G::oR1, lane, seed, gw0);
        // E row of round 0: lieutenants 1 .. L-1 (general g's word is in[g])
        const uint64_t* in = img + G::oIN + lw * NIN;
        uint64_t* erow = img + G::oE + lw * (C + 1);
        if (act) erow[la] = in[la + 2];
        __builtin_amdgcn_wave_barrier();
        // ---- subtree rounds ------------------------------------------------------
        const uint64_t gw = gw0 + lw;
        for (uint32_t j1 = 0; j1 < (uint32_t)L; ++j1) {
            // the issue priority of the SIMD's two waves alternates every round
            // (round 6: a one-stream launch 50.0 -> 48.8 us, two steps in flight the
            // same, profiles/r06za_om3w_prio_ab.log; round 2's kernel had measured
            // it 2.5 us slower).  DIAG & 8: lab, without
            if constexpr ((DIAG & 8) == 0) wave_alternate_priority(j1);
            const uint64_t r1 = om3_round<N, true>(in, act ? img[G::oL0 + lw * L + j1] : 0ull,
                                                   img + G::oR2, lw, la, act, j1, seed, gw,
                                                   erow, &lofs);
            FUSED_STAMP(1);
            // R1[j1, b] is root input j1 of receiver column j2(b)
            if constexpr (BA_OM3W_LAB_NO_R1T) asm volatile("" ::"v"(r1));  // lab ablation (wrong results)
            else if (act) img[G::oR1 + (lw * L + la + (la >= j1 ? 1u : 0u)) * G::LP + j1] = r1;
            FUSED_STAMP(2);
        }
        __builtin_amdgcn_wave_barrier();
        roots_r1t<L, W, G::LP>(img + G::oR1, img + G::oAU, lane);
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(3);
        {
            TrialCounts tc;
            wave_epilogue<N, W, ME, DIAG>(img + G::oIN, img + G::oAU, lane, w0, batch, decisions,
                                          outcome, tc);
            wave_fold(tc, lane, folded);
        }
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(4);
    }
    wave_flush_folded(folded, threadIdx.x & 63, wv, wpb, counters, sk, (DIAG & 4) != 0);
#ifdef BA_FUSED_STAMPS
    if ((threadIdx.x & 63) == 0 && blockIdx.x * wpb + wv < (uint32_t)kPartialRows)
    {
        for (int i = 0; i < 6; ++i) g_fused_stamps[blockIdx.x * wpb + wv][i] = st_acc[i];
        g_fused_stamps[blockIdx.x * wpb + wv][6] = rt0;
        // [5]: HW_ID | XCC_ID << 32 (s_getreg: id | offset << 6 | (size - 1) << 11)
        g_fused_stamps[blockIdx.x * wpb + wv][5] =
            __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) |
            ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)) << 32);
        g_fused_stamps[blockIdx.x * wpb + wv][7] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ---------------------------------------------------------------------------
// k_om4w: effective depth 4 (n=13, m=4 is SURVEY config 3).  Same wave-task
// design one level deeper: a round is a second-level subtree (j1, j2), whose
// C2 = L-2 level-2 slots (j1, j2, a) are C2 leaf blocks, so lane (w, a),
// w < W = 64 / C2, owns leaf block (j1, j2, a) of word w.  Per round:
//   1. one interleaved Philox group: L1[j1, j2], L2[j1, j2, a] (the lane's
//      leaf parent) and the level-3 diagonal pairs of its block
//   2. leaf block: R3[j1, j2, a, *] into LDS receiver-major (L2 on the
//      diagonal), as R2 in k_om3w
//   3. lane (w, b): R2[j1, j2, b] = maj over C2 contiguous words (carry-save),
//      added into the R1 counter of (w, j1, receiver), and L1[j1, j2] into
//      the R1 counter of (w, j1, j2)
// After the C1 = L-1 rounds of j1, R1[j1, c] (strict majority of C1 inputs)
// is added into the root counters; roots and epilogue are k_om3w's.
// LDS per wave: IN[W][N+3] | L0[W][L] | R3T[W][C2][C2] | R1C[W][C1][P1] |
// RC[W][L][P] ; A/U roots reuse R3T when it fits.
// ---------------------------------------------------------------------------
// k_om4w's occupancy target: 3 blocks of 4 waves per CU (3 waves per SIMD,
// <= 168 VGPRs; the launch cap below follows it).  Round 3: the column-ordered
// leaf schedule and staged inputs brought the kernel from 224 to 186 VGPRs, and
// the 3-wave bound costs a few spills outside the round loop (per first hop).
#ifndef BA_OM4W_BLOCKS_PER_CU
#define BA_OM4W_BLOCKS_PER_CU 3
#endif
// BA_OM4W_PAIRS = 1 (round 6): a round's Philox group drops from S/2 + 3 calls
// per lane to (S+1)/2.  (a) The level-1 lie words of a j1's C1 rounds come from
// ONE call per lane per j1 (W x NP1 pairs over the wave's lanes, into L1W in
// LDS), where every lane drew its round's level-1 pair.  (b) For odd S and even
// C2 (n = 7, 9, 11, 13) lanes 2k, 2k+1 hold blocks x2 even / odd of one word:
// they share the level-2 pair x2 >> 1 and the level-3 pair that straddles their
// blocks, so the even lane draws its five level-3 pairs (the straddling one
// last), the odd lane its four others and the level-2 pair, and each takes the
// missing one from its partner with a DPP swap -- and the diagonal lie words
// become one select per half between the two lanes' layouts, where the odd
// block's half-pair offset cost three ops per half.  0 = the round-5 group
// (lab A/B only).
#ifndef BA_OM4W_PAIRS
#define BA_OM4W_PAIRS 3  // bit 0: (a), bit 1: (b)
#endif
#define BA_OM4W_L1W ((BA_OM4W_PAIRS & 1) != 0)
#define BA_OM4W_XCH ((BA_OM4W_PAIRS & 2) != 0)
template <int N>
struct Om4W {
    static constexpr int L = N - 1, S = N - 4, C1 = L - 1, C2 = L - 2;
    static constexpr int W = 64 / C2;
    static constexpr int BPC = BA_OM4W_BLOCKS_PER_CU;  // launch cap: blocks per CU
    static constexpr int LANES = W * C2;
    static constexpr int P = planes_c(L), P1 = planes_c(C1);
    static constexpr int NIN = N + 3;
    static constexpr int oIN = 0, oL0 = oIN + W * NIN, oR3 = oL0 + W * L;
    static constexpr int oR1 = oR3 + W * C2 * C2, oRC = oR1 + W * C1 * P1;
    static constexpr int oE = oRC + W * L * P;   // E2[W][C2 + 1] (members, see k_om4w)
    // L1W[W][C1]: the level-1 lie words of the current j1's C1 rounds (BA_OM4W_PAIRS)
    static constexpr int NP1 = C1 / 2 + 1;       // Philox pairs that cover C1 slots
    static constexpr int oL1 = oE + W * (C2 + 1);
    static constexpr int end0 = oL1 + (BA_OM4W_L1W ? W * C1 : 0);
    static constexpr bool au_in_r3 = 2 * L <= C2 * C2;
    static constexpr int oAU = au_in_r3 ? oR3 : end0;
    static constexpr int words = ((au_in_r3 ? end0 : end0 + W * 2 * L) + 1) & ~1;
};

template <int N, bool STAGED = false>
__global__ __launch_bounds__(kWaveThreads, BA_OM4W_BLOCKS_PER_CU) void k_om4w(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk) {
    using G = Om4W<N>;
    constexpr int L = G::L, S = G::S, C1 = G::C1, C2 = G::C2, W = G::W, P = G::P, P1 = G::P1;
    constexpr int NIN = G::NIN;
    constexpr uint32_t ME = 4;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6,
                   wpb = blockDim.x >> 6;
    uint64_t* img = lds + (uint64_t)wv * G::words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W;
    // lane-derived values once per wave (k_om3w forms them per task; here that
    // measured 3% slower with staged inputs: profiles/r05n_om4w_lane_ab.log)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lw_ = lane / C2, la = lane - lw_ * C2;
    const bool act = lane < (uint32_t)G::LANES;
    const uint32_t lw = act ? lw_ : 0;
    // member a of lane la's leaf block is E2[a + (a >= la)]; member d's R3T row
    // is d + (d >= la) (the k_om3w tables, E2 in place of E, C2 in place of C + 1)
    const LaneBytes<S> mem([la](int a) { return 8u * (a + ((uint32_t)a >= la ? 1u : 0u)); });
    const LaneBytes<S> r3o([la](int d) { return (uint32_t)d >= la ? 8u * C2 : 0u; });
    uint64_t folded = 0;  // run counters folded per task (wave_fold)
    // tasks: the first wave-round static, then (sk.tasks != nullptr: a persistent
    // launch) each further task from the launch's atomic counter, fetched at the
    // start of the current task so its latency hides behind the task: a wave
    // that issues faster (a SIMD's older wave wins arbitration) takes more
    // tasks, instead of finishing its fixed share early and leaving its SIMD to
    // one wave for the rest of the launch
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    for (uint64_t task = (uint64_t)blockIdx.x * wpb + wv; task < ntasks;) {
        uint32_t next_raw = 0;
        if (sk.tasks != nullptr && lane == 0) next_raw = atomicAdd(sk.tasks, 1u);
        const uint64_t w0 = task * W;
        const uint64_t gw0 = (first_trial >> 6) + w0;
        if constexpr (STAGED)
            stage_words<N, W>(img + G::oIN, lane, w0, batch, faulty, order);
        else
            wave_inputs<N, W, 0>(img + G::oIN, lane, w0, seed, gs, first_trial, batch, faulty, order);
        __builtin_amdgcn_wave_barrier();
        wave_level0<N, W, P>(img + G::oIN, img + G::oL0, img + G::oRC, lane, seed, gw0);
        __builtin_amdgcn_wave_barrier();
        const uint64_t* in = img + G::oIN + lw * NIN;
        uint64_t* erow = img + G::oE + lw * (C2 + 1);
        const uint64_t gw = gw0 + lw;
        uint32_t round = 0;
        for (uint32_t j1 = 0; j1 < (uint32_t)L; ++j1) {
            // R1 counters of this j1 start at zero
            for (uint32_t it = lane; it < (uint32_t)(W * C1 * P1); it += 64) img[G::oR1 + it] = 0;
            // E2 of round (j1, c2 = 0): the lieutenants other than j1 and j2 = the
            // first non-j1, ascending, i.e. non-j1 ranks 1 .. C1-1 (a faulty word of
            // lieutenant j sits at in[j + 1]).  Each round c2 then moves E2 by one
            // entry: E2[c2] becomes j2(c2)'s word (below).
            if (act) {
                const uint32_t r = la + 1;
                erow[la] = in[r + (r >= j1 ? 1u : 0u) + 1];
            }
            __builtin_amdgcn_wave_barrier();
            const uint64_t fj1 = in[j1 + 1];
            const uint64_t l0j1 = img[G::oL0 + lw * L + j1];
            if constexpr (BA_OM4W_L1W) {
                // L1W[w][c2] = the lie word of level-1 slot j1*C1 + c2 of word w:
                // lane (w, i) draws pair (j1*C1 >> 1) + i and keeps its in-range halves
                static_assert(W * G::NP1 <= 64, "one L1 pair per lane");
                const uint32_t s0 = j1 * C1;
                if (lane < (uint32_t)(W * G::NP1)) {
                    const uint32_t w = lane / G::NP1, i = lane - w * G::NP1, pr = (s0 >> 1) + i;
                    const uint64_t g1 = gw0 + w;
                    P4 q[1] = {P4{pr, 1u, (uint32_t)g1, (uint32_t)(g1 >> 32)}};
                    philox_groups<1>(q, (uint32_t)seed, (uint32_t)(seed >> 32));  // the rounds' code shape
                    const uint64_t h0 = (uint64_t)q[0].y << 32 | q[0].x, h1 = (uint64_t)q[0].w << 32 | q[0].z;
                    const uint32_t c0 = 2 * pr - s0;  // c2 of the pair's first half (may be -1)
                    if (c0 < (uint32_t)C1) img[G::oL1 + w * C1 + c0] = h0;
                    if (c0 + 1 < (uint32_t)C1) img[G::oL1 + w * C1 + c0 + 1] = h1;
                }
                __builtin_amdgcn_wave_barrier();
            }
            for (uint32_t c2 = 0; c2 < (uint32_t)C1; ++c2, ++round) {
                // unlike k_om3w, the per-round priority alternation pays here
                // (config 3 A/B, round 2: without it 2.8% slower; R3T rows padded
                // as k_om3w's R2T: 0.6% slower)
                wave_alternate_priority(round);
                const uint32_t j2 = c2 + (c2 >= j1);
                const uint32_t x1 = j1 * C1 + c2;     // level-1 slot (j1, j2)
                const uint32_t x2 = x1 * C2 + la;     // level-2 slot (j1, j2, j3): leaf block
                // j3 = E2[la] (the la-th lieutenant other than j1, j2); its rank
                // among the non-j1 lieutenants is la + (la >= c2)
                uint64_t par = 0, l1v = 0;
                // the byte tables pass through an empty asm each round, so their
                // addresses are formed here, not hoisted into 2S live VGPRs
                LaneBytes<S> memr = mem, r3r = r3o;
                static_for<0, LaneBytes<S>::NB>([&](auto k) {
                    opaque_v(memr.b[k()]);
                    opaque_v(r3r.b[k()]);
                });
                if (act) {
                    const uint32_t x3 = x2 * S;
                    constexpr int NPD = (S + 1) / 2;
                    auto lo = [](const P4& q) { return (uint64_t)q.y << 32 | q.x; };
                    auto hi = [](const P4& q) { return (uint64_t)q.w << 32 | q.z; };
                    uint64_t lie3[S], lie2, lie1;
                    if constexpr (BA_OM4W_XCH && S % 2 == 1 && C2 % 2 == 0) {
                        // (b): x2 & 1 == la & 1; the odd lane's x3 >> 1 is the
                        // straddling pair, its own pairs follow it
                        const bool odd = (la & 1u) != 0;
                        P4 pc[NPD];
                        static_for<0, NPD - 1>([&](auto qd) {
                            pc[qd()] = P4{(x3 >> 1) + qd() + (odd ? 1u : 0u), 3u, (uint32_t)gw,
                                          (uint32_t)(gw >> 32)};
                        });
                        pc[NPD - 1] = odd ? P4{x2 >> 1, 2u, (uint32_t)gw, (uint32_t)(gw >> 32)}
                                          : P4{(x3 >> 1) + NPD - 1, 3u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                        philox_groups<NPD>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
                        // the half the partner needs of this lane's last call: the even
                        // lane's straddling pair's second half (the odd block's first
                        // slot), the odd lane's level-2 pair's first half (x2 even)
                        const P4& l4 = pc[NPD - 1];
                        const uint32_t s0x = odd ? l4.x : l4.z, s0y = odd ? l4.y : l4.w;
                        const uint64_t rcv = (uint64_t)swap_pair(s0y) << 32 | swap_pair(s0x);
                        // slot x3 + d: even lane half d&1 of pair d>>1; odd lane d = 0 the
                        // straddling pair's second half, else half (d-1)&1 of pair (d-1)>>1
                        static_for<0, S>([&](auto d) {
                            constexpr int e = d();
                            const uint64_t ev = (e & 1) ? hi(pc[e >> 1]) : lo(pc[e >> 1]);
                            uint64_t ov;
                            if constexpr (e == 0) ov = rcv;
                            else ov = ((e - 1) & 1) ? hi(pc[(e - 1) >> 1]) : lo(pc[(e - 1) >> 1]);
                            lie3[e] = odd ? ov : ev;
                        });
                        lie2 = odd ? hi(l4) : rcv;
                        if constexpr (!BA_OM4W_L1W) {  // lab A/B (bit 0 off): the round's own level-1 call
                            uint64_t h0, h1;
                            lie_pair(seed, 1, x1 >> 1, gw, h0, h1);
                            lie1 = (x1 & 1u) ? h1 : h0;
                        }
                    } else {
                        constexpr int NG = NPD + (BA_OM4W_L1W ? 1 : 2);
                        P4 pc[NG];
                        static_for<0, NPD>([&](auto qd) {
                            pc[qd()] = P4{(x3 >> 1) + qd(), 3u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                        });
                        pc[NPD] = P4{x2 >> 1, 2u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                        if constexpr (!BA_OM4W_L1W) pc[NG - 1] = P4{x1 >> 1, 1u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                        // at most 4 calls in flight (philox10_n's one-statement rounds;
                        // 7 interleaved calls held ~70 VGPRs at once)
                        philox_groups<NG>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
                        uint64_t lw3[2 * NPD];
                        static_for<0, NPD>([&](auto qd) {
                            lw3[2 * qd()] = lo(pc[qd()]);
                            lw3[2 * qd() + 1] = hi(pc[qd()]);
                        });
                        const uint64_t oddmask = 0ull - (uint64_t)(x3 & 1u);
                        static_for<0, S>([&](auto d) {
                            if constexpr (S % 2 == 1) lie3[d()] = lw3[d()] ^ ((lw3[d()] ^ lw3[d() + 1]) & oddmask);
                            else lie3[d()] = lw3[d()];
                        });
                        lie2 = (x2 & 1u) ? hi(pc[NPD]) : lo(pc[NPD]);
                        if constexpr (!BA_OM4W_L1W) lie1 = (x1 & 1u) ? hi(pc[NG - 1]) : lo(pc[NG - 1]);
                    }
                    if constexpr (BA_OM4W_L1W) lie1 = img[G::oL1 + lw * C1 + c2];  // (a)
                    l1v = (fj1 & lie1) | (~fj1 & l0j1);              // L1[j1, j2], sender j1
                    const uint64_t fj2 = in[j2 + 1];
                    par = (fj2 & lie2) | (~fj2 & l1v);               // L2[j1, j2, j3], sender j2
                    // members of leaf block (j1, j2, j3): the lieutenants not in
                    // {j1, j2, j3}, ascending = E2 without its entry la
                    const uint64_t fs = erow[la];  // level-3 sender: j3
                    const char* eb = (const char*)erow;
                    uint64_t diag[S], Fm[S];
                    static_for<0, S>([&](auto d) {
                        diag[d()] = (fs & lie3[d()]) | (~fs & par);
                        Fm[d()] = *(const uint64_t*)(eb + memr.template get<d()>());
                    });
                    uint64_t* r3t = img + G::oR3 + lw * C2 * C2 + la;
                    char* rb = (char*)r3t;
                    leaf_block_emit<S>(ME, seed, gw, x2, diag, Fm, [&](auto d, uint64_t v) {
                        *(uint64_t*)(rb + r3r.template get<d()>() + 8 * C2 * d()) = v;
                    });
                    r3t[la * C2] = par;
                }
                __builtin_amdgcn_wave_barrier();
                if (act) {
                    // R2[j1, j2, b], b = la (receiver: the la-th lieutenant not in {j1, j2})
                    const uint64_t* col = img + G::oR3 + (lw * C2 + la) * C2;
                    Csa<planes_c(C2)> cnt;
                    static_for<0, C2>([&](auto a) { cnt.template add<a()>(col[a()]); });
                    const uint64_t r2 = cnt.template ge<C2, C2 / 2 + 1>();  // inner tie -> non-attack
                    // receiver j3 as a rank among the non-j1 lieutenants
                    planes_add<P1>(img + G::oR1 + (lw * C1 + la + (la >= c2 ? 1u : 0u)) * P1, r2);
                    // E2 for round c2 + 1: E2[c2] = j2's word (this round's E2 reads
                    // were issued above, and one wave's LDS operations complete in
                    // order); the other lanes store to the spare slot E2[C2]
                    erow[la == c2 ? la : (uint32_t)C2] = in[j2 + 1];
                }
                __builtin_amdgcn_wave_barrier();
                if (act && la == 0) planes_add<P1>(img + G::oR1 + (lw * C1 + c2) * P1, l1v);
                __builtin_amdgcn_wave_barrier();
            }
            // R1[j1, c] -> root column c (rank among the non-j1) -> general rank
            for (uint32_t it = lane; it < (uint32_t)(W * C1); it += 64) {
                const uint32_t w = it / C1, c = it - w * C1;
                const uint64_t* r1c = img + G::oR1 + (w * C1 + c) * P1;
                Count<P1> cnt;
                static_for<0, P1>([&](auto q) { cnt.c[q()] = r1c[q()]; });
                const uint64_t r1 = cnt.ge(C1 / 2 + 1);  // inner tie -> non-attack
                planes_add<P>(img + G::oRC + (w * L + c + (c >= j1 ? 1u : 0u)) * P, r1);
            }
            __builtin_amdgcn_wave_barrier();
        }
        wave_roots<L, W, P>(img + G::oRC, img + G::oAU, lane);
        __builtin_amdgcn_wave_barrier();
        {
            TrialCounts tc;
            wave_epilogue<N, W, ME, 0>(img + G::oIN, img + G::oAU, lane, w0, batch, decisions, outcome, tc);
            wave_fold(tc, lane, folded);
        }
        __builtin_amdgcn_wave_barrier();
        task = sk.tasks != nullptr ? nwaves + __builtin_amdgcn_readfirstlane(next_raw) : task + nwaves;
    }
    wave_flush_folded(folded, lane, wv, wpb, counters, sk, false);
}

// WAVE engine launch: one wave per W-word task, 4 independent waves per block,
// at most two blocks per CU (two waves per SIMD, the kernels' register budget)
// and a persistent task loop.  `staged` (optional) replaces `kernel` when both
// inputs are given.
template <typename G, typename K>
inline hipError_t launch_wave(const RunArgs& a, K kernel, const char* name, K staged = nullptr,
                              bool dyn_tasks = false) {
    if (staged && a.gen.faulty_mode == 0 && a.gen.order_mode == 0) kernel = staged;
    constexpr uint32_t wpb = kWaveThreads / 64;
    const uint64_t words = (a.batch + 63) / 64, tasks = (words + G::W - 1) / G::W;
    uint64_t blocks = (tasks + wpb - 1) / wpb;
    uint64_t cap = (uint64_t)G::BPC * a.cu_count;
    if (const char* e = getenv("BA_WAVE_MAX_BLOCKS")) {  // tests: force the persistent task loop
        const uint64_t c = strtoull(e, nullptr, 0);
        if (c >= 1 && c < cap) cap = c;
    }
    if (blocks > cap) blocks = cap;
    // persistent launch (more tasks than waves) of a kernel with the dynamic loop
    // (k_om4w): task assignment from the ctx's counter, zeroed on the launch's
    // stream (BA_WAVE_STATIC_TASKS=1: the static stride loop, A/B only)
    Sink sk = a.sink;
    const bool stat = getenv("BA_WAVE_STATIC_TASKS") && atoi(getenv("BA_WAVE_STATIC_TASKS")) != 0;
    if (!dyn_tasks || stat || tasks <= blocks * wpb || sk.tasks == nullptr) {
        sk.tasks = nullptr;
    } else {
        const hipError_t e = hipMemsetAsync(sk.tasks, 0, sizeof(unsigned int), a.stream);
        if (e != hipSuccess) return e;
    }
    ProfScope ps(a.prof, name, a.stream);
    hipLaunchKernelGGL(kernel, dim3((uint32_t)blocks), dim3(kWaveThreads), wpb * G::words * 8,
                       a.stream, a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order,
                       a.decisions, a.outcome, a.counters, sk);
    return hipGetLastError();
}

}  // namespace ba
