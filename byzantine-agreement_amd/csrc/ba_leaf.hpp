// ba_leaf.hpp -- device code shared by the leaf-fused engines (k_leaf,
// k_fused*, the WAVE kernels): compile-time loops, the leaf-block column
// majorities, and the diagnostic phase stamps of the lab builds.
#pragma once
#include "ba_engine.hpp"

namespace ba {

constexpr int planes_c(int s) { return s < 2 ? 1 : (s < 4 ? 2 : (s < 8 ? 3 : (s < 16 ? 4 : 5))); }

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  Every
// register-array index in the leaf code goes through this, so no index is ever
// dynamic (a dynamic index would send the array to scratch memory).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Column majorities of one leaf block.  diag[a] = L_{me-1}[sigma.j_a] (the
// direct value, also every loyal row's broadcast), Fm[a] = faulty word of j_a.
// Column b counts diag[b] then rows a != b in row order, so the carry-save
// counters see a compile-time input schedule (Csa, ba_device.hpp).
// The S(S-1)/2 Philox calls run in interleaved groups of PG (philox10_n);
// each group's 2*PG lie words feed the counters before the next group starts.
// The S = 11 leaf (config 5, n=16 m=5: 55 pairs) in groups of 5: 11 full groups
// where groups of 3 left a lone call at the end; one lease, A B A B
// (profiles/r05i_c5_leaf_groups_ab.log): 1024-instance calls 59.4-60.4 vs
// 60.7-61.1 us on one stream, 48.7-49.4 vs 49.9-50.3 us with two in flight
// (groups of 6: 61.9-62.5); one instance 16.8-16.9 vs 16.5 us.
constexpr int leaf_philox_group(int npair) {
    return npair == 55 ? 5 : (npair % 3 == 0 ? 3 : (npair % 4 == 0 ? 4 : (npair % 2 == 0 ? 2 : 3)));
}

// Column-ordered schedule (S - 1 even: a slot pair never straddles two rows).
// Step t takes pair q(t) = a (S-1)/2 + cp with cp = t / S, a = t % S: the pairs
// of one column pair cp = c/2 for every row a, then the next cp.  Receiver
// b = c + (c >= a) of a slot (a, c) stays within {c, c+1, c+2}, so a column is
// complete a few steps after it starts and its majority is taken right then:
// about three columns' counters are live at a time instead of all S (row order
// feeds every column from the first row to the last).  Counts do not depend on
// the input order, so the results are identical.
struct LeafSched {
    static constexpr int slot_recv(int S, int e) {
        const int a = e / (S - 1), c = e % (S - 1);
        return c + (c >= a ? 1 : 0);
    }
    static constexpr int step_pair(int S, int t) { return (t % S) * ((S - 1) / 2) + t / S; }
    // inputs column b holds before slot h of step t (its diag value counts as one)
    static constexpr int inputs_before(int S, int b, int t, int h) {
        int k = 1;
        for (int u = 0; u <= t; ++u)
            for (int hh = 0; hh < 2; ++hh) {
                if (u == t && hh >= h) return k;
                if (slot_recv(S, 2 * step_pair(S, u) + hh) == b) ++k;
            }
        return k;
    }
    static constexpr int last_step(int S, int b) {
        int last = -1;
        for (int u = 0; u < S * (S - 1) / 2; ++u)
            for (int hh = 0; hh < 2; ++hh)
                if (slot_recv(S, 2 * step_pair(S, u) + hh) == b) last = u;
        return last;
    }
};

// emit(b, R_b) receives column b's majority as soon as the column is complete
// (a caller that stores it right away keeps no result registers live).
template <int S, typename Emit>
__device__ __forceinline__ void leaf_block_cols(uint32_t me, uint64_t seed, uint64_t gw,
                                                uint32_t sr, const uint64_t (&diag)[S],
                                                const uint64_t (&Fm)[S], Emit&& emit) {
    constexpr int NL = planes_c(S);
    constexpr int NPAIR = S * (S - 1) / 2;
    constexpr int PG = leaf_philox_group(NPAIR);
    Csa<NL> cnt[S];
    static_for<0, S>([&](auto b) { cnt[b()].template add<0>(diag[b()]); });
    const uint32_t pair0 = sr * (uint32_t)NPAIR;
    static_for<0, (NPAIR + PG - 1) / PG>([&](auto grp) {
        constexpr int t0 = grp() * PG, ng = NPAIR - t0 < PG ? NPAIR - t0 : PG;
        P4 c[ng];
        static_for<0, ng>([&](auto g) {
            uint32_t cx = pair0 + (uint32_t)LeafSched::step_pair(S, t0 + g());
#ifndef BA_LEAF_CTR_FOLD
            // opaque: the round-0 product is one v_mad_u64_u32 of this word, not a
            // 64-bit add of M0 * pair0 and an SGPR-pair constant M0 * q (21 such
            // pairs per leaf block held 42 SGPRs and spilled SGPRs to VGPR lanes)
            asm("" : "+v"(cx));
#endif
            c[g()] = P4{cx, me, (uint32_t)gw, (uint32_t)(gw >> 32)};
        });
        philox10_n<ng>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        static_for<0, ng>([&](auto g) {
            constexpr int t = t0 + g(), q = LeafSched::step_pair(S, t);
            static_for<0, 2>([&](auto h) {
                constexpr int e = 2 * q + h();
                constexpr int a = e / (S - 1);
                constexpr int b = LeafSched::slot_recv(S, e);
                constexpr int K = LeafSched::inputs_before(S, b, t, h());
                const uint64_t lw = h() == 0 ? ((uint64_t)c[g()].y << 32 | c[g()].x)
                                             : ((uint64_t)c[g()].w << 32 | c[g()].z);
                cnt[b].template add<K>((Fm[a] & lw) | (~Fm[a] & diag[a]));
            });
            // columns whose last input was this step: majority now, counters die
            static_for<0, S>([&](auto b) {
                if constexpr (LeafSched::last_step(S, b()) == t)
                    emit(b, cnt[b()].template ge<S, S / 2 + 1>());
            });
        });
    });
}

template <int S>
__device__ __forceinline__ void leaf_block(uint32_t me, uint64_t seed, uint64_t gw, uint32_t sr,
                                           const uint64_t (&diag)[S], const uint64_t (&Fm)[S],
                                           uint64_t (&R)[S]) {
#ifndef BA_LEAF_ROW_ORDER
    if constexpr (S >= 3 && (S - 1) % 2 == 0) {
        leaf_block_cols<S>(me, seed, gw, sr, diag, Fm,
                           [&](auto b, uint64_t v) { R[b()] = v; });
        return;
    }
#endif
    constexpr int NL = planes_c(S);
    constexpr int NPAIR = S * (S - 1) / 2;
    constexpr int PG = leaf_philox_group(NPAIR);
    Csa<NL> cnt[S];
    static_for<0, S>([&](auto b) { cnt[b()].template add<0>(diag[b()]); });
    const uint32_t pair0 = sr * (uint32_t)NPAIR;  // leaf block base slot sr*S*(S-1) is even
    static_for<0, (NPAIR + PG - 1) / PG>([&](auto grp) {
        constexpr int q0 = grp() * PG, ng = NPAIR - q0 < PG ? NPAIR - q0 : PG;
        uint64_t lw[2 * ng];
        lie_pairs<ng>(seed, me, pair0 + q0, gw, lw);
        static_for<0, 2 * ng>([&](auto h) {
            constexpr int e = 2 * q0 + h();      // slot within the block: row a, column c
            constexpr int a = e / (S - 1);
            constexpr int c = e % (S - 1);
            constexpr int b = c + (c >= a);      // receiver's rank among the S members
            constexpr int K = 1 + a - (b < a ? 1 : 0);  // inputs column b holds so far
            cnt[b].template add<K>((Fm[a] & lw[h()]) | (~Fm[a] & diag[a]));
        });
    });
    // S inputs per column; strict majority, inner tie -> non-attack
    static_for<0, S>([&](auto b) { R[b()] = cnt[b()].template ge<S, S / 2 + 1>(); });
}

// leaf_block with the results handed to emit(b, R_b) (std::integral_constant b):
// right when each column completes under the column schedule, at the end
// otherwise.
template <int S, typename Emit>
__device__ __forceinline__ void leaf_block_emit(uint32_t me, uint64_t seed, uint64_t gw,
                                                uint32_t sr, const uint64_t (&diag)[S],
                                                const uint64_t (&Fm)[S], Emit&& emit) {
#ifndef BA_LEAF_ROW_ORDER
    if constexpr (S >= 3 && (S - 1) % 2 == 0) {
        leaf_block_cols<S>(me, seed, gw, sr, diag, Fm, emit);
        return;
    }
#endif
    uint64_t R[S];
    leaf_block<S>(me, seed, gw, sr, diag, Fm, R);
    static_for<0, S>([&](auto b) { emit(b, R[b()]); });
}

// Bit-sliced count of one matrix column in an LDS word image: the direct value
// img[diag] plus the child results of rows a != b of prefix sr (s members).
template <int P>
__device__ __forceinline__ Count<P> column_count(const uint64_t* img, uint32_t diag,
                                                 uint32_t child, uint32_t sr, uint32_t s,
                                                 uint32_t b) {
    Count<P> cnt;
    cnt.add(img[diag]);
    const uint32_t base = child + sr * s * (s - 1);
    for (uint32_t a = 0; a < b; ++a) cnt.add(img[base + a * (s - 1) + b - 1]);
    for (uint32_t a = b + 1; a < s; ++a) cnt.add(img[base + a * (s - 1) + b]);
    return cnt;
}

// Diagnostic build only (tools/fused_lab.hip defines BA_FUSED_STAMPS): thread 0
// of every block sums s_memtime cycles per phase; no output depends on them.
#ifdef BA_FUSED_STAMPS
__device__ unsigned long long g_fused_stamps[kPartialRows][8];
#define FUSED_STAMP_INIT() unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_acc[6] = {0, 0, 0, 0, 0, 0}
#define FUSED_STAMP(i)                                              \
    do {                                                            \
        const unsigned long long st_now = __builtin_amdgcn_s_memtime(); \
        st_acc[i] += st_now - st_prev;                              \
        st_prev = st_now;                                           \
    } while (0)
#define FUSED_STAMP_STORE()                                                      \
    if (tid == 0)                                                                \
        for (int i = 0; i < 6; ++i) g_fused_stamps[blockIdx.x][i] = st_acc[i]
#else
#define FUSED_STAMP_INIT()
#define FUSED_STAMP(i)
#define FUSED_STAMP_STORE()
#endif

}  // namespace ba
