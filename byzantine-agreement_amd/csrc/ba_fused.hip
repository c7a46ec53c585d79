// ba_fused.hip -- leaf-fused OM(m) kernels for gfx950.
//
// The leaf level L_me holds 84-90% of an OM tree's slots (n=10,m=3: 3024 of
// 3609), yet every leaf is a pure function of its parent and a lie bit:
//     L_me[sigma.j.r] = F[j] ? lie(me, slot) : L_{me-1}[sigma.j]
// so the leaf-parent majority R_{me-1}[sigma.r] can be computed straight from
// L_{me-1}[sigma.*] and freshly generated lies, without ever writing L_me.
// One thread owns one leaf block (sigma, 64-trial word): S = n - me members,
// S(S-1) leaf slots = S(S-1)/2 Philox4x32-10 calls (two slot-words each), and
// S bit-sliced column counters in registers.  Fully unrolled on S, so every
// (row, column) index is a compile-time constant.
//
//   k_leaf<S>   LEVELS engine: reads L_{me-1} from HBM, writes R_{me-1} to HBM.
//   k_fused<S>  FUSED engine: a block owns WPB trial words and runs the whole
//               tree for them in LDS (input bit-slicing, top relay levels,
//               leaf blocks, inner majorities, root + quorum epilogue).  HBM
//               traffic is the per-trial outputs only.
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
constexpr int leaf_philox_group(int npair) { return npair % 3 == 0 ? 3 : (npair % 4 == 0 ? 4 : (npair % 2 == 0 ? 2 : 3)); }

template <int S>
__device__ __forceinline__ void leaf_block(uint32_t me, uint64_t seed, uint64_t gw, uint32_t sr,
                                           const uint64_t (&diag)[S], const uint64_t (&Fm)[S],
                                           uint64_t (&R)[S]) {
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

// ---------------------------------------------------------------------------
// LEVELS: one thread per (leaf block, word)
// ---------------------------------------------------------------------------
// Leaf blocks sr = srbase + idx / W (a first-hop subtree range of level me-2);
// L_{me-1} / R_{me-1} are indexed from the range's first block.
template <int S>
__global__ __launch_bounds__(256) void k_leaf(uint32_t me, uint64_t seed, uint64_t gw0,
                                              FastDiv divW, uint32_t work, uint32_t srbase,
                                              const uint64_t* __restrict__ Lm1,
                                              const uint64_t* __restrict__ F,
                                              const uint64_t* __restrict__ members,
                                              uint64_t* __restrict__ Rm1) {
    const uint32_t W = divW.d;
    for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < work; idx += gridDim.x * 256) {
        const uint32_t sl = fdiv(idx, divW);
        const uint32_t w = idx - sl * W;
        const uint32_t sr = srbase + sl;
        const uint64_t mem = members[sr];  // S member ids, 5 bits each
        uint64_t diag[S], Fm[S], R[S];
        static_for<0, S>([&](auto a) {
            const uint64_t x = (uint64_t)sl * S + a();
            diag[a()] = Lm1[x * W + w];
            Fm[a()] = F[((mem >> (5 * a())) & 31u) * W + w];
        });
        leaf_block<S>(me, seed, gw0 + w, sr, diag, Fm, R);
        static_for<0, S>([&](auto b) { Rm1[((uint64_t)sl * S + b()) * W + w] = R[b()]; });
    }
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

// ---------------------------------------------------------------------------
// FUSED: one block per group of WPB trial words, everything in LDS
// ---------------------------------------------------------------------------
// Per-word LDS image (uint64 words), offsets from FusedPlan:
//   F[n] OB OO VAL | L_0 .. L_{me-2} | R_1 .. R_{me-1}
// The plan is read through a device pointer (scalar loads): its per-level
// arrays are indexed by runtime level numbers, which a by-value kernel
// argument would turn into a private (scratch) copy.
template <int S>
__global__ __launch_bounds__(kFusedThreads, (S <= 7 ? 4 : 2)) void k_fused(
    const FusedPlan* __restrict__ fpp, uint64_t seed, GenSpec gs, uint64_t first_trial,
    uint64_t batch, const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    const uint8_t* __restrict__ sender, const uint64_t* __restrict__ members,
    uint64_t* __restrict__ decisions,
    uint8_t* __restrict__ outcome, uint64_t* __restrict__ counters, Sink sk) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    // run counters live in LDS (not in registers across the leaf stage)
    __shared__ __attribute__((aligned(16))) unsigned long long blockcnt[16];
    const FusedPlan& fp = *fpp;
    const uint32_t n = fp.n, L = n - 1, me = fp.me, WPB = fp.wpb, T = blockDim.x;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t stride = fp.word_stride;  // uint64 words per trial word in LDS
    if (tid < 16) blockcnt[tid] = 0;
    FUSED_STAMP_INIT();
    const uint64_t total_words = (batch + 63) / 64;
    // balanced persistent grid: block b owns a contiguous run of words, taken
    // in groups of at most WPB (the grid is one block per resident slot, so a
    // partial last round of groups never idles most of the chip)
    const uint64_t per_block = (total_words + gridDim.x - 1) / gridDim.x;
    const uint64_t wbeg = (uint64_t)blockIdx.x * per_block;
    const uint64_t wend = wbeg + per_block < total_words ? wbeg + per_block : total_words;
    for (uint64_t w0 = wbeg; w0 < wend; w0 += WPB) {
        const uint32_t nw = (uint32_t)(wend - w0 < WPB ? wend - w0 : WPB);  // words this group
        // ---- A: inputs -> bit-sliced words (one wave per word) -----------------
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            uint64_t* img = lds + (uint64_t)lw * stride;
            const uint64_t i = (w0 + lw) * 64 + lane;
            const bool valid = (w0 + lw) < total_words && i < batch;
            uint32_t fm = 0, oc = 0;
            if (valid) {
                if (gs.faulty_mode == 0) fm = faulty[i];
                if (gs.order_mode == 0) oc = order[i];
                gen_trial(n, seed, gs, first_trial + i, fm, oc);
            }
            uint64_t mine = 0;
            for (uint32_t g = 0; g < n; ++g) {
                const uint64_t b = __ballot(valid && ((fm >> g) & 1u));
                if (lane == g) mine = b;
            }
            const uint64_t ob = __ballot(valid && oc == 1);
            const uint64_t oo = __ballot(valid && oc == 2);
            const uint64_t vv = __ballot(valid);
            if (lane < n) img[lane] = mine;
            if (lane == 0) {
                img[n] = ob;
                img[n + 1] = oo;
                img[n + 2] = vv;
            }
        }
        __syncthreads();
        FUSED_STAMP(0);
        const uint64_t gwg = (first_trial >> 6) + w0;  // global word of lw = 0
        // ---- B: relay levels 0..me-2, one Philox per (slot pair, word) ----------
        // (level me-1, the leaf blocks' diagonal, is generated by the leaf
        // threads themselves in stage C)
        for (uint32_t k = 0; k + 2 <= me; ++k) {
            const uint32_t outk = fp.offL[k];
            const uint32_t Sk = fp.S[k], npair = (Sk + 1) / 2, items = npair * nw;
            auto relay = [&](uint32_t item, uint64_t lie0, uint64_t lie1) {
                const uint32_t lw = item / npair, pair = item - lw * npair;
                uint64_t* img = lds + (uint64_t)lw * stride;
                static_for<0, 2>([&](auto h) {
                    const uint32_t x = 2 * pair + h();
                    if (x >= Sk) return;
                    uint64_t parent, fw;
                    if (k == 0) {
                        parent = img[n];
                        fw = img[0];
                    } else {
                        const uint32_t y = x / (L - k);
                        parent = img[fp.offL[k - 1] + y];
                        fw = img[sender[fp.snd_off[k - 1] + y]];
                    }
                    const uint64_t lie = h() ? lie1 : lie0;
                    img[outk + x] = (fw & lie) | (~fw & parent);
                });
            };
            // two items per thread per pass: two independent Philox chains in flight
            for (uint32_t it = tid; it < items; it += 2 * T) {
                const uint32_t it2 = it + T < items ? it + T : it;
                const uint32_t lwa = it / npair, lwb = it2 / npair;
                uint64_t a0, a1, b0, b1;
                lie_pair(seed, k, it - lwa * npair, gwg + lwa, a0, a1);
                lie_pair(seed, k, it2 - lwb * npair, gwg + lwb, b0, b1);
                relay(it, a0, a1);
                if (it2 != it) relay(it2, b0, b1);
            }
            __syncthreads();
        }
        FUSED_STAMP(1);
        // ---- C: leaf blocks (sigma at level me-2), R_{me-1} into LDS -------------
        {
            const uint32_t Q = fp.S[me - 2];
            for (uint32_t it = tid; it < Q * nw; it += T) {
                const uint32_t lw = it / Q, sr = it - lw * Q;
                uint64_t* img = lds + (uint64_t)lw * stride;
                const uint64_t gw = gwg + lw;
                const uint32_t x0 = sr * S;
                const uint64_t mem = members[sr];  // S member ids, 5 bits each
                // level me-1 for this block (the diagonal): what each member
                // received from sigma's last relayer, F[last] ? lie : L_{me-2}[sigma]
                const uint64_t par = img[fp.offL[me - 2] + sr];
                const uint64_t fs = img[sender[fp.snd_off[me - 2] + sr]];
                // S odd: x0 = sr*S has either parity and (S+1)/2 pairs cover the
                // S slots from x0; S even: x0 is even and S/2 pairs suffice
                constexpr int NPD = (S + 1) / 2;
                uint64_t lw2[2 * NPD];
                static_for<0, NPD>([&](auto q) {
                    lie_pair(seed, me - 1, (x0 >> 1) + q(), gw, lw2[2 * q()], lw2[2 * q() + 1]);
                });
                // bitwise select: a ternary here becomes lw2[a + odd], a dynamic index (scratch)
                const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
                uint64_t diag[S], Fm[S], R[S];
                static_for<0, S>([&](auto a) {
                    uint64_t lie;
                    if constexpr (S % 2 == 1) lie = lw2[a()] ^ ((lw2[a()] ^ lw2[a() + 1]) & oddmask);
                    else lie = lw2[a()];
                    diag[a()] = (fs & lie) | (~fs & par);
                    Fm[a()] = img[(mem >> (5 * a())) & 31u];
                });
#ifdef BA_FUSED_SCHED_BARRIER
                __builtin_amdgcn_sched_barrier(0);  // keep leaf Philox below the diagonal's
#endif
                leaf_block<S>(me, seed, gw, sr, diag, Fm, R);
                const uint32_t offR = fp.offR[me - 1] + x0;
                static_for<0, S>([&](auto b) { img[offR + b()] = R[b()]; });
            }
            __syncthreads();
        }
        FUSED_STAMP(2);
        // ---- D: inner majorities p = me-2 .. 1 ----------------------------------
        for (int p = (int)me - 2; p >= 1; --p) {
            const uint32_t Sp = fp.S[p], s = L - (uint32_t)p, thr = s / 2 + 1;
            for (uint32_t it = tid; it < Sp * nw; it += T) {
                const uint32_t lw = it / Sp, y = it - lw * Sp;
                uint64_t* img = lds + (uint64_t)lw * stride;
                const uint32_t sr = y / s, b = y - sr * s;
                const uint32_t d = fp.offL[p] + y, c = fp.offR[p + 1];
                img[fp.offR[p] + y] = s < 8    ? column_count<3>(img, d, c, sr, s, b).ge(thr)
                                      : s < 16 ? column_count<4>(img, d, c, sr, s, b).ge(thr)
                                               : column_count<5>(img, d, c, sr, s, b).ge(thr);
            }
            __syncthreads();
        }
        FUSED_STAMP(3);
        // ---- E: root majority (tie -> undefined) + per-trial epilogue -----------
        // roots go to the (now dead) R_{me-1} area: A at +0, U at +L
        for (uint32_t it = tid; it < L * nw; it += T) {
            const uint32_t lw = it / L, b = it - lw * L;
            uint64_t* img = lds + (uint64_t)lw * stride;
            uint64_t att, tie;
            if (L < 16) {
                const Count<4> cnt = column_count<4>(img, fp.offL[0] + b, fp.offR[1], 0, L, b);
                att = cnt.ge(L / 2 + 1);
                tie = (L & 1u) ? 0ull : (cnt.ge(L / 2) & ~att);
            } else {
                const Count<5> cnt = column_count<5>(img, fp.offL[0] + b, fp.offR[1], 0, L, b);
                att = cnt.ge(L / 2 + 1);
                tie = (L & 1u) ? 0ull : (cnt.ge(L / 2) & ~att);
            }
            // stash after the word image's live data: use the R_{me-1} region
            img[fp.offRoot + b] = att;
            img[fp.offRoot + L + b] = tie;
        }
        __syncthreads();
        FUSED_STAMP(4);
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            const uint64_t* img = lds + (uint64_t)lw * stride;
            const uint64_t w = w0 + lw;
            const uint64_t i = w * 64 + lane;
            const bool live = w < total_words && ((img[n + 2] >> lane) & 1ull);
            uint32_t A = 0, U = 0, fm = 0;
            for (uint32_t b = 0; b < L; ++b) {
                A |= (uint32_t)((img[fp.offRoot + b] >> lane) & 1ull) << (b + 1);
                U |= (uint32_t)((img[fp.offRoot + L + b] >> lane) & 1ull) << (b + 1);
            }
            for (uint32_t g = 0; g < n; ++g) fm |= (uint32_t)((img[g] >> lane) & 1ull) << g;
            const uint32_t ob = (uint32_t)(img[n] >> lane) & 1u;
            const uint32_t oo = (uint32_t)(img[n + 1] >> lane) & 1u;
            const TrialResult r = trial_result(n, me, fm, oo ? 2u : ob, A, U);
            if (live) {
                if (decisions) decisions[i] = r.dec;
                if (outcome) outcome[i] = (uint8_t)r.out;
            }
            wave_counts_add(live, r, blockcnt);  // ballots: one LDS add per counter per wave
        }
        __syncthreads();
        FUSED_STAMP(5);
    }
    // integer sums commute: the block's totals go through the replicated sink
    // (no k_reduce launch, no single-line atomic hot spot)
    __syncthreads();
    if (wv == 0) sink_counters(lane, lane < C_NUM ? blockcnt[lane] : 0, blockIdx.x, gridDim.x, counters, sk);
    FUSED_STAMP_STORE();
}

// ---------------------------------------------------------------------------
// FUSED, effective depth 3, N generals known at compile time (n=10, m=3 is
// the BASELINE config).  Same algorithm and LDS image as k_fused, but every
// index is arithmetic on compile-time constants:
//   lieutenant ranks 0..L-1 (general = rank+1); level-1 slot y = j1*(L-1) + c
//   names j1 = y/(L-1) and j2 = c + (c >= j1); the a-th member of prefix
//   (j1, j2) is a + (a >= lo) + (a >= hi-1), lo/hi = min/max(j1, j2).
// Relay levels 0 and 1 run as ONE pass: every level-1 slot pair recomputes
// its parent's level-0 value (one extra Philox call), so no barrier between.
// The root + per-trial epilogue of a word is done by one wave (no barrier).
// ---------------------------------------------------------------------------
template <int N>
struct Om3 {
    static constexpr int L = N - 1, S = N - 3;               // lieutenants, leaf members
    static constexpr int S1 = L * (L - 1), S2 = S1 * (L - 2);  // level-1 / level-2 slots
    static constexpr int oF = 0, oOB = N, oOO = N + 1, oVAL = N + 2;
    static constexpr int oL0 = N + 3, oL1 = oL0 + L, oR2 = oL1 + S1, oR1 = oR2 + S2;
    static constexpr int words = ((oR1 + S1) + 1) & ~1;  // per trial word, 16-B aligned
    static_assert(2 * L <= S2, "root stash reuses the R2 area");
};

template <int N>
__global__ __launch_bounds__(kFusedThreads, ((N - 3) <= 7 ? 4 : 2)) void k_fused3(
    uint32_t wpb, uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk) {
    using G = Om3<N>;
    constexpr int L = G::L, S = G::S, S1 = G::S1, STRIDE = G::words;
    constexpr uint32_t ME = 3;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    __shared__ __attribute__((aligned(16))) unsigned long long blockcnt[16];
    const uint32_t T = kFusedThreads, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < 16) blockcnt[tid] = 0;
    FUSED_STAMP_INIT();
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t per_block = (total_words + gridDim.x - 1) / gridDim.x;
    const uint64_t wbeg = (uint64_t)blockIdx.x * per_block;
    const uint64_t wend = wbeg + per_block < total_words ? wbeg + per_block : total_words;
    for (uint64_t w0 = wbeg; w0 < wend; w0 += wpb) {
        const uint32_t nw = (uint32_t)(wend - w0 < wpb ? wend - w0 : wpb);
        const uint64_t gwg = (first_trial >> 6) + w0;
        // ---- A: inputs -> bit-sliced words (one wave per word) -------------------
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            uint64_t* img = lds + lw * STRIDE;
            const uint64_t i = (w0 + lw) * 64 + lane;
            const bool valid = i < batch;
            uint32_t fm = 0, oc = 0;
            if (valid) {
                if (gs.faulty_mode == 0) fm = faulty[i];
                if (gs.order_mode == 0) oc = order[i];
                gen_trial(N, seed, gs, first_trial + i, fm, oc);
            }
            uint64_t mine = 0;
            static_for<0, N>([&](auto g) {
                const uint64_t b = __ballot(valid && ((fm >> g()) & 1u));
                if (lane == g()) mine = b;
            });
            const uint64_t ob = __ballot(valid && oc == 1);
            const uint64_t oo = __ballot(valid && oc == 2);
            const uint64_t vv = __ballot(valid);
            if (lane < N) img[G::oF + lane] = mine;
            if (lane == 0) {
                img[G::oOB] = ob;
                img[G::oOO] = oo;
                img[G::oVAL] = vv;
            }
        }
        __syncthreads();
        FUSED_STAMP(0);
        // ---- B: levels 0 and 1 in one pass: item = (word, level-1 slot pair) ------
        {
            constexpr uint32_t NP = S1 / 2;  // S1 = L(L-1) is even
            for (uint32_t it = tid; it < NP * nw; it += T) {
                const uint32_t lw = it / NP, q = it - lw * NP;
                uint64_t* img = lds + lw * STRIDE;
                const uint64_t gw = gwg + lw;
                const uint64_t F0 = img[G::oF], ob = img[G::oOB];
                uint32_t x[2], y[2];
                x[0] = 2 * q;
                x[1] = 2 * q + 1;
                y[0] = x[0] / (L - 1);
                y[1] = x[1] / (L - 1);
                uint64_t l1a, l1b, p0a, p0b, p1a, p1b;
                lie_pair(seed, 1, q, gw, l1a, l1b);               // level-1 pair
                lie_pair(seed, 0, y[0] >> 1, gw, p0a, p0b);       // parent of x0 (level 0)
                uint64_t L0v[2];
                L0v[0] = (F0 & ((y[0] & 1) ? p0b : p0a)) | (~F0 & ob);
                if constexpr ((L - 1) % 2 == 0) {                 // both slots share a parent
                    L0v[1] = L0v[0];
                    (void)p1a;
                    (void)p1b;
                } else {
                    lie_pair(seed, 0, y[1] >> 1, gw, p1a, p1b);
                    L0v[1] = (F0 & ((y[1] & 1) ? p1b : p1a)) | (~F0 & ob);
                }
                const uint64_t lie1[2] = {l1a, l1b};
                static_for<0, 2>([&](auto h) {
                    const uint64_t fj = img[G::oF + y[h()] + 1];  // sender: lieutenant y
                    img[G::oL1 + x[h()]] = (fj & lie1[h()]) | (~fj & L0v[h()]);
                    img[G::oL0 + y[h()]] = L0v[h()];              // identical value from
                });                                               // every sibling pair
            }
        }
        __syncthreads();
        FUSED_STAMP(1);
        // ---- C: leaf blocks, one per (word, level-1 slot) ------------------------
        for (uint32_t it = tid; it < (uint32_t)S1 * nw; it += T) {
            const uint32_t lw = it / S1, sr = it - lw * S1;
            uint64_t* img = lds + lw * STRIDE;
            const uint64_t gw = gwg + lw;
            const uint32_t j1 = sr / (L - 1), c = sr - j1 * (L - 1), j2 = c + (c >= j1);
            const uint32_t lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
            const uint64_t par = img[G::oL1 + sr];
            const uint64_t fs = img[G::oF + j2 + 1];  // level-2 sender: j2
            const uint32_t x0 = sr * S;
            constexpr int NPD = (S + 1) / 2;
            uint64_t lw2[2 * NPD];
            static_for<0, NPD>([&](auto qd) {
                lie_pair(seed, 2, (x0 >> 1) + qd(), gw, lw2[2 * qd()], lw2[2 * qd() + 1]);
            });
            // bitwise select: a ternary here becomes lw2[a + odd], a dynamic index (scratch)
                const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
            uint64_t diag[S], Fm[S], R[S];
            static_for<0, S>([&](auto a) {
                uint64_t lie;
                if constexpr (S % 2 == 1) lie = lw2[a()] ^ ((lw2[a()] ^ lw2[a() + 1]) & oddmask);
                else lie = lw2[a()];
                diag[a()] = (fs & lie) | (~fs & par);
                const uint32_t ida = a() + (a() >= lo) + (a() + 1 >= hi);  // member a's rank
                Fm[a()] = img[G::oF + ida + 1];
            });
            leaf_block<S>(ME, seed, gw, sr, diag, Fm, R);
            static_for<0, S>([&](auto b) { img[G::oR2 + x0 + b()] = R[b()]; });
        }
        __syncthreads();
        FUSED_STAMP(2);
        // ---- D: R1[j1*(L-1) + b] over L1 and R2 (s = L-1 inputs) -------------------
        for (uint32_t it = tid; it < (uint32_t)S1 * nw; it += T) {
            const uint32_t lw = it / S1, y = it - lw * S1;
            uint64_t* img = lds + lw * STRIDE;
            const uint32_t j1 = y / (L - 1), b = y - j1 * (L - 1);
            Count<planes_c(L - 1)> cnt;
            cnt.add(img[G::oL1 + y]);
            const uint32_t base = G::oR2 + j1 * (L - 1) * (L - 2);
            static_for<0, L - 1>([&](auto a) {
                if (a() == b) return;
                cnt.add(img[base + a() * (L - 2) + (a() < b ? b - 1 : b)]);
            });
            img[G::oR1 + y] = cnt.ge((L - 1) / 2 + 1);
        }
        __syncthreads();
        FUSED_STAMP(3);
        // ---- E: per wave and word: roots (lanes 0..L-1), then every trial ---------
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            uint64_t* img = lds + lw * STRIDE;
            if (lane < (uint32_t)L) {
                const uint32_t b = lane;
                Count<planes_c(L)> cnt;
                cnt.add(img[G::oL0 + b]);
                static_for<0, L>([&](auto a) {
                    if (a() == b) return;
                    cnt.add(img[G::oR1 + a() * (L - 1) + (a() < b ? b - 1 : b)]);
                });
                const uint64_t att = cnt.ge(L / 2 + 1);
                const uint64_t tie = (L & 1) ? 0ull : (cnt.ge(L / 2) & ~att);
                img[G::oR2 + b] = att;       // R2 is dead after stage D
                img[G::oR2 + L + b] = tie;
            }
            __builtin_amdgcn_wave_barrier();
            // LDS ops of one wave complete in order: the root words written above
            // are visible to this wave's reads below without a block barrier
            const uint64_t w = w0 + lw, i = w * 64 + lane;
            const bool live = (img[G::oVAL] >> lane) & 1ull;
            uint32_t A = 0, U = 0, fm = 0;
            static_for<0, L>([&](auto b) {
                A |= (uint32_t)((img[G::oR2 + b()] >> lane) & 1ull) << (b() + 1);
                U |= (uint32_t)((img[G::oR2 + L + b()] >> lane) & 1ull) << (b() + 1);
            });
            static_for<0, N>([&](auto g) { fm |= (uint32_t)((img[G::oF + g()] >> lane) & 1ull) << g(); });
            const uint32_t ob = (uint32_t)(img[G::oOB] >> lane) & 1u;
            const uint32_t oo = (uint32_t)(img[G::oOO] >> lane) & 1u;
            const TrialResult r = trial_result(N, ME, fm, oo ? 2u : ob, A, U);
            if (live) {
                if (decisions) decisions[i] = r.dec;
                if (outcome) outcome[i] = (uint8_t)r.out;
            }
            wave_counts_add(live, r, blockcnt);
        }
        __syncthreads();
        FUSED_STAMP(5);
    }
    // integer sums commute: the block's totals go through the replicated sink
    // (no k_reduce launch, no single-line atomic hot spot)
    __syncthreads();
    if (wv == 0) sink_counters(lane, lane < C_NUM ? blockcnt[lane] : 0, blockIdx.x, gridDim.x, counters, sk);
    FUSED_STAMP_STORE();
}

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
// Lie bits are keyed exactly as in k_fused3 (level, global slot pair, global
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
        gen_words<N, W, -1>(in0, lane, w0, seed, gs, first_trial, batch, faulty, order);
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

// Per-trial epilogue (lane = trial) of W words, two words per iteration:
// their LDS reads and logic interleave without the register blow-up (and
// spills) of unrolling all W words at once.
template <int N, int W, uint32_t ME, int DIAG>
__device__ __forceinline__ void wave_epilogue(const uint64_t* in0, const uint64_t* au0,
                                              uint32_t lane, uint64_t w0, uint64_t batch,
                                              uint64_t* __restrict__ decisions,
                                              uint8_t* __restrict__ outcome, TrialCounts& tc) {
    constexpr int L = N - 1, NIN = N + 3;
    if constexpr ((DIAG & 32) != 0) {  // lab: near-free stand-in epilogue
        static_for<0, W>([&](auto wq) {
            const uint64_t i = (w0 + wq()) * 64 + lane;
            if (i < batch) decisions[i] = au0[wq() * 2 * L + (lane & 15)];
        });
        return;
    }
    constexpr int EW = 2;
#pragma unroll 1
    for (int wb = 0; wb < W; wb += EW) {
        uint64_t dec_out[EW];
        uint32_t out_out[EW];
        static_for<0, EW>([&](auto wq) {
            const int w = wb + wq();
            out_out[wq()] = 0xFFu;  // 0xFF: not a trial of this batch
            dec_out[wq()] = 0;
            if (W % EW != 0 && w >= W) return;
            const uint64_t* inw = in0 + w * NIN;
            const uint64_t* au = au0 + w * 2 * L;
            const bool live = (inw[N + 2] >> lane) & 1ull;
            uint32_t A = 0, U = 0, fm = 0;
            static_for<0, L>([&](auto b) {
                A |= (uint32_t)((au[b()] >> lane) & 1ull) << (b() + 1);
                U |= (uint32_t)((au[L + b()] >> lane) & 1ull) << (b() + 1);
            });
            static_for<0, N>([&](auto g) { fm |= (uint32_t)((inw[g()] >> lane) & 1ull) << g(); });
            const uint32_t ob = (uint32_t)(inw[N] >> lane) & 1u;
            const uint32_t oo = (uint32_t)(inw[N + 1] >> lane) & 1u;
            const TrialResult r = trial_result(N, ME, fm, oo ? 2u : ob, A, U);
            const uint32_t lv = live ? 1u : 0u;
            const uint32_t q = r.out & 3, agree = (r.out >> 2) & 1, appl = (r.out >> 3) & 1;
            const uint32_t valid = (r.out >> 4) & 1, inb = (r.out >> 5) & 1;
            tc.v[C_TRIALS] += lv;
            tc.v[C_AGREE] += lv & agree;
            tc.v[C_VAPPL] += lv & appl;
            tc.v[C_VALID] += lv & valid;
            tc.v[C_QR] += lv & (q == 0);
            tc.v[C_QA] += lv & (q == 1);
            tc.v[C_QU] += lv & (q == 2);
            tc.v[C_UNDEF] += lv * r.nU;
            tc.v[C_INB] += lv & inb;
            tc.v[C_VIOL] += lv & inb & ((agree ^ 1u) | (appl & (valid ^ 1u)));
            tc.v[C_FTOT] += lv * r.nf;
            tc.v[C_ATT] += lv * r.nA;
            dec_out[wq()] = r.dec;
            out_out[wq()] = live ? r.out : 0xFFu;
        });
        static_for<0, EW>([&](auto wq) {
            const uint64_t i = (w0 + wb + wq()) * 64 + lane;
            if (out_out[wq()] != 0xFFu) {
                if (!(DIAG & 1) && decisions) decisions[i] = dec_out[wq()];
                if (!(DIAG & 2) && outcome) outcome[i] = (uint8_t)out_out[wq()];
            }
        });
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
// k_om3w: effective depth 3 (see the WAVE engine note above)
// ---------------------------------------------------------------------------
template <int N>
struct Om3W {
    static constexpr int L = N - 1, S = N - 3, C = L - 1;
    static constexpr int W = 64 / C;               // trial words per wave task
    static constexpr int LANES = W * C;            // lanes busy in the subtree rounds
    static constexpr int P = planes_c(L);          // root counter planes (L inputs)
    static constexpr int NIN = N + 3;
    static constexpr int oIN = 0, oL0 = oIN + W * NIN, oR2 = oL0 + W * L, oRC = oR2 + W * C * C;
    static constexpr int end0 = oRC + W * L * P;
    static constexpr bool au_in_r2 = 2 * L <= C * C;
    static constexpr int oAU = au_in_r2 ? oR2 : end0;
    static constexpr int words = ((au_in_r2 ? end0 : end0 + W * 2 * L) + 1) & ~1;
};

// DIAG: lab-only ablation switches (tools/om3_lab.hip); the product uses 0.
template <int N, int DIAG = 0>
__global__ __launch_bounds__(kWaveThreads, 2) void k_om3w(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk) {
    using G = Om3W<N>;
    constexpr int L = G::L, S = G::S, C = G::C, W = G::W, P = G::P, NIN = G::NIN;
    constexpr uint32_t ME = 3;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint64_t* img = lds + (uint64_t)wv * G::words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W;
    // this lane's (word, leaf block) in the subtree rounds
    const uint32_t lw_ = lane / C, la = lane - lw_ * C;
    const bool act = lane < (uint32_t)G::LANES;
    const uint32_t lw = act ? lw_ : 0;
    TrialCounts tc;
    FUSED_STAMP_INIT();
#ifdef BA_FUSED_STAMPS
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (uint64_t task = (uint64_t)blockIdx.x * wpb + wv; task < ntasks;
         task += (uint64_t)gridDim.x * wpb) {
        const uint64_t w0 = task * W;
        const uint64_t gw0 = (first_trial >> 6) + w0;
        wave_inputs<N, W, DIAG>(img + G::oIN, lane, w0, seed, gs, first_trial, batch, faulty, order);
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(0);
        wave_level0<N, W, P>(img + G::oIN, img + G::oL0, img + G::oRC, lane, seed, gw0);
        __builtin_amdgcn_wave_barrier();
        // ---- subtree rounds ------------------------------------------------------
        const uint64_t* in = img + G::oIN + lw * NIN;
        const uint64_t gw = gw0 + lw;
        for (uint32_t j1 = 0; j1 < (uint32_t)L; ++j1) {
            if constexpr ((DIAG & 8) == 0) wave_alternate_priority(j1);
            const uint32_t sr = j1 * C + la;             // level-1 slot (j1, j2)
            const uint32_t j2 = la + (la >= j1);
            uint64_t par = 0;
            if (act) {
                // 1. L1[j1, a] (sender j1 relays L0[j1]) and the level-2 diagonal
                //    pairs of leaf block (j1, a): one interleaved Philox group
                const uint32_t x0 = sr * S;
                constexpr int NPD = (S + 1) / 2;
                P4 pc[NPD + 1];
                static_for<0, NPD>([&](auto qd) {
                    pc[qd()] = P4{(x0 >> 1) + qd(), 2u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                });
                pc[NPD] = P4{sr >> 1, 1u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                philox10_n<NPD + 1>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
                uint64_t lw2[2 * NPD];
                static_for<0, NPD>([&](auto qd) {
                    lw2[2 * qd()] = (uint64_t)pc[qd()].y << 32 | pc[qd()].x;
                    lw2[2 * qd() + 1] = (uint64_t)pc[qd()].w << 32 | pc[qd()].z;
                });
                const uint64_t lie = (sr & 1u) ? ((uint64_t)pc[NPD].w << 32 | pc[NPD].z)
                                               : ((uint64_t)pc[NPD].y << 32 | pc[NPD].x);
                const uint64_t fj = in[j1 + 1];
                par = (fj & lie) | (~fj & img[G::oL0 + lw * L + j1]);
                // 2. leaf block (j1, a): level-2 diagonal, then S(S-1) leaves
                const uint32_t lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
                const uint64_t fs = in[j2 + 1];  // level-2 sender: j2
                const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
                uint64_t diag[S], Fm[S], R[S];
                static_for<0, S>([&](auto a) {
                    uint64_t lie2;
                    if constexpr (S % 2 == 1) lie2 = lw2[a()] ^ ((lw2[a()] ^ lw2[a() + 1]) & oddmask);
                    else lie2 = lw2[a()];
                    diag[a()] = (fs & lie2) | (~fs & par);
                    const uint32_t ida = a() + (a() >= lo) + (a() + 1 >= hi);  // member a's rank
                    Fm[a()] = in[ida + 1];
                });
                leaf_block<S>(ME, seed, gw, sr, diag, Fm, R);
                // receiver-major: member d of block a is receiver b = d + (d >= a)
                uint64_t* r2t = img + G::oR2 + lw * C * C + la;
                r2t[la * C] = par;
                static_for<0, S>([&](auto d) { r2t[(d() + (d() >= la ? 1u : 0u)) * C] = R[d()]; });
            }
            __builtin_amdgcn_wave_barrier();
            FUSED_STAMP(1);
            if (act) {
                // 3. R1[j1, b], b = la: L1[j1, b] (this lane's own parent) plus
                //    column b of the word's other leaf blocks a' != b
                const uint64_t* col = img + G::oR2 + (lw * C + la) * C;
                Csa<planes_c(C)> cnt;
                static_for<0, C>([&](auto a) { cnt.template add<a()>(col[a()]); });
                const uint64_t r1 = cnt.template ge<C, C / 2 + 1>();  // inner tie -> non-attack
                // root column j2 += R1[j1, b] (ripple add on the bit-sliced planes)
                planes_add<P>(img + G::oRC + (lw * L + j2) * P, r1);
            }
            __builtin_amdgcn_wave_barrier();
            FUSED_STAMP(2);
        }
        wave_roots<L, W, P>(img + G::oRC, img + G::oAU, lane);
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(3);
        wave_epilogue<N, W, ME, DIAG>(img + G::oIN, img + G::oAU, lane, w0, batch, decisions,
                                      outcome, tc);
        __builtin_amdgcn_wave_barrier();
        FUSED_STAMP(4);
    }
    wave_flush(tc, lane, wv, wpb, counters, sk, (DIAG & 4) != 0);
#ifdef BA_FUSED_STAMPS
    if (lane == 0 && blockIdx.x * wpb + wv < (uint32_t)kPartialRows)
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
template <int N>
struct Om4W {
    static constexpr int L = N - 1, S = N - 4, C1 = L - 1, C2 = L - 2;
    static constexpr int W = 64 / C2;
    static constexpr int LANES = W * C2;
    static constexpr int P = planes_c(L), P1 = planes_c(C1);
    static constexpr int NIN = N + 3;
    static constexpr int oIN = 0, oL0 = oIN + W * NIN, oR3 = oL0 + W * L;
    static constexpr int oR1 = oR3 + W * C2 * C2, oRC = oR1 + W * C1 * P1;
    static constexpr int end0 = oRC + W * L * P;
    static constexpr bool au_in_r3 = 2 * L <= C2 * C2;
    static constexpr int oAU = au_in_r3 ? oR3 : end0;
    static constexpr int words = ((au_in_r3 ? end0 : end0 + W * 2 * L) + 1) & ~1;
};

template <int N>
__global__ __launch_bounds__(kWaveThreads, 2) void k_om4w(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk) {
    using G = Om4W<N>;
    constexpr int L = G::L, S = G::S, C1 = G::C1, C2 = G::C2, W = G::W, P = G::P, P1 = G::P1;
    constexpr int NIN = G::NIN;
    constexpr uint32_t ME = 4;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint64_t* img = lds + (uint64_t)wv * G::words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W;
    const uint32_t lw_ = lane / C2, la = lane - lw_ * C2;
    const bool act = lane < (uint32_t)G::LANES;
    const uint32_t lw = act ? lw_ : 0;
    TrialCounts tc;
    for (uint64_t task = (uint64_t)blockIdx.x * wpb + wv; task < ntasks;
         task += (uint64_t)gridDim.x * wpb) {
        const uint64_t w0 = task * W;
        const uint64_t gw0 = (first_trial >> 6) + w0;
        wave_inputs<N, W, 0>(img + G::oIN, lane, w0, seed, gs, first_trial, batch, faulty, order);
        __builtin_amdgcn_wave_barrier();
        wave_level0<N, W, P>(img + G::oIN, img + G::oL0, img + G::oRC, lane, seed, gw0);
        __builtin_amdgcn_wave_barrier();
        const uint64_t* in = img + G::oIN + lw * NIN;
        const uint64_t gw = gw0 + lw;
        uint32_t round = 0;
        for (uint32_t j1 = 0; j1 < (uint32_t)L; ++j1) {
            // R1 counters of this j1 start at zero
            for (uint32_t it = lane; it < (uint32_t)(W * C1 * P1); it += 64) img[G::oR1 + it] = 0;
            __builtin_amdgcn_wave_barrier();
            const uint64_t fj1 = in[j1 + 1];
            const uint64_t l0j1 = img[G::oL0 + lw * L + j1];
            for (uint32_t c2 = 0; c2 < (uint32_t)C1; ++c2, ++round) {
                wave_alternate_priority(round);
                const uint32_t j2 = c2 + (c2 >= j1);
                const uint32_t lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
                const uint32_t x1 = j1 * C1 + c2;     // level-1 slot (j1, j2)
                const uint32_t x2 = x1 * C2 + la;     // level-2 slot (j1, j2, j3): leaf block
                const uint32_t j3 = la + (la >= lo) + (la + 1 >= hi);  // the a-th other lieutenant
                uint64_t par = 0, l1v = 0;
                if (act) {
                    const uint32_t x3 = x2 * S;
                    constexpr int NPD = (S + 1) / 2;
                    P4 pc[NPD + 2];
                    static_for<0, NPD>([&](auto qd) {
                        pc[qd()] = P4{(x3 >> 1) + qd(), 3u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                    });
                    pc[NPD] = P4{x2 >> 1, 2u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                    pc[NPD + 1] = P4{x1 >> 1, 1u, (uint32_t)gw, (uint32_t)(gw >> 32)};
                    philox10_n<NPD + 2>(pc, (uint32_t)seed, (uint32_t)(seed >> 32));
                    uint64_t lw3[2 * NPD];
                    static_for<0, NPD>([&](auto qd) {
                        lw3[2 * qd()] = (uint64_t)pc[qd()].y << 32 | pc[qd()].x;
                        lw3[2 * qd() + 1] = (uint64_t)pc[qd()].w << 32 | pc[qd()].z;
                    });
                    const uint64_t lie2 = (x2 & 1u) ? ((uint64_t)pc[NPD].w << 32 | pc[NPD].z)
                                                    : ((uint64_t)pc[NPD].y << 32 | pc[NPD].x);
                    const uint64_t lie1 = (x1 & 1u) ? ((uint64_t)pc[NPD + 1].w << 32 | pc[NPD + 1].z)
                                                    : ((uint64_t)pc[NPD + 1].y << 32 | pc[NPD + 1].x);
                    l1v = (fj1 & lie1) | (~fj1 & l0j1);              // L1[j1, j2], sender j1
                    const uint64_t fj2 = in[j2 + 1];
                    par = (fj2 & lie2) | (~fj2 & l1v);               // L2[j1, j2, j3], sender j2
                    // members of leaf block (j1, j2, j3): the lieutenants not in
                    // {j1, j2, j3}, ascending
                    const uint32_t e0 = lo < j3 ? lo : j3;
                    const uint32_t e2 = hi > j3 ? hi : j3;
                    const uint32_t e1 = lo + hi + j3 - e0 - e2;
                    const uint64_t fs = in[j3 + 1];  // level-3 sender: j3
                    const uint64_t oddmask = 0ull - (uint64_t)(x3 & 1u);
                    uint64_t diag[S], Fm[S], R[S];
                    static_for<0, S>([&](auto d) {
                        uint64_t lie3;
                        if constexpr (S % 2 == 1) lie3 = lw3[d()] ^ ((lw3[d()] ^ lw3[d() + 1]) & oddmask);
                        else lie3 = lw3[d()];
                        diag[d()] = (fs & lie3) | (~fs & par);
                        uint32_t m = d();
                        m += m >= e0 ? 1u : 0u;
                        m += m >= e1 ? 1u : 0u;
                        m += m >= e2 ? 1u : 0u;
                        Fm[d()] = in[m + 1];
                    });
                    leaf_block<S>(ME, seed, gw, x2, diag, Fm, R);
                    uint64_t* r3t = img + G::oR3 + lw * C2 * C2 + la;
                    r3t[la * C2] = par;
                    static_for<0, S>([&](auto d) { r3t[(d() + (d() >= la ? 1u : 0u)) * C2] = R[d()]; });
                }
                __builtin_amdgcn_wave_barrier();
                if (act) {
                    // R2[j1, j2, b], b = la (receiver: the la-th lieutenant not in {j1, j2})
                    const uint64_t* col = img + G::oR3 + (lw * C2 + la) * C2;
                    Csa<planes_c(C2)> cnt;
                    static_for<0, C2>([&](auto a) { cnt.template add<a()>(col[a()]); });
                    const uint64_t r2 = cnt.template ge<C2, C2 / 2 + 1>();  // inner tie -> non-attack
                    // receiver j3 (same formula as above) as a rank among the non-j1
                    planes_add<P1>(img + G::oR1 + (lw * C1 + (j3 - (j3 > j1 ? 1u : 0u))) * P1, r2);
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
        wave_epilogue<N, W, ME, 0>(img + G::oIN, img + G::oAU, lane, w0, batch, decisions, outcome, tc);
        __builtin_amdgcn_wave_barrier();
    }
    wave_flush(tc, lane, wv, wpb, counters, sk, false);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Trees the WAVE kernels are compiled for (k_om3w / k_om4w instantiations).
bool wave_supported(const Geometry& g) {
    return (g.me == 3 && g.n >= 5 && g.n <= 14) || (g.me == 4 && g.n >= 6 && g.n <= kWave4MaxN);
}

bool leaf_supported(const Geometry& g) {
    const uint32_t S = g.n - g.me;
    return g.me >= 2 && S >= 2 && S <= kMaxLeafS;
}

template <int S>
static void launch_leaf_s(uint32_t me, uint64_t seed, uint64_t gw0, uint32_t W, uint32_t work,
                          uint32_t srbase, const uint64_t* Lm1, const uint64_t* F,
                          const uint64_t* snd, uint64_t* Rm1, hipStream_t st) {
    uint64_t b = (work + 255) / 256;
    if (b > 16384) b = 16384;
    if (b < 1) b = 1;
    hipLaunchKernelGGL(k_leaf<S>, dim3((uint32_t)b), dim3(256), 0, st, me, seed, gw0,
                       make_fastdiv(W), work, srbase, Lm1, F, snd, Rm1);
}

hipError_t launch_leaf(const Geometry& g, uint64_t seed, uint64_t gw0, uint32_t W,
                       uint32_t srbase, uint32_t srcnt, const uint64_t* Lm1, const uint64_t* F,
                       const uint64_t* d_members, uint64_t* Rm1, hipStream_t st, Prof* prof) {
    ProfScope ps(prof, "k_leaf", st);
    const uint32_t S = g.n - g.me;
    const uint32_t work = (uint32_t)((uint64_t)srcnt * W);
    if (work == 0) return hipSuccess;
    const uint64_t* snd = d_members;
    switch (S) {
#define LEAF_CASE(s) \
    case s: launch_leaf_s<s>(g.me, seed, gw0, W, work, srbase, Lm1, F, snd, Rm1, st); break;
        LEAF_CASE(2) LEAF_CASE(3) LEAF_CASE(4) LEAF_CASE(5) LEAF_CASE(6) LEAF_CASE(7)
        LEAF_CASE(8) LEAF_CASE(9) LEAF_CASE(10) LEAF_CASE(11) LEAF_CASE(12)
#undef LEAF_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Plan the FUSED LDS image; false if the tree does not fit a block.
bool plan_fused(const Geometry& g, FusedPlan& fp) {
    if (!leaf_supported(g) || g.me > kFusedMaxDepth) return false;
    fp = FusedPlan{};
    fp.n = g.n;
    fp.me = g.me;
    const uint32_t L = g.L;
    uint32_t o = g.n + 3;
    for (uint32_t k = 0; k <= g.me; ++k) fp.S[k] = (uint32_t)g.S[k];
    for (uint32_t k = 0; k + 2 <= g.me; ++k) { fp.offL[k] = o; o += fp.S[k]; }
    for (uint32_t p = 1; p <= g.me - 1; ++p) { fp.offR[p] = o; o += fp.S[p]; }
    // root stash (2L words) reuses R_{me-1}, dead after stage D (me >= 3), or a
    // fresh area when R_{me-1} == R_1 is still being read by the roots (me == 2)
    if (g.me >= 3) {
        fp.offRoot = fp.offR[g.me - 1];
    } else {
        fp.offRoot = o;
        o += 2 * L;
    }
    o = (o + 1) & ~1u;  // keep each word image 16-byte aligned
    fp.word_stride = o;
    for (uint32_t k = 0; k < g.me; ++k) fp.snd_off[k] = (uint32_t)g.sender_off[k];
    const uint64_t bytes_per_word = (uint64_t)o * 8;
    const uint32_t Q = fp.S[g.me - 2];
    if (bytes_per_word > kFusedLdsBudget) return false;
    // words per block: the LDS image fits the budget, and the leaf stage (Q
    // blocks per word over 256 threads) wastes the fewest thread-passes
    // (n=10, m=3: 7 words -> 504 leaf blocks in two passes of 256, 98% busy)
    const uint32_t T = kFusedThreads;
    uint32_t wpb = 0;
    double best = -1.0;
    for (uint32_t w = 1; w <= 16; ++w) {
        if (bytes_per_word * w > kFusedLdsBudget) break;
        const uint32_t passes = (Q * w + T - 1) / T;
        const double eff = (double)(Q * w) / (double)(passes * T) + 1e-3 * w;  // tie -> more words
        if (eff > best) {
            best = eff;
            wpb = w;
        }
    }
    if (wpb == 0) return false;
    fp.wpb = wpb;
    fp.threads = T;
    fp.lds_bytes = (uint32_t)(bytes_per_word * wpb);
    return true;
}

template <int S>
static void launch_fused_s(const FusedPlan& fp, const FusedPlan* d_fp, uint32_t blocks,
                           uint32_t lds_bytes, const RunArgs& a, const uint8_t* d_sender,
                           uint64_t* partials) {
    hipLaunchKernelGGL(k_fused<S>, dim3(blocks), dim3(fp.threads), lds_bytes, a.stream, d_fp,
                       a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order, d_sender, a.members,
                       a.decisions, a.outcome, a.counters, a.sink);
}

// WAVE engine launch: one wave per W-word task, 4 independent waves per block,
// at most two blocks per CU (two waves per SIMD, the kernels' register budget)
// and a persistent task loop.
template <typename G, typename K>
static hipError_t launch_wave(const RunArgs& a, K kernel, const char* name) {
    constexpr uint32_t wpb = kWaveThreads / 64;
    const uint64_t words = (a.batch + 63) / 64, tasks = (words + G::W - 1) / G::W;
    uint64_t blocks = (tasks + wpb - 1) / wpb;
    uint64_t cap = 2ull * a.cu_count;
    if (const char* e = getenv("BA_WAVE_MAX_BLOCKS")) {  // tests: force the persistent task loop
        const uint64_t c = strtoull(e, nullptr, 0);
        if (c >= 1 && c < cap) cap = c;
    }
    if (blocks > cap) blocks = cap;
    ProfScope ps(a.prof, name, a.stream);
    hipLaunchKernelGGL(kernel, dim3((uint32_t)blocks), dim3(kWaveThreads), wpb * G::words * 8,
                       a.stream, a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order,
                       a.decisions, a.outcome, a.counters, a.sink);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_om3w_n(const RunArgs& a) {
    return launch_wave<Om3W<N>>(a, k_om3w<N>, "k_om3w");
}

template <int N>
static hipError_t launch_om4w_n(const RunArgs& a) {
    return launch_wave<Om4W<N>>(a, k_om4w<N>, "k_om4w");
}

hipError_t launch_fused(const RunArgs& a, const Geometry& g, bool plan_ok, const FusedPlan& fp,
                        const FusedPlan* d_fp, const uint8_t* d_sender, uint64_t* partials) {
    const uint64_t words = (a.batch + 63) / 64;
    // effective depth 3 or 4 within wave_supported: the WAVE kernels.
    // BA_FUSED_KIND selects the alternatives for cross-checks: 1 = block
    // kernel k_fused3 (depth 3), 2 = generic k_fused (trees that fit its plan).
    const char* kenv = getenv("BA_FUSED_KIND");
    const int kind = kenv ? atoi(kenv) : 0;
    if (wave_supported(g) && kind == 0) {
        if (g.me == 3) {
            switch (g.n) {
#define OM3W_CASE(nn) \
    case nn: return launch_om3w_n<nn>(a);
                OM3W_CASE(5) OM3W_CASE(6) OM3W_CASE(7) OM3W_CASE(8) OM3W_CASE(9) OM3W_CASE(10)
                OM3W_CASE(11) OM3W_CASE(12) OM3W_CASE(13) OM3W_CASE(14)
#undef OM3W_CASE
                default: return hipErrorInvalidValue;
            }
        }
        switch (g.n) {
#define OM4W_CASE(nn) \
    case nn: return launch_om4w_n<nn>(a);
            OM4W_CASE(6) OM4W_CASE(7) OM4W_CASE(8) OM4W_CASE(9) OM4W_CASE(10) OM4W_CASE(11)
            OM4W_CASE(12) OM4W_CASE(13) OM4W_CASE(14)
#undef OM4W_CASE
            default: return hipErrorInvalidValue;
        }
    }
    if (!plan_ok) return hipErrorInvalidValue;  // BA_FUSED_KIND forced a kernel this tree lacks
    // BA_FUSED_KIND=1: the compile-time-specialised block kernel k_fused3
    const bool spec3 = g.me == 3 && g.n >= 5 && g.n <= 14 && kind != 2;
    // one block per resident slot (occupancy x CUs): each owns an equal run of words
    int occ = 0;
    if (spec3) {
        switch (g.n) {
#define OCC3_CASE(nn) \
    case nn: (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused3<nn>, kFusedThreads, fp.lds_bytes); break;
            OCC3_CASE(5) OCC3_CASE(6) OCC3_CASE(7) OCC3_CASE(8) OCC3_CASE(9) OCC3_CASE(10)
            OCC3_CASE(11) OCC3_CASE(12) OCC3_CASE(13) OCC3_CASE(14)
#undef OCC3_CASE
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (g.n - g.me) {
#define OCC_CASE(s) \
    case s: (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused<s>, fp.threads, fp.lds_bytes); break;
            OCC_CASE(2) OCC_CASE(3) OCC_CASE(4) OCC_CASE(5) OCC_CASE(6) OCC_CASE(7)
            OCC_CASE(8) OCC_CASE(9) OCC_CASE(10) OCC_CASE(11) OCC_CASE(12)
#undef OCC_CASE
            default: return hipErrorInvalidValue;
        }
    }
    if (occ < 1) occ = 1;
    uint32_t lds_bytes = fp.lds_bytes;
#ifdef BA_FUSED_STAMPS
    // diagnostic: BA_FUSED_BLOCKS_PER_CU=k pads LDS so that only k blocks fit a CU
    if (const char* s = getenv("BA_FUSED_BLOCKS_PER_CU")) {
        const int k = atoi(s);
        if (k >= 1 && k < occ) {
            lds_bytes = 160 * 1024 / k - 1024;
            occ = k;
        }
    }
#endif
    uint64_t slots = (uint64_t)occ * a.cu_count;
    if (slots > (uint64_t)kPartialRows) slots = kPartialRows;
    const uint32_t blocks = (uint32_t)(words < slots ? words : slots);
    {
        ProfScope ps(a.prof, "k_fused", a.stream);
        if (spec3) {
            switch (g.n) {
#define FUSED3_CASE(nn)                                                                          \
    case nn:                                                                                     \
        hipLaunchKernelGGL(k_fused3<nn>, dim3(blocks), dim3(kFusedThreads), lds_bytes, a.stream, \
                           fp.wpb, a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order,     \
                           a.decisions, a.outcome, a.counters, a.sink);                         \
        break;
                FUSED3_CASE(5) FUSED3_CASE(6) FUSED3_CASE(7) FUSED3_CASE(8) FUSED3_CASE(9)
                FUSED3_CASE(10) FUSED3_CASE(11) FUSED3_CASE(12) FUSED3_CASE(13) FUSED3_CASE(14)
#undef FUSED3_CASE
                default: return hipErrorInvalidValue;
            }
        } else {
            switch (g.n - g.me) {
#define FUSED_CASE(s) \
    case s: launch_fused_s<s>(fp, d_fp, blocks, lds_bytes, a, d_sender, partials); break;
                FUSED_CASE(2) FUSED_CASE(3) FUSED_CASE(4) FUSED_CASE(5) FUSED_CASE(6) FUSED_CASE(7)
                FUSED_CASE(8) FUSED_CASE(9) FUSED_CASE(10) FUSED_CASE(11) FUSED_CASE(12)
#undef FUSED_CASE
                default: return hipErrorInvalidValue;
            }
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    (void)partials;
    return hipSuccess;
}

}  // namespace ba
