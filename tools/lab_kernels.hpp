// lab_kernels.hpp -- kernels measured and rejected, kept for the lab harnesses
// only (tools/om3_lab.hip, tools/om3q_lab.hip); NOT part of libba_hip.so.
//   k_fused3<N>  block-synchronous depth-3 kernel (98.6 us per 1M trials vs
//                k_om3w's 52; DESIGN.md §4 "FUSED block engine")
//   k_om3h<N,P>  k_om3w with each task split over P units and a last-arriver
//                epilogue (98.5 us vs 50.1, profiles/r03i_split_ab.log)
//   k_om3q<N>    k_om3w with a block-level work queue (slower)
// Include after the product sources (ba_fused.hip, ba_wave3.hip).
#pragma once
namespace ba {
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
// k_om3h: k_om3w with each task split into two halves of its first-hop rounds
// (staged inputs; BA_WAVE_SPLIT=1).  A unit is (task, half): half 0 runs rounds
// j1 in [0, H0), half 1 rounds [H0, L), H0 = ceil(L/2).  Both halves stage the
// task's inputs and level 0 (5 of ~230 Philox calls per word); each publishes
// its R1 entries R1T[w][col][j1] (its j1 range) to the task's exchange block in
// L2 and arrives at the task's counter; the second arrival merges the other
// half's entries into its LDS image and runs the roots, the epilogue and the
// counts.  No wave waits for another (the k_cascade hand-off), and units come
// from the ctx's dynamic counter: 2 units per task halve the granule a wave
// takes, so a one-step launch's tail (the SIMD's younger wave running alone
// after its older partner finished) should be about half as long.
// MEASURED SLOWER (round 3, profiles/r03i_split_ab.log): 98.5 us per 1M-trial
// launch against k_om3w's 50.1 (thirds: 105 us), bit-identical; the kernel
// compiles to 238 VGPRs without a bound (46 spills at the 3-block bound)
// against k_om3w's 170.  Kept as a lab switch (A/B, parity-tested), off by
// default.
// xch: [tasks][W][L][L] words; xcnt: [tasks] counters, zero between launches
// (the last arriver resets its counter).
// ---------------------------------------------------------------------------
template <int N, int P = 2>
__global__ __launch_bounds__(kWaveThreads, BA_OM3W_MIN_BLOCKS(N)) void k_om3h(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk, uint64_t* __restrict__ xch,
    uint32_t* __restrict__ xcnt) {
    using G = Om3W<N>;
    constexpr int L = G::L, C = G::C, W = G::W, NIN = G::NIN;
    constexpr uint32_t ME = 3;
    static_assert(P >= 2 && P <= L, "k_om3h: 2..L parts per task");
    (void)gs;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint64_t* img = lds + (uint64_t)wv * G::words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W, nunits = (uint64_t)P * ntasks;
    const uint32_t lw_ = lane / C, la = lane - lw_ * C;
    const bool act = lane < (uint32_t)G::LANES;
    const uint32_t lw = act ? lw_ : 0;
    const Om3LaneOffsets<N> lofs(la);
    uint64_t folded = 0;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    for (uint64_t u = (uint64_t)blockIdx.x * wpb + wv; u < nunits;) {
        uint32_t next_raw = 0;
        if (sk.tasks != nullptr && lane == 0) next_raw = atomicAdd(sk.tasks, 1u);
        const uint64_t task = u / P;
        const uint32_t part = (uint32_t)(u - task * P);
        // part p runs rounds [p L / P, (p + 1) L / P)
        const uint32_t jb = part * L / P, je = (part + 1) * L / P;
        const uint64_t w0 = task * W;
        const uint64_t gw0 = (first_trial >> 6) + w0;
        stage_words<N, W>(img + G::oIN, lane, w0, batch, faulty, order);
        __builtin_amdgcn_wave_barrier();
        level0_r1t<N, W>(img + G::oIN, img + G::oL0, img + G::oR1, lane, seed, gw0);
        const uint64_t* in = img + G::oIN + lw * NIN;
        uint64_t* erow = img + G::oE + lw * (C + 1);
        // E row of round jb: the lieutenants other than jb in rank order
        if (act) erow[la] = in[la + (la >= jb ? 1u : 0u) + 1];
        __builtin_amdgcn_wave_barrier();
        const uint64_t gw = gw0 + lw;
        for (uint32_t j1 = jb; j1 < je; ++j1) {
            const uint64_t r1 = om3_round<N, true>(in, act ? img[G::oL0 + lw * L + j1] : 0ull,
                                                   img + G::oR2, lw, la, act, j1, seed, gw,
                                                   erow, &lofs);
            if (act) img[G::oR1 + (lw * L + la + (la >= j1 ? 1u : 0u)) * L + j1] = r1;
        }
        __builtin_amdgcn_wave_barrier();
        // publish this part's entries R1T[w][col][j1], j1 in [jb, je), col != j1
        uint64_t* xt = xch + task * (uint64_t)(W * L * L);
        const uint32_t nj = je - jb;
        for (uint32_t it = lane; it < (uint32_t)(W * L) * nj; it += 64) {
            const uint32_t row = it / nj, j1 = jb + (it - row * nj);  // row = w * L + col
            if (row % L != j1) store_sc1(xt + row * L + j1, img[G::oR1 + row * L + j1]);
        }
        drain_stores();
        if (arrive_last(xcnt + task, (uint32_t)P, lane)) {
            // every other part's entries (all of R1T outside [jb, je))
            const uint32_t no = (uint32_t)L - nj;
            for (uint32_t it = lane; it < (uint32_t)(W * L) * no; it += 64) {
                const uint32_t row = it / no, k = it - row * no;
                const uint32_t j1 = k < jb ? k : k + nj;
                if (row % L != j1) img[G::oR1 + row * L + j1] = load_sc1(xt + row * L + j1);
            }
            __builtin_amdgcn_wave_barrier();
            roots_r1t<L, W>(img + G::oR1, img + G::oAU, lane);
            __builtin_amdgcn_wave_barrier();
            TrialCounts tc;
            wave_epilogue<N, W, ME, 0>(img + G::oIN, img + G::oAU, lane, w0, batch, decisions,
                                       outcome, tc);
            wave_fold(tc, lane, folded);
        }
        __builtin_amdgcn_wave_barrier();
        u = sk.tasks != nullptr ? nwaves + __builtin_amdgcn_readfirstlane(next_raw) : u + nwaves;
    }
    wave_flush_folded(folded, lane, wv, wpb, counters, sk, false);
}

// ---------------------------------------------------------------------------
// k_om3q: effective depth 3 with a block-level work queue (A/B only:
// BA_WAVE_KIND=2; k_om3w is the bench kernel, DESIGN.md §4 on why the queue
// did not pay).
//
// k_om3w gives each wave a whole task (W words x all L first-hop rounds).  At
// two waves per SIMD the SIMD's older wave wins VALU arbitration, finishes its
// task first and leaves the younger wave alone for the last ~25% of the
// launch at about half the issue rate (tools/om3_lab HW_ID trace, round 2).
// k_om3q cuts the work finer: a block of 8 waves (two per SIMD) holds up to
// kQueueMaxTasks tasks in LDS, and a UNIT is one first-hop round j1 of one
// task (one om3_round: 1/L of the task).  Waves take units from an LDS
// counter, so a faster wave simply takes more of them; the wave that finishes
// the L-th unit of a task resolves that task's roots and epilogue while the
// others keep taking units.  Phases per group of tasks:
//   A. inputs + level 0 of each task (one wave per task), L0 also written on
//      the diagonal of the task's R1T
//   B. units (task-major, so tasks complete one after another): om3_round,
//      then R1[j1, b] stored receiver-major, R1T[w][j2][j1]; no counters are
//      accumulated per round (k_om3w's LDS read-modify-write of root planes)
//   C. (by the L-th unit's wave) roots = compile-time carry-save counts of the
//      L contiguous R1T words, then the shared epilogue
// Bit-identical to k_om3w (same lie keying, same majorities).
// LDS: per task IN[W][N+3] | L0[W][L] | R1T[W][L][L]; per wave the R2T
// scratch [W][C][C+1] (the roots' A/U reuse it).
// ---------------------------------------------------------------------------
constexpr int kQueueThreads = 512;  // 8 waves: two per SIMD
constexpr int kQueueMaxTasks = 8;   // tasks a block holds in LDS at once

template <int N, int THREADS = kQueueThreads>
struct Om3Q {
    static constexpr int L = N - 1, S = N - 3, C = L - 1, CP = C + 1;
    static constexpr int W = 64 / C;
    static constexpr int LANES = W * C;
    static constexpr int NIN = N + 3;
    static constexpr int tIN = 0, tL0 = W * NIN, tR1 = tL0 + W * L;
    static constexpr int task_words = ((tR1 + W * L * L) + 1) & ~1;
    static constexpr int wave_words = ((W * C * CP > W * 2 * L ? W * C * CP : W * 2 * L) + 1) & ~1;
    static constexpr int waves = THREADS / 64;
    static constexpr int lds_bytes = (kQueueMaxTasks * task_words + waves * wave_words) * 8;
};

// Level 0 of a task's W words (one Philox per slot pair) into l0[w*L + j] and
// the diagonal r1t[(w*L + j)*L + j] (root column j counts L0[j] as its own input).
template <int N, int W>
__device__ __forceinline__ void queue_level0(const uint64_t* in0, uint64_t* l0, uint64_t* r1t,
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
                r1t[(w * L + j) * L + j] = v;
            }
        });
    }
}

// Run counters of a block of WAVES waves: wave sums (lane c holds counter c),
// combined in LDS, then one sink unit per block (contains a block barrier).
template <int WAVES>
__device__ __forceinline__ void block_flush(const TrialCounts& tc, uint32_t lane, uint32_t wv,
                                            uint64_t* __restrict__ counters, const Sink& sk) {
    uint64_t mine = 0;
#pragma unroll
    for (int c = 0; c < C_NUM; ++c) {
        uint32_t x = tc.v[c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if (lane == (uint32_t)c) mine = x;
    }
    __shared__ unsigned long long wcnt[WAVES][16];
    if (lane < 16) wcnt[wv][lane] = mine;
    __syncthreads();
    if (wv == 0) {
        uint64_t tot = 0;
        for (uint32_t k = 0; k < (uint32_t)WAVES; ++k) tot += lane < 16 ? wcnt[k][lane] : 0;
        sink_counters(lane, tot, blockIdx.x, gridDim.x, counters, sk);
    }
}

// One trial word's epilogue with lane = trial (ba.py:197-255 via trial_result,
// the restatement the oracle tests pin): the task's bit-sliced root words
// A/U and input planes are read once each with wave-uniform (broadcast) LDS
// reads, each lane gathers its own bits into lieutenant / general masks, and
// stores its decision word and outcome byte.  A whole wave per word keeps the
// epilogue parallel across waves (k_om3q queues it per word).
template <int N, uint32_t ME>
__device__ __forceinline__ void word_epilogue(const uint64_t* inw, const uint64_t* au,
                                              uint32_t lane, uint64_t i, uint64_t batch,
                                              uint64_t* __restrict__ decisions,
                                              uint8_t* __restrict__ outcome, TrialCounts& tc) {
    constexpr int L = N - 1;
    const bool hi = lane >= 32;
    const uint32_t sh = lane & 31;
    auto bit = [&](uint64_t v) -> uint32_t {
        return __builtin_amdgcn_ubfe(hi ? (uint32_t)(v >> 32) : (uint32_t)v, sh, 1);
    };
    uint64_t av[L], fv[N + 3];
    static_for<0, L>([&](auto b) { av[b()] = au[b()]; });
    static_for<0, N + 3>([&](auto g) { fv[g()] = inw[g()]; });
    uint32_t A = 0, U = 0, fm = 0;
    static_for<0, L>([&](auto b) { A |= bit(av[b()]) << (b() + 1); });
    if constexpr (L % 2 == 0) {  // an even number of root inputs can tie: undefined
        uint64_t uv[L];
        static_for<0, L>([&](auto b) { uv[b()] = au[L + b()]; });
        static_for<0, L>([&](auto b) { U |= bit(uv[b()]) << (b() + 1); });
    }
    static_for<0, N>([&](auto g) { fm |= bit(fv[g()]) << g(); });
    const uint32_t live = bit(fv[N + 2]);
    const uint32_t oc = bit(fv[N + 1]) ? 2u : bit(fv[N]);
    if (live) {
        uint64_t dec;
        uint32_t out;
        finish_trial(N, ME, fm, oc, A, U, dec, out, tc);
        if (decisions) decisions[i] = dec;
        if (outcome) outcome[i] = (uint8_t)out;
    }
}

// Lab builds only (tools/om3q_lab.hip defines BA_QUEUE_STAMPS): per wave, the
// s_memtime cycles spent in each phase and the units it took.  No output
// depends on them.
#ifdef BA_QUEUE_STAMPS
__device__ unsigned long long g_q_stamps[4096][10];
#define QSTAMP_INIT() unsigned long long qs_prev = __builtin_amdgcn_s_memtime(), qs_acc[10] = {0}
#define QSTAMP(i)                                                   \
    do {                                                            \
        const unsigned long long qs_now = __builtin_amdgcn_s_memtime(); \
        qs_acc[i] += qs_now - qs_prev;                              \
        qs_prev = qs_now;                                           \
    } while (0)
#define QCOUNT(i) (qs_acc[i] += 1)
#define QSTAMP_STORE()                                                                   \
    if (lane == 0 && blockIdx.x * WAVES + wv < 4096)                                     \
        for (int i = 0; i < 10; ++i) g_q_stamps[blockIdx.x * WAVES + wv][i] = qs_acc[i]
#else
#define QSTAMP_INIT()
#define QSTAMP(i)
#define QCOUNT(i)
#define QSTAMP_STORE()
#endif

// STAGED: both inputs given (ba_gen_inputs_device buffers): loads only, the
// draw code is not compiled in.  EPI: 1 = the epilogue as W word units (lane =
// trial) in the queue; 0 = the bit-sliced epilogue of the whole task by the
// wave that wrote its roots (lab A/B).
template <int N, bool STAGED, int EPI = 1, int LAB = 0, int THREADS = kQueueThreads>
__global__ __launch_bounds__(THREADS, THREADS / 256) void k_om3q(
    uint64_t seed, GenSpec gs, uint64_t first_trial, uint64_t batch,
    const uint32_t* __restrict__ faulty, const uint8_t* __restrict__ order,
    uint64_t* __restrict__ decisions, uint8_t* __restrict__ outcome,
    uint64_t* __restrict__ counters, Sink sk, uint32_t tasks_per_group) {
    using G = Om3Q<N, THREADS>;
    constexpr int L = G::L, C = G::C, W = G::W, NIN = G::NIN, WAVES = G::waves;
    constexpr uint32_t ME = 3;
    static_assert(G::W * G::L <= 128, "roots: two items per lane");
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    // queue state: round units (q_next), per-task round completions (q_done);
    // a task's W epilogue word units become available when its roots are
    // written (e_ready) and are claimed one at a time (e_taken, e_claimed)
    __shared__ uint32_t q_next, q_done[kQueueMaxTasks], e_ready[kQueueMaxTasks],
        e_taken[kQueueMaxTasks], e_claimed;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t* wimg = lds + kQueueMaxTasks * G::task_words + wv * G::wave_words;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t ntasks = (total_words + W - 1) / W;
    const uint64_t ngroups = (ntasks + tasks_per_group - 1) / tasks_per_group;
    const uint32_t lw_ = lane / C, la = lane - lw_ * C;
    const bool act = lane < (uint32_t)G::LANES;
    const uint32_t lw = act ? lw_ : 0;
    TrialCounts tc;
    QSTAMP_INIT();
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t t0 = grp * tasks_per_group;
        const uint32_t nt = (uint32_t)(ntasks - t0 < tasks_per_group ? ntasks - t0 : tasks_per_group);
        if (threadIdx.x == 0) {
            q_next = 0;
            e_claimed = 0;
        }
        if (threadIdx.x < (uint32_t)kQueueMaxTasks) {
            q_done[threadIdx.x] = 0;
            e_ready[threadIdx.x] = 0;
            e_taken[threadIdx.x] = 0;
        }
        // A. inputs + level 0, one wave per task
        for (uint32_t t = wv; t < nt; t += WAVES) {
            uint64_t* timg = lds + t * G::task_words;
            const uint64_t w0 = (t0 + t) * W;
            if constexpr (STAGED)
                stage_words<N, W>(timg + G::tIN, lane, w0, batch, faulty, order);
            else
                wave_inputs<N, W, 0>(timg + G::tIN, lane, w0, seed, gs, first_trial, batch, faulty, order);
            __builtin_amdgcn_wave_barrier();
            queue_level0<N, W>(timg + G::tIN, timg + G::tL0, timg + G::tR1, lane, seed,
                               (first_trial >> 6) + w0);
        }
        QSTAMP(0);
        __syncthreads();
        QSTAMP(5);
        const uint32_t nunits = nt * (uint32_t)L, nepi = EPI ? nt * (uint32_t)W : 0u;
        // lab switches (tools/om3q_lab.hip; the product uses LAB = 0):
        //   1: static units (wave v takes units v, v+8, ...), 2: s_setprio 1 for
        //   waves 4-7, 4: waves 4-7 start phase B ~6k cycles late
        if constexpr ((LAB & 2) != 0) {
            if (wv >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
        }
        if constexpr ((LAB & 4) != 0) {
            if (wv >= WAVES / 2) {
                __builtin_amdgcn_s_sleep(47);
                __builtin_amdgcn_s_sleep(47);
            }
        }
        uint32_t lab_next = wv;
        while (true) {
            // 1. an epilogue word unit of a task whose roots are written, if any
            uint32_t e = 0xFFFFFFFFu;
            if (lane == 0) {
                for (uint32_t t = 0; t < nt; ++t) {
                    if (__hip_atomic_load(&e_ready[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                        __hip_atomic_load(&e_taken[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
                            (uint32_t)W) {
                        const uint32_t w = atomicAdd(&e_taken[t], 1u);
                        if (w < (uint32_t)W) {
                            atomicAdd(&e_claimed, 1u);
                            e = t * W + w;
                            break;
                        }
                    }
                }
            }
            e = __builtin_amdgcn_readfirstlane(e);
            if (e != 0xFFFFFFFFu) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint32_t t = e / W, w = e - t * W;
                const uint64_t* timg = lds + t * G::task_words;
                const uint64_t wg = (t0 + t) * W + w;  // trial word within the batch
                if (wg < total_words)
                    word_epilogue<N, ME>(timg + G::tIN + w * NIN, timg + G::tR1 + w * 2 * L, lane,
                                         wg * 64 + lane, batch, decisions, outcome, tc);
                QSTAMP(3);
                QCOUNT(8);
                continue;
            }
            // 2. a round unit (task, j1), task-major
            uint32_t u = 0;
            if constexpr ((LAB & 1) != 0) {
                u = lab_next;
                lab_next += WAVES;
            } else {
                if (lane == 0) u = atomicAdd(&q_next, 1u);
                u = __builtin_amdgcn_readfirstlane(u);
            }
            if (u < nunits) {
                const uint32_t t = u / (uint32_t)L, j1 = u - t * (uint32_t)L;
                uint64_t* timg = lds + t * G::task_words;
                const uint64_t gw = (first_trial >> 6) + (t0 + t) * W + lw;
                const uint64_t r1 = om3_round<N>(timg + G::tIN + lw * NIN,
                                                 act ? timg[G::tL0 + lw * L + j1] : 0ull, wimg, lw,
                                                 la, act, j1, seed, gw);
                if (act) timg[G::tR1 + (lw * L + la + (la >= j1 ? 1u : 0u)) * L + j1] = r1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                uint32_t d = 0;
                if (lane == 0) d = atomicAdd(&q_done[t], 1u);
                d = __builtin_amdgcn_readfirstlane(d);
                QSTAMP(1);
                QCOUNT(7);
                if (d + 1 != (uint32_t)L) continue;
                // the task's L-th round: its roots (compile-time carry-save counts of
                // L contiguous R1T words, L0 on the diagonal; strict majority
                // attacks, a tie is undefined, ba.py:188-195), written over R1T as
                // AU[W][2L], then its W epilogue word units are queued
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                uint64_t att[2] = {0, 0}, tie[2] = {0, 0};
                static_for<0, 2>([&](auto k) {
                    const uint32_t it = lane + 64 * k();
                    if (it < (uint32_t)(W * L)) {
                        const uint32_t w = it / L, col = it - w * L;
                        const uint64_t* r1t = timg + G::tR1 + (w * L + col) * L;
                        Csa<planes_c(L)> cnt;
                        static_for<0, L>([&](auto j) { cnt.template add<j()>(r1t[j()]); });
                        att[k()] = cnt.template ge<L, L / 2 + 1>();
                        if constexpr (L % 2 == 0) tie[k()] = cnt.template ge<L, L / 2>() & ~att[k()];
                    }
                });
                __builtin_amdgcn_wave_barrier();
                static_for<0, 2>([&](auto k) {
                    const uint32_t it = lane + 64 * k();
                    if (it < (uint32_t)(W * L)) {
                        const uint32_t w = it / L, col = it - w * L;
                        timg[G::tR1 + w * 2 * L + col] = att[k()];
                        timg[G::tR1 + w * 2 * L + L + col] = tie[k()];
                    }
                });
                QSTAMP(2);
                if constexpr (EPI == 0) {
                    __builtin_amdgcn_wave_barrier();
                    wave_epilogue<N, W, ME, 0>(timg + G::tIN, timg + G::tR1, lane, (t0 + t) * W, batch,
                                               decisions, outcome, tc);
                    QSTAMP(3);
                    continue;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(&e_ready[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                continue;
            }
            // 3. nothing to take: done once every epilogue unit is claimed, else a
            //    task's rounds are still running and its word units will appear
            if (__hip_atomic_load(&e_claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= nepi) break;
            __builtin_amdgcn_s_sleep(2);
            QSTAMP(4);
        }
        QSTAMP(4);
        __syncthreads();
        QSTAMP(6);
    }
    block_flush<WAVES>(tc, lane, wv, counters, sk);
    QSTAMP(6);
    QSTAMP_STORE();
}

template <int N>
inline hipError_t launch_om3q(const RunArgs& a) {
    using G = Om3Q<N>;
    const uint64_t words = (a.batch + 63) / 64, tasks = (words + G::W - 1) / G::W;
    // enough groups for every CU, at most kQueueMaxTasks tasks per group
    uint64_t tpg = (tasks + a.cu_count - 1) / a.cu_count;
    if (tpg < 1) tpg = 1;
    if (tpg > (uint64_t)kQueueMaxTasks) tpg = kQueueMaxTasks;
    const uint64_t groups = (tasks + tpg - 1) / tpg;
    uint64_t blocks = groups < a.cu_count ? groups : a.cu_count;  // one 8-wave block per CU
    if (const char* e = getenv("BA_WAVE_MAX_BLOCKS")) {  // tests: force the persistent group loop
        const uint64_t c = strtoull(e, nullptr, 0);
        if (c >= 1 && c < blocks) blocks = c;
    }
    const bool staged = a.gen.faulty_mode == 0 && a.gen.order_mode == 0;
    ProfScope ps(a.prof, "k_om3q", a.stream);
    if (staged)
        hipLaunchKernelGGL((k_om3q<N, true>), dim3((uint32_t)blocks), dim3(kQueueThreads),
                           G::lds_bytes, a.stream, a.seed, a.gen, a.first_trial, a.batch, a.faulty,
                           a.order, a.decisions, a.outcome, a.counters, a.sink, (uint32_t)tpg);
    else
        hipLaunchKernelGGL((k_om3q<N, false>), dim3((uint32_t)blocks), dim3(kQueueThreads),
                           G::lds_bytes, a.stream, a.seed, a.gen, a.first_trial, a.batch, a.faulty,
                           a.order, a.decisions, a.outcome, a.counters, a.sink, (uint32_t)tpg);
    return hipGetLastError();
}

}  // namespace ba
