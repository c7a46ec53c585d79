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
template <int S>
__device__ __forceinline__ void leaf_block(uint32_t me, uint64_t seed, uint64_t gw, uint32_t sr,
                                           const uint64_t (&diag)[S], const uint64_t (&Fm)[S],
                                           uint64_t (&R)[S]) {
    constexpr int P = planes_c(S);
    constexpr int NPAIR = S * (S - 1) / 2;
    Count<P> cnt[S];
    static_for<0, S>([&](auto b) { cnt[b()].add(diag[b()]); });
    const uint32_t pair0 = sr * (uint32_t)NPAIR;  // leaf block base slot sr*S*(S-1) is even
    static_for<0, NPAIR>([&](auto q) {
        uint64_t lw[2];
        lie_pair(seed, me, pair0 + q(), gw, lw[0], lw[1]);
        static_for<0, 2>([&](auto h) {
            constexpr int e = 2 * q() + h();     // slot within the block: row a, column c
            constexpr int a = e / (S - 1);
            constexpr int c = e % (S - 1);
            constexpr int b = c + (c >= a);      // receiver's rank among the S members
            cnt[b].add((Fm[a] & lw[h()]) | (~Fm[a] & diag[a]));
        });
    });
    static_for<0, S>([&](auto b) { R[b()] = cnt[b()].ge(S / 2 + 1); });  // inner tie -> non-attack
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
template <int S>
__global__ __launch_bounds__(256) void k_leaf(uint32_t me, uint64_t seed, uint64_t gw0,
                                              FastDiv divW, uint32_t work,
                                              const uint64_t* __restrict__ Lm1,
                                              const uint64_t* __restrict__ F,
                                              const uint64_t* __restrict__ members,
                                              uint64_t* __restrict__ Rm1) {
    const uint32_t W = divW.d;
    for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < work; idx += gridDim.x * 256) {
        const uint32_t sr = fdiv(idx, divW);
        const uint32_t w = idx - sr * W;
        const uint64_t mem = members[sr];  // S member ids, 5 bits each
        uint64_t diag[S], Fm[S], R[S];
        static_for<0, S>([&](auto a) {
            const uint64_t x = (uint64_t)sr * S + a();
            diag[a()] = Lm1[x * W + w];
            Fm[a()] = F[((mem >> (5 * a())) & 31u) * W + w];
        });
        leaf_block<S>(me, seed, gw0 + w, sr, diag, Fm, R);
        static_for<0, S>([&](auto b) { Rm1[((uint64_t)sr * S + b()) * W + w] = R[b()]; });
    }
}

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
    uint8_t* __restrict__ outcome, uint64_t* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    // run counters live in LDS (not in registers across the leaf stage)
    __shared__ __attribute__((aligned(16))) unsigned long long blockcnt[16];
    const FusedPlan& fp = *fpp;
    const uint32_t n = fp.n, L = n - 1, me = fp.me, WPB = fp.wpb, T = blockDim.x;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t stride = fp.word_stride;  // uint64 words per trial word in LDS
    if (tid < 16) blockcnt[tid] = 0;
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
        const uint64_t gwg = (first_trial >> 6) + w0;  // global word of lw = 0
        // ---- B: relay levels 0..me-1, one Philox per (slot pair, word) ----------
        // level me-1 (the leaf blocks' diagonal) goes into the R_{me-1} area:
        // each leaf block later reads its S words there before overwriting
        // exactly those S words with its S majorities.
        for (uint32_t k = 0; k + 1 <= me; ++k) {
            const uint32_t outk = (k + 1 == me) ? fp.offR[me - 1] : fp.offL[k];
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
        // ---- C: leaf blocks (sigma at level me-2), R_{me-1} into LDS -------------
        {
            const uint32_t Q = fp.S[me - 2];
            for (uint32_t it = tid; it < Q * nw; it += T) {
                const uint32_t lw = it / Q, sr = it - lw * Q;
                uint64_t* img = lds + (uint64_t)lw * stride;
                const uint64_t gw = gwg + lw;
                const uint32_t x0 = sr * S;
                const uint64_t mem = members[sr];  // S member ids, 5 bits each
                const uint32_t offR = fp.offR[me - 1] + x0;  // L_{me-1}[sigma.*], then R_{me-1}
                uint64_t diag[S], Fm[S], R[S];
                static_for<0, S>([&](auto a) {
                    diag[a()] = img[offR + a()];
                    Fm[a()] = img[(mem >> (5 * a())) & 31u];
                });
                leaf_block<S>(me, seed, gw, sr, diag, Fm, R);
                static_for<0, S>([&](auto b) { img[offR + b()] = R[b()]; });
            }
            __syncthreads();
        }
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
    }
    if (tid < 16) partial[(uint64_t)blockIdx.x * 16 + tid] = blockcnt[tid];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool leaf_supported(const Geometry& g) {
    const uint32_t S = g.n - g.me;
    return g.me >= 2 && S >= 2 && S <= kMaxLeafS;
}

template <int S>
static void launch_leaf_s(uint32_t me, uint64_t seed, uint64_t gw0, uint32_t W, uint32_t work,
                          const uint64_t* Lm1, const uint64_t* F, const uint64_t* snd,
                          uint64_t* Rm1, hipStream_t st) {
    uint64_t b = (work + 255) / 256;
    if (b > 16384) b = 16384;
    if (b < 1) b = 1;
    hipLaunchKernelGGL(k_leaf<S>, dim3((uint32_t)b), dim3(256), 0, st, me, seed, gw0,
                       make_fastdiv(W), work, Lm1, F, snd, Rm1);
}

hipError_t launch_leaf(const Geometry& g, uint64_t seed, uint64_t gw0, uint32_t W,
                       const uint64_t* Lm1, const uint64_t* F, const uint64_t* d_members,
                       uint64_t* Rm1, hipStream_t st, Prof* prof) {
    ProfScope ps(prof, "k_leaf", st);
    const uint32_t S = g.n - g.me;
    const uint32_t work = (uint32_t)(g.S[g.me - 2] * W);
    const uint64_t* snd = d_members;
    switch (S) {
#define LEAF_CASE(s) \
    case s: launch_leaf_s<s>(g.me, seed, gw0, W, work, Lm1, F, snd, Rm1, st); break;
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
                           const RunArgs& a, const uint8_t* d_sender, uint64_t* partials) {
    hipLaunchKernelGGL(k_fused<S>, dim3(blocks), dim3(fp.threads), fp.lds_bytes, a.stream, d_fp,
                       a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order, d_sender, a.members,
                       a.decisions, a.outcome, partials);
}

hipError_t launch_fused(const RunArgs& a, const Geometry& g, const FusedPlan& fp,
                        const FusedPlan* d_fp, const uint8_t* d_sender, uint64_t* partials) {
    const uint64_t words = (a.batch + 63) / 64;
    // one block per resident slot (occupancy x CUs): each owns an equal run of words
    int occ = 0;
    switch (g.n - g.me) {
#define OCC_CASE(s) \
    case s: (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused<s>, fp.threads, fp.lds_bytes); break;
        OCC_CASE(2) OCC_CASE(3) OCC_CASE(4) OCC_CASE(5) OCC_CASE(6) OCC_CASE(7)
        OCC_CASE(8) OCC_CASE(9) OCC_CASE(10) OCC_CASE(11) OCC_CASE(12)
#undef OCC_CASE
        default: return hipErrorInvalidValue;
    }
    if (occ < 1) occ = 1;
    uint64_t slots = (uint64_t)occ * a.cu_count;
    if (slots > (uint64_t)kPartialRows) slots = kPartialRows;
    const uint32_t blocks = (uint32_t)(words < slots ? words : slots);
    {
        ProfScope ps(a.prof, "k_fused", a.stream);
        switch (g.n - g.me) {
#define FUSED_CASE(s) \
    case s: launch_fused_s<s>(fp, d_fp, blocks, a, d_sender, partials); break;
            FUSED_CASE(2) FUSED_CASE(3) FUSED_CASE(4) FUSED_CASE(5) FUSED_CASE(6) FUSED_CASE(7)
            FUSED_CASE(8) FUSED_CASE(9) FUSED_CASE(10) FUSED_CASE(11) FUSED_CASE(12)
#undef FUSED_CASE
            default: return hipErrorInvalidValue;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_reduce(partials, (int)blocks, a.counters, a.stream, a.prof);
}

}  // namespace ba
