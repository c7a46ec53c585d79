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
#include "ba_leaf.hpp"

namespace ba {

// ---------------------------------------------------------------------------
// LEVELS: one thread per (leaf block, word)
// ---------------------------------------------------------------------------
// Leaf blocks sr = srbase + idx / W (a first-hop subtree range of level me-2).
// Relay level me-1 is fused in: the S diagonal values of block sr all relay
// its parent L_{me-2}[sr] through the same sender (the last general of sr,
// snd2[sr]), so the thread reads one parent word and draws the level me-1
// lies itself (the same Philox pairs k_relay would draw: keyed by global slot
// pair, so the bits are identical).  L_{me-1} and L_me are never materialised.
// L_{me-2} is indexed from lbase (its range's first slot; level 0 is whole),
// R_{me-1} from the range's first block.
template <int S>
__global__ __launch_bounds__(256) void k_leaf(uint32_t me, uint64_t seed, uint64_t gw0,
                                              FastDiv divW, uint32_t work, uint32_t srbase,
                                              uint32_t lbase, const uint64_t* __restrict__ Lm2,
                                              const uint8_t* __restrict__ snd2,
                                              const uint64_t* __restrict__ F,
                                              const uint64_t* __restrict__ members,
                                              uint64_t* __restrict__ Rm1) {
    constexpr int NPD = (S + 1) / 2;  // level me-1 slot pairs a block's S slots touch
    const uint32_t W = divW.d;
    for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < work; idx += gridDim.x * 256) {
        const uint32_t sl = fdiv(idx, divW);
        const uint32_t w = idx - sl * W;
        const uint32_t sr = srbase + sl;
        const uint64_t gw = gw0 + w;
        const uint64_t mem = members[sr];  // S member ids, 5 bits each
        const uint64_t par = Lm2[(uint64_t)(sr - lbase) * W + w];
        const uint64_t fs = F[(uint64_t)snd2[sr] * W + w];
        const uint32_t x0 = sr * (uint32_t)S;  // first level me-1 slot of the block
        uint64_t lw[2 * NPD];
        lie_pairs<NPD>(seed, me - 1, x0 >> 1, gw, lw);
        const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);  // odd S only: block starts mid-pair
        uint64_t diag[S], Fm[S], R[S];
        static_for<0, S>([&](auto a) {
            uint64_t lie;
            if constexpr (S % 2 == 1) lie = lw[a()] ^ ((lw[a()] ^ lw[a() + 1]) & oddmask);
            else lie = lw[a()];
            diag[a()] = (fs & lie) | (~fs & par);
            Fm[a()] = F[((mem >> (5 * a())) & 31u) * W + w];
        });
        leaf_block<S>(me, seed, gw, sr, diag, Fm, R);
        static_for<0, S>([&](auto b) { Rm1[((uint64_t)sl * S + b()) * W + w] = R[b()]; });
    }
}

// LEVELS leaf-up (me >= 3): the S+1 sibling leaf blocks rho.x (x < G = S+1,
// the children of one level me-3 slot rho) of one word run on G lanes of one
// wave, and the wave also takes the next majority up,
//     R_{me-2}[rho.x] = maj(L_{me-2}[rho.x], R_{me-1}[rho.a.x] : a != x)
// (G inputs, inner tie -> non-attack).  Receiver x's inputs sit in the OTHER
// blocks' columns (member d of block a is sibling d + (d >= a)), so the lanes
// swap them through LDS, receiver-major T[x][a] with L_{me-2}[rho.x] on the
// diagonal, as the WAVE kernels' om3_round does for R1.  R_{me-1} is never
// stored: one k_majority launch and the S words per block it read go away.
// A unit = (rho, word), GPW = 64 / G units per wave; slot rho.x = srbase +
// unit's rho rank * G + x (the level me-2 range starts at its first child).
template <int S>
__global__ __launch_bounds__(256) void k_leaf_up(uint32_t me, uint64_t seed, uint64_t gw0,
                                                 FastDiv divW, uint32_t units, uint32_t srbase,
                                                 uint32_t lbase, const uint64_t* __restrict__ Lm2,
                                                 const uint8_t* __restrict__ snd2,
                                                 const uint64_t* __restrict__ F,
                                                 const uint64_t* __restrict__ members,
                                                 uint64_t* __restrict__ Rm2) {
    constexpr int G = S + 1, GP = G + 1, GPW = 64 / G, NPD = (S + 1) / 2;
    __shared__ uint64_t tr[4][GPW][G][GP];  // [wave][unit][receiver x][sender a], rows padded
    const uint32_t W = divW.d;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t g = lane / G, x = lane - g * G;
    const bool act = g < (uint32_t)GPW;
    const uint32_t gg = act ? g : 0;
    for (uint32_t u0 = blockIdx.x * 4 * GPW; u0 < units; u0 += gridDim.x * 4 * GPW) {
        const uint32_t u = u0 + wv * GPW + gg;
        const bool ok = act && u < units;
        const uint32_t rl = fdiv(ok ? u : 0u, divW);
        const uint32_t w = (ok ? u : 0u) - rl * W;
        const uint32_t sl = rl * G + x;
        const uint32_t sr = srbase + sl;
        uint64_t par = 0;
        if (ok) {
            const uint64_t gw = gw0 + w;
            const uint64_t mem = members[sr];
            par = Lm2[(uint64_t)(sr - lbase) * W + w];
            const uint64_t fs = F[(uint64_t)snd2[sr] * W + w];
            const uint32_t x0 = sr * (uint32_t)S;
            uint64_t lw[2 * NPD];
            lie_pairs<NPD>(seed, me - 1, x0 >> 1, gw, lw);
            const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
            uint64_t diag[S], Fm[S], R[S];
            static_for<0, S>([&](auto a) {
                uint64_t lie;
                if constexpr (S % 2 == 1) lie = lw[a()] ^ ((lw[a()] ^ lw[a() + 1]) & oddmask);
                else lie = lw[a()];
                diag[a()] = (fs & lie) | (~fs & par);
                Fm[a()] = F[((mem >> (5 * a())) & 31u) * W + w];
            });
            leaf_block<S>(me, seed, gw, sr, diag, Fm, R);
            uint64_t* t = &tr[wv][gg][0][x];
            t[x * GP] = par;
            static_for<0, S>([&](auto d) { t[(d() + (d() >= x ? 1u : 0u)) * GP] = R[d()]; });
        }
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            const uint64_t* col = &tr[wv][gg][x][0];
            Csa<planes_c(G)> cnt;
            static_for<0, G>([&](auto a) { cnt.template add<a()>(col[a()]); });
            Rm2[(uint64_t)sl * W + w] = cnt.template ge<G, G / 2 + 1>();
        }
        __builtin_amdgcn_wave_barrier();  // tr is rewritten by the next unit
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
// host side
// ---------------------------------------------------------------------------
bool leaf_supported(const Geometry& g) {
    const uint32_t S = g.n - g.me;
    return g.me >= 2 && S >= 2 && S <= kMaxLeafS;
}

template <int S>
static void launch_leaf_s(uint32_t me, uint64_t seed, uint64_t gw0, uint32_t W, uint32_t work,
                          uint32_t srbase, uint32_t lbase, const uint64_t* Lm2,
                          const uint8_t* snd2, const uint64_t* F, const uint64_t* mem,
                          uint64_t* Rout, bool up, hipStream_t st) {
    if (up) {  // work = units (rho, word); GPW units per wave, 4 waves per block
        constexpr uint32_t GPW = 64 / (S + 1);
        uint64_t b = (work + 4 * GPW - 1) / (4 * GPW);
        if (b > 16384) b = 16384;
        if (b < 1) b = 1;
        hipLaunchKernelGGL(k_leaf_up<S>, dim3((uint32_t)b), dim3(256), 0, st, me, seed, gw0,
                           make_fastdiv(W), work, srbase, lbase, Lm2, snd2, F, mem, Rout);
        return;
    }
    uint64_t b = (work + 255) / 256;
    if (b > 16384) b = 16384;
    if (b < 1) b = 1;
    hipLaunchKernelGGL(k_leaf<S>, dim3((uint32_t)b), dim3(256), 0, st, me, seed, gw0,
                       make_fastdiv(W), work, srbase, lbase, Lm2, snd2, F, mem, Rout);
}

hipError_t launch_leaf(const Geometry& g, uint64_t seed, uint64_t gw0, uint32_t W,
                       uint32_t srbase, uint32_t srcnt, uint32_t lbase, const uint64_t* Lm2,
                       const uint8_t* d_sender, const uint64_t* F, const uint64_t* d_members,
                       uint64_t* Rm1, bool up, hipStream_t st, Prof* prof) {
    ProfScope ps(prof, up ? "k_leaf_up" : "k_leaf", st);
    if (up && g.me < 3) return hipErrorInvalidValue;  // R_{me-2} would be the root level
    const uint32_t S = g.n - g.me;
    if (up && srcnt % (S + 1) != 0) return hipErrorInvalidValue;  // whole sibling groups only
    // work items: (leaf block, word), or (sibling group, word) for leaf-up
    const uint32_t work = (uint32_t)((uint64_t)(up ? srcnt / (S + 1) : srcnt) * W);
    if (work == 0) return hipSuccess;
    const uint8_t* snd2 = d_sender + g.sender_off[g.me - 2];  // last general of each level me-2 slot
    switch (S) {
#define LEAF_CASE(s) \
    case s: launch_leaf_s<s>(g.me, seed, gw0, W, work, srbase, lbase, Lm2, snd2, F, d_members, Rm1, up, st); break;
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

hipError_t launch_fused(const RunArgs& a, const Geometry& g, bool plan_ok, const FusedPlan& fp,
                        const FusedPlan* d_fp, const uint8_t* d_sender, uint64_t* partials) {
    const uint64_t words = (a.batch + 63) / 64;
    // effective depth 3 or 4 within wave_supported: the WAVE kernels.
    // BA_FUSED_KIND=2 runs the generic k_fused on such a tree instead (a
    // cross-check of two independent kernels in the GPU tests).
    const char* kenv = getenv("BA_FUSED_KIND");
    const int kind = kenv ? atoi(kenv) : 0;
    if (wave_supported(g) && kind != 2) return launch_wave_engine(a, g);
    if (!plan_ok) return hipErrorInvalidValue;  // BA_FUSED_KIND forced a kernel this tree lacks
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
        switch (g.n - g.me) {
#define FUSED_CASE(s) \
    case s: launch_fused_s<s>(fp, d_fp, blocks, lds_bytes, a, d_sender, partials); break;
            FUSED_CASE(2) FUSED_CASE(3) FUSED_CASE(4) FUSED_CASE(5) FUSED_CASE(6) FUSED_CASE(7)
            FUSED_CASE(8) FUSED_CASE(9) FUSED_CASE(10) FUSED_CASE(11) FUSED_CASE(12)
#undef FUSED_CASE
            default: return hipErrorInvalidValue;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    (void)partials;
    return hipSuccess;
}

}  // namespace ba
