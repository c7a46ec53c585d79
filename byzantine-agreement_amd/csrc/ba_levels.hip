// ba_levels.hip -- LEVELS engine: level-synchronous OM(m) over bit-packed HBM
// arrays, plus the ba.py table-mode (OM(1) canonical draw order) kernel.
//
// Layout: level k is an array L_k[slot][word] of uint64, word-fastest, so the
// 64 lanes of a wave touch 64 consecutive words of one slot (512 B, coalesced).
//
//   k_input     bit-slices per-trial inputs: F[g][w] = ballot(general g faulty)
//               (k_input_given: staged inputs, four words per wave)
//   k_relay     L_k[x] = F[sender] ? lie(x) : L_{k-1}[parent(x)]   (ba.py:42-57, 263-277)
//   k_relay_top levels 0..K in one launch (ancestor chains)
//   k_majority  R_p[sigma.r] = [2a > s] over L_p[sigma.r] and R_{p+1}[sigma.j.r] (ba.py:159-195)
//   k_epilogue  root majority (tie -> undefined), quorum, IC flags    (ba.py:188-255)
// The leaf-fused kernels (k_leaf, k_leaf_up) are in ba_fused.hip; the small-batch
// tail (k_tail) and the big-batch epilogue (k_epilogue_w) in ba_tail.hip.
#include "ba_engine.hpp"

namespace ba {

constexpr int kBlock = 256;
constexpr uint32_t kLoadChunk = 8;  // child loads issued together by the majority kernels

__device__ __forceinline__ uint32_t grid_threads() { return gridDim.x * kBlock; }

// ---------------------------------------------------------------------------
// input bit-slicing: one wave per 64-trial word
// ---------------------------------------------------------------------------
// The planes of word w (lane = trial): F[g] for the n generals, OB (order is
// attack), OO (order is "other"), VAL (trial of the batch); lane g < n returns
// F[g] in `mine`, every lane returns ob / oo / vv.
__device__ __forceinline__ void word_inputs(uint32_t n, uint64_t seed, const GenSpec& gs, uint64_t t0,
                                            uint64_t ntrials, const uint32_t* __restrict__ faulty,
                                            const uint8_t* __restrict__ order, uint64_t w,
                                            uint32_t lane, uint64_t& mine, uint64_t& ob,
                                            uint64_t& oo, uint64_t& vv) {
    const uint64_t i = w * 64 + lane;  // trial index within the chunk
    const bool valid = i < ntrials;
    uint32_t fm = 0, oc = 0;
    if (valid) {
        if (gs.faulty_mode == 0) fm = faulty[i];
        if (gs.order_mode == 0) oc = order[i];
        gen_trial(n, seed, gs, t0 + i, fm, oc);
    }
    mine = 0;
    for (uint32_t g = 0; g < n; ++g) {
        const uint64_t b = __ballot(valid && ((fm >> g) & 1u));
        if (lane == g) mine = b;
    }
    ob = __ballot(valid && oc == 1);
    oo = __ballot(valid && oc == 2);
    vv = __ballot(valid);
}

__global__ __launch_bounds__(kBlock) void k_input(uint32_t n, uint64_t seed, GenSpec gs,
                                                  uint64_t t0, uint64_t ntrials,
                                                  const uint32_t* __restrict__ faulty,
                                                  const uint8_t* __restrict__ order,
                                                  uint64_t* __restrict__ scratch, uint64_t W,
                                                  uint64_t offF, uint64_t offOB, uint64_t offOO,
                                                  uint64_t offVAL) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t words_per_grid = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < W;
         w += words_per_grid) {
        uint64_t mine, ob, oo, vv;
        word_inputs(n, seed, gs, t0, ntrials, faulty, order, w, lane, mine, ob, oo, vv);
        if (lane < n) scratch[offF + (uint64_t)lane * W + w] = mine;
        if (lane == 0) {
            scratch[offOB + w] = ob;
            scratch[offOO + w] = oo;
            scratch[offVAL + w] = vv;
        }
    }
}

// Given (staged) inputs: a wave slices kInGivenWPW words, every load of them in
// flight before the first ballot (one wave per word waited one round trip each
// and needed 4x the waves).
constexpr uint32_t kInGivenWPW = 4;
__global__ __launch_bounds__(kBlock) void k_input_given(uint32_t n, uint64_t ntrials,
                                                        const uint32_t* __restrict__ faulty,
                                                        const uint8_t* __restrict__ order,
                                                        uint64_t* __restrict__ scratch, uint64_t W,
                                                        uint64_t offF, uint64_t offOB, uint64_t offOO,
                                                        uint64_t offVAL) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t base = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); base < W;
         base += nwaves * kInGivenWPW) {
        uint32_t fm[kInGivenWPW], oc[kInGivenWPW];
#pragma unroll
        for (uint32_t k = 0; k < kInGivenWPW; ++k) {
            const uint64_t w = base + k * nwaves, i = w * 64 + lane;
            const bool ok = w < W && i < ntrials;
            fm[k] = ok ? faulty[i] : 0u;
            oc[k] = ok ? order[i] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kInGivenWPW; ++k) {
            const uint64_t w = base + k * nwaves;
            if (w >= W) break;
            const bool valid = w * 64 + lane < ntrials;
            uint64_t mine = 0;
            for (uint32_t g = 0; g < n; ++g) {
                const uint64_t b = __ballot(valid && ((fm[k] >> g) & 1u));
                if (lane == g) mine = b;
            }
            const uint64_t ob = __ballot(valid && oc[k] == 1), oo = __ballot(valid && oc[k] == 2);
            const uint64_t vv = __ballot(valid);
            if (lane < n) scratch[offF + (uint64_t)lane * W + w] = mine;
            if (lane == 0) {
                scratch[offOB + w] = ob;
                scratch[offOO + w] = oo;
                scratch[offVAL + w] = vv;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// relay level k: one thread per (slot pair, word); one Philox call per thread.
// Level k holds global slots [xbase, xbase + xcnt) (a first-hop subtree range;
// the whole level by default), its parent level starts at global slot pbase.
// Lies stay keyed by the GLOBAL slot pair, so any split gives the same bits.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_relay(uint32_t k, uint32_t xbase, uint32_t xcnt,
                                                  uint32_t pbase, FastDiv divW, FastDiv divFan,
                                                  uint32_t work, uint64_t seed, uint64_t gw0,
                                                  const uint64_t* __restrict__ Lprev,
                                                  uint64_t* __restrict__ Lk,
                                                  const uint64_t* __restrict__ F,
                                                  const uint8_t* __restrict__ sender) {
    const uint32_t W = divW.d;
    const uint32_t pair0 = xbase >> 1, xend = xbase + xcnt;
    for (uint32_t idx = blockIdx.x * kBlock + threadIdx.x; idx < work; idx += grid_threads()) {
        const uint32_t pl = fdiv(idx, divW);
        const uint32_t w = idx - pl * W;
        const uint32_t pair = pair0 + pl;
        uint64_t lie[2];
        lie_pair(seed, k, pair, gw0 + w, lie[0], lie[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t x = 2 * pair + h;
            if (x < xbase || x >= xend) continue;
            uint64_t parent, fw;
            if (k == 0) {  // commander -> lieutenant x (ba.py:263-277)
                parent = Lprev[w];
                fw = F[w];
            } else {
                const uint32_t y = fdiv(x, divFan);
                parent = Lprev[(uint64_t)(y - pbase) * W + w];
                fw = F[(uint64_t)sender[y] * W + w];
            }
            Lk[(uint64_t)(x - xbase) * W + w] = (fw & lie[h]) | (~fw & parent);
        }
    }
}

// ---------------------------------------------------------------------------
// Bit-sliced root + quorum epilogue (4 <= n <= 16, me >= 1): a block owns 64
// consecutive trial words, and the quorum is decided for all 64 trials of a
// word at once with bit-plane counters (lane = word), as the WAVE engines'
// epilogue does; trial_result (ba_device.hpp, the per-trial restatement of
// ba.py:197-255 the oracle pins) is the reference it must equal.
//   1. wave v computes the root majorities of receivers b = v, v+4, ...
//      for the 64 words (lane = word: coalesced loads) into LDS A/U planes
//   2. wave 0 (lane = word): quorum, IC1/IC2 and bound flags from the planes,
//      run counters by popcount; six outcome planes + the live mask to LDS
//   3. wave v extracts words v, v+4, ... per trial (lane = trial) and stores
//      the decision word and outcome byte
// LDS: [2L + 7 + n][64] uint64 (A planes, U planes, 6 outcome planes, live
// mask, faulty planes).  Used from 64 words per launch up (one block per 64
// words; below that the per-trial k_epilogue has more parallelism).
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(kBlock) void k_epilogue_bs(uint32_t n, uint32_t me, uint64_t W,
                                                        const uint64_t* __restrict__ scratch,
                                                        uint64_t offF, uint64_t offOB,
                                                        uint64_t offOO, uint64_t offVAL,
                                                        uint64_t offL0,
                                                        const uint64_t* __restrict__ C1,
                                                        uint64_t* __restrict__ decisions,
                                                        uint8_t* __restrict__ outcome,
                                                        uint64_t* __restrict__ counters, Sink sk) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sp[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t L = n - 1;
    const uint32_t needed = 2 * ((n - 1) / 3) + 1;  // quorum of n >= 4 live generals
    const uint32_t K0 = L - needed;                 // retreat: #(A|U) <= K0 (+1 if the order is retreat)
    uint64_t* sOut = sp + 2 * L * 64;               // q1 q2 agree appl valid inb live
    uint64_t* sF = sOut + 7 * 64;                   // faulty planes of the n generals
    TrialCounts tc;
    const uint64_t groups = (W + 63) / 64;
    for (uint64_t gi = blockIdx.x; gi < groups; gi += gridDim.x) {
        const uint64_t w = gi * 64 + lane;
        const bool wok = w < W;
        // 1. faulty planes to LDS (rows g = v, v+4, ...), then the root
        //    majorities (L inputs: L_0[b] and the level-1 votes about b); every
        //    load of a chunk is in flight before the first add
        for (uint32_t g = wv; g < n; g += kBlock / 64)
            sF[g * 64 + lane] = wok ? scratch[offF + (uint64_t)g * W + w] : 0ull;
        for (uint32_t b = wv; b < L; b += kBlock / 64) {
            Count<P> c;
            if (wok) {
                for (uint32_t a0 = 0; a0 < L; a0 += kLoadChunk) {  // a == b: the direct value L_0[b]
                    uint64_t v[kLoadChunk];
#pragma unroll
                    for (uint32_t q = 0; q < kLoadChunk; ++q) {
                        const uint32_t a = a0 + q;
                        const uint64_t cs = (uint64_t)a * (L - 1) + (b - (b > a));
                        v[q] = a >= L ? 0ull
                                      : (a == b ? scratch[offL0 + (uint64_t)b * W + w] : C1[cs * W + w]);
                    }
#pragma unroll
                    for (uint32_t q = 0; q < kLoadChunk; ++q) c.add(v[q]);
                }
            }
            const uint64_t att = c.ge(L / 2 + 1);                        // strict majority
            const uint64_t tie = (L & 1u) ? 0ull : (c.ge(L / 2) & ~att);  // root tie: undefined
            sp[b * 64 + lane] = att;
            sp[(L + b) * 64 + lane] = tie;
        }
        __syncthreads();
        // 2. quorum and flags, lane = word
        if (wv == 0) {
            uint64_t val = 0, obr = 0, oo = 0;
            if (wok) {
                val = scratch[offVAL + w];
                obr = scratch[offOB + w];
                oo = scratch[offOO + w];
            }
            const uint64_t f0 = sF[lane];
            const uint64_t ob = obr & ~oo, orr = ~obr & ~oo;  // commander attack / retreat
            Count<P> cA, cX, cF;
            cF.add(f0);
            uint64_t anyA = 0, anyU = 0, anyR = 0, allA = ~0ull, allR = ~0ull;
            uint32_t nA = 0, nU = 0, nf = (uint32_t)__popcll(f0 & val);
            for (uint32_t b = 0; b < L; ++b) {
                const uint64_t a = sp[b * 64 + lane], u = sp[(L + b) * 64 + lane], x = a | u;
                const uint64_t f = sF[(b + 1) * 64 + lane];
                cA.add(a);
                cX.add(x);
                cF.add(f);
                anyA |= a & ~f;
                anyU |= u & ~f;
                anyR |= ~(x | f);
                allA &= a | f;
                allR &= ~x | f;
                nA += (uint32_t)__popcll(a & val);
                nU += (uint32_t)__popcll(u & val);
                nf += (uint32_t)__popcll(f & val);
            }
            const uint64_t retreat = ~cX.ge(K0 + 1) | (orr & ~cX.ge(K0 + 2));
            const uint64_t attc = cA.ge(needed) | (ob & cA.ge(needed - 1));
            const uint64_t q1 = ~retreat & attc, q2 = ~retreat & ~attc;
            const uint64_t agree = ~maj3(anyA, anyU, anyR);  // loyal lieutenants: one decision kind
            const uint64_t appl = ~f0;
            const uint64_t valid = appl & ((ob & allA) | (~ob & allR));
            const uint64_t inb = n > 3 * me ? ~cF.ge(me + 1) : 0ull;
            tc.v[C_TRIALS] += (uint32_t)__popcll(val);
            tc.v[C_AGREE] += (uint32_t)__popcll(agree & val);
            tc.v[C_VAPPL] += (uint32_t)__popcll(appl & val);
            tc.v[C_VALID] += (uint32_t)__popcll(valid & val);
            tc.v[C_QR] += (uint32_t)__popcll(retreat & val);
            tc.v[C_QA] += (uint32_t)__popcll(q1 & val);
            tc.v[C_QU] += (uint32_t)__popcll(q2 & val);
            tc.v[C_UNDEF] += nU;
            tc.v[C_INB] += (uint32_t)__popcll(inb & val);
            tc.v[C_VIOL] += (uint32_t)__popcll(inb & (~agree | (appl & ~valid)) & val);
            tc.v[C_FTOT] += nf;
            tc.v[C_ATT] += nA;
            sOut[0 * 64 + lane] = q1;
            sOut[1 * 64 + lane] = q2;
            sOut[2 * 64 + lane] = agree;
            sOut[3 * 64 + lane] = appl;
            sOut[4 * 64 + lane] = valid;
            sOut[5 * 64 + lane] = inb;
            sOut[6 * 64 + lane] = val;
        }
        __syncthreads();
        // 3. per-trial decision words and outcome bytes, lane = trial
        const uint32_t half = lane >> 5, sh = lane & 31;
        auto bit = [&](const uint64_t* q) -> uint32_t {
            return __builtin_amdgcn_ubfe(reinterpret_cast<const uint32_t*>(q)[half], sh, 1);
        };
        const uint32_t nw = (uint32_t)(W - gi * 64 < 64 ? W - gi * 64 : 64);
        for (uint32_t j = wv; j < nw; j += kBlock / 64) {
            if (!bit(sOut + 6 * 64 + j)) continue;  // not a trial of this batch
            uint64_t dec = 0;
            for (uint32_t b = 0; b < L; ++b) {
                dec |= (uint64_t)bit(sp + b * 64 + j) << (2 * b);
                dec |= (uint64_t)bit(sp + (L + b) * 64 + j) << (2 * b + 1);
            }
            uint32_t out = 0;
#pragma unroll
            for (int k = 0; k < 6; ++k) out |= bit(sOut + k * 64 + j) << k;
            const uint64_t i = (gi * 64 + j) * 64 + lane;
            if (decisions) decisions[i] = dec;
            if (outcome) outcome[i] = (uint8_t)out;
        }
        __syncthreads();
    }
    block_counts_sink<kBlock>(tc, counters, sk);
}

// ---------------------------------------------------------------------------
// relay levels 0..K in ONE launch (the levels above the leaf blocks are small:
// for n=16, m=5 they are 15 + 210 + 2730 + 32760 slots, where four k_relay
// launches cost more in launch gaps than in work).  Items [0, np0*W) write
// level 0 (always whole).  The other items own one level-K slot pair of the
// range and word: each walks its slots' ancestor chain from the commander down,
// drawing the lie pair of every ancestor (keyed by global slot pair, as
// k_relay), and writes its level-K slots plus every ancestor it is the first
// descendant of (x == a * D[k]).  Redundant draws: K per level-K pair, ~4%
// of a depth-5 tree's Philox calls.
// ---------------------------------------------------------------------------
constexpr int kTopMax = 6;
struct TopPlan {
    uint32_t K, L;                     // deepest level; lieutenants (= level-0 slots)
    uint32_t np0;                      // level-0 slot pairs
    uint32_t xbK, xeK;                 // level-K slot range [xbK, xeK)
    uint32_t base[kTopMax + 1];        // first slot of level k's range (level 0: 0)
    uint64_t off[kTopMax + 1];         // scratch offset of level k
    uint32_t snd_off[kTopMax + 1];     // sender table offset of level k (k < K)
    FastDiv D[kTopMax + 1];            // D[k] = prod_{i=k+1..K} (L - i): level-K slots per level-k slot
};

// Inputs fused in (IN.fuse): every block bit-slices the batch's inputs itself
// into LDS (a wave per word) and reads F / OB from there, and block 0 also
// stores them to scratch for the later kernels -- one launch (k_input) less on
// the latency-bound small batches of config 5.  Every block re-slices the
// whole batch, so this pays only for tiny batches: at 16 words (config 5's
// 1024 instances) the fused launch measured 4.6 us slower per call than
// k_input + k_relay_top, with staged and with drawn inputs (tools/config5_ab.py).
constexpr uint32_t kTopFuseWords = 2;
constexpr uint32_t kTopFuseGivenWords = kTopFuseWords;
struct TopInputs {
    uint32_t fuse, n;
    uint64_t seed, t0, ntrials;
    GenSpec gs;
    const uint32_t* faulty;
    const uint8_t* order;
    uint64_t offOO, offVAL;
};

// The ancestor chain of level-K slot x: levels 0..K-1, each a relay of the
// one above (commander first), drawn from the Philox pair of the ancestor's
// global slot pair (k_relay's keying, so the bits are identical).  Returns
// the value of x's level K-1 ancestor and writes every ancestor x is the first
// descendant of.  All table and F loads are issued before the first store (a
// store to scratch may alias F, so interleaving them would serialise one
// memory round trip per level), and the K Philox calls -- plus, with EXTRA,
// the caller's level-K pair `xc` -- run as one interleaved group.
template <int K, bool EXTRA>
__device__ __forceinline__ uint64_t top_chain(const TopPlan& tp, uint32_t x, uint32_t w,
                                              uint32_t W, uint64_t gw, uint64_t seed,
                                              const uint64_t* F, uint64_t ob,
                                              const uint8_t* __restrict__ sender,
                                              uint64_t* __restrict__ scratch, P4& xc) {
    uint32_t a[K], snd[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = fdiv(x, tp.D[k]);
    snd[0] = 0;  // level 0: the commander relays
#pragma unroll
    for (int k = 1; k < K; ++k) snd[k] = sender[tp.snd_off[k - 1] + a[k - 1]];
    uint64_t fw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) fw[k] = F[(uint64_t)snd[k] * W + w];
    constexpr int G = K + (EXTRA ? 1 : 0);
    P4 c[G];
#pragma unroll
    for (int k = 0; k < K; ++k) c[k] = P4{a[k] >> 1, (uint32_t)k, (uint32_t)gw, (uint32_t)(gw >> 32)};
    if constexpr (EXTRA) c[K] = xc;
    philox10_n<G>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    if constexpr (EXTRA) xc = c[K];
    uint64_t v = ob;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t lie = (a[k] & 1u) ? ((uint64_t)c[k].w << 32 | c[k].z)
                                         : ((uint64_t)c[k].y << 32 | c[k].x);
        v = (fw[k] & lie) | (~fw[k] & v);
        if (k >= 1 && x == a[k] * tp.D[k].d)  // first descendant writes the ancestor
            scratch[tp.off[k] + (uint64_t)(a[k] - tp.base[k]) * W + w] = v;
    }
    return v;
}

template <int K>
__global__ __launch_bounds__(kBlock) void k_relay_top(TopPlan tp, FastDiv divW, uint32_t work,
                                                      uint64_t seed, uint64_t gw0,
                                                      const uint8_t* __restrict__ sender,
                                                      uint64_t* __restrict__ scratch,
                                                      uint64_t offF, uint64_t offOB, TopInputs IN) {
    const uint32_t W = divW.d;
    const uint32_t work0 = tp.np0 * W;
    const uint64_t* F = scratch + offF;
    const uint64_t* OBp = scratch + offOB;
    __shared__ uint64_t sIn[kTopFuseGivenWords * (kMaxN + 1)];  // F[g][w] rows, then OB[w]
    if (IN.fuse) {
        const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        auto put = [&](uint32_t w, uint64_t mine, uint64_t ob, uint64_t oo, uint64_t vv) {
            if (lane < IN.n) sIn[lane * W + w] = mine;
            if (lane == 0) sIn[IN.n * W + w] = ob;
            if (blockIdx.x == 0) {
                if (lane < IN.n) scratch[offF + (uint64_t)lane * W + w] = mine;
                if (lane == 0) {
                    scratch[offOB + w] = ob;
                    scratch[IN.offOO + w] = oo;
                    scratch[IN.offVAL + w] = vv;
                }
            }
        };
        if (IN.gs.faulty_mode == 0 && IN.gs.order_mode == 0) {
            // given (staged) inputs: every load of the wave's words in flight
            // before the first ballot (a load-ballot loop waits one round trip
            // per word)
            constexpr uint32_t PW = (kTopFuseGivenWords + kBlock / 64 - 1) / (kBlock / 64);
            uint32_t fm[PW], oc[PW];
#pragma unroll
            for (uint32_t j = 0; j < PW; ++j) {
                const uint32_t w = wv + j * (kBlock / 64);
                const uint64_t i = (uint64_t)w * 64 + lane;
                const bool ok = w < W && i < IN.ntrials;
                fm[j] = ok ? IN.faulty[i] : 0u;
                oc[j] = ok ? IN.order[i] : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < PW; ++j) {
                const uint32_t w = wv + j * (kBlock / 64);
                if (w >= W) break;
                const uint64_t i = (uint64_t)w * 64 + lane;
                const bool valid = i < IN.ntrials;
                uint64_t mine = 0;
                for (uint32_t g = 0; g < IN.n; ++g) {
                    const uint64_t b = __ballot(valid && ((fm[j] >> g) & 1u));
                    if (lane == g) mine = b;
                }
                put(w, mine, __ballot(valid && oc[j] == 1), __ballot(valid && oc[j] == 2),
                    __ballot(valid));
            }
        } else {
            for (uint32_t w = wv; w < W; w += kBlock / 64) {
                uint64_t mine, ob, oo, vv;
                word_inputs(IN.n, IN.seed, IN.gs, IN.t0, IN.ntrials, IN.faulty, IN.order, w, lane,
                            mine, ob, oo, vv);
                put(w, mine, ob, oo, vv);
            }
        }
        __syncthreads();
        F = sIn;
        OBp = sIn + IN.n * W;
    }
    for (uint32_t idx = blockIdx.x * kBlock + threadIdx.x; idx < work; idx += grid_threads()) {
        if (idx < work0) {  // level 0, whole: commander -> lieutenant x (ba.py:263-277)
            const uint32_t p = fdiv(idx, divW), w = idx - p * W;
            uint64_t lie[2];
            lie_pair(seed, 0, p, gw0 + w, lie[0], lie[1]);
            const uint64_t f0 = F[w], ob = OBp[w];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t x = 2 * p + h;
                if (x < tp.L) scratch[tp.off[0] + (uint64_t)x * W + w] = (f0 & lie[h]) | (~f0 & ob);
            }
            continue;
        }
        if constexpr (K >= 1) {
            const uint32_t it = idx - work0;
            const uint32_t pl = fdiv(it, divW), w = it - pl * W;
            const uint64_t gw = gw0 + w;
            const uint32_t pairK = (tp.xbK >> 1) + pl;
            const uint32_t x0 = 2 * pairK, x1 = x0 + 1;
            const bool ok0 = x0 >= tp.xbK && x0 < tp.xeK, ok1 = x1 >= tp.xbK && x1 < tp.xeK;
            const uint32_t xa = ok0 ? x0 : x1;  // chain anchor: the first slot of the range
            const uint32_t par0 = fdiv(x0, tp.D[K - 1]), par1 = fdiv(x1, tp.D[K - 1]);
            const uint32_t para = ok0 ? par0 : par1;
            // level-K senders (loads issued before the chain's stores)
            const uint64_t fw0 = ok0 ? F[(uint64_t)sender[tp.snd_off[K - 1] + par0] * W + w] : 0ull;
            const uint64_t fw1 = ok1 ? F[(uint64_t)sender[tp.snd_off[K - 1] + par1] * W + w] : 0ull;
            const uint64_t ob = OBp[w];
            P4 xc{pairK, (uint32_t)K, (uint32_t)gw, (uint32_t)(gw >> 32)};
            const uint64_t va = top_chain<K, true>(tp, xa, w, W, gw, seed, F, ob, sender, scratch, xc);
            const uint64_t lieK0 = (uint64_t)xc.y << 32 | xc.x, lieK1 = (uint64_t)xc.w << 32 | xc.z;
            if (ok0) scratch[tp.off[K] + (uint64_t)(x0 - tp.base[K]) * W + w] = (fw0 & lieK0) | (~fw0 & va);
            if (ok1) {
                uint64_t v1 = va;
                if (par1 != para) {  // the pair straddles two parents (odd L-K only): second chain
                    P4 none{};
                    v1 = top_chain<K, false>(tp, x1, w, W, gw, seed, F, ob, sender, scratch, none);
                }
                scratch[tp.off[K] + (uint64_t)(x1 - tp.base[K]) * W + w] = (fw1 & lieK1) | (~fw1 & v1);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// inner majority level p (1 <= p < me): one thread per (slot, word).  Level p
// starts at global slot ybase, its child level at cbase (subtree ranges).
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(kBlock) void k_majority(uint32_t s, FastDiv divW, FastDiv divS,
                                                     uint32_t work, uint32_t ybase, uint32_t cbase,
                                                     const uint64_t* __restrict__ Lp,
                                                     const uint64_t* __restrict__ C,
                                                     uint64_t* __restrict__ Rp) {
    const uint32_t W = divW.d;
    const uint32_t thr = s / 2 + 1;  // strict majority; inner tie -> non-attack
    for (uint32_t idx = blockIdx.x * kBlock + threadIdx.x; idx < work; idx += grid_threads()) {
        const uint32_t yl = fdiv(idx, divW);
        const uint32_t w = idx - yl * W;
        const uint32_t y = ybase + yl;
        const uint32_t sr = fdiv(y, divS);
        const uint32_t b = y - sr * s;
        Count<P> cnt;
        cnt.add(Lp[(uint64_t)yl * W + w]);
        const uint64_t base = (uint64_t)sr * s;
        // children in chunks of kLoadChunk: every load of a chunk is in flight
        // before the first add (a load-add loop waits one HBM latency per child)
        for (uint32_t a0 = 0; a0 < s; a0 += kLoadChunk) {
            uint64_t v[kLoadChunk];
#pragma unroll
            for (uint32_t q = 0; q < kLoadChunk; ++q) {
                const uint32_t a = a0 + q;
                const uint64_t cs = (base + a) * (s - 1) + (b - (b > a)) - cbase;
                v[q] = (a < s && a != b) ? C[cs * W + w] : 0ull;
            }
#pragma unroll
            for (uint32_t q = 0; q < kLoadChunk; ++q) cnt.add(v[q]);  // absent children add 0
        }
        Rp[(uint64_t)yl * W + w] = cnt.ge(thr);
    }
}

// ---------------------------------------------------------------------------
// root majority + quorum epilogue: one wave per word
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(kBlock) void k_epilogue(uint32_t n, uint32_t me, uint64_t W,
                                                     uint64_t ntrials,
                                                     const uint64_t* __restrict__ scratch,
                                                     uint64_t offF, uint64_t offOB, uint64_t offOO,
                                                     uint64_t offVAL, uint64_t offL0,
                                                     const uint64_t* __restrict__ C1,
                                                     uint64_t* __restrict__ decisions,
                                                     uint8_t* __restrict__ outcome,
                                                     uint64_t* __restrict__ counters, Sink sk) {
    __shared__ uint64_t sA[kBlock / 64][kMaxN], sU[kBlock / 64][kMaxN], sF[kBlock / 64][kMaxN];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t L = n - 1;
    TrialCounts tc;
    const uint64_t words_per_grid = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t win = (W + (kBlock / 64) - 1) / (kBlock / 64) * (kBlock / 64);
    for (uint64_t w0 = (uint64_t)blockIdx.x * (kBlock / 64); w0 < win; w0 += words_per_grid) {
        const uint64_t w = w0 + wv;
        const bool wok = w < W;
        if (wok && lane < L) {  // root for lieutenant r = lane + 1 (bit-sliced)
            const uint32_t b = lane;
            Count<P> cnt;
            cnt.add(scratch[offL0 + (uint64_t)b * W + w]);
            if (me >= 1) {
                for (uint32_t a0 = 0; a0 < L; a0 += kLoadChunk) {  // loads in flight together
                    uint64_t v[kLoadChunk];
#pragma unroll
                    for (uint32_t q = 0; q < kLoadChunk; ++q) {
                        const uint32_t a = a0 + q;
                        const uint64_t cs = (uint64_t)a * (L - 1) + (b - (b > a));
                        v[q] = (a < L && a != b) ? C1[cs * W + w] : 0ull;
                    }
#pragma unroll
                    for (uint32_t q = 0; q < kLoadChunk; ++q) cnt.add(v[q]);
                }
            }
            const uint32_t c = me >= 1 ? L : 1u;  // OM(0): the direct value alone
            const uint64_t att = cnt.ge(c / 2 + 1);
            const uint64_t tie = (c & 1u) ? 0ull : (cnt.ge(c / 2) & ~att);
            sA[wv][lane] = att;
            sU[wv][lane] = tie;
        }
        if (wok && lane < n) sF[wv][lane] = scratch[offF + (uint64_t)lane * W + w];
        __syncthreads();
        if (wok) {
            const uint64_t i = w * 64 + lane;
            const uint64_t vv = scratch[offVAL + w];
            if ((vv >> lane) & 1ull) {
                uint32_t A = 0, U = 0, fm = 0;
                for (uint32_t b = 0; b < L; ++b) {
                    A |= (uint32_t)((sA[wv][b] >> lane) & 1ull) << (b + 1);
                    U |= (uint32_t)((sU[wv][b] >> lane) & 1ull) << (b + 1);
                }
                for (uint32_t g = 0; g < n; ++g) fm |= (uint32_t)((sF[wv][g] >> lane) & 1ull) << g;
                const uint32_t ob = (uint32_t)(scratch[offOB + w] >> lane) & 1u;
                const uint32_t oo = (uint32_t)(scratch[offOO + w] >> lane) & 1u;
                const uint32_t oc = oo ? 2u : ob;
                uint64_t dec;
                uint32_t out;
                finish_trial(n, me, fm, oc, A, U, dec, out, tc);
                if (decisions) decisions[i] = dec;
                if (outcome) outcome[i] = (uint8_t)out;
            }
        }
        __syncthreads();
    }
    block_counts_sink<kBlock>(tc, counters, sk);  // run counters: no k_reduce launch
}

// ---------------------------------------------------------------------------
// ba.py OM(1) in its canonical draw order (lie table), one thread per trial
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_table(uint32_t n, uint32_t relay, uint32_t me,
                                                  uint64_t seed, GenSpec gs, uint64_t first_trial,
                                                  uint64_t batch, const uint32_t* __restrict__ faulty,
                                                  const uint8_t* __restrict__ order,
                                                  const uint32_t* __restrict__ table,
                                                  uint32_t stride, const uint32_t* __restrict__ poll,
                                                  uint64_t* __restrict__ decisions,
                                                  uint8_t* __restrict__ outcome,
                                                  uint64_t* __restrict__ partial) {
    TrialCounts tc;
    const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < batch;
         i += (uint64_t)gridDim.x * kBlock) {
        uint32_t fm = gs.faulty_mode == 0 ? faulty[i] : 0;
        uint32_t oc = gs.order_mode == 0 ? order[i] : 0;
        gen_trial(n, seed, gs, first_trial + i, fm, oc);
        fm &= all;
        const uint32_t ob = oc == 1;
        const uint32_t* row = table + i * stride;
        // the coin stream: coin c is bit c & 31 of row[c >> 5].  take(k) = the next
        // k <= 31 coins as bits 0..k-1 (a word or two, not one load per coin)
        uint32_t c = 0;
        auto take = [&](uint32_t k) -> uint32_t {
            if (k == 0) return 0u;
            const uint32_t w = c >> 5, sh = c & 31u;
            uint32_t v = row[w] >> sh;
            if (sh + k > 32u) v |= row[w + 1] << (32u - sh);  // coins c..c+k-1 exist
            c += k;
            return v & ((1u << k) - 1u);
        };
        const uint32_t cf = fm & 1u, lts = all & ~1u;
        // ba.py:263-277: lieutenant r gets coin r-1 from a faulty commander
        const uint32_t V = cf ? take(n - 1) << 1 : (ob ? lts : 0u);
        const uint32_t pm = poll ? poll[i] & all & ~1u : 0u;
        // ba.py:159-195, receiver-major: receiver r counts V_r, the commander's
        // answer to a stale poll, then every other lieutenant j ascending -- a coin
        // from a faulty j, V_j from a loyal one.  Only the counts matter, so the
        // loyal relays are one popcount and the faulty ones the popcount of their
        // run of coins (the stream order is unchanged).
        const uint32_t nfl = __popc(fm & lts), loyalV = V & ~fm & lts;
        uint32_t A = 0, U = 0;
        for (uint32_t r = 1; r < n; ++r) {
            uint32_t a = (V >> r) & 1u, cnt = 1;
            if (relay) {
                if ((pm >> r) & 1u) {  // stale primary_port: the commander answers too
                    a += cf ? take(1) : ob;
                    ++cnt;
                }
                a += __popc(loyalV & ~(1u << r)) + __popc(take(nfl - ((fm >> r) & 1u)));
                cnt += n - 2;
            }
            if (2 * a > cnt) A |= 1u << r;
            else if (2 * a == cnt) U |= 1u << r;
        }
        uint64_t dec;
        uint32_t out;
        finish_trial(n, me, fm, oc, A, U, dec, out, tc);
        if (decisions) decisions[i] = dec;
        if (outcome) outcome[i] = (uint8_t)out;
    }
    block_counts_out<kBlock>(tc, partial);
}

// Sum the per-block counter rows: 64 row groups x 16 columns, then a fixed
// LDS tree over the groups (deterministic integer sums).
constexpr int kReduceThreads = 1024;
__global__ __launch_bounds__(kReduceThreads) void k_reduce(const uint64_t* __restrict__ partial,
                                                           int rows,
                                                           uint64_t* __restrict__ counters) {
    __shared__ uint64_t red[kReduceThreads];
    const int t = threadIdx.x, col = t & 15, grp = t >> 4;
    uint64_t s = 0;
#pragma unroll 8
    for (int r = grp; r < rows; r += kReduceThreads / 16) s += partial[(uint64_t)r * 16 + col];
    red[t] = s;
    __syncthreads();
    for (int stride = kReduceThreads / 2; stride >= 16; stride >>= 1) {
        if (t < stride) red[t] += red[t + stride];
        __syncthreads();
    }
    // atomic adds: two table-mode calls in flight on two ctx streams may share
    // one counter array, like the sink of the other engines
    if (t < 16)
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(counters) + t,
                               (unsigned long long)red[t], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static uint32_t blocks_for(uint64_t work, uint32_t cap) {
    uint64_t b = (work + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    return (uint32_t)(b < cap ? b : cap);
}

hipError_t launch_reduce(const uint64_t* partials, int rows, uint64_t* counters, hipStream_t s,
                         Prof* prof) {
    ProfScope ps(prof, "k_reduce", s);
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kReduceThreads), 0, s, partials, rows, counters);
    return hipGetLastError();
}

// Synthetic per-trial inputs to HBM (ba_gen_inputs_device): one thread per
// trial, the draws of gen_trial, so a GIVEN-mode run on them equals the run
// that draws them itself.
__global__ __launch_bounds__(kBlock) void k_gen_inputs(uint32_t n, uint64_t seed, GenSpec gs,
                                                        uint64_t first_trial, uint64_t batch,
                                                        uint32_t* __restrict__ faulty_out,
                                                        uint8_t* __restrict__ order_out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < batch;
         i += (uint64_t)gridDim.x * kBlock) {
        uint32_t fm = 0, oc = 0;
        gen_trial(n, seed, gs, first_trial + i, fm, oc);
        if (faulty_out) faulty_out[i] = fm;
        if (order_out) order_out[i] = (uint8_t)oc;
    }
}

hipError_t launch_gen_inputs(const RunArgs& a, uint32_t* faulty_out, uint8_t* order_out) {
    uint64_t blocks = (a.batch + kBlock - 1) / kBlock;
    if (blocks > 8ull * a.cu_count) blocks = 8ull * a.cu_count;
    if (blocks < 1) blocks = 1;
    ProfScope ps(a.prof, "k_gen_inputs", a.stream);
    hipLaunchKernelGGL(k_gen_inputs, dim3((uint32_t)blocks), dim3(kBlock), 0, a.stream, a.n, a.seed,
                       a.gen, a.first_trial, a.batch, faulty_out, order_out);
    return hipGetLastError();
}

hipError_t launch_table(const RunArgs& a, uint64_t* partials) {
    const uint32_t blocks = blocks_for(a.batch, kPartialRows);
    ProfScope ps(a.prof, "k_table", a.stream);
    hipLaunchKernelGGL(k_table, dim3(blocks), dim3(kBlock), 0, a.stream, a.n, (uint32_t)(a.m >= 1),
                       a.me, a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order, a.table,
                       a.table_stride, a.poll, a.decisions, a.outcome, partials);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_reduce(partials, (int)blocks, a.counters, a.stream, a.prof);
}

template <int P>
static void launch_majority_p(uint32_t s, uint32_t W, uint32_t work, uint32_t ybase,
                              uint32_t cbase, const uint64_t* Lp, const uint64_t* C, uint64_t* Rp,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_majority<P>, dim3(blocks_for(work, 16384)), dim3(kBlock), 0, st, s,
                       make_fastdiv(W), make_fastdiv(s), work, ybase, cbase, Lp, C, Rp);
}

template <int P>
static void launch_epilogue_p(uint32_t blocks, const RunArgs& a, uint64_t W, uint64_t nt,
                              const uint64_t* scratch, const LevelsLayout& lay, const uint64_t* C1,
                              uint64_t* dec, uint8_t* out, uint64_t* partials) {
    hipLaunchKernelGGL(k_epilogue<P>, dim3(blocks), dim3(kBlock), 0, a.stream, a.n, a.me, W, nt,
                       scratch, lay.F, lay.OB, lay.OO, lay.VAL, lay.Lk[0], C1, dec, out,
                       a.counters, a.sink);
    (void)partials;
}

hipError_t launch_levels_chunk(const RunArgs& a, const Geometry& g, const uint8_t* d_sender,
                               uint64_t* scratch, const LevelsLayout& lay, uint64_t trial0,
                               uint64_t ntrials, uint64_t* partials, const LevelsJob& job) {
    const uint64_t W = (ntrials + 63) / 64;
    const uint64_t gw0 = (a.first_trial + trial0) / 64;
    hipStream_t st = a.stream;
    // small batches: the inputs are bit-sliced inside k_relay_top (TopInputs)
    const bool no_fuse_in = getenv("BA_NO_INPUT_FUSION") && atoi(getenv("BA_NO_INPUT_FUSION")) != 0;
    TopInputs tin{};
    const bool given_in = a.gen.faulty_mode == 0 && a.gen.order_mode == 0;
    tin.fuse = (!no_fuse_in && a.n <= (uint32_t)kMaxN &&
                W <= (given_in ? kTopFuseGivenWords : kTopFuseWords)) ? 1u : 0u;
    tin.n = a.n;
    tin.seed = a.seed;
    tin.t0 = a.first_trial + trial0;
    tin.ntrials = ntrials;
    tin.gs = a.gen;
    tin.faulty = a.faulty ? a.faulty + trial0 : nullptr;
    tin.order = a.order ? a.order + trial0 : nullptr;
    tin.offOO = lay.OO;
    tin.offVAL = lay.VAL;
    hipError_t e = hipSuccess;
    if (!tin.fuse && given_in) {
        ProfScope ps(a.prof, "k_input", st);
        hipLaunchKernelGGL(k_input_given, dim3(blocks_for(W * 64 / kInGivenWPW, 4096)), dim3(kBlock), 0,
                           st, a.n, ntrials, a.faulty + trial0, a.order + trial0, scratch, W, lay.F,
                           lay.OB, lay.OO, lay.VAL);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (!tin.fuse) {
        ProfScope ps(a.prof, "k_input", st);
        hipLaunchKernelGGL(k_input, dim3(blocks_for(W * 64, 4096)), dim3(kBlock), 0, st, a.n, a.seed,
                           a.gen, a.first_trial + trial0, ntrials,
                           a.faulty ? a.faulty + trial0 : nullptr, a.order ? a.order + trial0 : nullptr,
                           scratch, W, lay.F, lay.OB, lay.OO, lay.VAL);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // where level k / majority p live: scratch, except the level-1 child
    // results (R_1, or L_1 at depth 1) that a subtree pass leaves in votes_out
    auto Lptr = [&](uint32_t k) -> uint64_t* {
        if (k == 1 && g.me == 1 && job.h == 1 && job.votes_out) return job.votes_out;
        return scratch + lay.Lk[k];
    };
    auto Rptr = [&](uint32_t p) -> uint64_t* {
        if (p == job.h && job.votes_out) return job.votes_out;
        return scratch + lay.Rp[p];
    };
    // relay, top-down (levels 0..me, or 0..me-2 when the two bottom levels
    // are fused into the leaf-block kernel and never materialised).  Level 0
    // is always whole; a root-only pass stops there.
    const uint32_t ktop = !job.tree ? job.h - 1 : (lay.leaf_fused ? g.me - 2 : g.me);
    // levels 0..kf in one k_relay_top launch; a materialised leaf level (no
    // leaf fusion) stays a k_relay launch, since a chain walk per leaf pair
    // would multiply the biggest level's draws.  BA_NO_TOP_RELAY=1: one
    // k_relay launch per level (A/B and parity tests).
    static const bool no_top = getenv("BA_NO_TOP_RELAY") && atoi(getenv("BA_NO_TOP_RELAY")) != 0;
    const uint32_t kf = (lay.leaf_fused || !job.tree || g.me == 0) ? ktop : g.me - 1;
    uint32_t k_first = 0;
    if (tin.fuse && (no_top || kf > (uint32_t)kTopMax)) {  // no k_relay_top: inputs on their own
        ProfScope ps(a.prof, "k_input", st);
        hipLaunchKernelGGL(k_input, dim3(blocks_for(W * 64, 4096)), dim3(kBlock), 0, st, a.n, a.seed,
                           a.gen, a.first_trial + trial0, ntrials, tin.faulty, tin.order, scratch, W,
                           lay.F, lay.OB, lay.OO, lay.VAL);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (!no_top && kf <= (uint32_t)kTopMax) {
        TopPlan tp{};
        tp.K = kf;
        tp.L = g.L;
        tp.np0 = (g.L + 1) / 2;
        tp.xbK = (uint32_t)lay.base[kf];
        tp.xeK = (uint32_t)(lay.base[kf] + lay.cnt[kf]);
        for (uint32_t k = 0; k <= kf; ++k) {
            tp.base[k] = (uint32_t)lay.base[k];
            tp.off[k] = lay.Lk[k];
            tp.snd_off[k] = k < g.me ? (uint32_t)g.sender_off[k] : 0u;
            uint64_t d = 1;
            for (uint32_t i = k + 1; i <= kf; ++i) d *= g.L - i;
            tp.D[k] = make_fastdiv((uint32_t)d);
        }
        const uint32_t npK = kf == 0 ? 0u : (tp.xeK + 1) / 2 - tp.xbK / 2;
        const uint32_t work = (uint32_t)((uint64_t)(tp.np0 + (tp.xeK > tp.xbK ? npK : 0u)) * W);
        ProfScope ps(a.prof, "k_relay_top", st);
        const dim3 grid(blocks_for(work, 16384)), blk(kBlock);
        const FastDiv dW = make_fastdiv((uint32_t)W);
        switch (kf) {
#define BA_TOP(KK)                                                                               \
    case KK:                                                                                     \
        hipLaunchKernelGGL(k_relay_top<KK>, grid, blk, 0, st, tp, dW, work, a.seed, gw0, d_sender, \
                           scratch, lay.F, lay.OB, tin);                                         \
        break;
            BA_TOP(0) BA_TOP(1) BA_TOP(2) BA_TOP(3) BA_TOP(4) BA_TOP(5) BA_TOP(6)
#undef BA_TOP
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        k_first = kf + 1;
    }
    for (uint32_t k = k_first; k <= ktop; ++k) {
        const uint32_t xbase = (uint32_t)lay.base[k], xcnt = (uint32_t)lay.cnt[k];
        if (xcnt == 0) continue;
        const uint32_t npair = (xbase + xcnt + 1) / 2 - xbase / 2;
        const uint32_t work = (uint32_t)((uint64_t)npair * W);
        const uint64_t* Lprev = k == 0 ? scratch + lay.OB : Lptr(k - 1);
        const uint32_t pbase = k == 0 ? 0u : (uint32_t)lay.base[k - 1];
        const uint8_t* snd = k == 0 ? nullptr : d_sender + g.sender_off[k - 1];
        ProfScope ps(a.prof, k == g.me ? "k_relay_leaf" : "k_relay_inner", st);
        hipLaunchKernelGGL(k_relay, dim3(blocks_for(work, 16384)), dim3(kBlock), 0, st, k, xbase,
                           xcnt, pbase, make_fastdiv((uint32_t)W), make_fastdiv(g.L - k), work,
                           a.seed, gw0, Lprev, Lptr(k), scratch + lay.F, snd);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // leaf-up (me >= 3): k_leaf also takes the majority of level me-2 from its
    // block's S column results, so R_{me-1} is never stored and the inner
    // majority launches start one level higher.  BA_NO_LEAF_UP=1: off (A/B).
    const bool no_up = getenv("BA_NO_LEAF_UP") && atoi(getenv("BA_NO_LEAF_UP")) != 0;
    // (a split's tree pass keeps its vote level: leaf-up only below it)
    const bool leaf_up = job.tree && lay.leaf_fused && g.me >= 3 && !no_up &&
                         g.me - 2 >= (job.votes_out ? job.h : 1u);
    if (job.tree && lay.leaf_fused) {  // L_{me-1} and L_me on the fly: R_{me-1} from L_{me-2}
        // leaf blocks = slots of level me-2; level 0 is stored whole, but its
        // subtree range is the first-hop lieutenants [jb, je) themselves
        const bool top = g.me == 2;
        const uint32_t srbase = top ? lay.jb : (uint32_t)lay.base[g.me - 2];
        const uint32_t srcnt = top ? lay.je - lay.jb : (uint32_t)lay.cnt[g.me - 2];
        e = launch_leaf(g, a.seed, gw0, (uint32_t)W, srbase, srcnt, (uint32_t)lay.base[g.me - 2],
                        Lptr(g.me - 2), d_sender, scratch + lay.F, a.members,
                        leaf_up ? Rptr(g.me - 2) : Rptr(g.me - 1), leaf_up, st, a.prof);
        if (e != hipSuccess) return e;
    }
    // inner majorities, bottom-up: levels me-1..1 (no leaf fusion), me-2..1
    // (k_leaf wrote R_{me-1}) or me-3..1 (k_leaf wrote R_{me-2}); a split's
    // tree pass stops at its vote level h, its root pass takes levels h-1..1
    // over the gathered votes
    const int pdeep = job.tree ? (int)g.me - (lay.leaf_fused ? (leaf_up ? 3 : 2) : 1) : (int)job.h - 1;
    const int plow = (job.tree && job.votes_out) ? (int)job.h : 1;
    // small batches: level 1 + roots + quorum in one k_tail launch (level 1 whole)
    const bool no_tail = getenv("BA_NO_TAIL") && atoi(getenv("BA_NO_TAIL")) != 0;
    const bool tail = !no_tail && job.root && plow == 1 && pdeep >= 1 && W <= kTailMaxWords &&
                      tail_supported(g) && lay.base[1] == 0 && lay.cnt[1] == g.S[1];
    for (int p = pdeep; p >= (tail ? 2 : plow); --p) {
        const uint32_t s = g.L - (uint32_t)p;
        const uint32_t work = (uint32_t)(lay.cnt[p] * W);
        const uint32_t ybase = (uint32_t)lay.base[p], cbase = (uint32_t)lay.base[p + 1];
        const uint64_t* C = (!job.tree && p + 1 == (int)job.h) ? job.votes_in
                            : (p + 1 == (int)g.me) ? Lptr(p + 1) : Rptr(p + 1);
        const uint64_t* Lp = Lptr(p);
        uint64_t* Rp = Rptr(p);
        ProfScope ps(a.prof, p + 1 == (int)g.me ? "k_majority_leaf" : "k_majority_inner", st);
        switch (planes_for(s)) {
            case 1: launch_majority_p<1>(s, (uint32_t)W, work, ybase, cbase, Lp, C, Rp, st); break;
            case 2: launch_majority_p<2>(s, (uint32_t)W, work, ybase, cbase, Lp, C, Rp, st); break;
            case 3: launch_majority_p<3>(s, (uint32_t)W, work, ybase, cbase, Lp, C, Rp, st); break;
            case 4: launch_majority_p<4>(s, (uint32_t)W, work, ybase, cbase, Lp, C, Rp, st); break;
            default: launch_majority_p<5>(s, (uint32_t)W, work, ybase, cbase, Lp, C, Rp, st); break;
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (!job.root) return hipSuccess;
    if (tail) {
        const uint64_t* C2 = (!job.tree && job.h == 2) ? job.votes_in
                             : (g.me == 2 ? Lptr(2) : Rptr(2));
        ProfScope ps(a.prof, "k_tail", st);
        return launch_tail(a, g, W, scratch, lay, Lptr(1), C2, (uint32_t)lay.base[2],
                           a.decisions ? a.decisions + trial0 : nullptr,
                           a.outcome ? a.outcome + trial0 : nullptr);
    }
    // root + quorum epilogue over L_0 and the level-1 child results
    const uint64_t* C1 = (job.votes_in && job.h == 1) ? job.votes_in
                         : (g.me >= 2 ? scratch + lay.Rp[1] : (g.me == 1 ? scratch + lay.Lk[1] : nullptr));
    const uint32_t blocks = blocks_for(W * 64, kPartialRows);
    uint64_t* dec = a.decisions ? a.decisions + trial0 : nullptr;
    uint8_t* out = a.outcome ? a.outcome + trial0 : nullptr;
    static const bool old_epi = getenv("BA_EPILOGUE_PER_TRIAL") && atoi(getenv("BA_EPILOGUE_PER_TRIAL")) != 0;
    const uint64_t groups = (W + 63) / 64;
    const bool no_epi_w = getenv("BA_NO_EPILOGUE_W") && atoi(getenv("BA_NO_EPILOGUE_W")) != 0;
    if (!old_epi && !no_epi_w && epilogue_w_supported(g) && groups >= 64) {  // ba_tail.hip
        ProfScope ps(a.prof, "k_epilogue", st);
        return launch_epilogue_w(a, g, W, scratch, lay, C1, dec, out);
    }
    if (!old_epi && g.n >= 4 && g.n <= 16 && g.me >= 1 && groups >= 64) {  // bit-sliced epilogue
        const uint32_t eb = (uint32_t)(groups < 4096 ? groups : 4096);
        const size_t lds = (size_t)(2 * g.L + 7 + g.n) * 64 * 8;
        ProfScope ps(a.prof, "k_epilogue", st);
        if (planes_for(g.n) <= 4)
            hipLaunchKernelGGL(k_epilogue_bs<4>, dim3(eb), dim3(kBlock), lds, st, a.n, a.me, W,
                               scratch, lay.F, lay.OB, lay.OO, lay.VAL, lay.Lk[0], C1, dec, out,
                               a.counters, a.sink);
        else
            hipLaunchKernelGGL(k_epilogue_bs<5>, dim3(eb), dim3(kBlock), lds, st, a.n, a.me, W,
                               scratch, lay.F, lay.OB, lay.OO, lay.VAL, lay.Lk[0], C1, dec, out,
                               a.counters, a.sink);
        return hipGetLastError();
    }
    { ProfScope ps(a.prof, "k_epilogue", st);
    switch (planes_for(g.L)) {
        case 1: launch_epilogue_p<1>(blocks, a, W, ntrials, scratch, lay, C1, dec, out, partials); break;
        case 2: launch_epilogue_p<2>(blocks, a, W, ntrials, scratch, lay, C1, dec, out, partials); break;
        case 3: launch_epilogue_p<3>(blocks, a, W, ntrials, scratch, lay, C1, dec, out, partials); break;
        case 4: launch_epilogue_p<4>(blocks, a, W, ntrials, scratch, lay, C1, dec, out, partials); break;
        default: launch_epilogue_p<5>(blocks, a, W, ntrials, scratch, lay, C1, dec, out, partials); break;
    } }
    return hipGetLastError();
}

}  // namespace ba
