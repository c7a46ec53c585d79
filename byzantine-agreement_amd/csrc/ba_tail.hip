// ba_tail.hip -- LEVELS small-batch tail (gfx950): the level-1 majorities, the
// root majorities and the quorum epilogue of one 64-trial word per block, in
// ONE launch instead of a k_majority launch plus k_epilogue.  Config 5's
// batches (n=16, m=5, 1..1024 instances = 1..16 words) are latency-bound: each
// launch costs a few us even when its work is tiny, and the per-trial epilogue
// (trial_result in one wave per word) is a long serial instruction stream.
// Here the epilogue is the WAVE engines' byte-sliced one (ba_wave.hpp,
// wave_epilogue: the quorum and IC flags of 8 trials per lane, then lane =
// trial extraction), compiled for N generals and the runtime depth me.
//
// Per word w (block):
//   1. R_1[y] for every level-1 slot y (L(L-1) of them; s = L-1 inputs: L_1[y]
//      and the level-2 results about y's receiver from y's other children),
//      every global load of a thread issued before its first add -> LDS
//   2. lanes b < L: the root of lieutenant b+1 = strict majority of L_0[b] and
//      the level-1 results about b (tie -> undefined, ba.py:188-195) -> LDS
//   3. wave 0: wave_epilogue over the word's input planes and root planes
// Bit-identical to k_majority + k_epilogue (same majorities, trial_result
// restated bit-sliced; GPU parity tests).
#include "ba_wave.hpp"

namespace ba {

constexpr int kTailBlock = 256;
constexpr int kTailMinN = 4, kTailMaxN = 16;

template <int N>
__global__ __launch_bounds__(kTailBlock) void k_tail(uint32_t me, uint64_t W,
                                                     const uint64_t* __restrict__ scratch,
                                                     uint64_t offF, uint64_t offOB, uint64_t offOO,
                                                     uint64_t offVAL, uint64_t offL0,
                                                     const uint64_t* __restrict__ L1,
                                                     const uint64_t* __restrict__ C2,
                                                     uint32_t c2base,
                                                     uint64_t* __restrict__ decisions,
                                                     uint8_t* __restrict__ outcome,
                                                     uint64_t* __restrict__ counters, Sink sk) {
    constexpr int L = N - 1, s = L - 1, S1 = L * s, NIN = N + 3, P = planes_c(L);
    __shared__ uint64_t sR1[S1];
    __shared__ uint64_t sIn[NIN];    // F[0..N) OB OO VAL (wave_epilogue's input planes)
    __shared__ uint64_t sAU[2 * L];  // A[0..L) U[0..L)
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    TrialCounts tc;
    for (uint64_t w = blockIdx.x; w < W; w += gridDim.x) {
        // 1. input planes; R_1 of every level-1 slot
        if (tid < (uint32_t)NIN) {
            const uint64_t o = tid < (uint32_t)N ? offF + (uint64_t)tid * W
                               : (tid == N ? offOB : (tid == N + 1 ? offOO : offVAL));
            sIn[tid] = scratch[o + w];
        }
        for (uint32_t y = tid; y < (uint32_t)S1; y += kTailBlock) {
            const uint32_t sr = y / s, b = y - sr * s;
            uint64_t v[s];
            v[0] = L1[(uint64_t)y * W + w];
#pragma unroll
            for (int a = 0; a + 1 < s; ++a) {
                const uint32_t aa = a + ((uint32_t)a >= b ? 1u : 0u);  // the a-th child != b
                const uint64_t cs = ((uint64_t)sr * s + aa) * (s - 1) + (b - (b > aa ? 1u : 0u)) - c2base;
                v[a + 1] = C2[cs * W + w];
            }
            Count<P> c;
#pragma unroll
            for (int a = 0; a < s; ++a) c.add(v[a]);
            sR1[y] = c.ge(s / 2 + 1);  // strict majority; inner tie -> non-attack
        }
        const uint64_t l0 = tid < (uint32_t)L ? scratch[offL0 + (uint64_t)tid * W + w] : 0ull;
        __syncthreads();
        // 2. roots
        if (tid < (uint32_t)L) {
            const uint32_t b = tid;
            Count<P> c;
            c.add(l0);
#pragma unroll
            for (int a = 0; a < L; ++a)
                if ((uint32_t)a != b) c.add(sR1[a * (L - 1) + (b - (b > (uint32_t)a ? 1u : 0u))]);
            const uint64_t att = c.ge(L / 2 + 1);
            sAU[b] = att;
            sAU[L + b] = (L & 1) ? 0ull : (c.ge(L / 2) & ~att);
        }
        __syncthreads();
        // 3. quorum epilogue (wave 0)
        if (tid < 64)
            wave_epilogue<N, 1, 0, 0>(sIn, sAU, lane, w, W * 64, decisions, outcome, tc, me);
        __syncthreads();
    }
    block_counts_sink<kTailBlock>(tc, counters, sk);
}

// ---------------------------------------------------------------------------
// Big-batch root + quorum epilogue (>= 64 groups of 64 words, 4 <= n <= 16):
// k_epilogue_w<N>, the successor of k_epilogue_bs.  A block of 4 waves owns a
// group of 64 words:
//   1. thread (wave v, lane = word) counts the roots of receivers b = v, v+4,
//      ... of its word -- L_0[b] and the level-1 votes about b -- with EVERY
//      load of all its receivers issued before the first add (compile-time N:
//      one memory round trip, where k_epilogue_bs waited one per chunk of 8
//      per receiver), and loads the word's input planes g = v, v+4, ... in the
//      same round trip; roots and planes go to LDS word-major
//   2. wave v runs wave_epilogue over its 16 words: the quorum and IC flags of
//      8 trials per lane (byte-sliced, all 64 lanes busy), then lane = trial
//      extraction and the stores
// k_epilogue_bs had wave 0 alone run the bit-sliced quorum (lane = word) while
// the other three waves waited at the barrier.
// ---------------------------------------------------------------------------
constexpr int kEpiBlock = 256;
constexpr int kEpiMinN = 4, kEpiMaxN = 16;

template <int N>
__global__ __launch_bounds__(kEpiBlock) void k_epilogue_w(uint32_t me, uint64_t W,
                                                          const uint64_t* __restrict__ scratch,
                                                          uint64_t offF, uint64_t offOB,
                                                          uint64_t offOO, uint64_t offVAL,
                                                          uint64_t offL0,
                                                          const uint64_t* __restrict__ C1,
                                                          uint64_t* __restrict__ decisions,
                                                          uint8_t* __restrict__ outcome,
                                                          uint64_t* __restrict__ counters, Sink sk) {
    constexpr int L = N - 1, NIN = N + 3, P = planes_c(L), NWV = kEpiBlock / 64;
    constexpr int KB = (L + NWV - 1) / NWV;      // receivers per thread
    constexpr int KG = (NIN + NWV - 1) / NWV;    // input planes per thread
    __shared__ uint64_t rec[64 * NIN];           // [word][F[0..N) OB OO VAL]
    __shared__ uint64_t au[64 * 2 * L];          // [word][A[0..L) U[0..L)]
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    TrialCounts tc;
    const uint64_t groups = (W + 63) / 64;
    for (uint64_t gi = blockIdx.x; gi < groups; gi += gridDim.x) {
        const uint64_t w = gi * 64 + lane;
        const bool wok = w < W;
        // 1. every load of this thread in flight at once
        uint64_t v[KB][L], pl[KG];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const uint32_t b = wv + (uint32_t)k * NWV;
#pragma unroll
            for (int a = 0; a < L; ++a) {
                const uint64_t cs = (uint64_t)a * (L - 1) + (b - (b > (uint32_t)a ? 1u : 0u));
                const bool ok = wok && b < (uint32_t)L;
                v[k][a] = !ok ? 0ull
                              : ((uint32_t)a == b ? scratch[offL0 + (uint64_t)b * W + w] : C1[cs * W + w]);
            }
        }
#pragma unroll
        for (int k = 0; k < KG; ++k) {
            const uint32_t g = wv + (uint32_t)k * NWV;
            const uint64_t o = g < (uint32_t)N ? offF + (uint64_t)g * W
                               : (g == N ? offOB : (g == N + 1 ? offOO : offVAL));
            pl[k] = (wok && g < (uint32_t)NIN) ? scratch[o + w] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const uint32_t b = wv + (uint32_t)k * NWV;
            if (b < (uint32_t)L) {
                Csa<P> c;
                static_for<0, L>([&](auto a) { c.template add<a()>(v[k][a()]); });
                const uint64_t att = c.template ge<L, L / 2 + 1>();  // strict majority
                au[lane * 2 * L + b] = att;
                // root tie (even L): undefined
                au[lane * 2 * L + L + b] = (L % 2 == 0) ? (c.template ge<L, L / 2>() & ~att) : 0ull;
            }
        }
#pragma unroll
        for (int k = 0; k < KG; ++k) {
            const uint32_t g = wv + (uint32_t)k * NWV;
            if (g < (uint32_t)NIN) rec[lane * NIN + g] = pl[k];  // VAL = 0 past the batch
        }
        __syncthreads();
        // 2. quorum + extraction, 16 words per wave
        wave_epilogue<N, 64 / NWV, 0, 0>(rec + wv * (64 / NWV) * NIN, au + wv * (64 / NWV) * 2 * L,
                                         lane, gi * 64 + wv * (64 / NWV), W * 64, decisions,
                                         outcome, tc, me);
        __syncthreads();
    }
    block_counts_sink<kEpiBlock>(tc, counters, sk);
}

bool epilogue_w_supported(const Geometry& g) {
    return g.me >= 1 && g.n >= (uint32_t)kEpiMinN && g.n <= (uint32_t)kEpiMaxN;
}

hipError_t launch_epilogue_w(const RunArgs& a, const Geometry& g, uint64_t W,
                             const uint64_t* scratch, const LevelsLayout& lay, const uint64_t* C1,
                             uint64_t* decisions, uint8_t* outcome) {
    if (!epilogue_w_supported(g) || W == 0) return hipErrorInvalidValue;
    const uint64_t groups = (W + 63) / 64;
    const uint32_t eb = (uint32_t)(groups < 4096 ? groups : 4096);
    switch (g.n) {
#define BA_EPI(NN)                                                                                 \
    case NN:                                                                                       \
        hipLaunchKernelGGL(k_epilogue_w<NN>, dim3(eb), dim3(kEpiBlock), 0, a.stream, a.me, W,     \
                           scratch, lay.F, lay.OB, lay.OO, lay.VAL, lay.Lk[0], C1, decisions,     \
                           outcome, a.counters, a.sink);                                          \
        break;
        BA_EPI(4) BA_EPI(5) BA_EPI(6) BA_EPI(7) BA_EPI(8) BA_EPI(9) BA_EPI(10) BA_EPI(11)
        BA_EPI(12) BA_EPI(13) BA_EPI(14) BA_EPI(15) BA_EPI(16)
#undef BA_EPI
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

bool tail_supported(const Geometry& g) {
    return g.me >= 2 && g.n >= (uint32_t)kTailMinN && g.n <= (uint32_t)kTailMaxN;
}

template <int N>
static void launch_tail_n(const RunArgs& a, uint64_t W, const uint64_t* scratch,
                          const LevelsLayout& lay, const uint64_t* L1, const uint64_t* C2,
                          uint32_t c2base, uint64_t* dec, uint8_t* out) {
    hipLaunchKernelGGL(k_tail<N>, dim3((uint32_t)W), dim3(kTailBlock), 0, a.stream, a.me, W,
                       scratch, lay.F, lay.OB, lay.OO, lay.VAL, lay.Lk[0], L1, C2, c2base, dec, out,
                       a.counters, a.sink);
}

hipError_t launch_tail(const RunArgs& a, const Geometry& g, uint64_t W, const uint64_t* scratch,
                       const LevelsLayout& lay, const uint64_t* L1, const uint64_t* C2,
                       uint32_t c2base, uint64_t* decisions, uint8_t* outcome) {
    if (!tail_supported(g) || W == 0 || W > kTailMaxWords) return hipErrorInvalidValue;
    switch (g.n) {
#define BA_TAIL(NN) \
    case NN: launch_tail_n<NN>(a, W, scratch, lay, L1, C2, c2base, decisions, outcome); break;
        BA_TAIL(4) BA_TAIL(5) BA_TAIL(6) BA_TAIL(7) BA_TAIL(8) BA_TAIL(9) BA_TAIL(10) BA_TAIL(11)
        BA_TAIL(12) BA_TAIL(13) BA_TAIL(14) BA_TAIL(15) BA_TAIL(16)
#undef BA_TAIL
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace ba
