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
