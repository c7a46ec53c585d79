// ba_device.hpp -- device building blocks shared by the OM(m) engines (gfx950).
//
// Data model: one 64-bit word holds one tree slot for 64 consecutive trials
// (bit b = trial 64*w + b), the natural product of a wave64 __ballot.  Relay
// is a per-word bit-select, majorities are bit-sliced counters over words, and
// a single Philox4x32-10 call yields the lie bits of two slots x 64 trials.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "ba_philox_asm.hpp"

namespace ba {

constexpr int kMaxN = 32;
constexpr uint32_t kGenTag = 0xFFFFFFFFu;  // Philox ctr word 1 of synthetic-input draws

// ---------------------------------------------------------------------------
// 3-input bitwise ops: one v_bitop3_b32 per 32-bit half on gfx950 (the
// truth-table immediate names the function of inputs 0xF0, 0xCC, 0xAA).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}
__host__ __device__ __forceinline__ uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) {
    return (uint64_t)xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32 |
           xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
__host__ __device__ __forceinline__ uint32_t maj3_32(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
    return (a & b) | (a & c) | (b & c);
#endif
}
__host__ __device__ __forceinline__ uint64_t maj3(uint64_t a, uint64_t b, uint64_t c) {
    return (uint64_t)maj3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32 |
           maj3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return xor3_32(a, b, c); }
__host__ __device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return maj3_32(a, b, c); }

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Each round is 2 x v_mad_u64_u32 +
// 2 x xor3 (tools/philox_bench: 9.5e11 calls/s on one MI355X vs 7.8e11 with
// 2-input xors).  The key is kernel-uniform.  Groups of 2-4 interleaved calls
// (philox10_n) take the round keys AND the two multipliers as VGPR operands
// (KeysV: a VALU op with an SGPR operand issues slower; VGPR
// multipliers +2.4% calls/s in tools/philox_bench), rounds 0-1 in C and rounds
// 2-9 as one generated asm statement (ba_philox_asm.hpp).  A single call
// (philox10, G = 1) is the round loop with its products pinned to
// v_mad_u64_u32 from round 2.  Same results on every path.
// ---------------------------------------------------------------------------
struct P4 {
    uint32_t x, y, z, w;
};

// Compile-time loop usable from host and device code (ba_leaf.hpp's static_for
// is device-only): f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, typename F>
__host__ __device__ __forceinline__ void static_for_h(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for_h<B + 1, E>(f);
    }
}

// The two 32x32 -> 64-bit products of Philox round I.  From round 2 on each
// is pinned to one v_mad_u64_u32 (inline asm).  Left alone, the compiler splits ~40 of a WAVE round's
// products into v_mul_hi_u32 + v_mul_lo_u32 pairs; pinned, the n=10 WAVE
// kernel runs ~3% faster (tools/om3_lab.hip A/B, same outputs).  Rounds 0-1
// stay plain C so the compiler can still share and strength-reduce the
// products common to a lane's calls (same level and word).
template <int I>
__host__ __device__ __forceinline__ void philox_mul2(uint32_t x, uint32_t z, uint64_t& p0,
                                                     uint64_t& p1) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (I >= 2) {
        // Both products in one asm statement: the hazard recognizer puts one
        // conservative s_nop after every inline-asm VALU def (it cannot see that
        // a v_mad_u64_u32 is neither a trans op nor an op_sel/SDWA write), so a
        // pair per statement halves them.  p0 is early-clobber: it is written
        // before z is read.
        uint64_t cc;
        asm("v_mad_u64_u32 %0, %2, %3, %5, 0\n\tv_mad_u64_u32 %1, %2, %4, %6, 0"
            : "=&v"(p0), "=v"(p1), "=&s"(cc)
            : "v"(x), "v"(z), "s"(0xD2511F53u), "s"(0xCD9E8D57u));
        return;
    }
#endif
    p0 = (uint64_t)0xD2511F53u * x;
    p1 = (uint64_t)0xCD9E8D57u * z;
}

// Both products of round I for G interleaved calls (philox10_n).  From round 2
// on, G = 2..4 calls' 2G products go into ONE asm statement: the hazard
// recognizer treats every inline-asm def as a possible dst-forwarding hazard
// and puts an s_nop between an asm and the next instruction that reads or
// writes any of its defs -- including the next asm's carry-out SGPR -- so one
// statement per group instead of one per call removes most of those nops.
template <int I, int G>
__host__ __device__ __forceinline__ void philox_mul2_n(const P4 (&c)[G], uint64_t (&p0)[G],
                                                       uint64_t (&p1)[G]) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (I >= 2 && G >= 2 && G <= 4) {
        uint64_t cc;
        constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
        if constexpr (G == 2)
            asm("v_mad_u64_u32 %0, %4, %5, %9, 0\n\tv_mad_u64_u32 %1, %4, %6, %10, 0\n\t"
                "v_mad_u64_u32 %2, %4, %7, %9, 0\n\tv_mad_u64_u32 %3, %4, %8, %10, 0"
                : "=&v"(p0[0]), "=&v"(p1[0]), "=&v"(p0[1]), "=&v"(p1[1]), "=&s"(cc)
                : "v"(c[0].x), "v"(c[0].z), "v"(c[1].x), "v"(c[1].z), "s"(M0), "s"(M1));
        else if constexpr (G == 3)
            asm("v_mad_u64_u32 %0, %6, %7, %13, 0\n\tv_mad_u64_u32 %1, %6, %8, %14, 0\n\t"
                "v_mad_u64_u32 %2, %6, %9, %13, 0\n\tv_mad_u64_u32 %3, %6, %10, %14, 0\n\t"
                "v_mad_u64_u32 %4, %6, %11, %13, 0\n\tv_mad_u64_u32 %5, %6, %12, %14, 0"
                : "=&v"(p0[0]), "=&v"(p1[0]), "=&v"(p0[1]), "=&v"(p1[1]), "=&v"(p0[2]),
                  "=&v"(p1[2]), "=&s"(cc)
                : "v"(c[0].x), "v"(c[0].z), "v"(c[1].x), "v"(c[1].z), "v"(c[2].x), "v"(c[2].z),
                  "s"(M0), "s"(M1));
        else
            asm("v_mad_u64_u32 %0, %8, %9, %17, 0\n\tv_mad_u64_u32 %1, %8, %10, %18, 0\n\t"
                "v_mad_u64_u32 %2, %8, %11, %17, 0\n\tv_mad_u64_u32 %3, %8, %12, %18, 0\n\t"
                "v_mad_u64_u32 %4, %8, %13, %17, 0\n\tv_mad_u64_u32 %5, %8, %14, %18, 0\n\t"
                "v_mad_u64_u32 %6, %8, %15, %17, 0\n\tv_mad_u64_u32 %7, %8, %16, %18, 0"
                : "=&v"(p0[0]), "=&v"(p1[0]), "=&v"(p0[1]), "=&v"(p1[1]), "=&v"(p0[2]),
                  "=&v"(p1[2]), "=&v"(p0[3]), "=&v"(p1[3]), "=&s"(cc)
                : "v"(c[0].x), "v"(c[0].z), "v"(c[1].x), "v"(c[1].z), "v"(c[2].x), "v"(c[2].z),
                  "v"(c[3].x), "v"(c[3].z), "s"(M0), "s"(M1));
        return;
    }
#endif
#pragma unroll
    for (int g = 0; g < G; ++g) philox_mul2<I>(c[g].x, c[g].z, p0[g], p1[g]);
}

__host__ __device__ __forceinline__ P4 philox10(P4 c, uint32_t k0, uint32_t k1) {
    static_for_h<0, 10>([&](auto i) {
        uint64_t p0, p1;
        philox_mul2<i()>(c.x, c.z, p0, p1);
        P4 n;
        n.x = xor3_32((uint32_t)(p1 >> 32), c.y, k0);
        n.y = (uint32_t)p1;
        n.z = xor3_32((uint32_t)(p0 >> 32), c.w, k1);
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    });
    return c;
}

// G independent Philox4x32-10 calls advanced round by round in lockstep: the
// source order interleaves the chains, so each v_mad_u64_u32 result is used G
// instructions later instead of right away (left to itself the scheduler runs
// the calls one after another and exposes the multiply latency).
// The key schedule of one seed in VGPRs (kv0[i], kv1[i] = round i's keys): a
// VALU op with an SGPR operand issues slower than one with VGPR operands only
// (tools/valu_cost operands: v_bitop3 xor3 4.5 vs 2.7 cycles per wave64
// instruction at 8 waves/SIMD), and every Philox xor3 takes one key.  The empty
// asm keeps the (uniform) values in VGPRs.
struct KeysV {
    uint32_t k0[10], k1[10];
    uint32_t m0, m1;  // the multipliers as VGPR operands too
    __device__ __forceinline__ explicit KeysV(uint64_t seed)
        : KeysV((uint32_t)seed, (uint32_t)(seed >> 32)) {}
    // the asm is not volatile: a pure function of the seed, so the compiler can
    // hoist it out of the loops and share it between call sites
    __device__ __forceinline__ KeysV(uint32_t a, uint32_t b) {
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            k0[i] = a + (uint32_t)i * 0x9E3779B9u;
            k1[i] = b + (uint32_t)i * 0xBB67AE85u;
            asm("" : "+v"(k0[i]), "+v"(k1[i]));
        }
        m0 = 0xD2511F53u;
        m1 = 0xCD9E8D57u;
        asm("" : "+v"(m0), "+v"(m1));
    }
};

// philox10_n with the round keys as VGPR operands (KeysV); same results.
template <int G>
__device__ __forceinline__ void philox10_n_vk(P4 (&c)[G], const KeysV& kv) {
    static_for_h<0, 2>([&](auto i) {
        uint64_t p0[G], p1[G];
        philox_mul2_n<i(), G>(c, p0, p1);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            P4 n;
            n.x = xor3_32((uint32_t)(p1[g] >> 32), c[g].y, kv.k0[i()]);
            n.y = (uint32_t)p1[g];
            n.z = xor3_32((uint32_t)(p0[g] >> 32), c[g].w, kv.k1[i()]);
            n.w = (uint32_t)p0[g];
            c[g] = n;
        }
    });
    if constexpr (G >= 2 && G <= 5) {
        uint32_t rk0[8], rk1[8], x[G], y[G], z[G], w[G];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            rk0[i] = kv.k0[i + 2];
            rk1[i] = kv.k1[i + 2];
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            x[g] = c[g].x;
            y[g] = c[g].y;
            z[g] = c[g].z;
            w[g] = c[g].w;
        }
        philox_r29_asm_vkm<G>(x, y, z, w, rk0, rk1, kv.m0, kv.m1);
#pragma unroll
        for (int g = 0; g < G; ++g) c[g] = P4{x[g], y[g], z[g], w[g]};
    } else {
        static_for_h<2, 10>([&](auto i) {
            uint64_t p0[G], p1[G];
            philox_mul2_n<i(), G>(c, p0, p1);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                P4 n;
                n.x = xor3_32((uint32_t)(p1[g] >> 32), c[g].y, kv.k0[i()]);
                n.y = (uint32_t)p1[g];
                n.z = xor3_32((uint32_t)(p0[g] >> 32), c[g].w, kv.k1[i()]);
                n.w = (uint32_t)p0[g];
                c[g] = n;
            }
        });
    }
}

template <int G>
__host__ __device__ __forceinline__ void philox10_n(P4 (&c)[G], uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
    // round keys as VGPR operands (KeysV, hoisted by the compiler): Philox calls
    // 8.4e11 -> 9.6e11 per second at 2 waves/SIMD (tools/philox_bench)
    if constexpr (G >= 2 && G <= 5) {
        philox10_n_vk<G>(c, KeysV(k0, k1));
        return;
    }
#endif
    static_for_h<0, 10>([&](auto i) {
        uint64_t p0[G], p1[G];
        philox_mul2_n<i(), G>(c, p0, p1);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            P4 n;
            n.x = xor3_32((uint32_t)(p1[g] >> 32), c[g].y, k0);
            n.y = (uint32_t)p1[g];
            n.z = xor3_32((uint32_t)(p0[g] >> 32), c[g].w, k1);
            n.w = (uint32_t)p0[g];
            c[g] = n;
        }
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    });
}

// G calls as consecutive groups of at most 4 interleaved calls (sizes as even as
// possible: 7 -> 4 + 3), so no more than four calls' state is live at once.
template <int G, int B = 0>
__host__ __device__ __forceinline__ void philox_groups(P4 (&c)[G], uint32_t k0, uint32_t k1) {
    if constexpr (B < G) {
        constexpr int left = G - B, ngrp = (left + 3) / 4, g = (left + ngrp - 1) / ngrp;
        P4 sub[g];
        static_for_h<0, g>([&](auto i) { sub[i()] = c[B + i()]; });
        philox10_n<g>(sub, k0, k1);
        static_for_h<0, g>([&](auto i) { c[B + i()] = sub[i()]; });
        philox_groups<G, B + g>(c, k0, k1);
    }
}

// Lie words of slots 2*pair and 2*pair+1 at level k for global trial word gw.
__device__ __forceinline__ void lie_pair(uint64_t seed, uint32_t k, uint32_t pair, uint64_t gw,
                                         uint64_t& lie0, uint64_t& lie1) {
    P4 o = philox10(P4{pair, k, (uint32_t)gw, (uint32_t)(gw >> 32)}, (uint32_t)seed,
                    (uint32_t)(seed >> 32));
    lie0 = (uint64_t)o.y << 32 | o.x;
    lie1 = (uint64_t)o.w << 32 | o.z;
}

// G consecutive slot pairs pair0 .. pair0+G-1 of level k, word gw, interleaved;
// lie[2q], lie[2q+1] = the two slot-words of pair pair0+q.
template <int G>
__device__ __forceinline__ void lie_pairs(uint64_t seed, uint32_t k, uint32_t pair0, uint64_t gw,
                                          uint64_t (&lie)[2 * G]) {
    P4 c[G];
#pragma unroll
    for (int g = 0; g < G; ++g) c[g] = P4{pair0 + (uint32_t)g, k, (uint32_t)gw, (uint32_t)(gw >> 32)};
    philox10_n<G>(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int g = 0; g < G; ++g) {
        lie[2 * g] = (uint64_t)c[g].y << 32 | c[g].x;
        lie[2 * g + 1] = (uint64_t)c[g].w << 32 | c[g].z;
    }
}

__device__ __forceinline__ uint32_t mulhi_range(uint32_t u, uint32_t range) {
    return (uint32_t)(((uint64_t)u * range) >> 32);
}

// ---------------------------------------------------------------------------
// Fast unsigned division by a launch-uniform divisor (Granlund-Montgomery).
// ---------------------------------------------------------------------------
struct FastDiv {
    uint32_t d, mul, shift;  // shift == 0xFFFFFFFF encodes d == 1
};

__host__ inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0, 0};
    if (d <= 1) {  // d == 0 never divides: callers skip empty levels
        f.shift = 0xFFFFFFFFu;
        return f;
    }
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    f.shift = l - 1;
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    if (f.shift == 0xFFFFFFFFu) return n;
    const uint32_t t = __umulhi(n, f.mul);
    return (t + ((n - t) >> 1)) >> f.shift;
}

// ---------------------------------------------------------------------------
// Bit-sliced counters over 64-trial words.  P planes count up to 2^P - 1.
// ---------------------------------------------------------------------------
template <int P>
struct Count {
    uint64_t c[P];
    __device__ __forceinline__ Count() {
#pragma unroll
        for (int i = 0; i < P; ++i) c[i] = 0;
    }
    __device__ __forceinline__ void add(uint64_t x) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const uint64_t t = c[i] & x;
            c[i] ^= x;
            x = t;
        }
    }
    // lanes whose count >= T (T uniform)
    __device__ __forceinline__ uint64_t ge(uint32_t T) const {
        if (T == 0) return ~0ull;
        if (T >= (1u << P)) return 0ull;
        uint64_t gt = 0, eq = ~0ull;
#pragma unroll
        for (int i = P - 1; i >= 0; --i) {
            if ((T >> i) & 1u) {
                eq &= c[i];
            } else {
                gt |= eq & c[i];
                eq &= ~c[i];
            }
        }
        return gt | eq;
    }
};

// ---------------------------------------------------------------------------
// Carry-save column counter for inputs added in a COMPILE-TIME order (the
// leaf blocks and fixed-fan-in majorities).  Level l holds an accumulated bit
// and at most one pending bit; the third bit of a level triggers one full adder
// (xor3 + maj3: two v_bitop3 per 32-bit half) whose carry moves up a level.
// Per input that is ~2 bitop3 per half, against 2 x planes ops for the ripple
// Count<P>::add.  Which levels are occupied after K inputs is a function of K
// alone, so every branch below is resolved at compile time.
// ---------------------------------------------------------------------------
template <int NL, typename T = uint64_t>
struct Csa {
    T acc[NL], pend[NL];

    // push the (N+1)-th event into level L
    template <int L, int N>
    __host__ __device__ __forceinline__ void push(T e) {
        static_assert(L < NL, "Csa: too few levels for this many inputs");
        if constexpr (N == 0) {
            acc[L] = e;
        } else if constexpr (N % 2 == 1) {
            pend[L] = e;
        } else {
            const T a = acc[L], p = pend[L];
            acc[L] = xor3(a, p, e);
            push<L + 1, (N - 2) / 2>(maj3(a, p, e));
        }
    }
    // add the (K+1)-th input
    template <int K>
    __host__ __device__ __forceinline__ void add(T x) {
        push<0, K>(x);
    }
    // binary digits r[0..NL) of the count after N events at level L (+ carry in)
    template <int L, int N, bool CIN>
    __host__ __device__ __forceinline__ void resolve(T (&r)[NL], T cin) const {
        if constexpr (L < NL) {
            constexpr bool hasA = N >= 1, hasP = N >= 2 && N % 2 == 0;
            constexpr int up = N >= 1 ? (N - 1) / 2 : 0;  // events level L passed up
            constexpr int terms = (int)hasA + (int)hasP + (int)CIN;
            if constexpr (terms == 0) {
                r[L] = 0;
                resolve<L + 1, up, false>(r, 0);
            } else if constexpr (terms == 1) {
                r[L] = hasA ? acc[L] : (hasP ? pend[L] : cin);
                resolve<L + 1, up, false>(r, 0);
            } else if constexpr (terms == 2) {
                const T x = hasA ? acc[L] : pend[L];
                const T y = CIN ? cin : pend[L];
                r[L] = x ^ y;
                resolve<L + 1, up, true>(r, x & y);
            } else {
                r[L] = xor3(acc[L], pend[L], cin);
                resolve<L + 1, up, true>(r, maj3(acc[L], pend[L], cin));
            }
        }
    }
    // Largest count the events from level L up can still represent (N events
    // pushed into level L), in units of 2^L.
    static constexpr int max_units(int L, int N) {
        if (L >= NL || N <= 0) return 0;
        const int nb = (N >= 1 ? 1 : 0) + (N >= 2 && N % 2 == 0 ? 1 : 0);
        return nb + 2 * max_units(L + 1, N >= 1 ? (N - 1) / 2 : 0);
    }
    // Lanes whose count from level L up (units of 2^L) is >= TH, straight from
    // the level bits (acc, pend) without resolving the binary sum: one level's
    // one or two bits decide between two neighbouring thresholds of the levels
    // above, G(t) and G(t + 1) with G(t) >= G(t + 1), so each step is
    // G(t+1) | (c & G(t)): about one 3-input op per level (majority of 9 from
    // the carry-save state: 3 ops per 32-bit half, where the ripple resolve and
    // the compare chain took ~8).
    template <int L, int N, int TH>
    __host__ __device__ __forceinline__ T ge_from() const {
        if constexpr (TH <= 0) return (T)~(T)0;
        else if constexpr (TH > max_units(L, N)) return (T)0;
        else {
            constexpr bool hasA = N >= 1, hasP = N >= 2 && N % 2 == 0;
            constexpr int up = N >= 1 ? (N - 1) / 2 : 0;
            if constexpr (!hasA && !hasP) {
                return ge_from<L + 1, up, (TH + 1) / 2>();
            } else if constexpr (hasA != hasP) {
                const T b = hasA ? acc[L] : pend[L];
                if constexpr (TH % 2 == 0) return ge_from<L + 1, up, TH / 2>();
                else return ge_from<L + 1, up, (TH + 1) / 2>() | (b & ge_from<L + 1, up, (TH - 1) / 2>());
            } else if constexpr (TH % 2 == 0) {
                // two bits: their sum is 2 iff both
                return ge_from<L + 1, up, TH / 2>() | (acc[L] & pend[L] & ge_from<L + 1, up, TH / 2 - 1>());
            } else {
                // sum >= 1 iff either
                return ge_from<L + 1, up, (TH + 1) / 2>() |
                       ((acc[L] | pend[L]) & ge_from<L + 1, up, (TH - 1) / 2>());
            }
        }
    }
    // lanes whose count (after K inputs) is >= TH
    template <int K, int TH>
    __host__ __device__ __forceinline__ T ge() const {
        if constexpr (TH <= 0) return (T)~(T)0;
        else if constexpr (TH > K) return (T)0;
#ifndef BA_CSA_GE_RESOLVE
        else if constexpr (true) return ge_from<0, K, TH>();
#endif
        else {
            T r[NL];
            resolve<0, K, false>(r, 0);
            T gt = 0, eq = (T)~(T)0;
#pragma unroll
            for (int i = NL - 1; i >= 0; --i) {
                if ((TH >> i) & 1) {
                    eq &= r[i];
                } else {
                    gt |= eq & r[i];
                    eq &= ~r[i];
                }
            }
            return gt | eq;
        }
    }
};

// planes needed to count s inputs
__host__ __device__ inline int planes_for(uint32_t s) {
    int p = 1;
    while ((1u << p) <= s) ++p;
    return p;
}

// ---------------------------------------------------------------------------
// Per-trial epilogue: quorum (ba.py:197-253), IC1/IC2, bound, outputs.
// A / U: lieutenant bitmasks (bit r, r = 1..n-1) of attack / undefined roots.
// ---------------------------------------------------------------------------
enum { C_TRIALS, C_AGREE, C_VAPPL, C_VALID, C_QR, C_QA, C_QU, C_UNDEF,
       C_INB, C_VIOL, C_FTOT, C_ATT, C_NUM = 12 };

__device__ __forceinline__ uint64_t part1by1(uint32_t v) {
    uint64_t x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// Sum of x over the wave's 64 lanes (uniform result): DPP within each 16-lane
// row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: four VALU
// adds), then the four row sums by readlane -- where a __shfl_xor tree is six
// dependent ds_bpermute round trips through LDS.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) + (uint32_t)__builtin_amdgcn_readlane((int)x, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)x, 32) + (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}

struct TrialCounts {
    uint32_t v[C_NUM];
    __device__ __forceinline__ TrialCounts() {
#pragma unroll
        for (int i = 0; i < C_NUM; ++i) v[i] = 0;
    }
};

struct TrialResult {
    uint64_t dec;
    uint32_t out, nU, nf, nA;
};

__device__ __forceinline__ TrialResult trial_result(uint32_t n, uint32_t me, uint32_t fm,
                                                    uint32_t oc, uint32_t A, uint32_t U) {
    const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    const uint32_t lts = all & ~1u;
    fm &= all;
    A &= lts;
    U &= lts & ~A;
    const uint32_t nA = __popc(A), nU = __popc(U), nR = (n - 1) - nA - nU;
    const uint32_t na = nA + (oc == 1), nu = nU + (oc == 2), nr = nR + (oc == 0);
    const uint32_t total = na + nr + nu;  // == n: every live general answers
    uint32_t needed = 2 * ((total - 1) / 3) + 1;
    if (total <= 3) needed = total - 1;
    if (total == 1) needed = 1;
    const uint32_t q = needed <= nr ? 0u : (needed <= na ? 1u : 2u);  // retreat first
    const uint32_t loyal = lts & ~fm;
    const uint32_t la = A & loyal, lu = U & loyal, lr = loyal & ~A & ~U;
    const uint32_t agree = ((la != 0) + (lu != 0) + (lr != 0)) <= 1;
    // bitwise & and selects only: a short-circuit && here became divergent
    // branches that split the WAVE epilogue into one basic block per word
    const uint32_t appl = (fm & 1u) == 0 ? 1u : 0u;
    const uint32_t okA = la == loyal ? 1u : 0u, okR = lr == loyal ? 1u : 0u;
    const uint32_t valid = appl & (oc == 1 ? okA : okR);
    const uint32_t nf = __popc(fm);
    const uint32_t inb = (nf <= me ? 1u : 0u) & (n > 3 * me ? 1u : 0u);
    TrialResult r;
    r.dec = part1by1(A >> 1) | (part1by1(U >> 1) << 1);
    r.out = q | agree << 2 | appl << 3 | valid << 4 | inb << 5;
    r.nU = nU;
    r.nf = nf;
    r.nA = nA;
    return r;
}

// Wave-level run counters from per-lane trial results: 0/1 flags by
// ballot+popcount, small integers bit-sliced (5 ballots each); lane 0 adds
// the wave's totals into a block counter array in LDS.
__device__ __forceinline__ void wave_counts_add(bool live, const TrialResult& r,
                                                unsigned long long* blockcnt) {
    const uint32_t o = r.out;
    const bool agree = (o >> 2) & 1, appl = (o >> 3) & 1, valid = (o >> 4) & 1, inb = (o >> 5) & 1;
    const uint32_t q = o & 3;
    uint64_t c[C_NUM];
    c[C_TRIALS] = __popcll(__ballot(live));
    c[C_AGREE] = __popcll(__ballot(live && agree));
    c[C_VAPPL] = __popcll(__ballot(live && appl));
    c[C_VALID] = __popcll(__ballot(live && valid));
    c[C_QR] = __popcll(__ballot(live && q == 0));
    c[C_QA] = __popcll(__ballot(live && q == 1));
    c[C_QU] = __popcll(__ballot(live && q == 2));
    c[C_INB] = __popcll(__ballot(live && inb));
    c[C_VIOL] = __popcll(__ballot(live && inb && (!agree || (appl && !valid))));
    c[C_UNDEF] = c[C_FTOT] = c[C_ATT] = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        c[C_UNDEF] += (uint64_t)__popcll(__ballot(live && ((r.nU >> b) & 1u))) << b;
        c[C_FTOT] += (uint64_t)__popcll(__ballot(live && ((r.nf >> b) & 1u))) << b;
        c[C_ATT] += (uint64_t)__popcll(__ballot(live && ((r.nA >> b) & 1u))) << b;
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int i = 0; i < C_NUM; ++i)
            if (c[i]) atomicAdd(&blockcnt[i], (unsigned long long)c[i]);
    }
}

// ---------------------------------------------------------------------------
// Run counter sink.  Device-scope atomics execute at the memory side, one
// request at a time per cache line, so thousands of waves adding into the
// caller's 12 counters (one line) at the end of a launch serialise: measured
// ~130 us for 2048 waves x 12 single-lane adds.  Instead each reporting unit
// (a wave or a block) adds its totals with ONE 12-lane instruction into
// replica (unit % R), every replica on a line of its own, and only the last
// unit of a replica folds it into the caller's counters: at most R units
// touch the caller's line.
//
// Memory ordering needs no fence: every replica word carries its own arrival
// count in its top 16 bits (each unit adds v + 2^48), so the unit whose
// returning add sees members-1 earlier arrivals on a word holds that word's
// complete sum -- an ordering on ONE location, which relaxed device-scope
// atomics guarantee (coherence order), unlike the ticket-on-another-word
// scheme it replaces, which relied on s_waitcnt draining the adds before the
// ticket.  That unit resets the word with an atomic exchange (no later
// access to it in this launch) and adds the sum into `out`.  Sums per launch
// and replica stay below 2^48; units per replica below 2^16.
// Units of one launch must all call sink_counters exactly once.
// ---------------------------------------------------------------------------
constexpr uint32_t kSinkReplicas = 64;
constexpr uint32_t kSinkRepStride = 16;  // uint64 per replica (128 B)
constexpr size_t kSinkBytes = kSinkReplicas * kSinkRepStride * 8;
constexpr uint32_t kSinkArrivalShift = 48;
constexpr uint32_t kSinkMaxUnitsPerReplica = (1u << (64 - kSinkArrivalShift)) - 1;  // 65535
constexpr unsigned long long kSinkValueMask = (1ull << kSinkArrivalShift) - 1;

struct Sink {
    unsigned long long* rep;  // [kSinkReplicas][kSinkRepStride], zero between launches
    // WAVE engines' dynamic task counter (ctx-owned, zeroed by the launch's stream
    // right before a persistent launch; nullptr = static task assignment)
    unsigned int* tasks = nullptr;
};
constexpr size_t kSinkTaskCounterBytes = 64;  // after the replicas, a line of its own

// Called by every lane of one wave; lane c < C_NUM passes the unit's total of
// counter c in v (other lanes: ignored).
__device__ __forceinline__ void sink_counters(uint32_t lane, uint64_t v, uint32_t unit,
                                              uint32_t nunits, uint64_t* __restrict__ out,
                                              const Sink& sk) {
    // at most one unit per replica (small launches: a handful of words or
    // blocks): no replica to combine in, so the unit adds straight into `out`
    // (<= 64 adds on its line, fire and forget), which spares the latency-bound
    // tail of a one-instance call a returning atomic and an exchange
    if (nunits <= kSinkReplicas) {
        if (lane < C_NUM && v)
            (void)__hip_atomic_fetch_add((unsigned long long*)out + lane, (unsigned long long)v,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint32_t r = unit % kSinkReplicas;
    const uint32_t members = (nunits - r + kSinkReplicas - 1) / kSinkReplicas;
    if (lane < C_NUM) {
        unsigned long long* w = sk.rep + r * kSinkRepStride + lane;
        const unsigned long long old =
            __hip_atomic_fetch_add(w, (unsigned long long)v + (1ull << kSinkArrivalShift),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(old >> kSinkArrivalShift) + 1u == members) {
            const unsigned long long tot = (old + v) & kSinkValueMask;
            (void)__hip_atomic_exchange(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tot)
                (void)__hip_atomic_fetch_add((unsigned long long*)out + lane, tot, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ __forceinline__ void finish_trial(uint32_t n, uint32_t me, uint32_t fm, uint32_t oc,
                                             uint32_t A, uint32_t U, uint64_t& dec,
                                             uint32_t& out, TrialCounts& tc) {
    const TrialResult r = trial_result(n, me, fm, oc, A, U);
    dec = r.dec;
    out = r.out;
    const uint32_t q = r.out & 3, agree = (r.out >> 2) & 1, appl = (r.out >> 3) & 1;
    const uint32_t valid = (r.out >> 4) & 1, inb = (r.out >> 5) & 1;
    tc.v[C_TRIALS] += 1;
    tc.v[C_AGREE] += agree;
    tc.v[C_VAPPL] += appl;
    tc.v[C_VALID] += valid;
    tc.v[C_QR] += q == 0;
    tc.v[C_QA] += q == 1;
    tc.v[C_QU] += q == 2;
    tc.v[C_UNDEF] += r.nU;
    tc.v[C_INB] += inb;
    tc.v[C_VIOL] += inb && (!agree || (appl && !valid));
    tc.v[C_FTOT] += r.nf;
    tc.v[C_ATT] += r.nA;
}

// Block-reduce per-thread counts into partial[blockIdx.x][0..15] (uint64).
// Deterministic: integer sums, fixed reduction tree, no atomics.
template <int BLOCK>
__device__ __forceinline__ void block_counts_out(const TrialCounts& tc, uint64_t* partial) {
    __shared__ uint64_t red[BLOCK / 64][C_NUM];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < C_NUM; ++i) {
        uint64_t x = tc.v[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if (lane == 0) red[wv][i] = x;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        uint64_t s = 0;
        if (threadIdx.x < C_NUM)
            for (int w = 0; w < BLOCK / 64; ++w) s += red[w][threadIdx.x];
        partial[(uint64_t)blockIdx.x * 16 + threadIdx.x] = s;
    }
}

// Block-reduce per-thread counts, then wave 0 adds the block's totals into
// `counters` through the sink (one reporting unit per block; every block of
// the launch must call it).  Replaces a partial-row write + k_reduce launch.
template <int BLOCK>
__device__ __forceinline__ void block_counts_sink(const TrialCounts& tc, uint64_t* counters,
                                                  const Sink& sk) {
    __shared__ uint64_t red[BLOCK / 64][C_NUM];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < C_NUM; ++i) {
        uint64_t x = tc.v[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if (lane == 0) red[wv][i] = x;
    }
    __syncthreads();
    if (wv == 0) {
        uint64_t s = 0;
        if (lane < (uint32_t)C_NUM)
            for (int w = 0; w < BLOCK / 64; ++w) s += red[w][lane];
        sink_counters(lane, s, blockIdx.x, gridDim.x, counters, sk);
    }
}

// Synthetic inputs (docs/SEMANTICS.md §4): u[i] = word i%4 of
// Philox(ctr = (i/4, 0xFFFFFFFF, t_lo, t_hi)).  The partial Fisher-Yates
// permutation lives in a per-thread LDS row (dynamic indices).
struct GenSpec {
    uint32_t faulty_mode, f, order_mode, order_value;
};

__device__ __forceinline__ uint32_t pick4(const P4& p, uint32_t i) {
    return i == 0 ? p.x : (i == 1 ? p.y : (i == 2 ? p.z : p.w));
}

// position of the j-th (0-based) set bit of v (j < popcount(v))
__device__ __forceinline__ uint32_t select_bit(uint32_t v, uint32_t j) {
    uint32_t base = 0;
#pragma unroll
    for (uint32_t s = 16; s >= 1; s >>= 1) {
        const uint32_t lo = v & ((1u << s) - 1u);
        const uint32_t c = __popc(lo);
        if (j >= c) {
            j -= c;
            v >>= s;
            base += s;
        } else {
            v = lo;
        }
    }
    return base;
}

// Overwrites fmask unless faulty_mode is GIVEN and oc unless order_mode is GIVEN
// (reference outputs: an address-taken local would live in scratch memory).
__device__ __forceinline__ void gen_trial(uint32_t n, uint64_t seed, const GenSpec& g, uint64_t t,
                                          uint32_t& fmask, uint32_t& oc) {
    if (g.faulty_mode == 0 && g.order_mode == 0) return;  // both given: no draw at all
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    P4 blk = philox10(P4{0u, kGenTag, (uint32_t)t, (uint32_t)(t >> 32)}, k0, k1);
    if (g.order_mode == 1) oc = blk.x >> 31;
    else if (g.order_mode == 2) oc = g.order_value;
    if (g.faulty_mode != 0) {
        uint32_t nf;
        if (g.faulty_mode == 1) {
            const uint32_t fmax = g.f < n ? g.f : n;
            nf = mulhi_range(blk.y, fmax + 1);
        } else {
            nf = g.f < n ? g.f : n;
        }
        // sequential selection without replacement (docs/SEMANTICS.md §4)
        const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
        uint32_t mask = 0, cur_call = 0;
        for (uint32_t i = 0; i < nf; ++i) {
            const uint32_t wi = 2 + i;
            if ((wi >> 2) != cur_call) {
                cur_call = wi >> 2;
                blk = philox10(P4{cur_call, kGenTag, (uint32_t)t, (uint32_t)(t >> 32)}, k0, k1);
            }
            const uint32_t j = mulhi_range(pick4(blk, wi & 3), n - i);
            mask |= 1u << select_bit(all & ~mask, j);
        }
        fmask = mask;
    }
}

}  // namespace ba
