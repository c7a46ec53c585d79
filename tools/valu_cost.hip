// valu_cost.hip -- issue cost (SIMD cycles per wave64 instruction) of the VALU
// instructions the OM kernels are made of, at 1, 2 and 8 resident waves per
// SIMD.  Each thread runs 16 independent chains of one instruction (inline asm,
// so the compiler cannot fold or split it) for ITERS iterations; the cost is
//   kernel time x in-kernel clock x 1024 SIMDs / wave-instructions issued.
// These weights turn the kernels' ISA instruction mix into an issue-cycle
// roofline: a v_mad_u64_u32 is not one "VALU slot".
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

enum Op { XOR3, ADD, MAD64, MULLO, MULHI, BFI, MAD24, LSHL_OR, XOR3_V, MAD64_V, ADD_S, ADD3_V,
          ADD_LIT, XOR_E32, XOR_E64, ADD_E64 };
static const char* kNames[] = {"v_bitop3_b32(xor3)", "v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32",
                               "v_mul_hi_u32", "v_bfi_b32", "v_mad_u32_u24", "v_lshl_or_b32",
                               "v_bitop3_b32(xor3, all VGPR)", "v_mad_u64_u32(VGPR multiplier)",
                               "v_add_u32(SGPR src0)", "v_add3_u32(all VGPR)",
                               "v_add_u32(literal src0, 8-byte VOP2)", "v_xor_b32_e32",
                               "v_xor_b32_e64 (VOP3 encoding)", "v_add_u32_e64 (VOP3 encoding)"};
constexpr int CH = 16;

// One asm statement issues the instruction once on each of 8 independent
// chains (a per-statement asm would get a conservative s_nop after it from the
// hazard recognizer, which then dominates the timing).
template <int OP>
__device__ __forceinline__ void op8(uint32_t (&a)[8], uint64_t (&r)[8], uint32_t x, uint32_t m) {
    if constexpr (OP == XOR3) {
        asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == ADD) {
        asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == MAD64) {
        uint64_t cc;  // the carry-out SGPR pair: an early-clobber OUTPUT, never an input
        asm volatile("v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mad_u64_u32 %1, %8, %9, %10, %1\n\tv_mad_u64_u32 %2, %8, %9, %10, %2\n\tv_mad_u64_u32 %3, %8, %9, %10, %3\n\tv_mad_u64_u32 %4, %8, %9, %10, %4\n\tv_mad_u64_u32 %5, %8, %9, %10, %5\n\tv_mad_u64_u32 %6, %8, %9, %10, %6\n\tv_mad_u64_u32 %7, %8, %9, %10, %7"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                       "+v"(r[6]), "+v"(r[7]), "=&s"(cc)
                     : "v"(x), "s"(m));
    } else if constexpr (OP == MULLO) {
        asm volatile("v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\tv_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == MULHI) {
        asm volatile("v_mul_hi_u32 %0, %0, %8\n\tv_mul_hi_u32 %1, %1, %8\n\tv_mul_hi_u32 %2, %2, %8\n\tv_mul_hi_u32 %3, %3, %8\n\tv_mul_hi_u32 %4, %4, %8\n\tv_mul_hi_u32 %5, %5, %8\n\tv_mul_hi_u32 %6, %6, %8\n\tv_mul_hi_u32 %7, %7, %8"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == BFI) {
        asm volatile("v_bfi_b32 %0, %8, %0, %9\n\tv_bfi_b32 %1, %8, %1, %9\n\tv_bfi_b32 %2, %8, %2, %9\n\tv_bfi_b32 %3, %8, %3, %9\n\tv_bfi_b32 %4, %8, %4, %9\n\tv_bfi_b32 %5, %8, %5, %9\n\tv_bfi_b32 %6, %8, %6, %9\n\tv_bfi_b32 %7, %8, %7, %9"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == MAD24) {
        asm volatile("v_mad_u32_u24 %0, %0, %8, %9\n\tv_mad_u32_u24 %1, %1, %8, %9\n\tv_mad_u32_u24 %2, %2, %8, %9\n\tv_mad_u32_u24 %3, %3, %8, %9\n\tv_mad_u32_u24 %4, %4, %8, %9\n\tv_mad_u32_u24 %5, %5, %8, %9\n\tv_mad_u32_u24 %6, %6, %8, %9\n\tv_mad_u32_u24 %7, %7, %8, %9"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == XOR3_V) {
        asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "v"(m));
    } else if constexpr (OP == MAD64_V) {
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mad_u64_u32 %1, %8, %9, %10, %1\n\tv_mad_u64_u32 %2, %8, %9, %10, %2\n\tv_mad_u64_u32 %3, %8, %9, %10, %3\n\tv_mad_u64_u32 %4, %8, %9, %10, %4\n\tv_mad_u64_u32 %5, %8, %9, %10, %5\n\tv_mad_u64_u32 %6, %8, %9, %10, %6\n\tv_mad_u64_u32 %7, %8, %9, %10, %7"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                       "+v"(r[6]), "+v"(r[7]), "=&s"(cc)
                     : "v"(x), "v"(m));
    } else if constexpr (OP == ADD_S) {
        asm volatile("v_add_u32 %0, %9, %0\n\tv_add_u32 %1, %9, %1\n\tv_add_u32 %2, %9, %2\n\tv_add_u32 %3, %9, %3\n\tv_add_u32 %4, %9, %4\n\tv_add_u32 %5, %9, %5\n\tv_add_u32 %6, %9, %6\n\tv_add_u32 %7, %9, %7"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == ADD3_V) {
        asm volatile("v_add3_u32 %0, %0, %8, %9\n\tv_add3_u32 %1, %1, %8, %9\n\tv_add3_u32 %2, %2, %8, %9\n\tv_add3_u32 %3, %3, %8, %9\n\tv_add3_u32 %4, %4, %8, %9\n\tv_add3_u32 %5, %5, %8, %9\n\tv_add3_u32 %6, %6, %8, %9\n\tv_add3_u32 %7, %7, %8, %9"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "v"(m));
    } else if constexpr (OP == ADD_LIT) {
        asm volatile("v_add_u32 %0, 0x12345, %0\n\tv_add_u32 %1, 0x12345, %1\n\tv_add_u32 %2, 0x12345, %2\n\tv_add_u32 %3, 0x12345, %3\n\tv_add_u32 %4, 0x12345, %4\n\tv_add_u32 %5, 0x12345, %5\n\tv_add_u32 %6, 0x12345, %6\n\tv_add_u32 %7, 0x12345, %7"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == XOR_E32) {
        asm volatile("v_xor_b32_e32 %0, %8, %0\n\tv_xor_b32_e32 %1, %8, %1\n\tv_xor_b32_e32 %2, %8, %2\n\tv_xor_b32_e32 %3, %8, %3\n\tv_xor_b32_e32 %4, %8, %4\n\tv_xor_b32_e32 %5, %8, %5\n\tv_xor_b32_e32 %6, %8, %6\n\tv_xor_b32_e32 %7, %8, %7"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == XOR_E64) {
        asm volatile("v_xor_b32_e64 %0, %8, %0\n\tv_xor_b32_e64 %1, %8, %1\n\tv_xor_b32_e64 %2, %8, %2\n\tv_xor_b32_e64 %3, %8, %3\n\tv_xor_b32_e64 %4, %8, %4\n\tv_xor_b32_e64 %5, %8, %5\n\tv_xor_b32_e64 %6, %8, %6\n\tv_xor_b32_e64 %7, %8, %7"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == ADD_E64) {
        asm volatile("v_add_u32_e64 %0, %8, %0\n\tv_add_u32_e64 %1, %8, %1\n\tv_add_u32_e64 %2, %8, %2\n\tv_add_u32_e64 %3, %8, %3\n\tv_add_u32_e64 %4, %8, %4\n\tv_add_u32_e64 %5, %8, %5\n\tv_add_u32_e64 %6, %8, %6\n\tv_add_u32_e64 %7, %8, %7"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    } else if constexpr (OP == LSHL_OR) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %8\n\tv_lshl_or_b32 %1, %1, 3, %8\n\tv_lshl_or_b32 %2, %2, 3, %8\n\tv_lshl_or_b32 %3, %3, 3, %8\n\tv_lshl_or_b32 %4, %4, 3, %8\n\tv_lshl_or_b32 %5, %5, 3, %8\n\tv_lshl_or_b32 %6, %6, 3, %8\n\tv_lshl_or_b32 %7, %7, 3, %8"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                       "+v"(a[6]), "+v"(a[7])
                     : "v"(x), "s"(m));
    }
}

template <int OP>
__global__ __launch_bounds__(256) void k_cost(uint32_t iters, uint32_t m, uint32_t* out,
                                              unsigned long long* stamps) {
    uint32_t a[CH / 8][8];
    uint64_t w[CH / 8][8];
    const uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
#pragma unroll
    for (int g = 0; g < CH / 8; ++g)
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            a[g][c] = x + c + 8 * g;
            w[g][c] = (uint64_t)(x ^ c) << 32 | (x + g);
        }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int g = 0; g < CH / 8; ++g) op8<OP>(a[g], w[g], x + i, m);
    }
    uint32_t r = 0;
#pragma unroll
    for (int g = 0; g < CH / 8; ++g)
#pragma unroll
        for (int c = 0; c < 8; ++c) r ^= a[g][c] ^ (uint32_t)w[g][c] ^ (uint32_t)(w[g][c] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int OP>
static void run(uint32_t W, uint32_t* d, unsigned long long* st) {
    const uint32_t blocks = 256 * W, iters = 4096 / W;
    for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_cost<OP>, dim3(blocks), dim3(256), 0, 0, iters, 0x9E3779B9u, d, st);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_cost<OP>, dim3(blocks), dim3(256), 0, 0, iters, 0x9E3779B9u, d, st);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
    }
    std::vector<unsigned long long> h(2 * blocks);
    (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (uint32_t b = 0; b < blocks; ++b)
        if (h[2 * b + 1]) clk.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    const double ghz = clk.empty() ? 2.4 : clk[clk.size() / 2];
    const double winst = (double)blocks * 4 * iters * CH;  // wave-instructions
    const double cyc = best * 1e-3 * ghz * 1e9 * 1024.0 / winst;
    printf("{\"inst\": \"%s\", \"waves_per_simd\": %u, \"cycles_per_wave_inst\": %.3f, \"clock_ghz\": %.3f, \"ms\": %.4f}\n",
           kNames[OP], W, cyc, ghz, best);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    const bool operands = argc > 1;  // "operands": SGPR vs VGPR operand variants only
    uint32_t* d;
    unsigned long long* st;
    (void)hipMalloc(&d, (size_t)256 * 8 * 256 * 4);
    (void)hipMalloc(&st, (size_t)256 * 8 * 2 * 8);
    for (uint32_t W : {1u, 2u, 8u}) {
        if (operands) {
            if (W == 1) continue;
            run<XOR3>(W, d, st);
            run<XOR3_V>(W, d, st);
            run<MAD64>(W, d, st);
            run<MAD64_V>(W, d, st);
            run<ADD>(W, d, st);
            run<ADD_S>(W, d, st);
            run<ADD3_V>(W, d, st);
            run<ADD_LIT>(W, d, st);
            run<XOR_E32>(W, d, st);
            run<XOR_E64>(W, d, st);
            run<ADD_E64>(W, d, st);
            continue;
        }
        run<XOR3>(W, d, st);
        run<ADD>(W, d, st);
        run<MAD64>(W, d, st);
        run<MULLO>(W, d, st);
        run<MULHI>(W, d, st);
        run<BFI>(W, d, st);
        run<MAD24>(W, d, st);
        run<LSHL_OR>(W, d, st);
    }
    (void)hipFree(d);
    (void)hipFree(st);
    return 0;
}
