// bank_cost.hip -- (round 3 lab; see DESIGN.md §8: identical asm measured at two
// different costs in one run, so treat its bank/SGPR columns with care) issue cost of 3-source VALU ops (v_bitop3_b32 xor3) by the
// VGPR banks of their sources (bank = register index mod 4 on CDNA), at 2, 3
// and 8 resident waves per SIMD.  Fixed registers (clobbers), 32 independent
// chains per wave, 64 instructions per asm statement.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

// dst/src0 = v[40 + i] (i = 0..31), src1 = A, src2 = B
#define OPS(A, B) \
  "v_bitop3_b32 v40, v40, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v41, v41, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v42, v42, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v43, v43, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v44, v44, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v45, v45, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v46, v46, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v47, v47, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v48, v48, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v49, v49, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v50, v50, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v51, v51, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v52, v52, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v53, v53, " A ", " B " bitop3:0x96\n\t" \
  "v_bitop3_b32 v54, v54, " A ", " B " bitop3:0x96\n\t" "v_bitop3_b32 v55, v55, " A ", " B " bitop3:0x96\n\t"
// 16 products into v[40:41] .. v[70:71] from x = v80 (bank 0), multiplier M
#define MADS(M) \
  "v_mad_u64_u32 v[40:41], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[42:43], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[44:45], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[46:47], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[48:49], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[50:51], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[52:53], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[54:55], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[56:57], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[58:59], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[60:61], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[62:63], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[64:65], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[66:67], s[2:3], v80, " M ", 0\n\t" \
  "v_mad_u64_u32 v[68:69], s[2:3], v80, " M ", 0\n\t" "v_mad_u64_u32 v[70:71], s[2:3], v80, " M ", 0\n\t"
#define MCLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55", \
  "v56","v57","v58","v59","v60","v61","v62","v63","v64","v65","v66","v67","v68","v69","v70","v71","s2","s3"
// bfi with sources x = v61 (bank 1), y = v62 (bank 2) / v65 (bank 1)
#define BFIS(A, B) \
  "v_bfi_b32 v40, v40, " A ", " B "\n\t" "v_bfi_b32 v41, v41, " A ", " B "\n\t" "v_bfi_b32 v42, v42, " A ", " B "\n\t" \
  "v_bfi_b32 v43, v43, " A ", " B "\n\t" "v_bfi_b32 v44, v44, " A ", " B "\n\t" "v_bfi_b32 v45, v45, " A ", " B "\n\t" \
  "v_bfi_b32 v46, v46, " A ", " B "\n\t" "v_bfi_b32 v47, v47, " A ", " B "\n\t" "v_bfi_b32 v48, v48, " A ", " B "\n\t" \
  "v_bfi_b32 v49, v49, " A ", " B "\n\t" "v_bfi_b32 v50, v50, " A ", " B "\n\t" "v_bfi_b32 v51, v51, " A ", " B "\n\t" \
  "v_bfi_b32 v52, v52, " A ", " B "\n\t" "v_bfi_b32 v53, v53, " A ", " B "\n\t" "v_bfi_b32 v54, v54, " A ", " B "\n\t" \
  "v_bfi_b32 v55, v55, " A ", " B "\n\t"
#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"

template <int V>
__global__ __launch_bounds__(256) void k_bank(uint32_t iters, uint32_t* out, unsigned long long* st) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("v_mov_b32 v60, %0\n\tv_mov_b32 v61, %0\n\tv_mov_b32 v62, %0\n\tv_mov_b32 v63, %0\n\tv_mov_b32 v64, %0\n\tv_mov_b32 v65, %0\n\tv_mov_b32 v66, %0\n\tv_mov_b32 v68, %0\n\tv_mov_b32 v80, %0\n\tv_mov_b32 v81, %0\n\tv_mov_b32 v84, %0" :: "v"(threadIdx.x) : "v60","v61","v62","v63","v64","v65","v66","v68","v80","v81","v84");
    for (uint32_t i = 0; i < iters; ++i) {
        // bank(v40+i) = i mod 4; v60/v64/v68 bank 0, v61 bank 1, v62 bank 2, v63 bank 3
        if constexpr (V == 0) asm volatile(OPS("v61", "v62") OPS("v61", "v62") OPS("v61", "v62") OPS("v61", "v62") ::: CLOB);  // sources in 3 banks (dst row varies)
        else if constexpr (V == 1) asm volatile(OPS("v60", "v64") OPS("v60", "v64") OPS("v60", "v64") OPS("v60", "v64") ::: CLOB); // src1, src2 same bank (0)
        else if constexpr (V == 2) asm volatile(OPS("v60", "s0") OPS("v60", "s0") OPS("v60", "s0") OPS("v60", "s0") ::: CLOB);   // SGPR src2
        else asm volatile(OPS("v61", "5") OPS("v61", "5") OPS("v61", "5") OPS("v61", "5") ::: CLOB);              // inline-constant src2
    }
    uint32_t r;
    asm volatile("v_mov_b32 %0, v40" : "=v"(r));
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int V>
static void run(const char* name, uint32_t W, uint32_t* d, unsigned long long* st) {
    const uint32_t blocks = 256 * W, iters = 2048 / W;
    for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_bank<V>, dim3(blocks), dim3(256), 0, 0, iters, d, st);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_bank<V>, dim3(blocks), dim3(256), 0, 0, iters, d, st);
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
    const double winst = (double)blocks * 4 * iters * ((V >= 4 && V <= 6) ? 32 : 64);
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %u, \"cycles_per_wave_inst\": %.3f, \"clock_ghz\": %.3f}\n",
           name, W, best * 1e-3 * ghz * 1e9 * 1024.0 / winst, ghz);
}

int main() {
    uint32_t* d;
    unsigned long long* st;
    (void)hipMalloc(&d, (size_t)256 * 8 * 256 * 4);
    (void)hipMalloc(&st, (size_t)256 * 8 * 2 * 8);
    for (uint32_t W : {2u, 8u}) {
        run<10>("xor3 v60,v64", W, d, st);
        run<20>("bfi v60,v64", W, d, st);
        run<11>("xor3 v61,v65", W, d, st);
        run<21>("bfi v61,v65", W, d, st);
        run<12>("xor3 v60,v62", W, d, st);
        run<22>("bfi v60,v62", W, d, st);
        run<13>("xor3 v60,v61", W, d, st);
        run<23>("bfi v60,v61", W, d, st);
        run<14>("xor3 v61,v63", W, d, st);
        run<24>("bfi v61,v63", W, d, st);
        run<15>("xor3 v60,v68", W, d, st);
        run<25>("bfi v60,v68", W, d, st);
        run<16>("xor3 v62,v66", W, d, st);
        run<26>("bfi v62,v66", W, d, st);
        run<17>("xor3 v63,v67", W, d, st);
        run<27>("bfi v63,v67", W, d, st);
    }
    for (uint32_t W : {1u, 2u, 3u, 8u}) {
        run<0>("xor3 sources in 3 banks", W, d, st);
        run<1>("xor3 src1/src2 same bank", W, d, st);
        run<2>("xor3 SGPR src2", W, d, st);
        run<3>("xor3 inline-constant src2", W, d, st);
        run<4>("mad_u64_u32 SGPR multiplier", W, d, st);
        run<5>("mad_u64_u32 VGPR multiplier, other bank", W, d, st);
        run<6>("mad_u64_u32 VGPR multiplier, same bank as x", W, d, st);
        run<7>("bfi sources in 3 banks", W, d, st);
        run<8>("bfi src1/src2 same bank", W, d, st);
    }
    return 0;
}
