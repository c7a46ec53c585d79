// philox_bench.hip -- Philox4x32-10 throughput ceiling on the GPU (calls/s),
// the VALU roofline of the OM(m) leaf kernels, for several code shapes:
//   mad64   : ba::philox10 as shipped (v_mad_u64_u32 + xor)
//   xor3    : v_mad_u64_u32 + v_bitop3 xor3 (2 x 3-input xors per round)
//   mulhilo : v_mul_hi_u32 + v_mul_lo_u32 + xor3
//   kernel_shape : ba::philox10_n as the OM kernels run it (pinned mads)
//   kernel_shape_vgpr_keys : ba::philox10_n_vk (round keys as VGPR operands)
// Each thread runs K independent counter-mode calls in CH interleaved chains
// and xors the outputs (so nothing is dead code).  Measured at 1, 2, 4 and 8
// resident waves per SIMD, after a warm-up, with the in-kernel clock.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../byzantine-agreement_amd/csrc/ba_device.hpp"

using ba::P4;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int V>
__device__ __forceinline__ P4 philox(P4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        P4 n;
        if constexpr (V == 0) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
            n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
            n.y = (uint32_t)p1;
            n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
            n.w = (uint32_t)p0;
        } else if constexpr (V == 1) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
            n.x = xor3((uint32_t)(p1 >> 32), c.y, k0);
            n.y = (uint32_t)p1;
            n.z = xor3((uint32_t)(p0 >> 32), c.w, k1);
            n.w = (uint32_t)p0;
        } else {
            n.x = xor3(__umulhi(0xCD9E8D57u, c.z), c.y, k0);
            n.y = 0xCD9E8D57u * c.z;
            n.z = xor3(__umulhi(0xD2511F53u, c.x), c.w, k1);
            n.w = 0xD2511F53u * c.x;
        }
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

template <int V>
__device__ __forceinline__ P4 philox_any(P4 c, uint32_t k0, uint32_t k1) {
    if constexpr (V == 3) return ba::philox10(c, k0, k1);  // the kernels' own code (pinned mads)
    else return philox<V>(c, k0, k1);
}

// Each thread: K counter-mode calls in CH interleaved chains.  Thread 0 of each
// block stamps s_memtime / s_memrealtime around its loop (in-kernel clock).
template <int V, int CH>
__global__ __launch_bounds__(256) void k_philox(uint64_t seed, uint32_t K, uint32_t* out,
                                                unsigned long long* stamps) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 0;
    const ba::KeysV kv(seed);
    for (uint32_t i = 0; i < K; i += CH) {
        P4 o[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) o[c] = P4{i + c, 3u, t, 0u};
        if constexpr (V == 3) {
            ba::philox10_n<CH>(o, (uint32_t)seed, (uint32_t)(seed >> 32));
        } else if constexpr (V == 7) {
            ba::philox10_n_vk<CH>(o, kv);
        } else {
#pragma unroll
            for (int c = 0; c < CH; ++c) o[c] = philox_any<V>(o[c], (uint32_t)seed, (uint32_t)(seed >> 32));
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] ^= o[c].x ^ o[c].y ^ o[c].z ^ o[c].w;
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) r ^= acc[c];
    out[t] = r;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// blocks = 256 CUs x W blocks of 4 waves -> W resident waves per SIMD (one wave
// per SIMD per block; the kernel's registers allow 8)
template <int V, int CH>
static void run(const char* name, uint32_t W, uint32_t* d, unsigned long long* st) {
    const uint32_t blocks = 256 * W, K = 8192 / W;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // >= 0.5 s of back-to-back launches first: the clock settles under this load
    for (int r = 0; r < 400; ++r)
        hipLaunchKernelGGL((k_philox<V, CH>), dim3(blocks), dim3(256), 0, 0, 1ull, K, d, st);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_philox<V, CH>), dim3(blocks), dim3(256), 0, 0, 1ull + r, K, d, st);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    std::vector<unsigned long long> h(2 * blocks);
    (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (uint32_t b = 0; b < blocks; ++b)
        if (h[2 * b + 1]) clk.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);  // 100 MHz ref
    std::sort(clk.begin(), clk.end());
    const double calls = (double)blocks * 256 * K;
    const double rate = calls / (best * 1e-3);
    // SIMD cycles per wave-call at 2.4 GHz over 1024 SIMDs
    const double cyc = 1024.0 * 2.4e9 / (rate / 64.0);
    printf("{\"variant\": \"%s\", \"chains\": %d, \"waves_per_simd\": %u, \"philox_calls_per_s\": %.4e, "
           "\"ms\": %.4f, \"simd_cycles_per_wave_call_at_2p4GHz\": %.1f, \"clock_ghz_median\": %.3f}\n",
           name, CH, W, rate, best, cyc, clk.empty() ? 0.0 : clk[clk.size() / 2]);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    uint32_t* d;
    unsigned long long* st;
    (void)hipMalloc(&d, (size_t)256 * 8 * 256 * 4);
    (void)hipMalloc(&st, (size_t)256 * 8 * 2 * 8);
    for (uint32_t W : {1u, 2u, 4u, 8u}) {
        run<1, 4>("xor3", W, d, st);
        run<3, 3>("kernel_shape", W, d, st);
        run<7, 3>("kernel_shape_vgpr_keys", W, d, st);
        run<3, 4>("kernel_shape_g4", W, d, st);
        run<7, 4>("kernel_shape_g4_vgpr_keys", W, d, st);
    }
    (void)hipFree(d);
    (void)hipFree(st);
    return 0;
}
