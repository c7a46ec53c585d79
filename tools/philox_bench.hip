// philox_bench.hip -- Philox4x32-10 throughput ceiling on the GPU (calls/s),
// the VALU roofline of the OM(m) leaf kernels, for several code shapes:
//   mad64   : ba::philox10 as shipped (v_mad_u64_u32 + xor)
//   xor3    : v_mad_u64_u32 + v_bitop3 xor3 (2 x 3-input xors per round)
//   mulhilo : v_mul_hi_u32 + v_mul_lo_u32 + xor3
// Each thread runs K independent counter-mode calls in CH interleaved chains
// and xors the outputs (so nothing is dead code).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

template <int V, int CH, int K>
__global__ __launch_bounds__(256) void k_philox(uint64_t seed, uint32_t* out) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 0;
    for (int i = 0; i < K; i += CH) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const P4 o = philox<V>(P4{(uint32_t)(i + c), 3u, t, 0u}, (uint32_t)seed,
                                   (uint32_t)(seed >> 32));
            acc[c] ^= o.x ^ o.y ^ o.z ^ o.w;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) r ^= acc[c];
    out[t] = r;
}

template <int V, int CH>
static void run(const char* name, uint32_t blocks, uint32_t* d) {
    constexpr int K = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k_philox<V, CH, K>), dim3(blocks), dim3(256), 0, 0, 1ull, d);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_philox<V, CH, K>), dim3(blocks), dim3(256), 0, 0, 1ull + r, d);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double calls = (double)blocks * 256 * K;
    const double rate = calls / (best * 1e-3);
    // SIMD cycles per wave-call at 2.4 GHz over 1024 SIMDs
    const double cyc = 1024.0 * 2.4e9 / (rate / 64.0);
    printf("{\"variant\": \"%s\", \"chains\": %d, \"philox_calls_per_s\": %.4e, \"ms\": %.4f, "
           "\"simd_cycles_per_wave_call_at_2p4GHz\": %.1f}\n", name, CH, rate, best, cyc);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    const uint32_t blocks = argc > 1 ? atoi(argv[1]) : 8192;
    uint32_t* d;
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    run<0, 1>("mad64", blocks, d);
    run<0, 2>("mad64", blocks, d);
    run<0, 4>("mad64", blocks, d);
    run<1, 2>("xor3", blocks, d);
    run<1, 4>("xor3", blocks, d);
    run<2, 2>("mulhilo", blocks, d);
    run<2, 4>("mulhilo", blocks, d);
    hipFree(d);
    return 0;
}
