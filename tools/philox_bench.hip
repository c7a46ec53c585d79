// philox_bench.hip -- Philox4x32-10 throughput ceiling on the GPU (calls/s),
// the VALU roofline of the OM(m) leaf kernels.  Each thread runs K independent
// counter-mode calls (2 interleaved streams for ILP) and xors the outputs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../byzantine-agreement_amd/csrc/ba_device.hpp"

template <int K>
__global__ __launch_bounds__(256) void k_philox(uint64_t seed, uint64_t* out) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint64_t acc0 = 0, acc1 = 0;
#pragma unroll 4
    for (int i = 0; i < K; i += 2) {
        uint64_t a, b, c, d;
        ba::lie_pair(seed, 3, (uint32_t)i, t, a, b);
        ba::lie_pair(seed, 3, (uint32_t)i + 1, t, c, d);
        acc0 ^= a ^ c;
        acc1 ^= b ^ d;
    }
    out[t] = acc0 ^ acc1;
}

int main(int argc, char** argv) {
    const uint32_t blocks = argc > 1 ? atoi(argv[1]) : 8192;
    constexpr int K = 256;
    uint64_t* d;
    hipMalloc(&d, (size_t)blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_philox<K>, dim3(blocks), dim3(256), 0, 0, 1ull, d);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_philox<K>, dim3(blocks), dim3(256), 0, 0, 1ull + r, d);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double calls = (double)blocks * 256 * K;
    const double rate = calls / (best * 1e-3);
    // wave-cycles per call per SIMD at 2.4 GHz over 1024 SIMDs
    const double cyc = 1024.0 * 2.4e9 / (rate / 64.0);
    printf("{\"philox_calls_per_s\": %.4e, \"ms\": %.4f, \"calls\": %.0f, "
           "\"simd_cycles_per_wave_call_at_2p4GHz\": %.1f}\n", rate, best, calls, cyc);
    hipFree(d);
    return 0;
}
