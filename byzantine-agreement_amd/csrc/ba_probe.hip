// ba_probe.hip -- engine-clock probe (ba_clock_probe_device, include/ba.h):
// every block's first lane reads its XCC / HW ids and the shader-clock
// (s_memtime) and 100 MHz (s_memrealtime) counters.  Two probes around a
// stretch of work give its average engine clock per XCD.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ba {

__global__ __launch_bounds__(64) void k_clock_probe(uint64_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    // s_getreg(id | offset << 6 | (size - 1) << 11): HW_REG_HW_ID = 4, HW_REG_XCC_ID = 20
    const uint64_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    const uint64_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)) & 0xfu;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const uint64_t rt = __builtin_amdgcn_s_memrealtime();
    uint64_t* o = out + 4 * (uint64_t)blockIdx.x;
    o[0] = xcc;
    o[1] = hw;
    o[2] = t;
    o[3] = rt;
}

hipError_t launch_clock_probe(uint64_t* d_out, uint32_t blocks, hipStream_t st) {
    hipLaunchKernelGGL(k_clock_probe, dim3(blocks), dim3(64), 0, st, d_out);
    return hipGetLastError();
}

}  // namespace ba
