// marker_cost.hip -- what a per-call "this call is done" marker costs a stream
// of back-to-back kernels (libba_hip's cross-stream ordering, ba_api.cpp
// ctx_mark).  A ~50 us VALU-bound kernel is launched K times back to back with
// one of these after every launch:
//   none | event (DisableTiming) | event+ReleaseToDevice | event+DisableSystemFence
//   | writevalue (hipStreamWriteValue64)
// and the average time per launch is reported (HIP events around the K launches).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_busy(uint32_t iters, uint32_t* out) {
    uint32_t a = threadIdx.x, b = blockIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        a = a * 1664525u + b;
        b = b ^ (a >> 7);
    }
    if (a == 0xFFFFFFFFu) out[0] = b;
}

int main() {
    uint32_t* d;
    uint64_t* flag;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&flag, 64);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t ev[4], t0, t1;
    (void)hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ev[2], hipEventDisableTiming | hipEventReleaseToDevice);
    (void)hipEventCreateWithFlags(&ev[3], hipEventDisableTiming | hipEventDisableSystemFence);
    (void)hipEventCreate(&t0);
    (void)hipEventCreate(&t1);
    const char* names[] = {"none", "event", "event_release_to_device", "event_no_system_fence",
                           "write_value64"};
    const uint32_t iters = 6000, K = 200;
    for (int rep = 0; rep < 3; ++rep)
        for (int v = 0; v < 5; ++v) {
            for (uint32_t k = 0; k < 50; ++k) hipLaunchKernelGGL(k_busy, dim3(2048), dim3(256), 0, s, iters, d);
            (void)hipStreamSynchronize(s);
            (void)hipEventRecord(t0, s);
            for (uint32_t k = 0; k < K; ++k) {
                hipLaunchKernelGGL(k_busy, dim3(2048), dim3(256), 0, s, iters, d);
                if (v >= 1 && v <= 3) (void)hipEventRecord(ev[v], s);
                if (v == 4) (void)hipStreamWriteValue64(s, flag, k + 1, 0);
            }
            (void)hipEventRecord(t1, s);
            (void)hipEventSynchronize(t1);
            float ms;
            (void)hipEventElapsedTime(&ms, t0, t1);
            printf("{\"marker\": \"%s\", \"rep\": %d, \"us_per_launch\": %.3f}\n", names[v], rep,
                   ms * 1e3 / K);
        }
    return 0;
}
