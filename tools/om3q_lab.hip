// om3q_lab.hip -- phase timing of the depth-3 queue kernel k_om3q (lab build:
// BA_QUEUE_STAMPS) against k_om3w on the bench workload (n=10, m=3, 1M trials,
// staged inputs).  Not the product; prints JSON lines.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/om3q_lab tools/om3q_lab.hip
#define BA_QUEUE_STAMPS 1
#include "../byzantine-agreement_amd/csrc/ba_wave3.hip"
#include "../byzantine-agreement_amd/csrc/ba_levels.hip"
#include "../byzantine-agreement_amd/csrc/ba_wave4.hip"
#include "../byzantine-agreement_amd/csrc/ba_fused.hip"
#include "lab_kernels.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ba;
void ba::Prof::begin(const char*, hipStream_t) {}
void ba::Prof::end() {}

template <typename K, typename... A>
static float time_k(K k, uint32_t grid, uint32_t threads, uint32_t lds, A... args) {
    for (int i = 0; i < 300; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, 0, args...);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int R = 50;
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, 0, args...);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
    return ms * 1000.f / R;
}

int main(int argc, char** argv) {
    const uint64_t B = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1u << 20);
    uint64_t *dec, *cnt;
    uint8_t *out, *so;
    uint32_t* sf;
    void* sp;
    (void)hipMalloc(&dec, B * 8);
    (void)hipMalloc(&out, B);
    (void)hipMalloc(&cnt, 128);
    (void)hipMalloc(&sf, B * 4);
    (void)hipMalloc(&so, B);
    (void)hipMalloc(&sp, kSinkBytes);
    (void)hipMemset(sp, 0, kSinkBytes);
    Sink sk{(unsigned long long*)sp};
    GenSpec gdraw{1, 3, 1, 1}, gstaged{0, 3, 0, 1};
    hipLaunchKernelGGL(k_gen_inputs, dim3(2048), dim3(256), 0, 0, 10u, 0xBA5EEDull, gdraw, 0ull, B, sf, so);
    (void)hipDeviceSynchronize();
    using G = Om3Q<10>;
    const uint64_t words = (B + 63) / 64, tasks = (words + G::W - 1) / G::W;
    uint64_t tpg = (tasks + 255) / 256;
    tpg = tpg < 1 ? 1 : (tpg > 8 ? 8 : tpg);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((tasks + tpg - 1) / tpg, 256);
    auto report = [&](const char* name, float us, uint32_t wpb = 8) {
        std::vector<unsigned long long> st(4096 * 10);
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_q_stamps), st.size() * 8);
        double ph[10] = {0};
        const uint32_t nw = grid * wpb;
        std::vector<double> tot;
        for (uint32_t w = 0; w < nw; ++w) {
            double t = 0;
            for (int i = 0; i < 10; ++i) ph[i] += (double)st[w * 10 + i];
            for (int i = 0; i < 7; ++i) t += (double)st[w * 10 + i];
            tot.push_back(t);
        }
        std::sort(tot.begin(), tot.end());
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"grid\": %u, \"tpg\": %llu, "
               "\"cycles_per_wave\": {\"inputs_l0\": %.0f, \"rounds\": %.0f, \"roots\": %.0f, "
               "\"epilogue\": %.0f, \"idle\": %.0f, \"barrier_A\": %.0f, \"barrier_end\": %.0f}, "
               "\"round_units_per_wave\": %.2f, \"epi_units_per_wave\": %.2f, \"total_p10\": %.0f, "
               "\"total_p90\": %.0f}\n", name, us, grid, (unsigned long long)tpg,
               ph[0] / nw, ph[1] / nw, ph[2] / nw, ph[3] / nw, ph[4] / nw, ph[5] / nw, ph[6] / nw,
               ph[7] / nw, ph[8] / nw, tot[nw / 10], tot[nw * 9 / 10]);
    };
    float us = time_k(k_om3q<10, true, 1>, grid, kQueueThreads, G::lds_bytes, 0xBA5EEDull, gstaged,
                      0ull, B, (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk, (uint32_t)tpg);
    report("om3q_word_epi", us);
    us = time_k(k_om3q<10, true, 0>, grid, kQueueThreads, G::lds_bytes, 0xBA5EEDull, gstaged,
                0ull, B, (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk, (uint32_t)tpg);
    report("om3q_task_epi", us);
    us = time_k(k_om3q<10, true, 1, 0, 768>, grid, 768, Om3Q<10, 768>::lds_bytes, 0xBA5EEDull, gstaged,
                0ull, B, (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk, (uint32_t)tpg);
    report("word_epi_12waves", us, 12);
    us = time_k(k_om3q<10, true, 1, 0, 1024>, grid, 1024, Om3Q<10, 1024>::lds_bytes, 0xBA5EEDull, gstaged,
                0ull, B, (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk, (uint32_t)tpg);
    report("word_epi_16waves", us, 16);
    const uint32_t ldsw = 4 * Om3W<10>::words * 8;
    const uint32_t gridw = (uint32_t)std::min<uint64_t>((tasks + 3) / 4, 512);
    const float usw = time_k(k_om3w<10>, gridw, 256, ldsw, 0xBA5EEDull, gstaged, 0ull, B,
                             (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk);
    const float usw2 = time_k(k_om3w<10, 0, true>, gridw, 256, ldsw, 0xBA5EEDull, gstaged, 0ull, B,
                              (const uint32_t*)sf, (const uint8_t*)so, dec, out, cnt, sk);
    const float usw3 = time_k(k_om3w<10, 0, false>, gridw, 256, ldsw, 0xBA5EEDull, gdraw, 0ull, B,
                              (const uint32_t*)nullptr, (const uint8_t*)nullptr, dec, out, cnt, sk);
    printf("{\"om3w_us\": %.2f, \"om3w_staged_specialised_us\": %.2f, \"om3w_drawn_us\": %.2f}\n",
           usw, usw2, usw3);
    return 0;
}
