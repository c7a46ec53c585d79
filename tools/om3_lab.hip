// om3_lab.hip -- diagnostic ablations of the FUSED n=10, m=3 kernel (not the
// product; outputs of the ablated variants are meaningless).  Each variant is
// k_fused3<10> with one stage replaced by a near-free stand-in, so the time a
// stage costs in situ is (baseline - variant).
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/om3_lab tools/om3_lab.hip
//   run:   tools/om3_lab [batch]
#define BA_FUSED_STAMPS 1
#include "../byzantine-agreement_amd/csrc/ba_fused.hip"
#include "../byzantine-agreement_amd/csrc/ba_wave3.hip"
#include "../byzantine-agreement_amd/csrc/ba_wave4.hip"
#include "../byzantine-agreement_amd/csrc/ba_levels.hip"
#include "lab_kernels.hpp"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <vector>

using namespace ba;
void ba::Prof::begin(const char*, hipStream_t) {}
void ba::Prof::end() {}

enum : int { NO_GEN = 1, NO_EPI = 2, CHEAP_LIE = 4, NO_LEAF = 8, NO_BARRIER_C = 16 };

__device__ __forceinline__ void cheap_pair(uint32_t k, uint32_t pair, uint64_t gw, uint64_t& a,
                                           uint64_t& b) {
    const uint32_t x = pair * 0x9E3779B9u ^ k * 0x85EBCA6Bu ^ (uint32_t)gw;
    a = (uint64_t)(x * 0xCC9E2D51u) << 32 | x;
    b = (uint64_t)(x ^ 0x1B873593u) << 32 | (x * 0xE6546B64u);
}

template <int S, int V>
__device__ __forceinline__ void leaf_block_v(uint32_t me, uint64_t seed, uint64_t gw, uint32_t sr,
                                             const uint64_t (&diag)[S], const uint64_t (&Fm)[S],
                                             uint64_t (&R)[S]) {
    constexpr int NL = planes_c(S);
    constexpr int NPAIR = S * (S - 1) / 2;
    Csa<NL> cnt[S];
    static_for<0, S>([&](auto b) { cnt[b()].template add<0>(diag[b()]); });
    const uint32_t pair0 = sr * (uint32_t)NPAIR;
    static_for<0, NPAIR>([&](auto q) {
        uint64_t lw[2];
        if constexpr (V & CHEAP_LIE) cheap_pair(me, pair0 + q(), gw, lw[0], lw[1]);
        else lie_pair(seed, me, pair0 + q(), gw, lw[0], lw[1]);
        static_for<0, 2>([&](auto h) {
            constexpr int e = 2 * q() + h();
            constexpr int a = e / (S - 1);
            constexpr int c = e % (S - 1);
            constexpr int b = c + (c >= a);
            constexpr int K = 1 + a - (b < a ? 1 : 0);
            cnt[b].template add<K>((Fm[a] & lw[h()]) | (~Fm[a] & diag[a]));
        });
    });
    static_for<0, S>([&](auto b) { R[b()] = cnt[b()].template ge<S, S / 2 + 1>(); });
}

template <int N, int V>
__global__ __launch_bounds__(kFusedThreads, 4) void lab3(uint32_t wpb, uint64_t seed, GenSpec gs,
                                                        uint64_t first_trial, uint64_t batch,
                                                        uint64_t* __restrict__ decisions,
                                                        uint8_t* __restrict__ outcome,
                                                        uint64_t* __restrict__ counters) {
    using G = Om3<N>;
    constexpr int L = G::L, S = G::S, S1 = G::S1, STRIDE = G::words;
    constexpr uint32_t ME = 3;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    __shared__ __attribute__((aligned(16))) unsigned long long blockcnt[16];
    const uint32_t T = kFusedThreads, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < 16) blockcnt[tid] = 0;
    const uint64_t total_words = (batch + 63) / 64;
    const uint64_t per_block = (total_words + gridDim.x - 1) / gridDim.x;
    const uint64_t wbeg = (uint64_t)blockIdx.x * per_block;
    const uint64_t wend = wbeg + per_block < total_words ? wbeg + per_block : total_words;
    for (uint64_t w0 = wbeg; w0 < wend; w0 += wpb) {
        const uint32_t nw = (uint32_t)(wend - w0 < wpb ? wend - w0 : wpb);
        const uint64_t gwg = (first_trial >> 6) + w0;
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            uint64_t* img = lds + lw * STRIDE;
            const uint64_t i = (w0 + lw) * 64 + lane;
            const bool valid = i < batch;
            uint32_t fm = 0, oc = 0;
            if (valid) {
                if constexpr (V & NO_GEN) {
                    const uint32_t h = (uint32_t)i * 0x9E3779B9u;
                    fm = (1u << (h >> 28)) | (1u << ((h >> 24) & 7));
                    fm &= (1u << N) - 1;
                    oc = (h >> 3) & 1;
                } else {
                    gen_trial(N, seed, gs, first_trial + i, fm, oc);
                }
            }
            uint64_t mine = 0;
            static_for<0, N>([&](auto g) {
                const uint64_t b = __ballot(valid && ((fm >> g()) & 1u));
                if (lane == g()) mine = b;
            });
            const uint64_t ob = __ballot(valid && oc == 1);
            const uint64_t oo = __ballot(valid && oc == 2);
            const uint64_t vv = __ballot(valid);
            if (lane < N) img[G::oF + lane] = mine;
            if (lane == 0) {
                img[G::oOB] = ob;
                img[G::oOO] = oo;
                img[G::oVAL] = vv;
            }
        }
        __syncthreads();
        {
            constexpr uint32_t NP = S1 / 2;
            for (uint32_t it = tid; it < NP * nw; it += T) {
                const uint32_t lw = it / NP, q = it - lw * NP;
                uint64_t* img = lds + lw * STRIDE;
                const uint64_t gw = gwg + lw;
                const uint64_t F0 = img[G::oF], ob = img[G::oOB];
                uint32_t x[2], y[2];
                x[0] = 2 * q;
                x[1] = 2 * q + 1;
                y[0] = x[0] / (L - 1);
                y[1] = x[1] / (L - 1);
                uint64_t l1a, l1b, p0a, p0b;
                lie_pair(seed, 1, q, gw, l1a, l1b);
                lie_pair(seed, 0, y[0] >> 1, gw, p0a, p0b);
                uint64_t L0v[2];
                L0v[0] = (F0 & ((y[0] & 1) ? p0b : p0a)) | (~F0 & ob);
                L0v[1] = L0v[0];
                const uint64_t lie1[2] = {l1a, l1b};
                static_for<0, 2>([&](auto h) {
                    const uint64_t fj = img[G::oF + y[h()] + 1];
                    img[G::oL1 + x[h()]] = (fj & lie1[h()]) | (~fj & L0v[h()]);
                    img[G::oL0 + y[h()]] = L0v[h()];
                });
            }
        }
        __syncthreads();
        for (uint32_t it = tid; it < (uint32_t)S1 * nw; it += T) {
            const uint32_t lw = it / S1, sr = it - lw * S1;
            uint64_t* img = lds + lw * STRIDE;
            const uint64_t gw = gwg + lw;
            const uint32_t j1 = sr / (L - 1), c = sr - j1 * (L - 1), j2 = c + (c >= j1);
            const uint32_t lo = j1 < j2 ? j1 : j2, hi = j1 < j2 ? j2 : j1;
            const uint64_t par = img[G::oL1 + sr];
            const uint64_t fs = img[G::oF + j2 + 1];
            const uint32_t x0 = sr * S;
            if constexpr (V & NO_LEAF) {
                static_for<0, S>([&](auto b) { img[G::oR2 + x0 + b()] = par ^ fs ^ b(); });
            } else {
                constexpr int NPD = (S + 1) / 2;
                uint64_t lw2[2 * NPD];
                static_for<0, NPD>([&](auto qd) {
                    if constexpr (V & CHEAP_LIE)
                        cheap_pair(2, (x0 >> 1) + qd(), gw, lw2[2 * qd()], lw2[2 * qd() + 1]);
                    else
                        lie_pair(seed, 2, (x0 >> 1) + qd(), gw, lw2[2 * qd()], lw2[2 * qd() + 1]);
                });
                const uint64_t oddmask = 0ull - (uint64_t)(x0 & 1u);
                uint64_t diag[S], Fm[S], R[S];
                static_for<0, S>([&](auto a) {
                    uint64_t lie;
                    if constexpr (S % 2 == 1) lie = lw2[a()] ^ ((lw2[a()] ^ lw2[a() + 1]) & oddmask);
                    else lie = lw2[a()];
                    diag[a()] = (fs & lie) | (~fs & par);
                    const uint32_t ida = a() + (a() >= lo) + (a() + 1 >= hi);
                    Fm[a()] = img[G::oF + ida + 1];
                });
                leaf_block_v<S, V>(ME, seed, gw, sr, diag, Fm, R);
                static_for<0, S>([&](auto b) { img[G::oR2 + x0 + b()] = R[b()]; });
            }
        }
        __syncthreads();
        for (uint32_t it = tid; it < (uint32_t)S1 * nw; it += T) {
            const uint32_t lw = it / S1, y = it - lw * S1;
            uint64_t* img = lds + lw * STRIDE;
            const uint32_t j1 = y / (L - 1), b = y - j1 * (L - 1);
            Count<planes_c(L - 1)> cnt;
            cnt.add(img[G::oL1 + y]);
            const uint32_t base = G::oR2 + j1 * (L - 1) * (L - 2);
            static_for<0, L - 1>([&](auto a) {
                if (a() == b) return;
                cnt.add(img[base + a() * (L - 2) + (a() < b ? b - 1 : b)]);
            });
            img[G::oR1 + y] = cnt.ge((L - 1) / 2 + 1);
        }
        __syncthreads();
        for (uint32_t lw = wv; lw < nw; lw += T / 64) {
            uint64_t* img = lds + lw * STRIDE;
            if (lane < (uint32_t)L) {
                const uint32_t b = lane;
                Count<planes_c(L)> cnt;
                cnt.add(img[G::oL0 + b]);
                static_for<0, L>([&](auto a) {
                    if (a() == b) return;
                    cnt.add(img[G::oR1 + a() * (L - 1) + (a() < b ? b - 1 : b)]);
                });
                const uint64_t att = cnt.ge(L / 2 + 1);
                const uint64_t tie = (L & 1) ? 0ull : (cnt.ge(L / 2) & ~att);
                img[G::oR2 + b] = att;
                img[G::oR2 + L + b] = tie;
            }
            __builtin_amdgcn_wave_barrier();
            const uint64_t w = w0 + lw, i = w * 64 + lane;
            const bool live = (img[G::oVAL] >> lane) & 1ull;
            if constexpr (V & NO_EPI) {
                if (live) decisions[i] = img[G::oR2 + (lane & 15)];
            } else {
                uint32_t A = 0, U = 0, fm = 0;
                static_for<0, L>([&](auto b) {
                    A |= (uint32_t)((img[G::oR2 + b()] >> lane) & 1ull) << (b() + 1);
                    U |= (uint32_t)((img[G::oR2 + L + b()] >> lane) & 1ull) << (b() + 1);
                });
                static_for<0, N>([&](auto g) { fm |= (uint32_t)((img[G::oF + g()] >> lane) & 1ull) << g(); });
                const uint32_t ob = (uint32_t)(img[G::oOB] >> lane) & 1u;
                const uint32_t oo = (uint32_t)(img[G::oOO] >> lane) & 1u;
                const TrialResult r = trial_result(N, ME, fm, oo ? 2u : ob, A, U);
                if (live) {
                    decisions[i] = r.dec;
                    outcome[i] = (uint8_t)r.out;
                }
                wave_counts_add(live, r, blockcnt);
            }
        }
        __syncthreads();
    }
    if (tid < C_NUM && blockcnt[tid]) atomicAdd((unsigned long long*)&counters[tid], blockcnt[tid]);
}

static float time_kernel(void (*k)(uint32_t, uint64_t, GenSpec, uint64_t, uint64_t, uint64_t*,
                                   uint8_t*, uint64_t*),
                         uint32_t grid, uint32_t lds, uint64_t B, uint64_t* dec, uint8_t* out,
                         uint64_t* cnt) {
    GenSpec gs{1, 3, 1, 1};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, 7u, 0xBA5EEDull, gs, 0ull, B, dec, out, cnt);
    (void)hipDeviceSynchronize();
    const int R = 20;
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < R; ++i)
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, 7u, 0xBA5EEDull, gs, 0ull, B, dec, out, cnt);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
    return ms * 1000.f / R;
}

template <typename K, typename... A>
static float time_launch(K k, uint32_t grid, uint32_t lds, A... args) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, args...);
    (void)hipDeviceSynchronize();
    const int R = 20;
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, args...);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
    return ms * 1000.f / R;
}

static Sink g_sink;

static int compare_wave(uint64_t B) {
    if (!g_sink.rep) {
        void* p = nullptr;
        (void)hipMalloc(&p, kSinkBytes);
        (void)hipMemset(p, 0, kSinkBytes);
        g_sink.rep = (unsigned long long*)p;
    }
    uint64_t *d1, *d2, *c1, *c2;
    uint8_t *o1, *o2;
    (void)hipMalloc(&d1, B * 8);
    (void)hipMalloc(&d2, B * 8);
    (void)hipMalloc(&o1, B);
    (void)hipMalloc(&o2, B);
    (void)hipMalloc(&c1, 16 * 8);
    (void)hipMalloc(&c2, 16 * 8);
    (void)hipMemset(c1, 0, 128);
    (void)hipMemset(c2, 0, 128);
    GenSpec gs{1, 3, 1, 1};
    const uint64_t first = 64ull * 12345;
    const uint32_t lds3 = 7 * Om3<10>::words * 8;
    hipLaunchKernelGGL(k_fused3<10>, dim3(1024), dim3(256), lds3, 0, 7u, 0xBA5EEDull, gs, first, B,
                       (const uint32_t*)nullptr, (const uint8_t*)nullptr, d1, o1, c1, g_sink);
    const uint64_t words = (B + 63) / 64, tasks = (words + Om3W<10>::W - 1) / Om3W<10>::W;
    const uint32_t ldsw = 4 * Om3W<10>::words * 8;
    const uint32_t gridw = (uint32_t)((tasks + 3) / 4);
    hipLaunchKernelGGL(k_om3w<10>, dim3(gridw), dim3(256), ldsw, 0, 0xBA5EEDull, gs, first, B,
                       (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h1(B), h2(B), k1(16), k2(16);
    std::vector<uint8_t> p1(B), p2(B);
    (void)hipMemcpy(h1.data(), d1, B * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), d2, B * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(p1.data(), o1, B, hipMemcpyDeviceToHost);
    (void)hipMemcpy(p2.data(), o2, B, hipMemcpyDeviceToHost);
    (void)hipMemcpy(k1.data(), c1, 128, hipMemcpyDeviceToHost);
    (void)hipMemcpy(k2.data(), c2, 128, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < B; ++i) bad += (h1[i] != h2[i]) || (p1[i] != p2[i]);
    int badc = 0;
    for (int i = 0; i < 12; ++i) badc += k1[i] != k2[i];
    printf("{\"compare_wave_vs_fused3\": {\"batch\": %llu, \"mismatched_trials\": %llu, "
           "\"mismatched_counters\": %d, \"trials\": %llu, \"attack_decisions\": %llu}}\n",
           (unsigned long long)B, (unsigned long long)bad, badc, (unsigned long long)k2[0],
           (unsigned long long)k2[11]);
    const float us3 = time_launch(k_fused3<10>, 1024, lds3, 7u, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d1, o1, c1, g_sink);
    const float usw = time_launch(k_om3w<10>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    printf("{\"fused3_us\": %.2f, \"wave_us\": %.2f, \"wave_trials_per_s\": %.4e, \"grid\": %u, \"lds\": %u}\n",
           us3, usw, B / (usw * 1e-6), gridw, ldsw);
    std::vector<unsigned long long> st(kPartialRows * 8);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_fused_stamps), st.size() * 8);
    double ph[6] = {0};
    uint64_t nw = 0;
    for (uint64_t wv = 0; wv < tasks && wv < (uint64_t)kPartialRows; ++wv, ++nw)
        for (int i = 0; i < 5; ++i) ph[i] += (double)st[wv * 8 + i];
    printf("{\"wave_phase_cycles\": {\"gen\": %.0f, \"l0_steps12\": %.0f, \"step3\": %.0f, \"roots\": %.0f, "
           "\"epilogue\": %.0f}}\n", ph[0] / nw, ph[1] / nw, ph[2] / nw, ph[3] / nw, ph[4] / nw);
    unsigned long long r0 = ~0ull, r1 = 0, smax = 0, emin = ~0ull;
    double cyc = 0, rt = 0;
    for (uint64_t wv = 0; wv < nw; ++wv) {
        const unsigned long long a = st[wv * 8 + 6], b = st[wv * 8 + 7];
        r0 = a < r0 ? a : r0;
        r1 = b > r1 ? b : r1;
        smax = a > smax ? a : smax;
        emin = b < emin ? b : emin;
        for (int i = 0; i < 5; ++i) cyc += (double)st[wv * 8 + i];
        rt += (double)(b - a);
    }
    {   // per-CU wave counts and durations (HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13])
        std::vector<std::pair<double, unsigned long long>> d;
        for (uint64_t wv = 0; wv < nw; ++wv) d.push_back({(st[wv * 8 + 7] - st[wv * 8 + 6]) * 0.01, st[wv * 8 + 5]});
        std::sort(d.begin(), d.end());
        std::map<unsigned long long, int> percu, persimd;
        for (auto& x : d) {
            const unsigned long long h = x.second;
            const unsigned long long cu = ((h >> 8) & 15) | ((h >> 12) & 1) << 4 | ((h >> 13) & 7) << 5 | (h >> 32 & 15) << 8;
            percu[cu]++;
            persimd[cu << 2 | ((h >> 4) & 3)]++;
        }
        std::map<int, int> hist_cu, hist_simd;
        for (auto& kv : percu) hist_cu[kv.second]++;
        for (auto& kv : persimd) hist_simd[kv.second]++;
        printf("{\"cus_used\": %zu, \"waves_per_cu_hist\": {", percu.size());
        for (auto& kv : hist_cu) printf("\"%d\": %d, ", kv.first, kv.second);
        printf("}, \"waves_per_simd_hist\": {");
        for (auto& kv : hist_simd) printf("\"%d\": %d, ", kv.first, kv.second);
        printf("}, \"dur_p10\": %.1f, \"dur_p50\": %.1f, \"dur_p90\": %.1f}\n", d[d.size() / 10].first,
               d[d.size() / 2].first, d[d.size() * 9 / 10].first);
        // the two waves of each SIMD: wave slot ids (HW_ID[3:0]) and who finishes first
        std::map<unsigned long long, std::vector<std::pair<int, double>>> bysimd;
        for (auto& x : d) {
            const unsigned long long h = x.second;
            const unsigned long long cu = ((h >> 8) & 15) | ((h >> 12) & 1) << 4 | ((h >> 13) & 7) << 5 | (h >> 32 & 15) << 8;
            bysimd[cu << 2 | ((h >> 4) & 3)].push_back({(int)(h & 15), x.first});
        }
        int pairs = 0, diffpar = 0, lowfirst = 0;
        std::map<int, int> slots;
        for (auto& kv : bysimd) {
            if (kv.second.size() != 2) continue;
            ++pairs;
            auto a = kv.second[0], b = kv.second[1];
            slots[a.first]++;
            slots[b.first]++;
            diffpar += (a.first & 1) != (b.first & 1);
            const auto& fast = a.second < b.second ? a : b;
            const auto& slow = a.second < b.second ? b : a;
            lowfirst += fast.first < slow.first;
        }
        printf("{\"simd_pairs\": %d, \"diff_slot_parity\": %d, \"lower_slot_finishes_first\": %d, \"slot_hist\": {", pairs, diffpar, lowfirst);
        for (auto& kv : slots) printf("\"%d\": %d, ", kv.first, kv.second);
        printf("}}\n");
    }
    printf("{\"clock_ghz\": %.3f, \"span_us\": %.2f, \"start_skew_us\": %.2f, \"first_end_us\": %.2f, "
           "\"mean_wave_us\": %.2f}\n",
           cyc / rt * 0.1, (r1 - r0) * 0.01, (smax - r0) * 0.01, (emin - r0) * 0.01, rt / nw * 0.01);
    const float v1 = time_launch(k_om3w<10, 1>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float v2 = time_launch(k_om3w<10, 2>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float v4 = time_launch(k_om3w<10, 4>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float v7 = time_launch(k_om3w<10, 7>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float vpad = time_launch(k_om3w<10>, gridw, 56u * 1024, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    printf("{\"wave_lds56k_us\": %.2f}\n", vpad);
    const float vprio = time_launch(k_om3w<10, 8>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    printf("{\"wave_prio_fixed_us\": %.2f}\n", vprio);  // DIAG 8: without the alternation
    {
        uint32_t* sf;
        uint8_t* so;
        (void)hipMalloc(&sf, B * 4);
        (void)hipMalloc(&so, B);
        hipLaunchKernelGGL(k_gen_inputs, dim3(2048), dim3(256), 0, 0, 10u, 0xBA5EEDull, gs, 0ull, B, sf, so);
        GenSpec gg{0, 3, 0, 1};
        const float vst = time_launch(k_om3w<10>, gridw, ldsw, 0xBA5EEDull, gg, 0ull, B,
                                      (const uint32_t*)sf, (const uint8_t*)so, d2, o2, c2, g_sink);
        const float vst2 = time_launch(k_om3w<10, 32>, gridw, ldsw, 0xBA5EEDull, gg, 0ull, B,
                                       (const uint32_t*)sf, (const uint8_t*)so, d2, o2, c2, g_sink);
        printf("{\"wave_staged_us\": %.2f, \"wave_staged_no_epi_us\": %.2f}\n", vst, vst2);
        // cold staged inputs: rotate over 64 batches (> the 256 MB Infinity Cache)
        const int NB = 64;
        uint32_t* cf;
        uint8_t* co;
        (void)hipMalloc(&cf, B * 4 * NB);
        (void)hipMalloc(&co, B * NB);
        for (int k = 0; k < NB; ++k)
            hipLaunchKernelGGL(k_gen_inputs, dim3(2048), dim3(256), 0, 0, 10u, 0xBA5EEDull, gs,
                               (uint64_t)k * B, B, cf + k * B, co + k * B);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        for (int k = 0; k < NB; ++k)
            hipLaunchKernelGGL(k_om3w<10>, dim3(gridw), dim3(256), ldsw, 0, 0xBA5EEDull, gg,
                               (uint64_t)k * B, B, (const uint32_t*)(cf + k * B),
                               (const uint8_t*)(co + k * B), d2, o2, c2, g_sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipEventRecord(e0, 0);
        for (int k = 0; k < NB; ++k)
            hipLaunchKernelGGL(k_om3w<10>, dim3(gridw), dim3(256), ldsw, 0, 0xBA5EEDull, gs,
                               (uint64_t)k * B, B, (const uint32_t*)nullptr, (const uint8_t*)nullptr,
                               d2, o2, c2, g_sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms2 = 0;
        (void)hipEventElapsedTime(&ms2, e0, e1);
        printf("{\"wave_staged_cold_us\": %.2f, \"wave_inkernel_same_seq_us\": %.2f}\n", ms * 1000 / NB, ms2 * 1000 / NB);
    }
    const float vng = time_launch(k_om3w<10, 16>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float vne = time_launch(k_om3w<10, 32>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    const float vnn = time_launch(k_om3w<10, 48>, gridw, ldsw, 0xBA5EEDull, gs, 0ull, B,
                                  (const uint32_t*)nullptr, (const uint8_t*)nullptr, d2, o2, c2, g_sink);
    printf("{\"wave_no_gen_us\": %.2f, \"wave_no_epi_us\": %.2f, \"wave_no_gen_no_epi_us\": %.2f}\n", vng, vne, vnn);
    printf("{\"wave_no_dec_us\": %.2f, \"wave_no_out_us\": %.2f, \"wave_no_atomic_us\": %.2f, \"wave_none_us\": %.2f}\n",
           v1, v2, v4, v7);
    return bad || badc;
}

int main(int argc, char** argv) {
    const uint64_t B = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1u << 20);
    uint64_t *dec, *cnt;
    uint8_t* out;
    (void)hipMalloc(&dec, B * 8);
    (void)hipMalloc(&out, B);
    (void)hipMalloc(&cnt, 16 * 8);
    if (argc > 2 && argv[2][0] == 'p') {  // PMC mode: only the WAVE kernel at batch B
        void* sp = nullptr;
        (void)hipMalloc(&sp, kSinkBytes);
        (void)hipMemset(sp, 0, kSinkBytes);
        Sink sk{(unsigned long long*)sp};
        const uint64_t words = (B + 63) / 64, tasks = (words + Om3W<10>::W - 1) / Om3W<10>::W;
        GenSpec gs{1, 3, 1, 1};
        const float us = time_launch(k_om3w<10>, (uint32_t)((tasks + 3) / 4), 4 * Om3W<10>::words * 8,
                                     0xBA5EEDull, gs, 0ull, B, (const uint32_t*)nullptr,
                                     (const uint8_t*)nullptr, dec, out, cnt, sk);
        printf("{\"wave_us\": %.2f}\n", us);
        return 0;
    }
    const uint32_t lds = 7 * Om3<10>::words * 8, grid = 1024;
    struct {
        const char* name;
        void (*k)(uint32_t, uint64_t, GenSpec, uint64_t, uint64_t, uint64_t*, uint8_t*, uint64_t*);
    } vs[] = {{"base", lab3<10, 0>},
              {"no_gen", lab3<10, NO_GEN>},
              {"no_epi", lab3<10, NO_EPI>},
              {"cheap_lie", lab3<10, CHEAP_LIE>},
              {"no_leaf", lab3<10, NO_LEAF>},
              {"no_gen_no_epi", lab3<10, NO_GEN | NO_EPI>},
              {"cheap_no_gen_no_epi", lab3<10, CHEAP_LIE | NO_GEN | NO_EPI>}};
    if (compare_wave(777 * 64 + 13) | compare_wave(B)) printf("MISMATCH\n");
    if (argc > 2) return 0;
    for (auto& v : vs) {
        const float us = time_kernel(v.k, grid, lds, B, dec, out, cnt);
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"trials_per_s\": %.4e}\n", v.name, us, B / (us * 1e-6));
    }
    return 0;
}
