// ba_wave3.hip -- WAVE engine, effective depth 3 (k_om3w), and the engine
// dispatch.
#include "ba_wave.hpp"

namespace ba {

hipError_t launch_wave4(const RunArgs& a, const Geometry& g);  // ba_wave4.hip

// Trees the WAVE kernels are compiled for (k_om3w / k_om4w instantiations).
bool wave_supported(const Geometry& g) {
    return (g.me == 3 && g.n >= 5 && g.n <= 14) || (g.me == 4 && g.n >= 6 && g.n <= kWave4MaxN);
}

// k_om3h: units = 2 per task, dynamic assignment from the ctx's task counter
template <int N, int P>
static hipError_t launch_om3h(const RunArgs& a) {
    using G = Om3W<N>;
    constexpr uint32_t wpb = kWaveThreads / 64;
    const uint64_t words = (a.batch + 63) / 64, units = P * ((words + G::W - 1) / G::W);
    uint64_t blocks = (units + wpb - 1) / wpb;
    uint64_t cap = (uint64_t)G::BPC * a.cu_count;
    if (const char* e = getenv("BA_WAVE_MAX_BLOCKS")) {  // tests: force the persistent unit loop
        const uint64_t c = strtoull(e, nullptr, 0);
        if (c >= 1 && c < cap) cap = c;
    }
    if (blocks > cap) blocks = cap;
    Sink sk = a.sink;
    if (units <= blocks * wpb || sk.tasks == nullptr) {
        sk.tasks = nullptr;
    } else {
        const hipError_t e = hipMemsetAsync(sk.tasks, 0, sizeof(unsigned int), a.stream);
        if (e != hipSuccess) return e;
    }
    ProfScope ps(a.prof, "k_om3h", a.stream);
    hipLaunchKernelGGL((k_om3h<N, P>), dim3((uint32_t)blocks), dim3(kWaveThreads), wpb * G::words * 8,
                       a.stream, a.seed, a.gen, a.first_trial, a.batch, a.faulty, a.order,
                       a.decisions, a.outcome, a.counters, sk, a.wave_xch, a.wave_cnt);
    return hipGetLastError();
}

bool wave_split_wanted(const RunArgs& a, const Geometry& g) {
    const char* e = getenv("BA_WAVE_SPLIT");  // read per call (tests and A/B switch it)
    return e && (atoi(e) == 2 || atoi(e) == 3 || atoi(e) == 1) && g.me == 3 && g.n >= 5 && g.n <= 14 && a.gen.faulty_mode == 0 &&
           a.gen.order_mode == 0 && a.faulty && a.order;
}
uint32_t wave_split_parts() {
    const char* e = getenv("BA_WAVE_SPLIT");
    return e && atoi(e) == 3 ? 3u : 2u;  // BA_WAVE_SPLIT=1 or 2: halves; 3: thirds
}
uint64_t wave_split_tasks(const Geometry& g, uint64_t batch) {
    const uint64_t C = g.L - 1, W = 64 / C;
    return ((batch + 63) / 64 + W - 1) / W;
}
uint64_t wave_split_xch_words(const Geometry& g, uint64_t batch) {
    const uint64_t C = g.L - 1, W = 64 / C;
    return wave_split_tasks(g, batch) * W * g.L * g.L;
}

hipError_t launch_wave_engine(const RunArgs& a, const Geometry& g) {
    if (g.me == 4) return launch_wave4(a, g);
    if (g.me != 3) return hipErrorInvalidValue;
    if (a.wave_xch && a.wave_cnt && a.faulty && a.order) {
        switch (g.n) {
#define OM3H_CASE(nn) \
    case nn: return a.wave_parts == 3 ? launch_om3h<nn, 3>(a) : launch_om3h<nn, 2>(a);
            OM3H_CASE(5) OM3H_CASE(6) OM3H_CASE(7) OM3H_CASE(8) OM3H_CASE(9) OM3H_CASE(10)
            OM3H_CASE(11) OM3H_CASE(12) OM3H_CASE(13) OM3H_CASE(14)
#undef OM3H_CASE
            default: return hipErrorInvalidValue;
        }
    }
    // depth 3: k_om3w; BA_WAVE_KIND=2 selects the block-queue kernel k_om3q (A/B,
    // cross-checks: DESIGN.md §4 on why the queue did not pay)
    const char* kind = getenv("BA_WAVE_KIND");
    if (kind && kind[0] == '2') {
        switch (g.n) {
#define OM3Q_CASE(nn) \
    case nn: return launch_om3q<nn>(a);
            OM3Q_CASE(5) OM3Q_CASE(6) OM3Q_CASE(7) OM3Q_CASE(8) OM3Q_CASE(9) OM3Q_CASE(10)
            OM3Q_CASE(11) OM3Q_CASE(12) OM3Q_CASE(13) OM3Q_CASE(14)
#undef OM3Q_CASE
            default: return hipErrorInvalidValue;
        }
    }
    switch (g.n) {
#define OM3W_CASE(nn) \
    case nn: return launch_wave<Om3W<nn>>(a, k_om3w<nn>, "k_om3w", k_om3w<nn, 0, true>);
        OM3W_CASE(5) OM3W_CASE(6) OM3W_CASE(7) OM3W_CASE(8) OM3W_CASE(9) OM3W_CASE(10)
        OM3W_CASE(11) OM3W_CASE(12) OM3W_CASE(13) OM3W_CASE(14)
#undef OM3W_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ba
