// ba_wave3.hip -- WAVE engine, effective depth 3 (k_om3w), and the engine
// dispatch.
#include "ba_wave.hpp"

// lab A/B builds only (tools/lab_variant.sh -DBA_OM3W_LAB_DIAG=...): k_om3w's DIAG switches
#ifndef BA_OM3W_LAB_DIAG
#define BA_OM3W_LAB_DIAG 0
#endif

namespace ba {

hipError_t launch_wave4(const RunArgs& a, const Geometry& g);  // ba_wave4.hip

// Trees the WAVE kernels are compiled for (k_om3w / k_om4w instantiations).
bool wave_supported(const Geometry& g) {
    return (g.me == 3 && g.n >= 5 && g.n <= 14) || (g.me == 4 && g.n >= 6 && g.n <= kWave4MaxN);
}

hipError_t launch_wave_engine(const RunArgs& a, const Geometry& g) {
    if (g.me == 4) return launch_wave4(a, g);
    if (g.me != 3) return hipErrorInvalidValue;
    // depth 3: k_om3w (the rejected alternatives live in tools/lab_kernels.hpp)
    switch (g.n) {
#define OM3W_CASE(nn) \
    case nn: return launch_wave<Om3W<nn>>(a, k_om3w<nn, BA_OM3W_LAB_DIAG>, "k_om3w", k_om3w<nn, BA_OM3W_LAB_DIAG, true>);
        OM3W_CASE(5) OM3W_CASE(6) OM3W_CASE(7) OM3W_CASE(8) OM3W_CASE(9) OM3W_CASE(10)
        OM3W_CASE(11) OM3W_CASE(12) OM3W_CASE(13) OM3W_CASE(14)
#undef OM3W_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ba
