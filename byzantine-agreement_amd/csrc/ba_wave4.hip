// ba_wave4.hip -- WAVE engine, effective depth 4 (k_om4w).
#include "ba_wave.hpp"

namespace ba {

hipError_t launch_wave4(const RunArgs& a, const Geometry& g) {
    switch (g.n) {
#define OM4W_CASE(nn) \
    case nn: return launch_wave<Om4W<nn>>(a, k_om4w<nn>, "k_om4w", k_om4w<nn, true>, true);
        OM4W_CASE(6) OM4W_CASE(7) OM4W_CASE(8) OM4W_CASE(9) OM4W_CASE(10) OM4W_CASE(11)
        OM4W_CASE(12) OM4W_CASE(13) OM4W_CASE(14)
#undef OM4W_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ba
