// writelane_probe.hip -- test-only translation unit (tests/test_lib.py): the
// staged-input k_om3w<10> on its own, so a copy built with
// -DBA_WRITELANE_NOP='""' shows that the code-object hazard check catches a
// writelane4 without its wait states.  Never linked into libba_hip.
#include "../../byzantine-agreement_amd/csrc/ba_wave.hpp"

template __global__ void ba::k_om3w<10, 0, true>(uint64_t, ba::GenSpec, uint64_t, uint64_t,
                                                 const uint32_t*, const uint8_t*, uint64_t*,
                                                 uint8_t*, uint64_t*, ba::Sink);
