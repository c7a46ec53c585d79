// ba_engine.hpp -- internal (C++) interface between the C ABI (ba_api.cpp) and
// the HIP engines.  Nothing here crosses the library boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "ba_device.hpp"

namespace ba {

// Optional per-kernel timing with HIP events recorded on the launch stream
// (ba_profile_enable / ba_profile_read).  Disabled: begin/end are no-ops.
struct Prof {
    struct Rec {
        const char* name;
        hipEvent_t a, b;
    };
    bool on = false;
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    hipStream_t stream = nullptr;
    hipEvent_t take();
    void begin(const char* name, hipStream_t s);
    void end();
};

// One call's resolved arguments; every pointer is a DEVICE pointer.
struct RunArgs {
    uint32_t n = 0, m = 0, me = 0;  // me = effective depth min(m, n-2)
    uint64_t seed = 0;
    uint32_t lie_mode = 0;
    GenSpec gen{};
    uint64_t first_trial = 0;  // global index of trial 0 (multiple of 64)
    uint32_t table_stride = 0;
    uint64_t batch = 0;
    const uint32_t* faulty = nullptr;
    const uint8_t* order = nullptr;
    const uint32_t* table = nullptr;
    const uint32_t* poll = nullptr;
    uint64_t* decisions = nullptr;
    uint8_t* outcome = nullptr;
    uint64_t* counters = nullptr;  // BA_NCOUNTERS, accumulated into
    hipStream_t stream = nullptr;
    Prof* prof = nullptr;
};

struct ProfScope {  // RAII: times one launch when profiling is on
    Prof* p;
    ProfScope(Prof* p_, const char* name, hipStream_t s) : p(p_) {
        if (p && p->on) p->begin(name, s);
    }
    ~ProfScope() {
        if (p && p->on) p->end();
    }
};

// Geometry of the OM(me) tree over L = n-1 lieutenants.  Level k holds one
// slot per (k+1)-permutation of lieutenants in lexicographic rank, so
// parent(x) = x / (L-k) and the children of a slot are contiguous.
struct Geometry {
    uint32_t n = 0, L = 0, me = 0;
    std::vector<uint64_t> S;           // S[k] = P(L, k+1), k = 0..me
    std::vector<uint64_t> sender_off;  // level k (< me): offset into sender[]
    std::vector<uint8_t> sender;       // general index of the last relayer of a slot
    uint64_t slots_total = 0;          // sum_k S[k]
    uint64_t inner_total = 0;          // sum_{1<=p<me} S[p] (inner majority levels)
    bool build(uint32_t n, uint32_t me, uint64_t max_level_slots);
};

// LEVELS engine scratch layout for a chunk of W trial words (uint64 words).
struct LevelsLayout {
    uint64_t W = 0;
    uint64_t F = 0, OB = 0, OO = 0, VAL = 0;
    std::vector<uint64_t> Lk, Rp;  // Rp[p] valid for 1 <= p < me
    uint64_t total = 0;
    void plan(const Geometry& g, uint64_t W);
    static uint64_t words_per_trial_word(const Geometry& g) {
        return g.n + 3 + g.slots_total + g.inner_total;
    }
};

constexpr int kPartialRows = 2048;  // max epilogue blocks per launch

hipError_t launch_table(const RunArgs& a, uint64_t* partials);
hipError_t launch_levels_chunk(const RunArgs& a, const Geometry& g, const uint8_t* d_sender,
                               uint64_t* scratch, const LevelsLayout& lay, uint64_t trial0,
                               uint64_t ntrials, uint64_t* partials);
hipError_t launch_reduce(const uint64_t* partials, int rows, uint64_t* counters, hipStream_t s,
                         Prof* prof);

}  // namespace ba
