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
    Sink sink{};                   // ctx-owned counter reduction slots (FUSED / WAVE)
    hipStream_t stream = nullptr;
    Prof* prof = nullptr;
    const uint64_t* members = nullptr;  // device copy of Geometry::members
    uint32_t cu_count = 256;            // compute units of the ctx device
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
    // leaf blocks (me >= 2, S = n-me <= 12): for every prefix sigma at level
    // me-2, the general ids of its S members packed 5 bits each, rank order
    std::vector<uint64_t> members;
    bool build(uint32_t n, uint32_t me, uint64_t max_level_slots);
};

// LEVELS engine scratch layout for a chunk of W trial words (uint64 words).
// A level may be restricted to the first-hop subtrees [jb, je) (SURVEY.md
// §8e): level k >= 1 then holds global slots [base[k], base[k] + cnt[k]) with
// base[k] = jb * S[k] / L; level 0 (L slots) is always whole.
struct LevelsLayout {
    uint64_t W = 0;
    // split units [jb, je) at level h-1: first-hop lieutenants (h = 1) or
    // level-1 slots, i.e. second-hop subtrees (h = 2).  Levels < h are whole,
    // except a second-hop tree pass's unit level (level 1: the range only).
    uint32_t jb = 0, je = 0, h = 1;
    uint64_t F = 0, OB = 0, OO = 0, VAL = 0;
    std::vector<uint64_t> Lk, Rp;  // Rp[p] valid for 1 <= p < me
    std::vector<uint64_t> base, cnt;
    uint64_t total = 0;
    bool leaf_fused = false;       // L_{me-1}, L_me not materialised (k_leaf)
    void plan(const Geometry& g, uint64_t W, bool leaf, uint32_t jb, uint32_t je, uint32_t h = 1);
    static uint64_t words_per_trial_word(const Geometry& g, bool leaf, uint32_t jb, uint32_t je,
                                         uint32_t h = 1);
};

// What one LEVELS pass computes.  The default is a whole trial batch.  A
// split at level h runs `tree` on a unit range (first-hop subtrees for h = 1,
// second-hop subtrees for h = 2) and leaves the units' level-h results (R_h,
// or L_1 at depth 1) in votes_out; `root` alone reads the gathered votes of
// every unit (votes_in), relays levels 0..h-1 itself, takes the majorities of
// levels h-1..1 and the root majorities + quorum.
struct LevelsJob {
    bool tree = true, root = true;
    uint32_t h = 1;                      // split level (1: first hop, 2: second hop)
    uint64_t* votes_out = nullptr;       // [ units' level-h slots ][ W ]
    const uint64_t* votes_in = nullptr;  // [ all level-h slots ][ W ]
};

constexpr int kPartialRows = 2048;  // max epilogue blocks per launch
constexpr int kMaxLeafS = 12;       // leaf-fused kernels instantiated for S = n-me in 2..12
constexpr int kFusedMaxDepth = 6;
constexpr uint64_t kFusedLdsBudget = 39 * 1024;  // per block: four blocks per CU
constexpr int kFusedThreads = 256;               // 4 waves: 4 blocks/CU at <= 128 VGPRs
constexpr int kWaveThreads = 256;                // WAVE engine: 4 independent waves per block
constexpr uint32_t kWave4MaxN = 14;              // k_om4w instantiated for 6 <= n <= 14

// LDS image of the FUSED engine (one per 64-trial word, WPB words per block).
struct FusedPlan {
    uint32_t n, me, wpb, threads, word_stride, lds_bytes, offRoot;
    uint32_t S[kFusedMaxDepth + 1];        // level sizes
    uint32_t offL[kFusedMaxDepth + 1];     // L_k, k = 0..me-2
    uint32_t offR[kFusedMaxDepth + 1];     // R_p, p = 1..me-1
    uint32_t snd_off[kFusedMaxDepth + 1];  // sender table offsets, levels 0..me-1
};

bool leaf_supported(const Geometry& g);
bool wave_supported(const Geometry& g);
hipError_t launch_wave_engine(const RunArgs& a, const Geometry& g);
bool plan_fused(const Geometry& g, FusedPlan& fp);
hipError_t launch_leaf(const Geometry& g, uint64_t seed, uint64_t gw0, uint32_t W,
                       uint32_t srbase, uint32_t srcnt, uint32_t lbase, const uint64_t* Lm2,
                       const uint8_t* d_sender, const uint64_t* F, const uint64_t* d_members,
                       uint64_t* Rm1, bool up, hipStream_t st, Prof* prof);
hipError_t launch_fused(const RunArgs& a, const Geometry& g, bool plan_ok, const FusedPlan& fp,
                        const FusedPlan* d_fp, const uint8_t* d_sender, uint64_t* partials);

// LEVELS small-batch tail (ba_tail.hip): level-1 majorities + roots + quorum
// of W <= kTailMaxWords words in one launch (config 5 A/B, one call: -3 us at
// 1 and 16 instances, neutral at 16 words = 1024 instances)
constexpr uint32_t kTailMaxWords = 16;
bool tail_supported(const Geometry& g);
hipError_t launch_tail(const RunArgs& a, const Geometry& g, uint64_t W, const uint64_t* scratch,
                       const LevelsLayout& lay, const uint64_t* L1, const uint64_t* C2,
                       uint32_t c2base, uint64_t* decisions, uint8_t* outcome);

// LEVELS big-batch root + quorum epilogue (ba_tail.hip, >= 64 groups of 64 words)
bool epilogue_w_supported(const Geometry& g);
hipError_t launch_epilogue_w(const RunArgs& a, const Geometry& g, uint64_t W,
                             const uint64_t* scratch, const LevelsLayout& lay, const uint64_t* C1,
                             uint64_t* decisions, uint8_t* outcome);

// LEVELS in one launch (ba_cascade.hip): leaf-up units plus an in-launch
// fan-in cascade of the majority levels above them, roots and quorum
struct CascJob {
    uint32_t h = 0;               // 0: the whole tree; 1 / 2: votes of the h-hop subtrees [ub, ue)
    uint32_t ub = 0, ue = 0;
    uint64_t* votes = nullptr;    // range mode: [(u - ub)(L - h) + c][W] (ba.h, ba_split_votes_device)
    const uint64_t* vin = nullptr;  // root mode: every unit's level-root_h votes (k_cascade_root)
    uint32_t root_h = 0;
    bool two = false;               // two launches: units, then the fan-in (k_cascade_top)
    bool co = false;                // one launch: units + co-resident fan-in blocks (whole tree, me >= 4)
    uint32_t check = 0;           // tests: 1 = epoch tags checked, 2 = and one stale tag injected
    uint64_t epoch = 0;           // check: this launch's tag
    uint64_t wait_ticks = 0;      // granule poll bound (0: the default; BA_TEST_GRANULE_TICKS)
};
bool cascade_supported(const Geometry& g);
bool cascade_check_supported(const Geometry& g);
bool cascade_range_supported(const Geometry& g, uint32_t h);
bool cascade_range_two_supported(const Geometry& g, uint32_t h);
uint64_t cascade_counters_per_word(const Geometry& g);       // 128-B counters per trial word
uint64_t cascade_scratch_words_per_word(const Geometry& g, bool co = false);  // R_1..R_{me-2} words per trial word (x2 with check tags)
bool cascade_root_pass_uses_scratch();                       // false: k_cascade_wtop (the default)
hipError_t launch_cascade(const RunArgs& a, const Geometry& g, const uint8_t* d_sender,
                          uint64_t* scratch, uint32_t* d_cnt, uint64_t trial0, uint64_t ntrials,
                          const CascJob& job);

hipError_t launch_table(const RunArgs& a, uint64_t* partials);
hipError_t launch_gen_inputs(const RunArgs& a, uint32_t* faulty_out, uint8_t* order_out);
// ba_mtdev.hip: ba.py's coin table on the device (ba_mt_table_device)
uint64_t mt_table_state_bytes_per_trial();
uint64_t mt_table_state_rows(uint64_t T);  // row length of the chunk's state: T rounded up to the kernel's blocks
hipError_t launch_mt_table(uint32_t n, uint32_t m, uint64_t T, const uint64_t* seeds,
                           const uint32_t* faulty, const uint32_t* poll, uint32_t stride,
                           uint32_t* table, uint32_t* next_word, uint32_t* state, hipStream_t s,
                           Prof* prof);
hipError_t launch_levels_chunk(const RunArgs& a, const Geometry& g, const uint8_t* d_sender,
                               uint64_t* scratch, const LevelsLayout& lay, uint64_t trial0,
                               uint64_t ntrials, uint64_t* partials, const LevelsJob& job);
hipError_t launch_reduce(const uint64_t* partials, int rows, uint64_t* counters, hipStream_t s,
                         Prof* prof);

}  // namespace ba
