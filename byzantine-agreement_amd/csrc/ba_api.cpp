// ba_api.cpp -- the C ABI of libba_hip.so (include/ba.h).
//
// Validation, context/device-memory ownership, engine selection and chunking
// live here; the arithmetic lives in the HIP engines.  There is no CPU compute
// path: without a HIP device every entry point fails with BA_EDEVICE.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ba.h"
#include "ba_engine.hpp"

using namespace ba;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// ba_multi.cpp reports its errors through the same thread-local message
extern "C" int ba_fail_internal(int code, const char* msg) { return fail(code, "%s", msg); }

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess)                                                         \
            return fail(BA_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(_e));   \
    } while (0)

// ---------------------------------------------------------------------------
// geometry
// ---------------------------------------------------------------------------
static uint64_t perm_count(uint32_t L, uint32_t len) {
    uint64_t p = 1;
    for (uint32_t i = 0; i < len; ++i) {
        if (L < i + 1) return 0;
        p *= (uint64_t)(L - i);
        if (p > (1ull << 40)) return 1ull << 40;  // saturate: far beyond any engine
    }
    return p;
}

static uint32_t effective_depth(uint32_t n, uint32_t m) {
    if (n < 2) return 0;
    return m < n - 2 ? m : n - 2;
}

namespace ba {
bool Geometry::build(uint32_t n_, uint32_t me_, uint64_t max_level_slots) {
    n = n_;
    L = n_ - 1;
    me = me_;
    S.assign(me + 1, 0);
    slots_total = inner_total = 0;
    for (uint32_t k = 0; k <= me; ++k) {
        S[k] = perm_count(L, k + 1);
        if (S[k] > max_level_slots) return false;
        slots_total += S[k];
        if (k >= 1 && k < me) inner_total += S[k];
    }
    // sender table: general index of the last relayer of every slot at levels
    // 0..me-1 (lexicographic DFS visits each level's slots in rank order).
    sender_off.assign(me, 0);
    uint64_t off = 0;
    for (uint32_t k = 0; k < me; ++k) {
        sender_off[k] = off;
        off += S[k];
    }
    sender.assign(off, 0);
    std::vector<uint64_t> fill(me, 0);
    // iterative DFS over relay paths of length 1..me in lexicographic order
    std::vector<uint32_t> next(me + 1, 0);
    std::vector<uint32_t> usedv(me + 1, 0);
    if (me > 0) {
        uint32_t depth = 0;
        usedv[0] = 0;
        next[0] = 0;
        while (true) {
            // find next candidate at this depth
            uint32_t c = next[depth];
            while (c < L && ((usedv[depth] >> c) & 1u)) ++c;
            if (c >= L) {
                if (depth == 0) break;
                --depth;
                continue;
            }
            next[depth] = c + 1;
            // path of length depth+1 ending in c -> slot of level `depth`
            sender[sender_off[depth] + fill[depth]++] = (uint8_t)(c + 1);
            if (depth + 1 < me) {
                usedv[depth + 1] = usedv[depth] | (1u << c);
                next[depth + 1] = 0;
                ++depth;
            }
        }
    }
    members.clear();
    const uint32_t S_leaf = n - me;
    if (me >= 2 && S_leaf <= 12) {
        members.assign(S[me - 2], 0);
        for (uint64_t sr = 0; sr < S[me - 2]; ++sr) {
            uint64_t packed = 0;
            for (uint32_t a = 0; a < S_leaf; ++a)
                packed |= (uint64_t)sender[sender_off[me - 1] + sr * S_leaf + a] << (5 * a);
            members[sr] = packed;
        }
    }
    return true;
}

void LevelsLayout::plan(const Geometry& g, uint64_t W_, bool leaf, uint32_t jb_, uint32_t je_,
                        uint32_t h_) {
    W = W_;
    jb = jb_;
    je = je_;
    h = h_;
    leaf_fused = leaf;
    base.assign(g.me + 1, 0);
    cnt.assign(g.me + 1, 0);
    for (uint32_t k = 0; k <= g.me; ++k) {
        if (k + 1 == h && h >= 2 && je > jb) {
            base[k] = jb;  // a second-hop tree pass: the units themselves (level-1 slots)
            cnt[k] = je - jb;
        } else if (k < h) {
            cnt[k] = g.S[k];  // levels above the split (and a root pass's levels < h): whole
        } else {
            const uint64_t q = g.S[k] / g.S[h - 1];  // slots per unit (a level h-1 slot)
            base[k] = (uint64_t)jb * q;
            cnt[k] = (uint64_t)(je - jb) * q;
        }
    }
    uint64_t o = 0;
    F = o; o += (uint64_t)g.n * W;
    OB = o; o += W;
    OO = o; o += W;
    VAL = o; o += W;
    Lk.assign(g.me + 1, 0);
    for (uint32_t k = 0; k <= g.me; ++k) {
        if (leaf && k + 1 >= g.me) break;  // L_{me-1}, L_me generated on the fly by k_leaf
        Lk[k] = o;
        o += cnt[k] * W;
    }
    Rp.assign(g.me + 1, 0);
    for (uint32_t p = 1; p < g.me; ++p) { Rp[p] = o; o += cnt[p] * W; }
    total = o;
}

uint64_t LevelsLayout::words_per_trial_word(const Geometry& g, bool leaf, uint32_t jb, uint32_t je,
                                            uint32_t h) {
    LevelsLayout l;
    l.plan(g, 1, leaf, jb, je, h);
    return l.total;
}
}  // namespace ba

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int grow(size_t need) {
        if (need <= bytes) return BA_OK;
        // kernels queued on any stream may still use the old buffer
        if (p) {
            (void)hipDeviceSynchronize();
            (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
        if (need == 0) return BA_OK;
        hipError_t e = hipMalloc(&p, need);
        if (e != hipSuccess)
            return fail(BA_ENOMEM, "hipMalloc(%zu) failed: %s", need, hipGetErrorString(e));
        bytes = need;
        return BA_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct GeoEntry {
    Geometry g;
    DevBuf sender;
    bool fused_ok = false;  // some FUSED kernel (WAVE or block) runs this tree
    bool plan_ok = false;   // the generic block kernel's LDS plan fits
    FusedPlan fp{};
    DevBuf fplan;    // device copy of fp (k_fused reads it through a pointer)
    DevBuf members;  // device copy of g.members
};

struct ProfTotal {
    uint64_t launches = 0;
    double ms = 0.0;
};

struct ba_ctx {
    int device = 0;
    uint32_t cu_count = 256;
    hipStream_t stream = nullptr;
    size_t scratch_budget = 8ull << 30;
    bool leaf_fusion = true;  // LEVELS uses k_leaf when available (BA_NO_LEAF_FUSION=1: off)
    DevBuf scratch, partials, io_faulty, io_order, io_table, io_poll, io_dec, io_out, io_cnt;
    DevBuf sink;  // counter sink replicas (zeroed once; kernels leave them zero)
    DevBuf casc;  // k_cascade's fan-in counters (zeroed when grown; kernels leave them zero)
    uint64_t casc_epoch = 0x5eed0000;  // k_cascade check builds: one tag per launch
    std::map<uint64_t, std::unique_ptr<GeoEntry>> geos;
    Prof prof;
    std::map<std::string, ProfTotal> prof_totals;
    // Stream ordering of the calls that share the ctx's scratch and counter sink:
    // the event marks the end of the last such call, on last_stream.
    hipEvent_t last_ev = nullptr;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    // CO cascade launches of this ctx that may still run (co_admit): the
    // stream of the last one and the polling blocks of the largest since the
    // stream was last seen idle.  Guarded by co_registry().mu.
    hipStream_t co_stream = nullptr;
    uint64_t co_pending = 0;
};

// Every live ctx, for the CO launch admission (co_admit).
struct CoRegistry {
    std::mutex mu;
    std::vector<ba_ctx*> ctxs;
};
static CoRegistry& co_registry() {
    static CoRegistry r;
    return r;
}

// A call about to use the ctx's scratch / sink on stream `s` first waits for
// the ctx's previous call if that ran on another stream (include/ba.h: calls of
// one ctx may come from any streams; the library orders them itself).  The
// ordering event is recorded on the previous call's stream only at that switch:
// it then follows everything queued there, the previous call included.  A
// record after EVERY call would cost every call's stream ~1.3-3 us before its
// next kernel (tools/marker_cost.hip: +3.0 us per launch for a DisableTiming
// event, +1.3 us without the system-scope fence; bench.py 1M trials 59.8 ->
// 57.0 us per step without it), which the single-stream case never needs.
// Skipped while `s` is capturing a graph: the replay's ordering is the caller's.
// The ctx's own stream (it lives as long as the ctx).  Library-internal: the
// communicators of ba_multi.cpp run their whole jobs on it, so the stream the
// ctx's ordering may record on never dies before the ctx does.
extern "C" __attribute__((visibility("hidden"))) hipStream_t ba_ctx_stream_internal(ba_ctx* ctx) {
    return ctx->stream;
}

static bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

static hipError_t ctx_order(ba_ctx* ctx, hipStream_t s) {
    if (!ctx->have_last || ctx->last_stream == s || stream_capturing(s)) return hipSuccess;
    hipError_t e = hipEventRecord(ctx->last_ev, ctx->last_stream);
    return e == hipSuccess ? hipStreamWaitEvent(s, ctx->last_ev, 0) : e;
}

static hipError_t ctx_mark(ba_ctx* ctx, hipStream_t s) {
    if (!stream_capturing(s)) {
        ctx->last_stream = s;
        ctx->have_last = true;
    }
    return hipSuccess;
}

namespace ba {
hipEvent_t Prof::take() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventReleaseToDevice);  // timing only: no system-scope fence
    return e;
}
void Prof::begin(const char* name, hipStream_t s) {
    stream = s;
    Rec r{name, take(), take()};
    (void)hipEventRecord(r.a, s);
    pending.push_back(r);
}
void Prof::end() { (void)hipEventRecord(pending.back().b, stream); }
}  // namespace ba

// Drain recorded events into per-kernel totals (synchronises on the events).
static void prof_collect(ba_ctx* ctx) {
    for (auto& r : ctx->prof.pending) {
        (void)hipEventSynchronize(r.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            ProfTotal& t = ctx->prof_totals[r.name];
            t.launches += 1;
            t.ms += ms;
        }
        ctx->prof.pool.push_back(r.a);
        ctx->prof.pool.push_back(r.b);
    }
    ctx->prof.pending.clear();
}

extern "C" int ba_profile_enable(ba_ctx* ctx, int on) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    prof_collect(ctx);
    ctx->prof_totals.clear();
    ctx->prof.on = on != 0;
    return BA_OK;
}

extern "C" int ba_profile_read(ba_ctx* ctx, int index, char* name, int name_len,
                               uint64_t* launches, double* total_ms) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    prof_collect(ctx);
    if (index < 0 || index >= (int)ctx->prof_totals.size())
        return fail(BA_EINVAL, "profile index %d out of range", index);
    auto it = ctx->prof_totals.begin();
    std::advance(it, index);
    if (name && name_len > 0) snprintf(name, (size_t)name_len, "%s", it->first.c_str());
    if (launches) *launches = it->second.launches;
    if (total_ms) *total_ms = it->second.ms;
    return BA_OK;
}

extern "C" int ba_version(void) { return BA_ABI_VERSION; }

extern "C" const char* ba_last_error(void) { return g_err.c_str(); }

extern "C" int ba_device_count(int* count) {
    if (!count) return fail(BA_EINVAL, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *count = 0;
        return fail(BA_EDEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = c;
    return BA_OK;
}

extern "C" int ba_ctx_create(int device, ba_ctx** out) {
    if (!out) return fail(BA_EINVAL, "out is NULL");
    *out = nullptr;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c == 0)
        return fail(BA_EDEVICE, "no HIP device visible (libba_hip has no CPU path)");
    if (device < 0 || device >= c) return fail(BA_EINVAL, "device %d out of range [0,%d)", device, c);
    HIP_TRY(hipSetDevice(device));
    auto* ctx = new ba_ctx();
    ctx->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        ctx->cu_count = (uint32_t)cus;
    if (const char* s = getenv("BA_SCRATCH_BYTES")) ctx->scratch_budget = strtoull(s, nullptr, 0);
    if (const char* s = getenv("BA_NO_LEAF_FUSION")) ctx->leaf_fusion = strcmp(s, "1") != 0;
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->last_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return fail(BA_EDEVICE, "hipStreamCreate/hipEventCreate: %s", hipGetErrorString(e));
    }
    if (ctx->sink.grow(kSinkBytes + kSinkTaskCounterBytes) != BA_OK ||
        hipMemset(ctx->sink.p, 0, kSinkBytes + kSinkTaskCounterBytes) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        (void)hipStreamDestroy(ctx->stream);
        (void)hipEventDestroy(ctx->last_ev);
        ctx->sink.release();
        delete ctx;
        return fail(BA_ENOMEM, "counter sink allocation failed");
    }
    {
        std::lock_guard<std::mutex> lk(co_registry().mu);
        co_registry().ctxs.push_back(ctx);
    }
    *out = ctx;
    return BA_OK;
}

extern "C" int ba_ctx_device(ba_ctx* ctx, int* device) {
    if (!ctx || !device) return fail(BA_EINVAL, "ctx and device are required");
    *device = ctx->device;
    return BA_OK;
}

namespace ba {
hipError_t launch_clock_probe(uint64_t* d_out, uint32_t blocks, hipStream_t st);  // ba_probe.hip
}

extern "C" int ba_clock_probe_device(ba_ctx* ctx, uint64_t* d_out, void* stream) {
    if (!ctx || !d_out) return fail(BA_EINVAL, "ctx and d_out are required");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(ba::launch_clock_probe(d_out, BA_PROBE_BLOCKS, stream ? (hipStream_t)stream : ctx->stream));
    return BA_OK;
}

extern "C" int ba_ctx_memory(ba_ctx* ctx, uint64_t* scratch_bytes, uint64_t* counter_bytes,
                             uint64_t* budget_bytes) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    if (scratch_bytes) *scratch_bytes = ctx->scratch.bytes;
    if (counter_bytes) *counter_bytes = ctx->casc.bytes;
    if (budget_bytes) *budget_bytes = ctx->scratch_budget;
    return BA_OK;
}

extern "C" int ba_ctx_stream(ba_ctx* ctx, void** stream) {
    if (!ctx || !stream) return fail(BA_EINVAL, "ctx and stream are required");
    *stream = (void*)ctx->stream;
    return BA_OK;
}

extern "C" void ba_ctx_destroy(ba_ctx* ctx) {
    if (!ctx) return;
    {
        std::lock_guard<std::mutex> lk(co_registry().mu);
        auto& v = co_registry().ctxs;
        v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
    }
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    prof_collect(ctx);
    for (hipEvent_t e : ctx->prof.pool) (void)hipEventDestroy(e);
    for (DevBuf* b : {&ctx->sink, &ctx->casc, &ctx->scratch, &ctx->partials, &ctx->io_faulty, &ctx->io_order, &ctx->io_table,
                      &ctx->io_poll, &ctx->io_dec, &ctx->io_out, &ctx->io_cnt})
        b->release();
    for (auto& kv : ctx->geos) {
        kv.second->sender.release();
        kv.second->fplan.release();
        kv.second->members.release();
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->last_ev) (void)hipEventDestroy(ctx->last_ev);
    delete ctx;
}

extern "C" uint64_t ba_level_slots(uint32_t n, uint32_t m, uint32_t k) {
    if (n < 1 || n > BA_MAX_GENERALS) return 0;
    if (k > effective_depth(n, m)) return 0;
    return perm_count(n - 1, k + 1);
}

extern "C" uint64_t ba_tree_slots(uint32_t n, uint32_t m) {
    if (n < 1 || n > BA_MAX_GENERALS) return 0;
    uint64_t s = 0;
    const uint32_t me = effective_depth(n, m);
    for (uint32_t k = 0; k <= me; ++k) s += perm_count(n - 1, k + 1);
    return s;
}

extern "C" int ba_engine_for(uint32_t n, uint32_t m) {
    if (n < 1 || n > BA_MAX_GENERALS || m > BA_MAX_DEPTH) return fail(BA_EINVAL, "n=%u m=%u", n, m);
    Geometry g;
    if (!g.build(n, effective_depth(n, m), 1ull << 31)) return BA_ENGINE_LEVELS;
    FusedPlan fp;
    return (wave_supported(g) || plan_fused(g, fp)) ? BA_ENGINE_FUSED : BA_ENGINE_LEVELS;
}

// ---------------------------------------------------------------------------
// validation
// ---------------------------------------------------------------------------
static int validate(const ba_params* p, uint64_t batch, bool has_faulty, bool has_order,
                    bool has_table) {
    if (!p) return fail(BA_EINVAL, "params is NULL");
    if (p->n < 1 || p->n > BA_MAX_GENERALS) return fail(BA_EINVAL, "n=%u outside [1,%d]", p->n, BA_MAX_GENERALS);
    if (p->m > BA_MAX_DEPTH) return fail(BA_EINVAL, "m=%u > %d", p->m, BA_MAX_DEPTH);
    if (p->lie_mode > BA_LIE_TABLE) return fail(BA_EINVAL, "lie_mode=%u", p->lie_mode);
    if (p->faulty_mode > BA_FAULTY_EXACT) return fail(BA_EINVAL, "faulty_mode=%u", p->faulty_mode);
    if (p->order_mode > BA_ORDER_CONST) return fail(BA_EINVAL, "order_mode=%u", p->order_mode);
    if (p->order_mode == BA_ORDER_CONST && p->order_value > BA_OTHER)
        return fail(BA_EINVAL, "order_value=%u", p->order_value);
    if (p->faulty_mode == BA_FAULTY_EXACT && p->f > p->n)
        return fail(BA_EINVAL, "exact f=%u > n=%u", p->f, p->n);
    if (p->engine > BA_ENGINE_LEVELS) return fail(BA_EINVAL, "engine=%u", p->engine);
    if (p->first_trial & 63) return fail(BA_EINVAL, "first_trial must be a multiple of 64");
    if (batch && p->faulty_mode == BA_FAULTY_GIVEN && !has_faulty)
        return fail(BA_EINVAL, "BA_FAULTY_GIVEN needs faulty_mask");
    if (batch && p->order_mode == BA_ORDER_GIVEN && !has_order)
        return fail(BA_EINVAL, "BA_ORDER_GIVEN needs order");
    if (p->lie_mode == BA_LIE_TABLE) {
        if (effective_depth(p->n, p->m) > 1)
            return fail(BA_ENOTSUP, "table (ba.py draw-order) mode exists for OM(1) only");
        const uint64_t L = p->n - 1, coins = L + L * L;
        if ((uint64_t)p->table_stride * 32 < coins)
            return fail(BA_EINVAL, "table_stride=%u words < %llu coins", p->table_stride,
                        (unsigned long long)coins);
        if (batch && !has_table) return fail(BA_EINVAL, "BA_LIE_TABLE needs lie_table");
    }
    return BA_OK;
}

// ba_multi.cpp validates a whole job on every rank before its collectives
extern "C" int ba_validate_internal(const ba_params* p, uint64_t batch) {
    return validate(p, batch, true, true, true);
}

static GeoEntry* geometry(ba_ctx* ctx, uint32_t n, uint32_t me, int* rc) {
    const uint64_t key = (uint64_t)n << 8 | me;
    auto it = ctx->geos.find(key);
    if (it != ctx->geos.end()) return it->second.get();
    auto ge = std::make_unique<GeoEntry>();
    if (!ge->g.build(n, me, 1ull << 31)) {
        *rc = fail(BA_ETOOBIG, "OM(%u) tree over %u generals has a level above 2^31 slots", me, n);
        return nullptr;
    }
    if (!ge->g.sender.empty()) {
        if ((*rc = ge->sender.grow(ge->g.sender.size())) != BA_OK) return nullptr;
        hipError_t e = hipMemcpy(ge->sender.p, ge->g.sender.data(), ge->g.sender.size(),
                                 hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            *rc = fail(BA_EDEVICE, "sender upload: %s", hipGetErrorString(e));
            return nullptr;
        }
    }
    if (!ge->g.members.empty()) {
        const size_t mb = ge->g.members.size() * sizeof(uint64_t);
        if ((*rc = ge->members.grow(mb)) != BA_OK) return nullptr;
        hipError_t e = hipMemcpy(ge->members.p, ge->g.members.data(), mb, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            *rc = fail(BA_EDEVICE, "members upload: %s", hipGetErrorString(e));
            return nullptr;
        }
    }
    ge->plan_ok = plan_fused(ge->g, ge->fp);
    ge->fused_ok = ge->plan_ok || wave_supported(ge->g);
    if (ge->plan_ok) {
        if ((*rc = ge->fplan.grow(sizeof(FusedPlan))) != BA_OK) return nullptr;
        hipError_t e = hipMemcpy(ge->fplan.p, &ge->fp, sizeof(FusedPlan), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            *rc = fail(BA_EDEVICE, "plan upload: %s", hipGetErrorString(e));
            return nullptr;
        }
    }
    GeoEntry* raw = ge.get();
    ctx->geos.emplace(key, std::move(ge));
    return raw;
}

// ---------------------------------------------------------------------------
// device entry points
// ---------------------------------------------------------------------------
static RunArgs make_args(ba_ctx* ctx, const ba_params* p, uint64_t batch, const uint32_t* d_faulty,
                         const uint8_t* d_order, const uint32_t* d_table, const uint32_t* d_poll,
                         uint64_t* d_decisions, uint8_t* d_outcome, uint64_t* d_counters,
                         void* stream) {
    RunArgs a;
    a.n = p->n;
    a.m = p->m;
    a.me = effective_depth(p->n, p->m);
    a.seed = p->seed;
    a.lie_mode = p->lie_mode;
    a.gen = GenSpec{p->faulty_mode, p->f, p->order_mode, p->order_value};
    a.first_trial = p->first_trial;
    a.table_stride = p->table_stride;
    a.batch = batch;
    a.faulty = p->faulty_mode == BA_FAULTY_GIVEN ? d_faulty : nullptr;
    a.order = p->order_mode == BA_ORDER_GIVEN ? d_order : nullptr;
    a.table = d_table;
    a.poll = d_poll;
    a.decisions = d_decisions;
    a.outcome = d_outcome;
    a.counters = d_counters;
    a.stream = (hipStream_t)stream;  // NULL = HIP's null stream (HIP convention)
    a.prof = &ctx->prof;
    a.cu_count = ctx->cu_count;
    a.sink.rep = (unsigned long long*)ctx->sink.p;
    a.sink.tasks = (unsigned int*)((char*)ctx->sink.p + kSinkBytes);
    return a;
}

// LEVELS over the first-hop subtrees [jb, je): chunk the batch so the scratch
// fits the budget and 32-bit indices hold.  `whole` = one chunk or BA_ETOOBIG
// (the subtree/vote entry points keep one vote stride for the whole batch).
static int run_levels(ba_ctx* ctx, const RunArgs& a, GeoEntry* ge, const LevelsJob& job,
                      uint32_t jb, uint32_t je, bool whole, uint64_t* partials) {
    const Geometry& g = ge->g;
    const bool leaf = ctx->leaf_fusion && leaf_supported(g);
    const uint64_t per_word = LevelsLayout::words_per_trial_word(g, leaf, jb, je, job.h) * sizeof(uint64_t);
    uint64_t max_level = 0;
    for (uint64_t s : g.S) max_level = s > max_level ? s : max_level;
    const uint64_t words = (a.batch + 63) / 64;
    uint64_t chunk = ctx->scratch_budget / per_word;
    const uint64_t idx_cap = (1ull << 31) / (max_level + 1);
    if (chunk > idx_cap) chunk = idx_cap;
    if (chunk > words) chunk = words;
    if (chunk == 0 || (whole && chunk < words))
        return fail(BA_ETOOBIG, "%llu 64-trial words need %llu bytes of scratch each (budget %zu%s)",
                    (unsigned long long)words, (unsigned long long)per_word, ctx->scratch_budget,
                    whole ? ", one chunk required: split the batch" : "");
    LevelsLayout lay;
    lay.plan(g, chunk, leaf, jb, je, job.h);
    int rc;
    if ((rc = ctx->scratch.grow(lay.total * sizeof(uint64_t))) != BA_OK) return rc;
    for (uint64_t w0 = 0; w0 < words; w0 += chunk) {
        const uint64_t wn = (words - w0) < chunk ? (words - w0) : chunk;
        const uint64_t trial0 = w0 * 64;
        const uint64_t nt = (a.batch - trial0) < wn * 64 ? (a.batch - trial0) : wn * 64;
        LevelsLayout cl;
        cl.plan(g, wn, leaf, jb, je, job.h);
        HIP_TRY(launch_levels_chunk(a, g, (const uint8_t*)ge->sender.p, (uint64_t*)ctx->scratch.p,
                                    cl, trial0, nt, partials, job));
    }
    return BA_OK;
}

// LEVELS in one launch per chunk (k_cascade, ba_cascade.hip): chunked like
// run_levels, with its own scratch plan (R_1 .. R_{me-2}, word-major) and the
// ctx's fan-in counters.  BA_NO_CASCADE=1 keeps the multi-launch pipeline (A/B).
static bool use_cascade(ba_ctx* ctx, const Geometry& g) {
    const char* e = getenv("BA_NO_CASCADE");  // read per call: tests switch it in-process
    const bool off = e && atoi(e) != 0;
    return !off && ctx->leaf_fusion && leaf_supported(g) && g.me >= 3 && cascade_supported(g);
}

constexpr uint64_t kCascTwoWords = 1;
constexpr uint64_t kCascCoWords = 4;

// BA_CASC_CHECK (tests only, read per call): 1 = the cascade's check build
// (epoch tags beside every hand-off word, mismatches counted into
// BA_C_CHECK_MISMATCH), 2 = the same with one stale tag injected.
static uint32_t cascade_check_mode(const Geometry& g) {
    const char* e = getenv("BA_CASC_CHECK");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2) && cascade_check_supported(g) ? (uint32_t)v : 0u;
}

// run_cascade's answer when the split's one-chunk cascade does not fit the
// scratch budget: the caller runs the per-range LEVELS kernels instead, whose
// scratch shrinks with the rank's unit range (internal, never returned)
constexpr int kCascadeNoFit = 1;

// CO launch admission.  A CO launch's fan-in blocks spin on granules; at me = 5
// the word's s0 = 0 block also waits for sibling fan-in blocks dispatched after
// it (ba_cascade.hip, casc_co_top), which need free block slots.  So the polling
// blocks of all CO launches that may run at once on a device are bounded by
// half the chip's block slots at the kernel's occupancy (3 blocks per CU): a
// call over the bound takes the two-launch cascade instead, whatever
// BA_CASC_CO says.  "May run at once": calls of one ctx are ordered (ctx_order),
// so a ctx contributes the largest CO launch it queued since its stream was
// last seen idle (hipStreamQuery: host-side, nothing is added to any stream);
// other ctxs' CO launches (other threads, other streams) count until their
// stream drains.  Launches captured into graphs are not counted (their replays
// are the caller's to schedule, include/ba.h).  Per process: other processes
// sharing the GPU are not seen -- a poll that still times out is an error,
// never a wrong answer (BA_EDEVICE, handoff_lost).
// BA_TEST_CO_BUDGET (tests only, read per call) replaces the bound.
static uint64_t co_poll_budget(const ba_ctx* ctx) {
    if (const char* e = getenv("BA_TEST_CO_BUDGET")) return strtoull(e, nullptr, 0);
    return (uint64_t)ctx->cu_count * 3 / 2;
}

static bool co_admit(ba_ctx* ctx, hipStream_t s, uint64_t pollers) {
    const uint64_t budget = co_poll_budget(ctx);
    if (pollers > budget) return false;
    if (stream_capturing(s)) return true;
    std::lock_guard<std::mutex> lk(co_registry().mu);
    uint64_t busy = 0;
    for (ba_ctx* c : co_registry().ctxs)  // fast path: everything counted as running fits
        if (c != ctx && c->device == ctx->device) busy += c->co_pending;
    if (busy + pollers <= budget) return true;
    busy = 0;
    const bool trace = getenv("BA_TEST_CO_TRACE") != nullptr;  // tests: the admission's view
    for (ba_ctx* c : co_registry().ctxs) {
        if (c == ctx || c->device != ctx->device || c->co_pending == 0) continue;
        // a stream being captured may not be queried: its launches count
        const bool cap = stream_capturing(c->co_stream);
        const hipError_t q = cap ? hipErrorNotReady : hipStreamQuery(c->co_stream);
        if (trace)
            fprintf(stderr, "co_admit ctx %p: other ctx %p pending %llu stream %p query %d\n", (void*)ctx,
                    (void*)c, (unsigned long long)c->co_pending, (void*)c->co_stream, (int)q);
        if (q == hipSuccess) {
            c->co_pending = 0;
            continue;
        }
        busy += c->co_pending;
    }
    if (trace)
        fprintf(stderr, "co_admit ctx %p: busy %llu + %llu vs budget %llu\n", (void*)ctx,
                (unsigned long long)busy, (unsigned long long)pollers, (unsigned long long)budget);
    return busy + pollers <= budget;
}

static void co_note(ba_ctx* ctx, hipStream_t s, uint64_t pollers) {
    if (stream_capturing(s)) return;
    std::lock_guard<std::mutex> lk(co_registry().mu);
    ctx->co_pending = std::max(ctx->co_pending, pollers);  // the previous ones finish first
    ctx->co_stream = s;
}

// The polling (fan-in) blocks of a CO launch over W words: one per level-(me-5)
// slot of every word (k_cascade_mtop's shape, CascMtop::PB)
static uint64_t co_pollers(const Geometry& g, uint64_t words) {
    return words * (g.me >= 5 ? g.S[g.me - 5] : 1u);
}

// A poll of a cascade hand-off that ran out of time (ba_cascade.hip) leaves a
// non-zero BA_C_CHECK_MISMATCH: the launch's results are invalid.
static int handoff_lost(uint64_t n) {
    return fail(BA_EDEVICE, "in-launch hand-off timed out (%llu stale granule poll(s), counter slot "
                "%d); results invalid", (unsigned long long)n, BA_C_CHECK_MISMATCH);
}

// job.h != 0 (the subtree split): one chunk (`whole`), no counters.
static int run_cascade(ba_ctx* ctx, const RunArgs& a, GeoEntry* ge, CascJob job = CascJob{}) {
    const Geometry& g = ge->g;
    const bool whole = job.h != 0 || job.vin != nullptr;  // vote rows span the whole batch
    job.check = whole ? 0u : cascade_check_mode(g);
    // Two launches (units, then the fan-in) from kCascTwoWords 64-trial words on:
    // the steps' latency-bound waves then no longer hold the slots the units use
    // (faster from one word up: profiles/r04h).  BA_CASC_TWO=0/1
    // (read per call) forces one or two.
    // The subtree split's range mode too (units, then k_cascade_mtop ending at the
    // vote level), where the shape has it.
    if (!job.vin && g.me >= 4 && (job.h == 0 || cascade_range_two_supported(g, job.h))) {
        const char* e = getenv("BA_CASC_TWO");
        job.two = e ? atoi(e) != 0 : (a.batch + 63) / 64 >= kCascTwoWords;
    }
    // The whole tree as ONE launch of units + co-resident fan-in blocks (no
    // units -> fan-in kernel boundary; ba_cascade.hip casc_co_top) up to
    // kCascCoWords 64-trial words.  BA_CASC_CO=0/1 (read per call) forces it.
    // The limit also bounds the launch's polling fan-in blocks (15 per word at
    // n=16, m=5: 60): forward progress needs the polling blocks of all CO
    // launches running at once to leave block slots for their units (768 at 3
    // blocks per CU), so a dozen such launches may run concurrently.
    if (job.two && job.h == 0) {
        const char* e = getenv("BA_CASC_CO");
        job.co = e ? atoi(e) != 0 : (a.batch + 63) / 64 <= kCascCoWords;
    }
    // per trial word: R_1 .. R_{me-2} (twice with check tags) and the fan-in
    // counters, one 128-B line each -- both count against the scratch budget
    // The split's root pass as k_cascade_wtop uses neither (the default)
    const bool uses = !job.vin || cascade_root_pass_uses_scratch();
    if (job.co) {  // CO keeps R_{me-2} as granules (2x): only where the batch fits one chunk
        const uint64_t co_bytes = cascade_scratch_words_per_word(g, true) * sizeof(uint64_t) *
                                      (job.check ? 2 : 1) + cascade_counters_per_word(g) * 128;
        if (ctx->scratch_budget / co_bytes < (a.batch + 63) / 64) job.co = false;
    }
    const uint64_t pollers = co_pollers(g, (a.batch + 63) / 64);
    if (job.co && !co_admit(ctx, a.stream, pollers)) job.co = false;  // forward progress bound
    if (const char* e = getenv("BA_TEST_GRANULE_TICKS")) job.wait_ticks = strtoull(e, nullptr, 0);
    const uint64_t r_bytes = uses ? cascade_scratch_words_per_word(g, job.co) * sizeof(uint64_t) *
                                        (job.check ? 2 : 1) : 0;
    const uint64_t c_bytes = uses ? cascade_counters_per_word(g) * 128 : 0;
    const uint64_t words = (a.batch + 63) / 64;
    uint64_t max_level = 0;
    for (uint32_t k = 0; k + 2 <= g.me; ++k) max_level = g.S[k] > max_level ? g.S[k] : max_level;
    uint64_t chunk = uses ? ctx->scratch_budget / (r_bytes + c_bytes) : words;
    const uint64_t idx_cap = (1ull << 31) / (max_level + 1);  // 32-bit slot indices in the kernel
    if (chunk > idx_cap) chunk = idx_cap;
    // the counter sink: one unit per word, < 2^16 units per replica (ba_device.hpp)
    const uint64_t sink_cap = (uint64_t)kSinkReplicas * kSinkMaxUnitsPerReplica;
    if (chunk > sink_cap) chunk = sink_cap;
    if (chunk > words) chunk = words;
    if (whole && chunk < words) return kCascadeNoFit;
    if (chunk == 0)
        return fail(BA_ETOOBIG, "a 64-trial word needs %llu bytes of scratch and counters (budget "
                    "%zu)", (unsigned long long)(r_bytes + c_bytes), ctx->scratch_budget);
    int rc;
    if ((rc = ctx->scratch.grow(chunk * r_bytes)) != BA_OK) return rc;
    const size_t cbytes = chunk * c_bytes;
    if (cbytes > ctx->casc.bytes) {
        // zeroed on the launch stream, ahead of the first kernel that uses them
        // (kernels leave them zero); a graph capture must follow an eager call
        // of at least its size (include/ba.h)
        if ((rc = ctx->casc.grow(cbytes)) != BA_OK) return rc;
        HIP_TRY(hipMemsetAsync(ctx->casc.p, 0, ctx->casc.bytes, a.stream));
    }
    for (uint64_t w0 = 0; w0 < words; w0 += chunk) {
        const uint64_t wn = (words - w0) < chunk ? (words - w0) : chunk;
        const uint64_t trial0 = w0 * 64;
        const uint64_t nt = (a.batch - trial0) < wn * 64 ? (a.batch - trial0) : wn * 64;
        job.epoch = ++ctx->casc_epoch;
        HIP_TRY(launch_cascade(a, g, (const uint8_t*)ge->sender.p, (uint64_t*)ctx->scratch.p,
                               (uint32_t*)ctx->casc.p, trial0, nt, job));
        if (job.co) co_note(ctx, a.stream, pollers);
    }
    return BA_OK;
}

static int run_trials_device_impl(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                  const uint32_t* d_faulty, const uint8_t* d_order,
                                  const uint32_t* d_table, const uint32_t* d_poll,
                                  uint64_t* d_decisions, uint8_t* d_outcome, uint64_t* d_counters,
                                  void* stream) {
    int rc = validate(p, batch, d_faulty != nullptr, d_order != nullptr, d_table != nullptr);
    if (rc != BA_OK) return rc;
    if (!d_counters) return fail(BA_EINVAL, "d_counters is required on the device path");
    if (batch == 0) return BA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    RunArgs a = make_args(ctx, p, batch, d_faulty, d_order, d_table, d_poll, d_decisions,
                          d_outcome, d_counters, stream);
    if ((rc = ctx->partials.grow(sizeof(uint64_t) * 16 * kPartialRows)) != BA_OK) return rc;
    uint64_t* partials = (uint64_t*)ctx->partials.p;

    if (p->lie_mode == BA_LIE_TABLE) {
        HIP_TRY(launch_table(a, partials));
        return BA_OK;
    }

    GeoEntry* ge = geometry(ctx, a.n, a.me, &rc);
    if (!ge) return rc;
    const Geometry& g = ge->g;
    a.members = (const uint64_t*)ge->members.p;
    const bool fused_ok = ge->fused_ok;
    if (p->engine == BA_ENGINE_FUSED && !fused_ok)
        return fail(BA_ENOTSUP, "FUSED engine needs m_eff = 3 (5 <= n <= 14) or 4 (6 <= n <= %u), "
                    "or 2 <= m_eff <= %d and n - m_eff <= %d with the per-word tree within "
                    "%llu B of LDS (n=%u, m_eff=%u)", kWave4MaxN, kFusedMaxDepth, kMaxLeafS,
                    (unsigned long long)kFusedLdsBudget, a.n, a.me);
    if (fused_ok && p->engine != BA_ENGINE_LEVELS) {
        HIP_TRY(launch_fused(a, g, ge->plan_ok, ge->fp, (const FusedPlan*)ge->fplan.p,
                             (const uint8_t*)ge->sender.p, partials));
        return BA_OK;
    }
    if (use_cascade(ctx, g)) return run_cascade(ctx, a, ge);
    return run_levels(ctx, a, ge, LevelsJob{}, 0, g.L, false, partials);
}

extern "C" int ba_gen_inputs_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                    uint32_t* d_faulty, uint8_t* d_order, void* stream) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    int rc = validate(p, batch, true, true, false);
    if (rc != BA_OK) return rc;
    if (d_faulty && p->faulty_mode == BA_FAULTY_GIVEN)
        return fail(BA_EINVAL, "faulty_mode is GIVEN: no faulty sets to generate");
    if (d_order && p->order_mode == BA_ORDER_GIVEN)
        return fail(BA_EINVAL, "order_mode is GIVEN: no orders to generate");
    if (batch == 0 || (!d_faulty && !d_order)) return BA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    RunArgs a = make_args(ctx, p, batch, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                          nullptr, stream);
    HIP_TRY(launch_gen_inputs(a, d_faulty, d_order));
    return BA_OK;
}

extern "C" uint64_t ba_split_units(uint32_t n, uint32_t m, uint32_t level) {
    if (n < 3 || n > BA_MAX_GENERALS) return 0;
    const uint32_t me = effective_depth(n, m);
    if (level == BA_SPLIT_FIRST_HOP) return me >= 1 ? n - 1 : 0;
    // second hop: R_2 must be a majority level, and leaf blocks (level me-2
    // slots) must lie inside one unit
    if (level == BA_SPLIT_SECOND_HOP) return (me >= 3 && n >= 4) ? (uint64_t)(n - 1) * (n - 2) : 0;
    return 0;
}

extern "C" uint64_t ba_split_vote_slots(uint32_t n, uint32_t m, uint32_t level, uint32_t u_begin,
                                        uint32_t u_end) {
    const uint64_t units = ba_split_units(n, m, level);
    if (units == 0 || u_begin > u_end || u_end > units) return 0;
    return (uint64_t)(u_end - u_begin) * (n - 1 - level);  // level-h children of a level h-1 slot
}

extern "C" uint64_t ba_vote_slots(uint32_t n, uint32_t m, uint32_t j_begin, uint32_t j_end) {
    return ba_split_vote_slots(n, m, BA_SPLIT_FIRST_HOP, j_begin, j_end);
}

static int validate_split(ba_ctx* ctx, const ba_params* p, uint64_t batch, const uint32_t* d_faulty,
                          const uint8_t* d_order, uint32_t level) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    int rc = validate(p, batch, d_faulty != nullptr, d_order != nullptr, false);
    if (rc != BA_OK) return rc;
    if (p->lie_mode != BA_LIE_PHILOX)
        return fail(BA_ENOTSUP, "the subtree split runs Philox lies only (table mode is OM(1))");
    if (p->engine == BA_ENGINE_FUSED)
        return fail(BA_ENOTSUP, "the subtree split runs on the LEVELS engine");
    if (effective_depth(p->n, p->m) == 0)
        return fail(BA_ENOTSUP, "OM(0) has no relay subtrees (n=%u, m=%u)", p->n, p->m);
    if (level != BA_SPLIT_FIRST_HOP && level != BA_SPLIT_SECOND_HOP)
        return fail(BA_EINVAL, "split level %u (1: first hop, 2: second hop)", level);
    if (ba_split_units(p->n, p->m, level) == 0)
        return fail(BA_ENOTSUP, "no level-%u split for n=%u, m=%u (the second-hop split needs "
                    "m_eff >= 3)", level, p->n, p->m);
    return BA_OK;
}

static int subtree_votes_impl(ba_ctx* ctx, const ba_params* p, uint64_t batch, uint32_t level,
                              uint32_t j_begin, uint32_t j_end, const uint32_t* d_faulty,
                              const uint8_t* d_order, uint64_t* d_votes, void* stream) {
    int rc = validate_split(ctx, p, batch, d_faulty, d_order, level);
    if (rc != BA_OK) return rc;
    const uint64_t units = ba_split_units(p->n, p->m, level);
    if (j_begin >= j_end || j_end > units)
        return fail(BA_EINVAL, "unit range [%u, %u) outside [0, %llu)", j_begin, j_end,
                    (unsigned long long)units);
    if (!d_votes) return fail(BA_EINVAL, "d_votes is NULL");
    if (batch == 0) return BA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    RunArgs a = make_args(ctx, p, batch, d_faulty, d_order, nullptr, nullptr, nullptr, nullptr,
                          nullptr, stream);
    GeoEntry* ge = geometry(ctx, a.n, a.me, &rc);
    if (!ge) return rc;
    a.members = (const uint64_t*)ge->members.p;
    if (use_cascade(ctx, ge->g) && cascade_range_supported(ge->g, level)) {
        CascJob cj;  // the one-launch cascade over the range's level-(me-3) units
        cj.h = level;
        cj.ub = j_begin;
        cj.ue = j_end;
        cj.votes = d_votes;
        if ((rc = run_cascade(ctx, a, ge, cj)) != kCascadeNoFit) return rc;
    }
    LevelsJob job;
    job.root = false;
    job.h = level;
    job.votes_out = d_votes;
    return run_levels(ctx, a, ge, job, j_begin, j_end, true, nullptr);
}

static int root_from_votes_impl(ba_ctx* ctx, const ba_params* p, uint64_t batch, uint32_t level,
                                const uint32_t* d_faulty, const uint8_t* d_order,
                                const uint64_t* d_votes, uint64_t* d_decisions, uint8_t* d_outcome,
                                uint64_t* d_counters, void* stream) {
    int rc = validate_split(ctx, p, batch, d_faulty, d_order, level);
    if (rc != BA_OK) return rc;
    if (!d_votes || !d_counters) return fail(BA_EINVAL, "d_votes and d_counters are required");
    if (batch == 0) return BA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    RunArgs a = make_args(ctx, p, batch, d_faulty, d_order, nullptr, nullptr, d_decisions,
                          d_outcome, d_counters, stream);
    if ((rc = ctx->partials.grow(sizeof(uint64_t) * 16 * kPartialRows)) != BA_OK) return rc;
    GeoEntry* ge = geometry(ctx, a.n, a.me, &rc);
    if (!ge) return rc;
    a.members = (const uint64_t*)ge->members.p;
    if (use_cascade(ctx, ge->g) && cascade_range_supported(ge->g, level)) {
        CascJob cj;  // one launch: step level-1 from the votes, roots, quorum
        cj.vin = d_votes;
        cj.root_h = level;
        if ((rc = run_cascade(ctx, a, ge, cj)) != kCascadeNoFit) return rc;
    }
    LevelsJob job;
    job.tree = false;
    job.h = level;
    job.votes_in = d_votes;
    // an empty unit range: only the inputs and levels 0..h-1 are materialised
    return run_levels(ctx, a, ge, job, 0, 0, true, (uint64_t*)ctx->partials.p);
}

// The ordered entry points: wait for the ctx's previous call if it ran on
// another stream, then mark this call's end (ctx_order / ctx_mark).
template <typename F>
static int ordered(ba_ctx* ctx, void* stream, F&& body) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    const hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(ctx_order(ctx, s));
    // marked whatever body() returned: a call that fails part-way may already
    // have queued work on s that uses the ctx's scratch, sink or task counter,
    // and the ctx's next call on another stream must wait for it
    const int rc = body();
    (void)ctx_mark(ctx, s);
    return rc;
}

// ba.py's coin table on the device: ba_mt_table's rows (random.seed(seed_t), then
// one round's coins in ba.py's draw order, ba.py:45, 269), chunked so the
// generators' states ([624][chunk] uint32, ba_mtdev.hip) fit the scratch budget.
extern "C" int ba_mt_table_device(ba_ctx* ctx, uint32_t n, uint32_t m, uint64_t batch,
                                  const uint64_t* d_seeds, const uint32_t* d_faulty_mask,
                                  const uint32_t* d_poll_commander, uint32_t stride,
                                  uint32_t* d_table, uint32_t* d_next_word, void* stream) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    if (n < 1 || n > BA_MAX_GENERALS) return fail(BA_EINVAL, "n=%u outside 1..%d", n, BA_MAX_GENERALS);
    const uint64_t L = n - 1;
    if ((uint64_t)stride * 32 < L + L * L)
        return fail(BA_EINVAL, "stride %u words < %llu coins of an n=%u round", stride,
                    (unsigned long long)(L + L * L), n);
    if (batch && (!d_seeds || !d_faulty_mask || !d_table))
        return fail(BA_EINVAL, "d_seeds, d_faulty_mask and d_table are required");
    if (batch == 0) return BA_OK;
    return ordered(ctx, stream, [&] {
        const hipStream_t s = (hipStream_t)stream;
        const uint64_t per = mt_table_state_bytes_per_trial();
        uint64_t chunk = ctx->scratch_budget / per;
        if (chunk > batch) chunk = batch;
        if (chunk > (1ull << 31)) chunk = 1ull << 31;
        if (chunk == 0) return fail(BA_ETOOBIG, "scratch budget %zu < %llu B", ctx->scratch_budget,
                                    (unsigned long long)per);
        int rc;
        if ((rc = ctx->scratch.grow(mt_table_state_rows(chunk) * per)) != BA_OK) return rc;
        for (uint64_t c0 = 0; c0 < batch; c0 += chunk) {
            const uint64_t T = batch - c0 < chunk ? batch - c0 : chunk;
            HIP_TRY(launch_mt_table(n, m, T, d_seeds + c0, d_faulty_mask + c0,
                                    d_poll_commander ? d_poll_commander + c0 : nullptr, stride,
                                    d_table + c0 * stride, d_next_word ? d_next_word + c0 : nullptr,
                                    (uint32_t*)ctx->scratch.p, s, &ctx->prof));
        }
        return BA_OK;
    });
}

extern "C" int ba_run_trials_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                    const uint32_t* d_faulty, const uint8_t* d_order,
                                    const uint32_t* d_table, const uint32_t* d_poll,
                                    uint64_t* d_decisions, uint8_t* d_outcome,
                                    uint64_t* d_counters, void* stream) {
    return ordered(ctx, stream, [&] {
        return run_trials_device_impl(ctx, p, batch, d_faulty, d_order, d_table, d_poll,
                                      d_decisions, d_outcome, d_counters, stream);
    });
}

extern "C" int ba_split_votes_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                     uint32_t level, uint32_t u_begin, uint32_t u_end,
                                     const uint32_t* d_faulty, const uint8_t* d_order,
                                     uint64_t* d_votes, void* stream) {
    return ordered(ctx, stream, [&] {
        return subtree_votes_impl(ctx, p, batch, level, u_begin, u_end, d_faulty, d_order, d_votes,
                                  stream);
    });
}

extern "C" int ba_root_from_split_votes_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                               uint32_t level, const uint32_t* d_faulty,
                                               const uint8_t* d_order, const uint64_t* d_votes,
                                               uint64_t* d_decisions, uint8_t* d_outcome,
                                               uint64_t* d_counters, void* stream) {
    return ordered(ctx, stream, [&] {
        return root_from_votes_impl(ctx, p, batch, level, d_faulty, d_order, d_votes, d_decisions,
                                    d_outcome, d_counters, stream);
    });
}

extern "C" int ba_subtree_votes_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                       uint32_t j_begin, uint32_t j_end, const uint32_t* d_faulty,
                                       const uint8_t* d_order, uint64_t* d_votes, void* stream) {
    return ba_split_votes_device(ctx, p, batch, BA_SPLIT_FIRST_HOP, j_begin, j_end, d_faulty,
                                 d_order, d_votes, stream);
}

extern "C" int ba_root_from_votes_device(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                         const uint32_t* d_faulty, const uint8_t* d_order,
                                         const uint64_t* d_votes, uint64_t* d_decisions,
                                         uint8_t* d_outcome, uint64_t* d_counters, void* stream) {
    return ba_root_from_split_votes_device(ctx, p, batch, BA_SPLIT_FIRST_HOP, d_faulty, d_order,
                                           d_votes, d_decisions, d_outcome, d_counters, stream);
}

// ---------------------------------------------------------------------------
// host entry point: copy in, run, copy out (PCIe-inclusive)
// ---------------------------------------------------------------------------
extern "C" int ba_run_trials(ba_ctx* ctx, const ba_params* p, uint64_t batch,
                             const uint32_t* faulty, const uint8_t* order,
                             const uint32_t* lie_table, const uint32_t* poll,
                             uint64_t* decisions, uint8_t* outcome, ba_counters* counters) {
    if (!ctx) return fail(BA_EINVAL, "ctx is NULL");
    int rc = validate(p, batch, faulty != nullptr, order != nullptr, lie_table != nullptr);
    if (rc != BA_OK) return rc;
    if (counters) memset(counters, 0, sizeof *counters);
    if (batch == 0) return BA_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    HIP_TRY(ctx_order(ctx, st));  // the io buffers follow the ctx's last call
    const bool need_f = p->faulty_mode == BA_FAULTY_GIVEN, need_o = p->order_mode == BA_ORDER_GIVEN;
    const bool need_t = p->lie_mode == BA_LIE_TABLE, need_p = need_t && poll;
    if (need_f && (rc = ctx->io_faulty.grow(batch * 4)) != BA_OK) return rc;
    if (need_o && (rc = ctx->io_order.grow(batch)) != BA_OK) return rc;
    if (need_t && (rc = ctx->io_table.grow(batch * p->table_stride * 4)) != BA_OK) return rc;
    if (need_p && (rc = ctx->io_poll.grow(batch * 4)) != BA_OK) return rc;
    if (decisions && (rc = ctx->io_dec.grow(batch * 8)) != BA_OK) return rc;
    if (outcome && (rc = ctx->io_out.grow(batch)) != BA_OK) return rc;
    if ((rc = ctx->io_cnt.grow(BA_NCOUNTERS * 8)) != BA_OK) return rc;
    if (need_f) HIP_TRY(hipMemcpyAsync(ctx->io_faulty.p, faulty, batch * 4, hipMemcpyHostToDevice, st));
    if (need_o) HIP_TRY(hipMemcpyAsync(ctx->io_order.p, order, batch, hipMemcpyHostToDevice, st));
    if (need_t)
        HIP_TRY(hipMemcpyAsync(ctx->io_table.p, lie_table, batch * p->table_stride * 4,
                               hipMemcpyHostToDevice, st));
    if (need_p) HIP_TRY(hipMemcpyAsync(ctx->io_poll.p, poll, batch * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(ctx->io_cnt.p, 0, BA_NCOUNTERS * 8, st));
    rc = ba_run_trials_device(ctx, p, batch, need_f ? (const uint32_t*)ctx->io_faulty.p : nullptr,
                              need_o ? (const uint8_t*)ctx->io_order.p : nullptr,
                              need_t ? (const uint32_t*)ctx->io_table.p : nullptr,
                              need_p ? (const uint32_t*)ctx->io_poll.p : nullptr,
                              decisions ? (uint64_t*)ctx->io_dec.p : nullptr,
                              outcome ? (uint8_t*)ctx->io_out.p : nullptr, (uint64_t*)ctx->io_cnt.p,
                              st);
    if (rc != BA_OK) return rc;
    if (decisions) HIP_TRY(hipMemcpyAsync(decisions, ctx->io_dec.p, batch * 8, hipMemcpyDeviceToHost, st));
    if (outcome) HIP_TRY(hipMemcpyAsync(outcome, ctx->io_out.p, batch, hipMemcpyDeviceToHost, st));
    uint64_t h_cnt[BA_NCOUNTERS];
    HIP_TRY(hipMemcpyAsync(h_cnt, ctx->io_cnt.p, BA_NCOUNTERS * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h_cnt[BA_C_CHECK_MISMATCH] != 0) return handoff_lost(h_cnt[BA_C_CHECK_MISMATCH]);
    if (counters) memcpy(counters->v, h_cnt, sizeof h_cnt);
    return BA_OK;
}
