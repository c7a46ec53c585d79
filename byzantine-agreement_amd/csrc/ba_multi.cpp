// ba_multi.cpp -- the multi-GPU layer inside the C ABI (SURVEY.md §8b/§8e:
// the library owns the RCCL communicators).  One process per GPU: rank 0 makes
// a unique id (ba_comm_unique_id), ships its 128 bytes to every rank out of
// band (MPI, a socket, a file, torch.distributed's store), every rank creates
// the communicator on its ctx's device (ba_comm_create).  Two ways the path
// shards, each with exactly the exchange it needs:
//
//  * trial data-parallel (ba_run_trials_multi, or per-batch runs plus
//    ba_comm_allreduce_device): each rank resolves a contiguous word-aligned
//    share of the trial index space; every draw is keyed by the global trial
//    index, so the shares give the same counters as one unsharded run.  The
//    only collective is an all-reduce of the 16 run counters.
//  * one huge instance split by first-hop subtree (ba_run_instance_split_multi,
//    or ba_subtree_votes_device + ba_comm_allgather_votes_device +
//    ba_root_from_votes_device): rank r owns the first hops ba_subtree_share
//    gives it, computes their level-1 child results in place in the full vote
//    array, and the ranks exchange them with one grouped broadcast per rank
//    (an all-gather of unequal shares, no padding or reassembly); every rank
//    then finishes the root majorities and quorum (ba.py:159-255).
//
// Error agreement: a rank whose local work fails still takes part in every
// collective of the call and raises an error flag that is all-reduced with
// the counters, so no rank blocks in a collective another rank skipped and
// every rank returns the error.
//
// Watchdog: a blocking whole job waits for its collectives by polling the
// comm's stream, and past the comm's timeout aborts the communicator
// (ncclCommAbort makes this rank's RCCL kernels return) and fails with
// BA_EABORTED.  A rank whose own transport fails (it cannot learn the agreed
// error flag, or cannot raise it) aborts itself at once: RCCL has no way to
// tell the peers, so they leave through their own watchdog.  Every rank's wait
// is bounded either way.
//
// RCCL is opened with dlopen on first use: torch's wheel bundles its own
// librccl.so, and a process that imports torch keeps that copy (RTLD_NOLOAD
// finds it) instead of loading a second RCCL beside it.  BA_RCCL_LIB names a
// replacement with the same entry points (test-only: tests/native/fake_rccl.c,
// a shared-memory stand-in that lets N processes share one GPU, which RCCL
// refuses, so these N>1 paths run on a one-GPU box).
#include <dlfcn.h>
#include <time.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/ba.h"

extern "C" int ba_fail_internal(int code, const char* msg);  // ba_api.cpp: sets ba_last_error
extern "C" int ba_validate_internal(const ba_params* p, uint64_t batch);  // ba_api.cpp

namespace {

struct Rccl {
    bool tried = false;
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    const char* over = getenv("BA_RCCL_LIB");  // test-only replacement (see the top)
    if (over && over[0]) {
        r.h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
    } else {
        for (const char* name : {"librccl.so", "librccl.so.1"}) {  // already loaded (torch's) first
            if ((r.h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
        }
        if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    if (!r.h) return r;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
    r.broadcast = (decltype(r.broadcast))dlsym(r.h, "ncclBroadcast");
    r.group_start = (decltype(r.group_start))dlsym(r.h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(r.h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
    r.comm_abort = (decltype(r.comm_abort))dlsym(r.h, "ncclCommAbort");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.broadcast ||
        !r.group_start || !r.group_end || !r.error_string || !r.comm_abort)
        r.h = nullptr;
    return r;
}

int failf(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return ba_fail_internal(code, buf);
}

constexpr int kErrSlot = BA_NCOUNTERS - 1;  // error flag, all-reduced with the counters
constexpr uint64_t kDefaultTimeoutMs = 300000;

uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// BA_TEST_PREAGREE_FAIL (test-only, read per call): make this rank's
// pre-exchange agreement transport fail -- "upload" (the flag upload; the
// device memset that replaces it works), "upload_memset" (both), "readback"
// (the agreed sum cannot be read back).
bool test_fail(const char* what) {
    const char* e = getenv("BA_TEST_PREAGREE_FAIL");
    return e && strcmp(e, what) == 0;
}

}  // namespace

struct ba_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    uint64_t* d_cnt = nullptr;  // BA_NCOUNTERS uint64 on the device, all-reduced in place
    uint64_t* d_votes = nullptr;  // full vote array of the split (grown on demand)
    size_t votes_bytes = 0;
    hipStream_t stream = nullptr;  // the ctx's own stream (not owned: the ctx outlives the comm)
    uint64_t* h_pin = nullptr;  // pinned host words: counter read-back, flag upload / read-back
    std::atomic<uint64_t> timeout_ms{kDefaultTimeoutMs};  // watchdog of the blocking jobs
    // ba_comm_abort may run on a supervisor thread while a job enqueues a
    // collective: `mu` guards `comm` and `aborted` -- every collective is
    // enqueued under it (with_comm), and the abort frees the communicator under
    // it, so no enqueue ever sees a freed or null communicator, and only one
    // thread ever calls ncclCommAbort
    std::mutex mu;
    std::atomic<bool> aborted{false};  // ncclCommAbort ran: the RCCL communicator is gone
    // recorded on the stream right before a job's first collective: the
    // watchdog's clock starts when the rank's own work ahead of it is done
    // (comm_wait), so a long local step is never taken for a peer that left
    hipEvent_t coll_ev = nullptr;
};

// Abort the RCCL communicator: this rank's pending collectives return (RCCL
// kernels poll the abort flag), the communicator is freed, and every further
// call on the comm fails with BA_EABORTED.  Safe from any thread.
static void abort_comm(ba_comm* c) {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->aborted.load()) return;
    if (c->comm && rccl().h) (void)rccl().comm_abort(c->comm);
    c->comm = nullptr;
    c->aborted.store(true);
}

// Enqueue a collective on the live communicator (under the comm's lock, so a
// concurrent ba_comm_abort waits for the enqueue, and the enqueue never sees a
// freed communicator); an aborted comm gives ncclInvalidUsage without a call.
template <typename F>
static ncclResult_t with_comm(ba_comm* c, F&& f) {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->aborted.load() || !c->comm) return ncclInvalidUsage;
    return f(c->comm);
}

static int fail_aborted(const ba_comm* c) {
    return failf(BA_EABORTED, "communicator of rank %d (of %d) was aborted; destroy it and create "
                 "a new one", c->rank, c->nranks);
}

// After an abort: RCCL's kernels see the abort flag and return, so the stream
// drains -- waited for at most this long (a hung kernel of the rank's own work
// must not block the caller forever; the comm is unusable either way, and
// ba_comm_destroy synchronizes the stream).
constexpr uint64_t kAbortDrainMs = 10000;

static void drain_after_abort(ba_comm* c) {
    const uint64_t t0 = now_ns();
    while (hipStreamQuery(c->stream) == hipErrorNotReady && now_ns() - t0 < kAbortDrainMs * 1000000ull) {
        timespec ts = {0, 200000};
        nanosleep(&ts, nullptr);
    }
}

// Wait for the comm's stream (the blocking jobs' collectives): poll it, and
// past the timeout abort the communicator so the stream drains, and fail.
// Only the exchange is timed: coll_ev is recorded right before the job's first
// collective, and when the clock runs out while it has not completed -- the
// rank's own kernels ahead of the exchange are still running -- the clock
// restarts instead of aborting.  When it has completed, the clock restarts once
// more (the exchange may have begun only just before), so the exchange always
// gets at least the whole timeout and at most twice it.  The event is queried
// only at an expiry: a job that completes in time pays one event record on its
// stream and nothing else (BA_MULTI_CLOCK=1, lab only: query the event on every
// poll and time from its completion; 0: time from the wait's start, round 5).
#ifndef BA_MULTI_CLOCK
#define BA_MULTI_CLOCK 2
#endif
static int comm_wait(ba_comm* c, const char* what) {
    const uint64_t lim = c->timeout_ms.load() * 1000000ull;
    uint64_t t0 = now_ns();
    bool timing = BA_MULTI_CLOCK == 0;
    for (uint32_t k = 0;; ++k) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return BA_OK;
        if (e != hipErrorNotReady) {
            abort_comm(c);
            return failf(BA_EDEVICE, "%s: %s (communicator aborted)", what, hipGetErrorString(e));
        }
        if (c->aborted.load()) {  // ba_comm_abort from another thread
            drain_after_abort(c);
            return failf(BA_EABORTED, "%s: communicator of rank %d aborted during the job", what,
                         c->rank);
        }
        if (BA_MULTI_CLOCK == 1 && !timing) {
            const hipError_t q = hipEventQuery(c->coll_ev);
            if (q == hipSuccess) {
                timing = true;
                t0 = now_ns();
            }
        } else if (now_ns() - t0 > lim) {
            if (BA_MULTI_CLOCK == 2 && !timing) {
                // an expiry: still in the rank's own work, or the exchange began
                // at an unknown time since -- restart the clock either way
                const hipError_t q = hipEventQuery(c->coll_ev);
                if (q != hipSuccess && q != hipErrorNotReady) {
                    abort_comm(c);
                    return failf(BA_EDEVICE, "%s: %s (communicator aborted)", what, hipGetErrorString(q));
                }
                timing = q == hipSuccess;  // in the exchange: the next expiry aborts
                t0 = now_ns();
                continue;
            }
            abort_comm(c);
            drain_after_abort(c);  // the aborted collectives return
            return failf(BA_EABORTED, "%s: no completion within %llu ms (a peer left the "
                         "exchange); communicator of rank %d aborted", what,
                         (unsigned long long)c->timeout_ms.load(), c->rank);
        }
        if (k > 2000) {  // a short spin first: most jobs complete within it
            timespec ts = {0, 50000};
            nanosleep(&ts, nullptr);
        }
    }
}

// Mark the start of the job's exchange (comm_wait's clock); a failed record
// leaves the clock to start at once, which only shortens the watchdog.
static void mark_exchange(ba_comm* c) {
    if (BA_MULTI_CLOCK == 0) return;
    if (hipEventRecord(c->coll_ev, c->stream) != hipSuccess) (void)hipEventRecord(c->coll_ev, nullptr);
}

// ba_api.cpp, library-internal
extern "C" hipStream_t ba_ctx_stream_internal(struct ba_ctx* ctx);

extern "C" int ba_comm_unique_id(unsigned char id[BA_COMM_ID_BYTES]) {
    if (!id) return failf(BA_EINVAL, "id is NULL");
    Rccl& r = rccl();
    if (!r.h) return failf(BA_EDEVICE, "RCCL (librccl.so.1) could not be loaded: %s", dlerror());
    ncclUniqueId u;
    const ncclResult_t e = r.get_unique_id(&u);
    if (e != ncclSuccess) return failf(BA_EDEVICE, "ncclGetUniqueId: %s", r.error_string(e));
    static_assert(sizeof(u) == BA_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, BA_COMM_ID_BYTES);
    return BA_OK;
}

extern "C" int ba_comm_create(struct ba_ctx* ctx, int nranks, int rank,
                              const unsigned char id[BA_COMM_ID_BYTES], struct ba_comm** out) {
    if (!ctx || !id || !out) return failf(BA_EINVAL, "ctx, id and out are required");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return failf(BA_EINVAL, "rank %d of %d ranks", rank, nranks);
    *out = nullptr;
    Rccl& r = rccl();
    if (!r.h) return failf(BA_EDEVICE, "RCCL (librccl.so.1) could not be loaded");
    int dev = 0;
    if (ba_ctx_device(ctx, &dev) != BA_OK) return BA_EINVAL;
    if (hipSetDevice(dev) != hipSuccess) return failf(BA_EDEVICE, "hipSetDevice(%d)", dev);
    ba_comm* c = new ba_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = dev;
    // whole jobs run on the ctx's own stream: a ctx call on another stream
    // afterwards orders itself after it by an event recorded on that stream
    // (ba_api.cpp ctx_order), so the stream must live as long as the ctx
    c->stream = ba_ctx_stream_internal(ctx);
    if (const char* t = getenv("BA_COMM_TIMEOUT_MS")) {
        const uint64_t v = strtoull(t, nullptr, 0);
        if (v > 0) c->timeout_ms = v;
    }
    if (hipMalloc(&c->d_cnt, BA_NCOUNTERS * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&c->h_pin, (BA_NCOUNTERS + 2) * sizeof(uint64_t), 0) != hipSuccess ||
        // a progress marker only (nothing is read through it): no system-scope
        // fence, which cost ~6 us per blocking call (profiles/r06h_watchdog_clock_ab.log)
        hipEventCreateWithFlags(&c->coll_ev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
        if (c->d_cnt) (void)hipFree(c->d_cnt);
        if (c->h_pin) (void)hipHostFree(c->h_pin);
        delete c;
        return failf(BA_ENOMEM, "communicator buffers");
    }
    ncclUniqueId u;
    memcpy(&u, id, BA_COMM_ID_BYTES);
    const ncclResult_t e = r.comm_init_rank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        (void)hipFree(c->d_cnt);
        (void)hipHostFree(c->h_pin);
        (void)hipEventDestroy(c->coll_ev);
        delete c;
        return failf(BA_EDEVICE, "ncclCommInitRank(%d ranks, rank %d): %s", nranks, rank,
                     r.error_string(e));
    }
    *out = c;
    return BA_OK;
}

extern "C" void ba_comm_destroy(struct ba_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm && !c->aborted.load() && rccl().h) (void)rccl().comm_destroy(c->comm);
    if (c->coll_ev) (void)hipEventDestroy(c->coll_ev);
    if (c->d_cnt) (void)hipFree(c->d_cnt);
    if (c->d_votes) (void)hipFree(c->d_votes);
    if (c->h_pin) (void)hipHostFree(c->h_pin);
    delete c;
}

extern "C" int ba_comm_rank(struct ba_comm* comm, int* nranks, int* rank) {
    if (!comm) return failf(BA_EINVAL, "comm is NULL");
    if (nranks) *nranks = comm->nranks;
    if (rank) *rank = comm->rank;
    return BA_OK;
}

extern "C" int ba_comm_set_timeout(struct ba_comm* comm, uint64_t timeout_ms) {
    if (!comm || timeout_ms == 0) return failf(BA_EINVAL, "comm is NULL or timeout is 0");
    comm->timeout_ms.store(timeout_ms);
    return BA_OK;
}

extern "C" int ba_comm_abort(struct ba_comm* comm) {
    if (!comm) return failf(BA_EINVAL, "comm is NULL");
    abort_comm(comm);
    return BA_OK;
}

// ---------------------------------------------------------------------------
// partition arithmetic (host only)
// ---------------------------------------------------------------------------
extern "C" int ba_trial_share(uint64_t total_trials, int nranks, int rank, uint64_t* first,
                              uint64_t* count) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count)
        return failf(BA_EINVAL, "rank %d of %d ranks", rank, nranks);
    const uint64_t words = (total_trials + 63) / 64;
    const uint64_t w0 = words * (uint64_t)rank / (uint64_t)nranks;
    const uint64_t w1 = words * (uint64_t)(rank + 1) / (uint64_t)nranks;
    const uint64_t f = w0 * 64, end = w1 * 64 < total_trials ? w1 * 64 : total_trials;
    *first = f;
    *count = end > f ? end - f : 0;
    return BA_OK;
}

extern "C" int ba_subtree_share(uint32_t n, int nranks, int rank, uint32_t* j_begin,
                                uint32_t* j_end) {
    if (n < 3 || n > BA_MAX_GENERALS || nranks < 1 || rank < 0 || rank >= nranks || !j_begin ||
        !j_end)
        return failf(BA_EINVAL, "n=%u, rank %d of %d ranks", n, rank, nranks);
    const uint64_t L = n - 1;  // first-hop lieutenants; ranks beyond L get empty shares
    *j_begin = (uint32_t)(L * (uint64_t)rank / (uint64_t)nranks);
    *j_end = (uint32_t)(L * (uint64_t)(rank + 1) / (uint64_t)nranks);
    return BA_OK;
}

extern "C" int ba_split_share(uint32_t n, uint32_t m, uint32_t level, int nranks, int rank,
                              uint32_t* u_begin, uint32_t* u_end) {
    const uint64_t U = ba_split_units(n, m, level);
    if (U == 0 || nranks < 1 || rank < 0 || rank >= nranks || !u_begin || !u_end)
        return failf(BA_EINVAL, "level-%u split of n=%u, m=%u, rank %d of %d ranks", level, n, m,
                     rank, nranks);
    *u_begin = (uint32_t)(U * (uint64_t)rank / (uint64_t)nranks);
    *u_end = (uint32_t)(U * (uint64_t)(rank + 1) / (uint64_t)nranks);
    return BA_OK;
}

// ---------------------------------------------------------------------------
// collectives (asynchronous on `stream`)
// ---------------------------------------------------------------------------
extern "C" int ba_comm_allreduce_device(struct ba_comm* comm, uint64_t* d_counters, void* stream) {
    if (!comm || !d_counters) return failf(BA_EINVAL, "comm and d_counters are required");
    if (comm->aborted.load()) return fail_aborted(comm);
    if (hipSetDevice(comm->device) != hipSuccess) return failf(BA_EDEVICE, "hipSetDevice");
    Rccl& r = rccl();
    const ncclResult_t e = with_comm(comm, [&](ncclComm_t cm) {
        return r.all_reduce(d_counters, d_counters, BA_NCOUNTERS, ncclUint64, ncclSum, cm,
                            (hipStream_t)stream);
    });
    if (comm->aborted.load()) return fail_aborted(comm);
    if (e != ncclSuccess) return failf(BA_EDEVICE, "ncclAllReduce: %s", r.error_string(e));
    return BA_OK;
}

extern "C" int ba_comm_allgather_split_votes_device(struct ba_comm* comm, uint32_t n, uint32_t m,
                                                    uint32_t level, uint64_t batch,
                                                    uint64_t* d_votes, void* stream) {
    if (!comm || !d_votes) return failf(BA_EINVAL, "comm and d_votes are required");
    const uint64_t units = ba_split_units(n, m, level);
    if (units == 0) return failf(BA_EINVAL, "no level-%u split votes for n=%u, m=%u", level, n, m);
    if (comm->aborted.load()) return fail_aborted(comm);
    if (hipSetDevice(comm->device) != hipSuccess) return failf(BA_EDEVICE, "hipSetDevice");
    const uint64_t W = (batch + 63) / 64, row = (uint64_t)(n - 1 - level) * W;  // words per unit
    Rccl& r = rccl();
    ncclResult_t e2 = ncclSuccess;
    const ncclResult_t e = with_comm(comm, [&](ncclComm_t cm) {
        ncclResult_t eb = r.group_start();
        for (int q = 0; q < comm->nranks && eb == ncclSuccess; ++q) {
            uint32_t ub = 0, ue = 0;
            (void)ba_split_share(n, m, level, comm->nranks, q, &ub, &ue);
            if (ue == ub) continue;
            uint64_t* part = d_votes + (uint64_t)ub * row;  // rank q's rows, in place on every rank
            eb = r.broadcast(part, part, (size_t)(ue - ub) * row, ncclUint64, q, cm, (hipStream_t)stream);
        }
        e2 = r.group_end();
        return eb;
    });
    if (comm->aborted.load()) return fail_aborted(comm);
    if (e != ncclSuccess || e2 != ncclSuccess)
        return failf(BA_EDEVICE, "vote all-gather (grouped ncclBroadcast): %s",
                     r.error_string(e != ncclSuccess ? e : e2));
    return BA_OK;
}

extern "C" int ba_comm_allgather_votes_device(struct ba_comm* comm, uint32_t n, uint32_t m,
                                              uint64_t batch, uint64_t* d_votes, void* stream) {
    return ba_comm_allgather_split_votes_device(comm, n, m, BA_SPLIT_FIRST_HOP, batch, d_votes,
                                                stream);
}

// ---------------------------------------------------------------------------
// blocking whole-job entry points
// ---------------------------------------------------------------------------
// Sum every rank's error flag -- and, for trial-DP, the counters (a split
// computes the same whole-job counters on every rank) -- over the ranks, copy
// them to the host and report: the local error, else "another rank failed",
// else OK.  A rank that cannot raise its flag, or whose collective cannot be
// enqueued, aborts itself (its peers then leave through their watchdog): it
// never returns as if nothing failed while its peers wait for it.
static int finish_job(ba_comm* comm, int local_rc, ba_counters* counters_out, bool sum_counters) {
    if (comm->aborted.load()) return local_rc != BA_OK ? local_rc : fail_aborted(comm);
    uint64_t* h = comm->h_pin;  // pinned: the copies below never block the host
    if (local_rc != BA_OK) {
        h[BA_NCOUNTERS] = 1;
        if (hipMemcpyAsync(comm->d_cnt + kErrSlot, h + BA_NCOUNTERS, sizeof(uint64_t),
                           hipMemcpyHostToDevice, comm->stream) != hipSuccess) {
            abort_comm(comm);
            return local_rc;
        }
    }
    Rccl& r = rccl();
    mark_exchange(comm);
    const ncclResult_t e = with_comm(comm, [&](ncclComm_t cm) {
        return sum_counters
            ? r.all_reduce(comm->d_cnt, comm->d_cnt, BA_NCOUNTERS, ncclUint64, ncclSum, cm, comm->stream)
            : r.all_reduce(comm->d_cnt + kErrSlot, comm->d_cnt + kErrSlot, 1, ncclUint64, ncclSum, cm,
                           comm->stream);
    });
    if (e != ncclSuccess) {
        const bool by_peer = comm->aborted.load();  // ba_comm_abort ran meanwhile
        abort_comm(comm);
        return local_rc != BA_OK ? local_rc
               : by_peer         ? fail_aborted(comm)
                                 : failf(BA_EDEVICE, "ncclAllReduce: %s (communicator aborted)",
                                         r.error_string(e));
    }
    int rc = BA_OK;
    if (hipMemcpyAsync(h, comm->d_cnt, BA_NCOUNTERS * sizeof(uint64_t), hipMemcpyDeviceToHost,
                       comm->stream) != hipSuccess)
        rc = failf(BA_EDEVICE, "counter read-back");
    const int rw = comm_wait(comm, "counter all-reduce");
    if (local_rc != BA_OK) return local_rc;
    if (rw != BA_OK) return rw;
    if (rc != BA_OK) return rc;
    ba_counters tmp;
    memcpy(tmp.v, h, sizeof tmp.v);
    if (tmp.v[kErrSlot] != 0)
        return failf(BA_EDEVICE, "%llu other rank(s) failed this call",
                     (unsigned long long)tmp.v[kErrSlot]);
    // a cascade hand-off poll that ran out of time (ba_cascade.hip): all-reduced
    // with the counters (trial-DP), so every rank of the job reports it
    if (tmp.v[BA_C_CHECK_MISMATCH] != 0)
        return failf(BA_EDEVICE, "in-launch hand-off timed out (%llu stale granule poll(s), counter "
                     "slot %d); results invalid", (unsigned long long)tmp.v[BA_C_CHECK_MISMATCH],
                     BA_C_CHECK_MISMATCH);
    tmp.v[kErrSlot] = 0;
    if (counters_out) *counters_out = tmp;
    return BA_OK;
}

// BA_FORCE_SPLIT=1: the split entry takes the vote-array path at one rank
// (test-only; read on every call, so a test can switch it in-process).
static bool force_split() {
    const char* e = getenv("BA_FORCE_SPLIT");
    return e && e[0] == '1';
}

// Sum every rank's error flag now, before a collective that a failed rank
// could not join.  Returns BA_OK when this rank is to join the exchange;
// otherwise this rank's own error, or "another rank failed" -- the same answer
// on every rank, so all of them leave the call together and the comm stays
// usable.  The error slot is left at 0 for finish_job when no rank failed.
// This rank's own agreement transport can fail while its local work is valid:
//  - flag upload: the flag is raised with a device memset instead (a failed
//    upload counts as a failure every rank sees), so all ranks leave together;
//    if the memset fails too, the flag cannot be raised at all;
//  - the all-reduce cannot be enqueued, or the agreed sum cannot be read back:
//    this rank cannot know whether its peers enter the exchange.
// In those last cases the rank aborts its communicator and fails: peers that
// wait for it in the all-reduce or the exchange leave through their watchdog
// (comm_wait), so no rank waits forever, and none trusts a half-done exchange.
static int preagree(ba_comm* comm, int local_rc) {
    uint64_t* up = comm->h_pin + BA_NCOUNTERS;      // pinned flag upload
    uint64_t* got = comm->h_pin + BA_NCOUNTERS + 1;  // pinned read-back
    *up = local_rc != BA_OK ? 1 : 0;
    *got = 0;
    Rccl& r = rccl();
    int up_rc = BA_OK;
    if (test_fail("upload") || test_fail("upload_memset") ||
        hipMemcpyAsync(comm->d_cnt + kErrSlot, up, sizeof *up, hipMemcpyHostToDevice,
                       comm->stream) != hipSuccess) {
        up_rc = failf(BA_EDEVICE, "error-flag upload");
        // raise it on the device: lowest byte 1 = a flag of 1
        if (test_fail("upload_memset") ||
            hipMemsetAsync(comm->d_cnt + kErrSlot, 0, sizeof(uint64_t), comm->stream) != hipSuccess ||
            hipMemsetAsync(comm->d_cnt + kErrSlot, 1, 1, comm->stream) != hipSuccess) {
            abort_comm(comm);
            return local_rc != BA_OK ? local_rc
                                     : failf(BA_EABORTED, "error flag could neither be uploaded "
                                             "nor set on the device; communicator aborted");
        }
    }
    mark_exchange(comm);
    const ncclResult_t e = with_comm(comm, [&](ncclComm_t cm) {
        return r.all_reduce(comm->d_cnt + kErrSlot, comm->d_cnt + kErrSlot, 1, ncclUint64, ncclSum, cm,
                            comm->stream);
    });
    if (e != ncclSuccess) {
        abort_comm(comm);
        return local_rc != BA_OK ? local_rc
                                 : failf(BA_EABORTED, "ncclAllReduce: %s (communicator aborted)",
                                         r.error_string(e));
    }
    if (test_fail("readback") ||
        hipMemcpyAsync(got, comm->d_cnt + kErrSlot, sizeof *got, hipMemcpyDeviceToHost,
                       comm->stream) != hipSuccess) {
        abort_comm(comm);
        return local_rc != BA_OK ? local_rc
               : up_rc != BA_OK  ? up_rc
                                 : failf(BA_EABORTED, "error-flag read-back; communicator aborted");
    }
    const int rw = comm_wait(comm, "pre-exchange error agreement");
    if (local_rc != BA_OK) return local_rc;
    if (up_rc != BA_OK) return up_rc;
    if (rw != BA_OK) return rw;
    if (*got != 0)
        return failf(BA_EDEVICE, "%llu other rank(s) failed this call before the vote exchange",
                     (unsigned long long)*got);
    return BA_OK;
}

static int begin_job(ba_comm* comm) {
    if (comm->aborted.load()) return fail_aborted(comm);
    if (hipSetDevice(comm->device) != hipSuccess || hipMemsetAsync(comm->d_cnt, 0,
            BA_NCOUNTERS * sizeof(uint64_t), comm->stream) != hipSuccess) {
        abort_comm(comm);  // this rank cannot take part: its peers leave through their watchdog
        return failf(BA_EDEVICE, "rank %d cannot reach its device (communicator aborted)",
                     comm->rank);
    }
    return BA_OK;
}

extern "C" int ba_run_trials_multi(struct ba_ctx* ctx, struct ba_comm* comm, const ba_params* p,
                                   uint64_t total_trials, uint64_t* d_decisions,
                                   uint8_t* d_outcome, ba_counters* counters_out,
                                   uint64_t* share_first, uint64_t* share_count) {
    if (!ctx || !comm || !p) return failf(BA_EINVAL, "ctx, comm and params are required");
    uint64_t first = 0, count = 0;
    int rc = ba_trial_share(total_trials, comm->nranks, comm->rank, &first, &count);
    if (rc != BA_OK) return rc;
    if (share_first) *share_first = first;
    if (share_count) *share_count = count;
    if ((rc = begin_job(comm)) != BA_OK) return rc;  // this rank cannot reach its device
    // every rank validates before any collective; a failure still joins the all-reduce
    int local = ba_validate_internal(p, total_trials);
    if (local == BA_OK && (p->faulty_mode == BA_FAULTY_GIVEN || p->order_mode == BA_ORDER_GIVEN ||
                           p->lie_mode == BA_LIE_TABLE))
        local = failf(BA_EINVAL, "ba_run_trials_multi draws its inputs (faulty/order modes other "
                      "than GIVEN, Philox lies); shard given inputs with ba_run_trials_device");
    if (local == BA_OK && count > 0) {
        ba_params q = *p;
        q.first_trial = p->first_trial + first;  // draws keyed by the global trial index
        local = ba_run_trials_device(ctx, &q, count, nullptr, nullptr, nullptr, nullptr, d_decisions,
                                     d_outcome, comm->d_cnt, comm->stream);
    }
    return finish_job(comm, local, counters_out, true);
}

extern "C" int ba_run_instance_split_level_multi(struct ba_ctx* ctx, struct ba_comm* comm,
                                                 const ba_params* p, uint32_t level,
                                                 uint64_t batch, const uint32_t* d_faulty_mask,
                                                 const uint8_t* d_order, uint64_t* d_decisions,
                                                 uint8_t* d_outcome, ba_counters* counters_out) {
    if (!ctx || !comm || !p) return failf(BA_EINVAL, "ctx, comm and params are required");
    int rc = begin_job(comm);
    if (rc != BA_OK) return rc;
    int local = ba_validate_internal(p, batch);
    const uint32_t n = p->n;
    const uint64_t units = local == BA_OK ? ba_split_units(n, p->m, level) : 0;
    const uint64_t slots = local == BA_OK ? ba_split_vote_slots(n, p->m, level, 0, (uint32_t)units) : 0;
    if (local == BA_OK && slots == 0)
        local = (level == BA_SPLIT_FIRST_HOP || level == BA_SPLIT_SECOND_HOP)
                    ? failf(BA_ENOTSUP, "no level-%u split for n=%u, m=%u (OM(0) has no relay "
                            "subtrees; the second-hop split needs m_eff >= 3)", level, n, p->m)
                    : failf(BA_EINVAL, "split level %u (1: first hop, 2: second hop)", level);
    // one rank owns every unit: the unsplit pass, no vote array -- unless
    // BA_FORCE_SPLIT=1 (test-only switch), which runs the vote array, the
    // grouped-broadcast exchange and the agreement steps on a one-rank
    // communicator, so the real RCCL code runs on a one-GPU box
    if (comm->nranks == 1 && !force_split()) {
        if (local == BA_OK && batch > 0)
            local = ba_run_trials_device(ctx, p, batch, d_faulty_mask, d_order, nullptr, nullptr,
                                         d_decisions, d_outcome, comm->d_cnt, comm->stream);
        return finish_job(comm, local, counters_out, false);
    }
    const uint64_t W = (batch + 63) / 64;
    const size_t need = (size_t)(slots * W * sizeof(uint64_t));
    const char* inj = getenv("BA_TEST_VOTE_ENOMEM");  // test-only: this call's allocation fails
    if (local == BA_OK && inj && inj[0] == '1') {
        local = failf(BA_ENOMEM, "vote buffer (%zu B; injected by BA_TEST_VOTE_ENOMEM)", need);
    } else if (local == BA_OK && need > comm->votes_bytes) {
        (void)hipStreamSynchronize(comm->stream);
        if (comm->d_votes) (void)hipFree(comm->d_votes);
        comm->d_votes = nullptr;
        comm->votes_bytes = 0;
        if (hipMalloc(&comm->d_votes, need) != hipSuccess)
            local = failf(BA_ENOMEM, "vote buffer (%zu B)", need);
        else
            comm->votes_bytes = need;
    }
    // Agree before the exchange: a rank that failed validation or could not
    // allocate its vote buffer cannot join the grouped broadcasts (its peers
    // would wait in them forever), so every rank learns of any failure here
    // and all of them skip the exchange together.
    {
        const int rc_pre = preagree(comm, local);
        if (rc_pre != BA_OK) return rc_pre;
    }
    if (local == BA_OK && batch > 0) {
        uint32_t ub = 0, ue = 0;
        (void)ba_split_share(n, p->m, level, comm->nranks, comm->rank, &ub, &ue);
        if (ue > ub)
            local = ba_split_votes_device(ctx, p, batch, level, ub, ue, d_faulty_mask, d_order,
                                          comm->d_votes + (uint64_t)ub * (n - 1 - level) * W,
                                          comm->stream);
    }
    // the exchange runs whatever happened locally (no rank may skip a collective)
    if (slots > 0 && batch > 0) {
        const int e = ba_comm_allgather_split_votes_device(comm, n, p->m, level, batch,
                                                           comm->d_votes, comm->stream);
        if (local == BA_OK) local = e;
    }
    if (local == BA_OK && batch > 0)
        local = ba_root_from_split_votes_device(ctx, p, batch, level, d_faulty_mask, d_order,
                                                comm->d_votes, d_decisions, d_outcome, comm->d_cnt,
                                                comm->stream);
    return finish_job(comm, local, counters_out, false);
}

extern "C" int ba_run_instance_split_multi(struct ba_ctx* ctx, struct ba_comm* comm,
                                           const ba_params* p, uint64_t batch,
                                           const uint32_t* d_faulty_mask, const uint8_t* d_order,
                                           uint64_t* d_decisions, uint8_t* d_outcome,
                                           ba_counters* counters_out) {
    return ba_run_instance_split_level_multi(ctx, comm, p, BA_SPLIT_FIRST_HOP, batch, d_faulty_mask,
                                             d_order, d_decisions, d_outcome, counters_out);
}
