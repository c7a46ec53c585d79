// ba_multi.cpp -- trial data-parallel runs across GPUs inside the C ABI
// (ba_run_trials_multi owns the RCCL communicators), for a
// host binding that does not bring torch.distributed.  One process per GPU:
// rank 0 makes a unique id (ba_comm_unique_id), ships its 128 bytes to every
// rank out of band (MPI, a socket, a file), every rank creates the
// communicator on its ctx's device (ba_comm_create), then each call resolves
// this rank's contiguous, word-aligned share of the trial index space and
// all-reduces the 16 run counters over RCCL (xGMI on one node).  No trial data
// crosses GPUs: every draw is keyed by the global trial index, so the shares
// give the same counters as one unsharded run.
//
// RCCL is opened with dlopen on first use: torch's wheel bundles its own
// librccl.so, and a process that imports torch keeps that copy (RTLD_NOLOAD
// finds it) instead of loading a second RCCL beside it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/ba.h"

extern "C" int ba_fail_internal(int code, const char* msg);  // ba_api.cpp: sets ba_last_error

namespace {

struct Rccl {
    bool tried = false;
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    for (const char* name : {"librccl.so", "librccl.so.1"}) {  // already loaded (torch's) first
        if ((r.h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
    }
    if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.h) return r;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
    r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce ||
        !r.error_string)
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

}  // namespace

struct ba_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    uint64_t* d_cnt = nullptr;  // BA_NCOUNTERS uint64 on the device, all-reduced in place
    hipStream_t stream = nullptr;
};

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
    if (hipMalloc(&c->d_cnt, BA_NCOUNTERS * sizeof(uint64_t)) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        if (c->d_cnt) (void)hipFree(c->d_cnt);
        delete c;
        return failf(BA_ENOMEM, "communicator buffers");
    }
    ncclUniqueId u;
    memcpy(&u, id, BA_COMM_ID_BYTES);
    const ncclResult_t e = r.comm_init_rank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        (void)hipFree(c->d_cnt);
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
    if (c->comm && rccl().h) (void)rccl().comm_destroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->d_cnt) (void)hipFree(c->d_cnt);
    delete c;
}

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

extern "C" int ba_run_trials_multi(struct ba_ctx* ctx, struct ba_comm* comm, const ba_params* p,
                                   uint64_t total_trials, uint64_t* d_decisions,
                                   uint8_t* d_outcome, ba_counters* counters_out,
                                   uint64_t* share_first, uint64_t* share_count) {
    if (!ctx || !comm || !p) return failf(BA_EINVAL, "ctx, comm and params are required");
    if (p->faulty_mode == BA_FAULTY_GIVEN || p->order_mode == BA_ORDER_GIVEN ||
        p->lie_mode == BA_LIE_TABLE)
        return failf(BA_EINVAL, "ba_run_trials_multi draws its inputs (faulty/order modes other "
                     "than GIVEN, Philox lies); shard given inputs with ba_run_trials_device");
    if (p->first_trial % 64 != 0) return failf(BA_EINVAL, "first_trial must be a multiple of 64");
    uint64_t first = 0, count = 0;
    int rc = ba_trial_share(total_trials, comm->nranks, comm->rank, &first, &count);
    if (rc != BA_OK) return rc;
    if (share_first) *share_first = first;
    if (share_count) *share_count = count;
    if (hipSetDevice(comm->device) != hipSuccess) return failf(BA_EDEVICE, "hipSetDevice");
    if (hipMemsetAsync(comm->d_cnt, 0, BA_NCOUNTERS * sizeof(uint64_t), comm->stream) != hipSuccess)
        return failf(BA_EDEVICE, "hipMemsetAsync");
    ba_params q = *p;
    q.first_trial = p->first_trial + first;  // draws keyed by the global trial index
    if (count > 0 &&
        (rc = ba_run_trials_device(ctx, &q, count, nullptr, nullptr, nullptr, nullptr, d_decisions,
                                   d_outcome, comm->d_cnt, comm->stream)) != BA_OK)
        return rc;
    // the only collective: the run counters, summed over ranks in place
    Rccl& r = rccl();
    const ncclResult_t e = r.all_reduce(comm->d_cnt, comm->d_cnt, BA_NCOUNTERS, ncclUint64,
                                        ncclSum, comm->comm, comm->stream);
    if (e != ncclSuccess) return failf(BA_EDEVICE, "ncclAllReduce: %s", r.error_string(e));
    if (counters_out &&
        hipMemcpyAsync(counters_out->v, comm->d_cnt, BA_NCOUNTERS * sizeof(uint64_t),
                       hipMemcpyDeviceToHost, comm->stream) != hipSuccess)
        return failf(BA_EDEVICE, "counter copy");
    if (hipStreamSynchronize(comm->stream) != hipSuccess) return failf(BA_EDEVICE, "sync");
    return BA_OK;
}
