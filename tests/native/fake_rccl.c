/* fake_rccl.c -- TEST INFRASTRUCTURE, never shipped or linked by the package.
 *
 * A stand-in for the RCCL entry points libba_hip resolves with dlsym
 * (byzantine-agreement_amd/csrc/ba_multi.cpp, rccl()), selected in a test
 * process with BA_RCCL_LIB=<this .so>.  It exists because RCCL refuses two
 * ranks on one GPU ("invalid usage"), so on a one-GPU box the library's N>1
 * paths -- the counter all-reduce, the grouped-broadcast vote all-gather, the
 * pre-exchange error agreement, the watchdog and its abort -- could otherwise
 * only first run on an 8-GPU node.  Here N processes share cuda:0 and exchange
 * through POSIX shared memory.
 *
 * Semantics kept from RCCL (what the library relies on):
 *  - collectives are ASYNCHRONOUS on the caller's stream: each one is a
 *    device->pinned-host copy, a host function (hipLaunchHostFunc) that does
 *    the exchange across the processes, and a pinned-host->device copy, all
 *    enqueued in stream order; the calling thread never blocks in them;
 *  - every rank must issue the same collectives in the same order; a rank that
 *    skips one leaves its peers' streams waiting in it (no error, no timeout
 *    of their own: a hang, as with RCCL);
 *  - ncclCommAbort acts on THIS rank only: its pending exchanges return and
 *    its communicator is freed; peers are not told (they stay in their
 *    exchange until their own watchdog aborts them);
 *  - ncclGroupStart/End: collectives between them are issued at GroupEnd;
 *  - ncclCommInitRank blocks until all ranks have joined.
 * A safety limit (FAKE_RCCL_TIMEOUT_S, default 120 s) ends any exchange that
 * waits longer, with an async error, so a broken test cannot hang forever.
 *
 * Shared memory per communicator (name from the unique id): a header with the
 * barrier state, then one slot of SLOT bytes per rank (FAKE_RCCL_SLOT_BYTES,
 * default 4 MiB; larger collectives go through in chunks).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

/* the RCCL ABI pieces used (rccl/rccl.h; values must match) */
typedef enum {
    ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
    ncclInvalidArgument = 4, ncclInvalidUsage = 5, ncclRemoteError = 6, ncclInProgress = 7
} ncclResult_t;
typedef enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3 } ncclRedOp_t;
typedef enum {
    ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
    ncclFloat64 = 8
} ncclDataType_t;
#define UID_BYTES 128
typedef struct { char internal[UID_BYTES]; } ncclUniqueId;

typedef struct {
    _Atomic uint32_t joined;
    _Atomic uint32_t arrive;
    _Atomic uint32_t gen;
    uint32_t pad[13];
} Header; /* 64 B; slots start at HDR */
#define HDR 4096

typedef struct Op Op;
typedef struct ncclComm {
    int nranks, rank;
    size_t slot;
    size_t map_bytes;
    unsigned char* base;         /* mapping: header, then nranks slots */
    _Atomic int aborted;         /* set by ncclCommAbort: pending exchanges return */
    _Atomic int async_err;       /* first exchange failure (ncclCommGetAsyncError) */
    Op* ops;                     /* issued, not yet retired */
    char name[UID_BYTES + 8];
} Comm, *ncclComm_t;

struct Op {
    Op* next;
    Comm* c;
    int bcast, root, dtype, redop;
    size_t bytes;
    unsigned char* stage;        /* pinned host buffer */
    hipEvent_t done;             /* recorded after the copy back */
    /* group queue */
    const void* send;
    void* recv;
    hipStream_t stream;
};

static double timeout_s(void) {
    const char* e = getenv("FAKE_RCCL_TIMEOUT_S");
    return e && *e ? atof(e) : 120.0;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static Header* hdr(Comm* c) { return (Header*)c->base; }
static unsigned char* slot(Comm* c, int r) { return c->base + HDR + (size_t)r * c->slot; }

/* all ranks meet; ncclRemoteError when this rank was aborted, ncclSystemError
 * past the safety limit */
static ncclResult_t barrier(Comm* c) {
    Header* h = hdr(c);
    if (atomic_load(&c->aborted)) return ncclRemoteError;  /* never arrive for an aborted rank */
    const uint32_t g = atomic_load(&h->gen);
    if (atomic_fetch_add(&h->arrive, 1) + 1 == (uint32_t)c->nranks) {
        atomic_store(&h->arrive, 0);
        atomic_fetch_add(&h->gen, 1);
        return ncclSuccess;
    }
    const double t0 = now_s(), lim = timeout_s();
    unsigned spins = 0;
    while (atomic_load(&h->gen) == g) {
        if (atomic_load(&c->aborted)) return ncclRemoteError;
        if (++spins > 1000) {
            struct timespec ts = {0, 20000};
            nanosleep(&ts, NULL);
            if ((spins & 255) == 0 && now_s() - t0 > lim) return ncclSystemError;
        } else {
            sched_yield();
        }
    }
    return ncclSuccess;
}

static size_t type_size(int dt) {
    switch (dt) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclInt32: case ncclUint32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

#define REDUCE(T)                                                                          \
    do {                                                                                   \
        T* d = (T*)dst;                                                                    \
        const T* s = (const T*)src;                                                        \
        for (size_t i = 0; i < n; ++i) {                                                   \
            if (op == ncclSum) d[i] += s[i];                                               \
            else if (op == ncclProd) d[i] *= s[i];                                         \
            else if (op == ncclMax) d[i] = s[i] > d[i] ? s[i] : d[i];                      \
            else d[i] = s[i] < d[i] ? s[i] : d[i];                                         \
        }                                                                                  \
    } while (0)

static void reduce_into(void* dst, const void* src, size_t bytes, int dt, int op) {
    const size_t n = bytes / type_size(dt);
    switch (dt) {
        case ncclInt8: REDUCE(int8_t); break;
        case ncclUint8: REDUCE(uint8_t); break;
        case ncclInt32: REDUCE(int32_t); break;
        case ncclUint32: REDUCE(uint32_t); break;
        case ncclInt64: REDUCE(int64_t); break;
        case ncclUint64: REDUCE(uint64_t); break;
        case ncclFloat64: REDUCE(double); break;
        default: break;
    }
}

/* the exchange, on HIP's host-function thread (no HIP calls allowed here) */
static void run_op(void* arg) {
    Op* o = (Op*)arg;
    Comm* c = o->c;
    ncclResult_t r = ncclSuccess;
    /* a failed or aborted comm stays failed: it never touches the shared state again */
    if (atomic_load(&c->async_err) != ncclSuccess || atomic_load(&c->aborted)) return;
    for (size_t off = 0; off < o->bytes && r == ncclSuccess; off += c->slot) {
        const size_t len = o->bytes - off < c->slot ? o->bytes - off : c->slot;
        if (o->bcast) {
            if (c->rank == o->root) memcpy(slot(c, 0), o->stage + off, len);
            if ((r = barrier(c)) != ncclSuccess) break;
            if (c->rank != o->root) memcpy(o->stage + off, slot(c, 0), len);
            r = barrier(c);
        } else {
            memcpy(slot(c, c->rank), o->stage + off, len);
            if ((r = barrier(c)) != ncclSuccess) break;
            memcpy(o->stage + off, slot(c, 0), len);
            for (int q = 1; q < c->nranks; ++q) reduce_into(o->stage + off, slot(c, q), len, o->dtype, o->redop);
            r = barrier(c);
        }
    }
    if (r != ncclSuccess) {
        int expect = ncclSuccess;
        atomic_compare_exchange_strong(&c->async_err, &expect, (int)r);
    }
}

/* retire finished ops (their copy back has completed) */
static void sweep(Comm* c, int wait) {
    Op** pp = &c->ops;
    while (*pp) {
        Op* o = *pp;
        if (wait) (void)hipEventSynchronize(o->done);
        if (hipEventQuery(o->done) == hipSuccess) {
            *pp = o->next;
            (void)hipEventDestroy(o->done);
            (void)hipHostFree(o->stage);
            free(o);
        } else {
            pp = &o->next;
        }
    }
}

static ncclResult_t issue(Op* o) {
    Comm* c = o->c;
    sweep(c, 0);
    if (hipHostMalloc((void**)&o->stage, o->bytes ? o->bytes : 1, 0) != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventCreateWithFlags(&o->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipHostFree(o->stage);
        return ncclUnhandledCudaError;
    }
    const int sends = !o->bcast || c->rank == o->root;
    if ((o->bytes && sends &&
         hipMemcpyAsync(o->stage, o->send, o->bytes, hipMemcpyDeviceToHost, o->stream) != hipSuccess) ||
        hipLaunchHostFunc(o->stream, run_op, o) != hipSuccess ||
        (o->bytes && hipMemcpyAsync(o->recv, o->stage, o->bytes, hipMemcpyHostToDevice, o->stream) != hipSuccess) ||
        hipEventRecord(o->done, o->stream) != hipSuccess) {
        (void)hipStreamSynchronize(o->stream);
        (void)hipEventDestroy(o->done);
        (void)hipHostFree(o->stage);
        return ncclUnhandledCudaError;
    }
    o->next = c->ops;
    c->ops = o;
    return ncclSuccess;
}

/* group queue (thread-local, as RCCL's group state) */
static __thread int g_depth = 0;
static __thread Op* g_head = NULL;
static __thread Op** g_tail = NULL;  /* NULL: &g_head */

static ncclResult_t submit(Op* o) {
    if (g_depth > 0) {
        o->next = NULL;
        if (!g_tail) g_tail = &g_head;
        *g_tail = o;
        g_tail = &o->next;
        return ncclSuccess;
    }
    const ncclResult_t r = issue(o);
    if (r != ncclSuccess) free(o);
    return r;
}

static ncclResult_t check_comm(Comm* c) {
    if (!c) return ncclInvalidArgument;
    if (atomic_load(&c->aborted)) return ncclInvalidUsage;
    return ncclSuccess;
}

/* ------------------------------------------------------------------------- */
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    static _Atomic unsigned counter = 0;
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof *id);
    struct timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    snprintf(id->internal, UID_BYTES, "/ba_fake_rccl_%d_%u_%ld", (int)getpid(),
             atomic_fetch_add(&counter, 1), (long)t.tv_nsec);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || id.internal[0] != '/') return ncclInvalidArgument;
    Comm* c = (Comm*)calloc(1, sizeof *c);
    if (!c) return ncclSystemError;
    const char* e = getenv("FAKE_RCCL_SLOT_BYTES");
    c->slot = e && *e ? (size_t)strtoull(e, NULL, 0) : ((size_t)4 << 20);
    c->slot = (c->slot + 63) & ~(size_t)63;
    c->nranks = nranks;
    c->rank = rank;
    c->map_bytes = HDR + (size_t)nranks * c->slot;
    memcpy(c->name, id.internal, UID_BYTES);
    c->name[UID_BYTES] = 0;
    const int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) { free(c); return ncclSystemError; }
    if (ftruncate(fd, (off_t)c->map_bytes) != 0) { close(fd); free(c); return ncclSystemError; }
    c->base = (unsigned char*)mmap(NULL, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (c->base == MAP_FAILED) { free(c); return ncclSystemError; }
    atomic_fetch_add(&hdr(c)->joined, 1);
    const ncclResult_t r = barrier(c);  /* every rank has mapped the segment */
    if (r != ncclSuccess) {
        munmap(c->base, c->map_bytes);
        free(c);
        return r;
    }
    if (rank == 0) shm_unlink(c->name);  /* the mappings stay; nothing is left in /dev/shm */
    *out = c;
    return ncclSuccess;
}

static void release(Comm* c) {
    sweep(c, 1);
    munmap(c->base, c->map_bytes);
    free(c);
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    release(c);
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    atomic_store(&c->aborted, 1);  /* this rank's pending exchanges return */
    release(c);
    return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* err) {
    if (!c || !err) return ncclInvalidArgument;
    *err = (ncclResult_t)atomic_load(&c->async_err);
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                           ncclRedOp_t op, ncclComm_t c, hipStream_t stream) {
    ncclResult_t r = check_comm(c);
    if (r != ncclSuccess) return r;
    if (!type_size(dt) || op < ncclSum || op > ncclMin) return ncclInvalidArgument;
    Op* o = (Op*)calloc(1, sizeof *o);
    if (!o) return ncclSystemError;
    *o = (Op){.c = c, .bcast = 0, .dtype = dt, .redop = op, .bytes = count * type_size(dt),
              .send = send, .recv = recv, .stream = stream};
    return submit(o);
}

ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, ncclDataType_t dt, int root,
                           ncclComm_t c, hipStream_t stream) {
    ncclResult_t r = check_comm(c);
    if (r != ncclSuccess) return r;
    if (!type_size(dt) || root < 0 || root >= c->nranks) return ncclInvalidArgument;
    Op* o = (Op*)calloc(1, sizeof *o);
    if (!o) return ncclSystemError;
    *o = (Op){.c = c, .bcast = 1, .root = root, .dtype = dt, .bytes = count * type_size(dt),
              .send = send, .recv = recv, .stream = stream};
    return submit(o);
}

ncclResult_t ncclGroupStart(void) {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void) {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    ncclResult_t first = ncclSuccess;
    Op* o = g_head;
    g_head = NULL;
    g_tail = NULL;
    while (o) {
        Op* nx = o->next;
        const ncclResult_t r = first == ncclSuccess ? issue(o) : ncclInternalError;
        if (r != ncclSuccess) {
            free(o);
            if (first == ncclSuccess) first = r;
        }
        o = nx;
    }
    return first;
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake_rccl)";
        case ncclUnhandledCudaError: return "unhandled HIP error (fake_rccl)";
        case ncclSystemError: return "system error / exchange timed out (fake_rccl)";
        case ncclInternalError: return "internal error (fake_rccl)";
        case ncclInvalidArgument: return "invalid argument (fake_rccl)";
        case ncclInvalidUsage: return "invalid usage: communicator aborted (fake_rccl)";
        case ncclRemoteError: return "exchange ended by this rank's abort (fake_rccl)";
        default: return "unknown (fake_rccl)";
    }
}
