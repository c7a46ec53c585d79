/*
 * ba.h -- C ABI of libba_hip.so, the MI355X-native batched OM(m)
 * Byzantine-agreement engine.
 *
 * The reference (mathiasplans/byzantine-agreement, /root/reference/ba.py) has no
 * FFI: its hot path is a set of in-process Python methods that the REPL calls
 * (ba.py:381 order, ba.py:386 wait_majority, ba.py:395 quorum, ba.py:399 clear)
 * plus the rpyc service surface between generals (Serv.exposed_*, ba.py:25-63).
 * Each entry point below names the reference interface it replaces.  The
 * ctypes binding a maintainer adds on the reference side is in INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns 0 (BA_OK) or a negative BA_E* code; no exception
 *     or C++ type crosses the ABI.  ba_last_error() gives a thread-local text.
 *   - Host-pointer entry points copy in/out over PCIe; *_device entry points
 *     take device pointers and a hipStream_t (as void*) and are asynchronous.
 *   - One ctx per host thread; a ctx is not thread-safe.  The library owns
 *     the device scratch it allocates inside the ctx (including the run
 *     counter reduction slots).  Calls of one ctx may be made on different
 *     streams: the library orders each call after the ctx's previous one
 *     (an event it records on the previous call's stream when the stream
 *     changes), except while the stream is capturing a graph -- a graph
 *     replay's ordering is the caller's.  So a stream that carried a call of
 *     a ctx must stay valid until that ctx's next call or ba_ctx_destroy.  Device
 *     buffers a captured graph holds stay valid until the ctx grows its
 *     scratch for a LARGER call: give a graph its own ctx.  Replays of graphs
 *     captured from one ctx must not run concurrently with each other or with
 *     an eager call of that ctx: they share the ctx's scratch, counter sink
 *     and persistent-kernel task counter (one replay at a time per ctx).
 *     Capture a ctx's calls only after an eager call of at least the same
 *     size on that ctx: growing scratch or the LEVELS cascade's fan-in
 *     counters allocates (and zeroes the counters on the call's stream),
 *     which a capturing stream cannot do.
 *
 * General indexing: the live generals sorted by id are
 * indexed 0..n-1; index 0 is the commander (lowest live id, ba.py:381 +
 * election ba.py:126-157); 1..n-1 are lieutenants.  n <= BA_MAX_GENERALS.
 */
#ifndef BA_H
#define BA_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BA_ABI_VERSION 1
#define BA_MAX_GENERALS 32
#define BA_MAX_DEPTH 8
#define BA_NCOUNTERS 16

/* error codes */
#define BA_OK 0
#define BA_EINVAL (-1)     /* bad argument (n, m, modes, sizes, null pointer)   */
#define BA_ENOMEM (-2)     /* device or host allocation failed                  */
#define BA_EDEVICE (-3)    /* HIP runtime error / no device                     */
#define BA_ENOTSUP (-4)    /* combination not supported (e.g. table mode, m>1)  */
#define BA_ETOOBIG (-5)    /* tree too large for the requested engine          */
#define BA_EABORTED (-6)   /* communicator aborted (watchdog timeout or a rank's  */
                           /* transport failure): destroy it, create a new one  */

/* lie source for faulty senders (ba.py:45, ba.py:269: random.randint(0,1)) */
#define BA_LIE_PHILOX 0 /* Philox4x32-10 keyed by (seed; trial word, level, slot) */
#define BA_LIE_TABLE 1  /* coins supplied in ba.py's canonical draw order (m=1)   */

/* faulty-set source (ba.py:401-407 g-state <id> faulty) */
#define BA_FAULTY_GIVEN 0  /* faulty_mask[] supplied by the caller               */
#define BA_FAULTY_RANDOM 1 /* f ~ U{0..f}, uniform f-subset of the n generals    */
#define BA_FAULTY_EXACT 2  /* exactly f faulty, uniform f-subset                 */

/* commander order source (ba.py:367-381 actual-order <o>) */
#define BA_ORDER_GIVEN 0  /* order[] supplied by the caller                     */
#define BA_ORDER_RANDOM 1 /* Bernoulli(1/2) attack/retreat                      */
#define BA_ORDER_CONST 2  /* every trial uses order_value                       */

/* order / decision codes.  Any order other than "attack" is relayed as
 * non-attack (ba.py:163-167, 177-181); the commander's own tally keeps it as
 * "other" (ba.py:208-215). */
#define BA_RETREAT 0
#define BA_ATTACK 1
#define BA_OTHER 2     /* order code only: e.g. `actual-order foo`           */
#define BA_UNDEFINED 2 /* decision code: root tie (ba.py:194-195)            */

/* quorum outcome codes (ba.py:246-253) */
#define BA_Q_RETREAT 0
#define BA_Q_ATTACK 1
#define BA_Q_UNDETERMINED 2

/* engines */
#define BA_ENGINE_AUTO 0
#define BA_ENGINE_FUSED 1  /* whole tree per 64-trial word resident on-chip     */
#define BA_ENGINE_LEVELS 2 /* level-synchronous, bit-packed levels in HBM       */

typedef struct ba_params {
    uint32_t n;            /* live generals, 1..32                                */
    uint32_t m;            /* OM depth; ba.py is m=1.  Effective depth min(m,n-2)   */
    uint64_t seed;         /* Philox key for lies and synthetic inputs           */
    uint32_t lie_mode;     /* BA_LIE_*                                            */
    uint32_t faulty_mode;  /* BA_FAULTY_*                                         */
    uint32_t f;            /* RANDOM: max f;  EXACT: f                            */
    uint32_t order_mode;   /* BA_ORDER_*                                          */
    uint32_t order_value;  /* BA_ORDER_CONST: BA_RETREAT/BA_ATTACK/BA_OTHER       */
    uint32_t engine;       /* BA_ENGINE_*                                         */
    uint64_t first_trial;  /* global index of trial 0; multiple of 64             */
    uint32_t table_stride; /* BA_LIE_TABLE: uint32 words per trial in lie_table   */
    uint32_t reserved[5];
} ba_params;

/* Run counters (integer sums; identical for any sharding of the trials). */
#define BA_C_TRIALS 0          /* trials resolved                                   */
#define BA_C_AGREEMENT 1       /* IC1: all loyal lieutenants decided alike          */
#define BA_C_VALID_APPL 2      /* commander loyal (IC2 applicable)                   */
#define BA_C_VALIDITY 3        /* IC2: loyal commander => loyal lts decide its order */
#define BA_C_Q_RETREAT 4       /* quorum outcome counts (ba.py:246-253)              */
#define BA_C_Q_ATTACK 5
#define BA_C_Q_UNDETERMINED 6
#define BA_C_UNDEF_DECISIONS 7 /* lieutenant decisions == undefined (root ties)      */
#define BA_C_IN_BOUND 8        /* trials with f <= m_eff and n > 3 m_eff             */
#define BA_C_BOUND_VIOL 9      /* in-bound trials violating IC1 or IC2               */
#define BA_C_FAULTY_TOTAL 10   /* sum of f over trials                               */
#define BA_C_ATTACK_DECISIONS 11 /* lieutenant decisions == attack                   */
/* Slot 14 (BA_C_CHECK_MISMATCH = BA_C_HANDOFF_LOST): non-zero means the call's
 * results are INVALID.  Every build counts there a granule hand-off of the
 * LEVELS cascade that stayed stale past its bounded poll (2 s; never on a
 * correct run -- a launch starved by other work on the GPU, or preempted that
 * long), and the check build (environment BA_CASC_CHECK=1, read per call; a
 * test switch) also counts hand-off tag mismatches there.  ba_run_trials and
 * the multi-rank jobs (ba_run_trials_multi, ba_run_instance_split*_multi) read
 * it back and return BA_EDEVICE ("in-launch hand-off timed out") instead of
 * results.  Callers of the asynchronous device entries (ba_run_trials_device,
 * ba_root_from_split_votes_device) MUST check slot 14 of their counters after
 * synchronizing before trusting decisions, outcomes or counters (ba_amd/lib.py:
 * check_handoff).  After such an error the ctx stays usable (every eager launch
 * tags its hand-offs with a new epoch); a captured graph repeats its launch's
 * epoch, so a graph whose replay reported it must be captured again.
 * BA_TEST_GRANULE_TICKS (tests only, read per call) shrinks the poll bound
 * (s_memrealtime ticks, 100 MHz) so a launch times out.
 * The cascade's in-launch hand-offs between workgroups rest on gfx950 / ROCm 7.2
 * behaviour measured in MI355X_MICROARCH.md, not on the HIP memory model:
 * granules ({32-bit value half, 32-bit launch tag} in one aligned 8-byte sc1
 * store, read with sc1 loads and re-read until the tag matches: the guide's R2
 * form, observed untorn) for R_1 and, in CO launches, R_{me-2}; drained sc1
 * stores + a relaxed agent-scope counter add + sc1 loads (the guide's
 * valid-forms row 1) only in the one-launch cascade and the non-default wave
 * fan-in (BA_CASC_MTOP=0). The check build and its
 * tests (tests/test_gpu_cascade.py, part of the GPU suite) watch both.
 * Slot 15 is the multi-GPU entries' error flag (always 0 in returned counters). */
#define BA_C_CHECK_MISMATCH 14
#define BA_C_HANDOFF_LOST BA_C_CHECK_MISMATCH

typedef struct ba_counters {
    uint64_t v[BA_NCOUNTERS];
} ba_counters;

/* Per-trial outputs
 *   decisions[t] : uint64, bits [2(r-1), 2(r-1)+1] = decision code of lieutenant r
 *                  (BA_RETREAT / BA_ATTACK / BA_UNDEFINED), r = 1..n-1.
 *                  Replaces Process.majority of each lieutenant (ba.py:188-195).
 *   outcome[t]   : uint8, bits 0-1 quorum code (ba.py:225-255), bit 2 IC1,
 *                  bit 3 IC2 applicable, bit 4 IC2, bit 5 in-bound.
 * Per-trial inputs
 *   faulty_mask[t] : uint32, bit i = general i faulty (ba.py:73, 407)
 *   order[t]       : uint8 order code (ba.py:381 cmd[1])
 *   lie_table      : table_stride uint32 words per trial; bit c (word c/32, bit
 *                    c%32) is the c-th coin of ba.py's canonical draw order,
 *                    1 = "attack" (random.randint(0,1) == 0).
 *   poll_commander : uint32 per trial (BA_LIE_TABLE only, NULL = none): bit r set
 *                    means lieutenant r also polls the commander in its relay
 *                    round.  ba.py:171 skips only the port a lieutenant believes is
 *                    the primary's; after g-add/g-kill that port can be stale or -1
 *                    (ba.py:86-102, 114-115), so the commander's answer is counted
 *                    too.  The stride must hold (n-1) + (n-1)^2 coins.
 */

/* ---- library / context (replaces Process/Serv lifecycle, ba.py:66-112) ---- */
int ba_version(void);
int ba_device_count(int* count);
int ba_ctx_create(int device, struct ba_ctx** out);
void ba_ctx_destroy(struct ba_ctx* ctx);
const char* ba_last_error(void);

/* ---- the hot path -------------------------------------------------------
 * One call resolves `batch` independent OM(m) trials: commander send
 * (Process.order, ba.py:257-285), the relay tree with the lie rule
 * (Serv.exposed_get_order, ba.py:42-57), the recursive majority
 * (Process.get_majority, ba.py:159-195) and the quorum epilogue
 * (get_majorities + quorum, ba.py:197-255).  Null optional pointers:
 * faulty_mask (unless BA_FAULTY_GIVEN), order (unless BA_ORDER_GIVEN),
 * lie_table (unless BA_LIE_TABLE), decisions, outcome, counters.
 * Counters are OVERWRITTEN with this call's totals.
 */
int ba_run_trials(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                  const uint32_t* faulty_mask, const uint8_t* order,
                  const uint32_t* lie_table, const uint32_t* poll_commander,
                  uint64_t* decisions, uint8_t* outcome, ba_counters* counters);

/* Same computation on device buffers, enqueued on `stream` (a hipStream_t as
 * void*; NULL is HIP's null stream, as in every HIP API -- NOT the ctx stream,
 * which only the host-pointer entry point uses).  d_counters (BA_NCOUNTERS uint64 on device) is ACCUMULATED
 * into, so repeated calls sum; zero it first for one call's totals. */
int ba_run_trials_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                         const uint32_t* d_faulty_mask, const uint8_t* d_order,
                         const uint32_t* d_lie_table, const uint32_t* d_poll_commander,
                         uint64_t* d_decisions, uint8_t* d_outcome, uint64_t* d_counters,
                         void* stream);

/* Synthetic inputs of trials [p->first_trial, p->first_trial + batch): the
 * faulty sets (p->faulty_mode RANDOM or EXACT) and commander orders
 * (p->order_mode RANDOM or CONST) that ba_run_trials_device would otherwise
 * draw itself -- the same Philox stream, so running the batch on these as
 * BA_FAULTY_GIVEN / BA_ORDER_GIVEN inputs gives bit-identical results.  This
 * stages a workload's per-trial inputs in HBM ahead of time (bench.py does so
 * before its timed region; the lies stay inside the run: they are the faulty
 * generals' coin flips during the protocol, ba.py:45, 269).  Either output may
 * be NULL; a non-NULL one whose mode is GIVEN is BA_EINVAL.  Asynchronous on
 * `stream` (NULL = HIP's null stream). */
int ba_gen_inputs_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                         uint32_t* d_faulty_mask, uint8_t* d_order, void* stream);

/* ---- one huge instance split by first-hop subtree --------
 * The subtree of first-hop lieutenant j (relay paths starting 0 -> j) needs
 * only L_0[j]; its relay levels and inner majorities are independent of the
 * other subtrees.  A rank owning subtrees [j_begin, j_end) (0-based lieutenant
 * ranks, j_end <= n-1) computes their level-1 child results -- R_1[j.r]
 * (m_eff >= 2) or L_1[j.r] (m_eff == 1), the votes each lieutenant r counts
 * about j (ba.py:169-186 generalised) -- into
 *     d_votes[(j - j_begin)(n-2) + c][w],  w < ceil(batch/64), c < n-2,
 * 64 trials per uint64 word.  Concatenating every rank's d_votes in j order
 * (an all-gather) gives the full [(n-1)(n-2)][W] array that
 * ba_root_from_votes_device turns into the root majorities, quorum and
 * counters -- bit-identical to ba_run_trials_device on the same params.
 * Both are asynchronous on `stream` (NULL = HIP's null stream).
 * LEVELS engine, Philox lies; the batch must fit one scratch chunk
 * (BA_ETOOBIG otherwise: split the batch). */
uint64_t ba_vote_slots(uint32_t n, uint32_t m, uint32_t j_begin, uint32_t j_end);
int ba_subtree_votes_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                            uint32_t j_begin, uint32_t j_end, const uint32_t* d_faulty_mask,
                            const uint8_t* d_order, uint64_t* d_votes, void* stream);
int ba_root_from_votes_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                              const uint32_t* d_faulty_mask, const uint8_t* d_order,
                              const uint64_t* d_votes, uint64_t* d_decisions, uint8_t* d_outcome,
                              uint64_t* d_counters, void* stream);

/* ---- the same split at either of two levels ------------------------------
 * level 1 (BA_SPLIT_FIRST_HOP): units = the n-1 first-hop subtrees; exactly
 *   the entries above (votes R_1 / L_1, n-2 per unit).
 * level 2 (BA_SPLIT_SECOND_HOP): units = the (n-1)(n-2) second-hop subtrees,
 *   one per level-1 slot (j, a) in path order u = j(n-2) + k, a = k + (k >= j);
 *   a unit's relay levels >= 2 and majorities >= 2 need only L_1[j.a], so a
 *   rank owning units [u_begin, u_end) computes their level-2 results
 *   R_2[j.a.r] (n-3 per unit, receivers r in rank order) into
 *       d_votes[(u - u_begin)(n-3) + c][w].
 *   The root pass relays levels 0 and 1 itself (cheap: (n-1)^2 slots), takes
 *   the level-1 majorities over the gathered R_2 and finishes as above.  Needs
 *   m_eff >= 3.  15 first hops split 1,2,..,2 over 8 ranks (slowest rank 2/15
 *   of the tree); 210 second hops split 26/27 (27/210).
 * ba_split_units: the units of a level (0 if the level does not apply);
 * ba_split_vote_slots: vote rows of units [u_begin, u_end);
 * ba_split_share: rank's contiguous unit range, units split as evenly as
 * possible (ranks beyond the unit count get empty ranges).  The level-1 forms
 * equal ba_vote_slots / ba_subtree_share / ba_subtree_votes_device /
 * ba_root_from_votes_device. */
#define BA_SPLIT_FIRST_HOP 1
#define BA_SPLIT_SECOND_HOP 2
uint64_t ba_split_units(uint32_t n, uint32_t m, uint32_t level);
uint64_t ba_split_vote_slots(uint32_t n, uint32_t m, uint32_t level, uint32_t u_begin,
                             uint32_t u_end);
int ba_split_share(uint32_t n, uint32_t m, uint32_t level, int nranks, int rank,
                   uint32_t* u_begin, uint32_t* u_end);
int ba_split_votes_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch, uint32_t level,
                          uint32_t u_begin, uint32_t u_end, const uint32_t* d_faulty_mask,
                          const uint8_t* d_order, uint64_t* d_votes, void* stream);
int ba_root_from_split_votes_device(struct ba_ctx* ctx, const ba_params* p, uint64_t batch,
                                    uint32_t level, const uint32_t* d_faulty_mask,
                                    const uint8_t* d_order, const uint64_t* d_votes,
                                    uint64_t* d_decisions, uint8_t* d_outcome,
                                    uint64_t* d_counters, void* stream);

/* ---- multi-GPU (no ba.py analogue: its generals are threads of
 * one process, ba.py:104-112) ----------------------------------------------
 * One process per GPU.  Rank 0 calls ba_comm_unique_id and ships the
 * BA_COMM_ID_BYTES bytes to every rank out of band (MPI, a socket, a file, a
 * torch.distributed store); every rank calls ba_comm_create on its ctx (the
 * communicator owns an RCCL communicator, a counter buffer and a vote buffer,
 * and runs its whole jobs on the ctx's own stream; destroy a comm before its
 * ctx).  RCCL is opened at run time (librccl.so.1, or the copy already loaded
 * in the process).  Every rank of a comm must make the same sequence of
 * collective calls with the same params. */
#define BA_COMM_ID_BYTES 128
struct ba_comm;
int ba_ctx_device(struct ba_ctx* ctx, int* device);
/* The ctx's own non-blocking HIP stream (the one ba_run_trials uses), valid as
 * long as the ctx.  Callers without a HIP binding of their own (ctypes) can pass
 * it to the *_device entry points; ctxs created one after another get streams
 * on different hardware queues, so their calls can run concurrently. */
int ba_ctx_stream(struct ba_ctx* ctx, void** stream);
int ba_comm_unique_id(unsigned char id[BA_COMM_ID_BYTES]);
int ba_comm_create(struct ba_ctx* ctx, int nranks, int rank,
                   const unsigned char id[BA_COMM_ID_BYTES], struct ba_comm** out);
void ba_comm_destroy(struct ba_comm* comm);
int ba_comm_rank(struct ba_comm* comm, int* nranks, int* rank);
/* Watchdog of the blocking whole jobs below.  A job waits for its collectives
 * by polling the comm's stream; past `timeout_ms` (default 300000, or
 * BA_COMM_TIMEOUT_MS at ba_comm_create) it aborts the communicator
 * (ncclCommAbort: this rank's collectives return) and fails with BA_EABORTED.
 * That bounds every rank's wait when a peer left the protocol (a dead process,
 * or a rank whose own transport failed and which aborted itself: it cannot
 * tell its peers, RCCL has no such message, so they learn it from their own
 * watchdog).  ba_comm_abort does the same on demand (e.g. from a host-side
 * watchdog of the asynchronous collectives).  An aborted comm fails every
 * further call with BA_EABORTED; ba_comm_destroy still frees it. */
int ba_comm_set_timeout(struct ba_comm* comm, uint64_t timeout_ms);
int ba_comm_abort(struct ba_comm* comm);

/* Partition arithmetic (host only).  ba_trial_share: rank's contiguous,
 * 64-trial-word-aligned share [first, first + count) of total_trials, words
 * split as evenly as possible.  ba_subtree_share: rank's first-hop lieutenant
 * range [j_begin, j_end) of the n-1 subtrees (15 over 8 ranks: 1,2,2,2,2,2,2,2;
 * ranks beyond n-1 get empty ranges). */
int ba_trial_share(uint64_t total_trials, int nranks, int rank, uint64_t* first,
                   uint64_t* count);
int ba_subtree_share(uint32_t n, int nranks, int rank, uint32_t* j_begin, uint32_t* j_end);

/* Collectives, asynchronous on `stream` (a hipStream_t as void*).
 * ba_comm_allreduce_device: d_counters (BA_NCOUNTERS uint64) summed over the
 * ranks in place -- the only exchange trial-DP needs.
 * ba_comm_allgather_votes_device: d_votes is the full [(n-1)(n-2)][W] vote
 * array of ba_subtree_votes_device (W = ceil(batch/64)) in which every rank
 * has written the rows of its ba_subtree_share; afterwards every rank holds
 * every row (one grouped RCCL broadcast per rank: an all-gather of unequal
 * shares in place, no padding). */
int ba_comm_allreduce_device(struct ba_comm* comm, uint64_t* d_counters, void* stream);
int ba_comm_allgather_votes_device(struct ba_comm* comm, uint32_t n, uint32_t m, uint64_t batch,
                                   uint64_t* d_votes, void* stream);
/* the same all-gather for a split at `level` (d_votes: the full
 * [ba_split_vote_slots(n, m, level, 0, units)][W] array) */
int ba_comm_allgather_split_votes_device(struct ba_comm* comm, uint32_t n, uint32_t m,
                                         uint32_t level, uint64_t batch, uint64_t* d_votes,
                                         void* stream);

/* Whole jobs, blocking (they return after the collectives, on the comm's
 * stream).  A rank whose local work fails still joins every collective and
 * raises an error flag all-reduced with the counters: every rank then returns
 * an error, none blocks.
 * ba_run_trials_multi: trial-DP over [p->first_trial, + total_trials) --
 *   inputs drawn on the device (faulty/order modes other than GIVEN), Philox
 *   lies, every draw keyed by the global trial index; this rank's share of the
 *   decisions / outcome bytes goes to the optional device buffers
 *   (share_count entries); counters_out = the whole job's totals on every
 *   rank, equal to one unsharded ba_run_trials.
 * ba_run_instance_split_multi: `batch` (normally few, huge) instances split by
 *   first-hop subtree -- subtree votes, vote all-gather, root majorities and
 *   quorum; decisions / outcome (batch entries) and counters_out identical on
 *   every rank and equal to an unsplit ba_run_trials on the same params
 *   (Philox lies, given or drawn inputs).  With one rank the rank owns every
 *   subtree and the call is the unsplit pass itself. */
int ba_run_trials_multi(struct ba_ctx* ctx, struct ba_comm* comm, const ba_params* p,
                        uint64_t total_trials, uint64_t* d_decisions, uint8_t* d_outcome,
                        ba_counters* counters_out, uint64_t* share_first,
                        uint64_t* share_count);
int ba_run_instance_split_multi(struct ba_ctx* ctx, struct ba_comm* comm, const ba_params* p,
                                uint64_t batch, const uint32_t* d_faulty_mask,
                                const uint8_t* d_order, uint64_t* d_decisions,
                                uint8_t* d_outcome, ba_counters* counters_out);
/* ba_run_instance_split_multi at a split level (1 = the call above, 2 =
 * second-hop units, m_eff >= 3) */
int ba_run_instance_split_level_multi(struct ba_ctx* ctx, struct ba_comm* comm,
                                      const ba_params* p, uint32_t level, uint64_t batch,
                                      const uint32_t* d_faulty_mask, const uint8_t* d_order,
                                      uint64_t* d_decisions, uint8_t* d_outcome,
                                      ba_counters* counters_out);

/* Per-kernel timing (tracing aux subsystem; replaces nothing in ba.py, which
 * only prints).  When enabled, every kernel the ctx launches is bracketed by
 * HIP events on its launch stream; ba_profile_read syncs those events and
 * returns the index-th kernel's name, launch count and summed milliseconds
 * (BA_EINVAL past the last kernel).  Enabling/disabling clears the totals. */
int ba_profile_enable(struct ba_ctx* ctx, int on);
int ba_profile_read(struct ba_ctx* ctx, int index, char* name, int name_len,
                    uint64_t* launches, double* total_ms);

/* Engine-clock probe (measurement aux; no ba.py analogue).  Enqueues on `stream`
 * one tiny launch of BA_PROBE_BLOCKS one-wave blocks; block b writes
 * d_out[4b .. 4b+3] = {XCC id, HW id, s_memtime, s_memrealtime}.  s_memtime
 * counts shader-clock cycles on a PER-CU counter (counters of different CUs are
 * not aligned), s_memrealtime a constant 100 MHz clock, so two probes bracketing
 * a stretch of work give that stretch's average engine clock per XCD from rows
 * of the SAME CU (HW id bits 8-15): (dmemtime / drealtime) x 100 MHz
 * (MI355X_MICROARCH.md).  BA_PROBE_BLOCKS = 2048 one-wave blocks reach every CU
 * in each probe.  bench.py brackets a replica of its timed region with two. */
/* Device memory a ctx holds for the engines: the LEVELS scratch and the
 * cascade's fan-in counters, and the budget both are chunked to (environment
 * BA_SCRATCH_BYTES at ba_ctx_create, 8 GiB by default): scratch + counters <=
 * budget for every call the budget admits. */
int ba_ctx_memory(struct ba_ctx* ctx, uint64_t* scratch_bytes, uint64_t* counter_bytes,
                  uint64_t* budget_bytes);

#define BA_PROBE_BLOCKS 2048
int ba_clock_probe_device(struct ba_ctx* ctx, uint64_t* d_out, void* stream);

/* ---- ba.py's coin source (host only, no device needed) --------------------
 * Replaces the unseeded global CPython MT19937 behind random.randint(0, 1)
 * (ba.py:45 relay lies, ba.py:269 commander lies).  ba_mt_seed(s) equals
 * random.seed(s) for 0 <= s < 2^64; ba_mt_next32 equals random.getrandbits(32);
 * each coin is one random.randint(0, 1) draw (1 = "attack", i.e. the draw was
 * 0).  Coins are packed in BA_LIE_TABLE layout, in ba.py's canonical draw
 * order, so a table row feeds ba_run_trials directly. */
typedef struct ba_mt {
    uint32_t state[624];
    uint32_t index;
} ba_mt;

void ba_mt_seed(ba_mt* mt, uint64_t seed);
uint32_t ba_mt_next32(ba_mt* mt);
/* coins one ba.py round draws: (n-1) if the commander is faulty (ba.py:263-273),
 * plus, per lieutenant r, one per other faulty lieutenant and one for a faulty
 * commander it polls (ba.py:169-186).  m == 0: commander coins only. */
uint32_t ba_om1_coin_count(uint32_t n, uint32_t m, uint32_t faulty_mask, uint32_t poll_commander);
/* draw `count` coins into packed[0..words) (zeroed first) */
int ba_mt_draw_coins(ba_mt* mt, uint32_t count, uint32_t* packed, uint32_t words);
/* Batched replay table: trial t is random.seed(seeds[t]) followed by one ba.py
 * round over (faulty_mask[t], poll_commander[t] or 0); row t of `table`
 * (stride uint32 words) receives its coins; next_word[t] (optional) the next
 * getrandbits(32) after the round.  threads <= 0: all host cores. */
int ba_mt_table(uint32_t n, uint32_t m, uint64_t batch, const uint64_t* seeds,
                const uint32_t* faulty_mask, const uint32_t* poll_commander, uint32_t stride,
                uint32_t* table, uint32_t* next_word, int threads);
/* The same table on the device (device buffers, asynchronous on `stream`, in
 * the ctx's call order): one thread per trial seeds CPython's MT19937 and draws
 * the round's coins; the rows equal ba_mt_table's.  Feeds ba_run_trials_device
 * in BA_LIE_TABLE mode without a host round trip (tools/run_configs.py config 1).
 * Uses 2,496 B of the ctx's scratch per trial of a chunk. */
int ba_mt_table_device(struct ba_ctx* ctx, uint32_t n, uint32_t m, uint64_t batch,
                       const uint64_t* d_seeds, const uint32_t* d_faulty_mask,
                       const uint32_t* d_poll_commander, uint32_t stride, uint32_t* d_table,
                       uint32_t* d_next_word, void* stream);

/* Tree geometry helpers (host only, no device needed). */
uint64_t ba_tree_slots(uint32_t n, uint32_t m);             /* sum_k |L_k|       */
uint64_t ba_level_slots(uint32_t n, uint32_t m, uint32_t k); /* |L_k|=P(n-1,k+1) */
int ba_engine_for(uint32_t n, uint32_t m);                  /* engine AUTO picks */

#ifdef __cplusplus
}
#endif
#endif
