"""bench.py -- OM(m) trial-decisions/s on MI355X (BASELINE.json metric, config 2).

A step resolves one batch of synthetic trials (n=10 generals, OM(3), 1M trials
per GPU by default: faulty set = uniform f-subset with f ~ U{0..3}, order ~
Bernoulli(1/2)).  Each trial's inputs (its faulty set and commander order) are
staged in HBM before the timed region by ba_gen_inputs_device (the same Philox
stream the kernel would draw; results are bit-identical either way), so `value`
has inputs resident as the measurement contract asks.  Everything the protocol
computes stays inside the timed region: every lie (a faulty general's coin
flip, ba.py:45, 269) is drawn from Philox in the kernel, every tree level and
majority is resolved, every lieutenant's root decision is written to HBM
(uint64/trial), plus the per-trial quorum/IC outcome byte and run counters.
`value_with_input_generation` repeats the timing with the inputs drawn inside
the kernel too.  Both passes follow a common warm-up of >= 1 s of back-to-back
steps, so neither pays the clock ramp.

Steps in flight (--streams, default 2): step i is enqueued on stream i % 2, each
stream with its own library ctx and output buffers, so two steps can run at
once.  A WAVE launch's last ~quarter runs one wave per SIMD (the SIMD's older
wave wins issue arbitration and finishes first); the next step's waves fill
those slots.  Every step is still a complete 1M-trial pass; the counters of
all K steps are checked against a one-stream pass of the same steps, reported
as `value_single_stream`, whose per-step HIP-event time is also the kernel's
launch time the roofline uses (and that rocprofv3 reports for --streams 1).

N>1: launched one process per GPU by torch.distributed.run.  Trials shard by
global index (weak scaling, no data-path collective); the run counters are
all-reduced once over RCCL inside the C ABI (ba_comm_allreduce_device) at the
end of the timed region, and that all-reduce is the closing barrier (it ends
on a rank only after every rank's steps have ended); the opening barrier is a
gloo barrier followed by an RCCL all-reduce of a dummy buffer, so the ranks
leave it together.  torch.distributed (gloo) carries the RCCL unique id and
the max-over-ranks of the wall time.  (A gloo barrier inside the timed region
would add a host TCP round trip to a ~1 ms region.)

Prints ONE JSON line (rank 0).  DESIGN.md §5 gives the roofline accounting:
`roofline` is the dominant kernel's HBM roofline on the bytes it must move
(its per-trial inputs and outputs), `valu_roofline` its vector-issue roofline
from the committed rocprofv3 counters of the same build, `compute_roofline`
its Philox floor; the level-synchronous byte count of SURVEY.md §8d is kept as
the labelled side figure `level_synchronous_equivalent`.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CLOCK_GHZ = 2.4        # MI355X_MICROARCH.md: max engine clock
SIMDS = 1024           # 256 CUs x 4 SIMDs
VALU_ISSUE_CYCLES = 2  # one wave64 VALU instruction per 2 cycles on a SIMD-32 (MI355X_MICROARCH.md)
# Philox4x32-10 issue ceilings of one MI355X (tools/philox_bench.hip: the best
# measured code shape per occupancy -- round 3: the kernels' grouped asm rounds
# with the keys as VGPR operands) by resident waves per SIMD
# the code shape the kernels ship: round keys and multipliers as VGPR operands
PHILOX_PEAK_SRC = "profiles/r04r_philox_bench_mvgpr.jsonl"
PHILOX_PEAK_FALLBACK = {2: 9.81e11, 4: 1.048e12, 8: 1.095e12}
PHILOX_BENCH_INSTS_PER_CALL = 40  # xor3 variant: 10 rounds x (2 v_mad_u64_u32 + 2 v_bitop3)
# bytes one trial's own inputs and outputs occupy: faulty mask (u32) + order (u8)
# read, decision word (u64) + outcome byte written (include/ba.h)
IO_BYTES_IN, IO_BYTES_OUT = 5, 9


def philox_peaks():
    """{waves per SIMD: calls/s} from the committed philox_bench run."""
    out = {}
    try:
        for line in open(os.path.join(ROOT, PHILOX_PEAK_SRC)):
            d = json.loads(line)
            if "waves_per_simd" in d and "philox_calls_per_s" in d:
                w = int(d["waves_per_simd"])
                out[w] = max(out.get(w, 0.0), float(d["philox_calls_per_s"]))
    except (OSError, ValueError):
        pass
    return out or dict(PHILOX_PEAK_FALLBACK)


def philox_calls_per_trial_word(n: int, m: int) -> int:
    """Fewest Philox4x32-10 calls that produce every lie bit of a 64-trial word:
    each call yields two slot-words, so level k needs ceil(|L_k| / 2) calls."""
    from ba_amd import lib as L
    lib = L.load()
    me = L.effective_depth(n, m)
    return sum((lib.ba_level_slots(n, m, k) + 1) // 2 for k in range(me + 1))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def level_synchronous_bytes_per_trial(n: int, m: int) -> int:
    """8 B per-trial I/O + 2 x ceil(bit-packed OM tree / 8) -- what a
    level-synchronous design (the LEVELS engine) writes and reads per trial."""
    from ba_amd import lib as L
    slots = L.load().ba_tree_slots(n, m)
    return 8 + 2 * ((slots + 7) // 8)


def kernel_io_bytes(name: str, n: int, m: int, batch: int, staged: bool) -> int:
    """Algorithmic HBM bytes of one launch of `name` over `batch` trials: the bytes
    the kernel cannot avoid moving."""
    from ba_amd import lib as L
    lib = L.load()
    me = L.effective_depth(n, m)
    S = [lib.ba_level_slots(n, m, k) for k in range(me + 1)]
    words = (batch + 63) // 64
    if name.startswith("k_om") or name.startswith("k_fused"):  # tree on chip: per-trial I/O only
        return (IO_BYTES_IN if staged else 0) * batch + IO_BYTES_OUT * batch
    if name == "k_leaf":  # levels me-1, me never materialised: read L_{me-2}, write R_{me-1}
        return 8 * words * (S[me - 2] + S[me - 1])
    if name == "k_leaf_up":  # read L_{me-2}, write R_{me-2} (the sibling-group majority)
        return 8 * words * 2 * S[me - 2]
    if name == "k_epilogue":  # read L_0, the level-1 votes and the n + 3 input planes; write I/O
        return 8 * words * (S[0] + S[1] + n + 3) + IO_BYTES_OUT * batch
    if name == "k_relay_top":  # write levels 0..me-2 once
        return 8 * words * sum(S[: me - 1])
    return 0


def so_digest() -> str:
    """sha256 (16 hex) of the library this process runs: ties committed PMC counters
    to the exact build (tools/pmc_summary.py records the same digest)."""
    from ba_amd import lib as L
    h = hashlib.sha256(open(L.LIB_PATH, "rb").read()).hexdigest()
    return h[:16]


def pmc_for(n, m, batch, engine, kernel, digest):
    """Per-launch counters of `kernel` from the newest committed rocprofv3 PMC summary
    of this workload (profiles/*pmc*.json).  Returns (entry, path, same_build)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        c = d.get("config") or {}
        if (c.get("n"), c.get("m"), c.get("batch"), c.get("engine")) != (n, m, batch, engine):
            continue
        for name, e in d.get("kernels", {}).items():
            if kernel in name and "traffic_bytes" in e:
                same = d.get("lib_sha16") == digest
                if same:
                    return e, os.path.relpath(path, ROOT), True
                if best is None:
                    best = (e, os.path.relpath(path, ROOT), False)
    return best if best else (None, None, False)


def cpu_threads() -> int:
    """The host threads this job may use: OMP_NUM_THREADS if the launcher set it (the
    GPU pool sets it to the job's CPU share), else the process's CPU affinity."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def run_cpu_baseline(n, m, seed, fmax, budget_s, ranges, gpu_counters, extra_first):
    """Time the word-sliced OpenMP C port (oracle/ba_sliced.c: 64 trials per word,
    one Philox call per two slot-words, the GPU engines' minimum draw count) on a
    bounded sample of the same workload, inputs staged first as on the GPU.

    The sample starts with exactly the trials this rank's GPU resolved in its
    timed steps, `ranges` = [(first, count), ...] (one contiguous range at world
    1; one range per step at world N, trials shard by step): the port's run
    counters over them must equal this rank's GPU counters from before the
    all-reduce (the quorum / IC tallies of ba.py:197-255), else the
    bench exits non-zero.  It then continues with trials from `extra_first` on
    (outside every rank's timed ranges) until ~budget_s of CPU work; `value` is
    all sampled trials over the time of both runs."""
    import oracle_c
    threads = cpu_threads()
    kw = dict(seed=seed, faulty_mode=1, f=fmax, order_mode=1)

    def timed_run(f0, cnt):
        fm, oc = oracle_c.sliced_gen(n, cnt, threads=threads, first_trial=f0, **kw)
        t0 = time.perf_counter()
        _, _, c = oracle_c.sliced_run(n, m, cnt, seed=seed, faulty=fm, order=oc, first_trial=f0,
                                      threads=threads, want_outputs=False)
        return c, time.perf_counter() - t0

    got, dt0, count = None, 0.0, 0
    for f0, cnt in ranges:
        c, dt = timed_run(f0, cnt)
        got = c if got is None else {k: got[k] + c[k] for k in got}
        dt0 += dt
        count += cnt
    want = {k: gpu_counters[k] for k in got}
    match = got == want
    if not match:
        raise SystemExit(f"cpu_baseline: the C port's counters over this GPU's timed trials "
                         f"({len(ranges)} ranges, {count} trials) differ from the GPU's: {got} vs {want}")
    rate = count / max(dt0, 1e-9)
    extra = int(min(max(rate * budget_s - count, 0), 1 << 27)) // 64 * 64
    dt1 = 0.0
    if extra:
        _, dt1 = timed_run(extra_first, extra)
    sample, dt = count + extra, dt0 + dt1
    value = sample / dt
    nproc = os.cpu_count() or 1
    where = (f"trials [{ranges[0][0]}, {ranges[0][0] + count})" if len(ranges) == 1 else
             f"this rank's {len(ranges)} step ranges of {ranges[0][1]} trials (first {ranges[0][0]})")
    return {"value": round(value, 1), "unit": "trial-decisions/s", "cores": threads, "kind": "port",
            "sample": f"word-sliced OpenMP C port (oracle/ba_sliced.c, x{threads} threads) on "
                      f"{where} of the same n={n}, m={m} synthetic stream: this GPU's {count} timed "
                      f"trials, then {extra} more from trial {extra_first} (inputs staged first, as "
                      f"on the GPU), {dt:.1f} s; host CPU: {cpu_model()}, nproc={nproc}; {threads} "
                      f"threads = this job's CPU share (OMP_NUM_THREADS / affinity)",
            "per_thread_value": round(value / threads, 1),
            "all_cores_projection": {"value": round(value / threads * nproc, 1), "cores": nproc,
                                     "note": "per-thread rate x nproc, not measured (the pool "
                                             "grants this job its CPU share only)"},
            "counters_match": match,
            "counters_checked": {"ranges": len(ranges), "first_trial": ranges[0][0], "trials": count,
                                 "what": "all 12 run counters of this rank's timed steps (before "
                                         "the all-reduce)"},
            "reference_ba_py": {"value_us_per_trial": 574.0, "config": "OM(1) n=10, one core",
                                "where": "dev container (Intel Xeon), BASELINE.md; ba.py cannot "
                                         "run on the GPU box (rpyc and the reference are absent)"}}


def clock_from_probes(p0, p1):
    """Average engine clock between two ba_clock_probe_device probes, per XCD:
    (d s_memtime / d s_memrealtime) x 100 MHz, rows {xcc, hw, memtime, realtime}.
    s_memtime is a per-CU counter (two CUs' counters differ by arbitrary offsets,
    even within one shader engine: profiles/r04w_probe_pairing.log), so a difference
    is only taken between rows of the SAME XCD and CU (HW_ID bits 8-15: CU, SH, SE)
    in the two probes; the XCD's clock is the median over those pairs.  An XCD whose
    probe blocks landed on no common CU is left out (a difference across CUs is not a
    clock).  Returns (median MHz over the XCDs measured, {xcc: MHz})."""
    import statistics

    def by_unit(rows):
        d = {}
        for xcc, hw, mt, rt in rows:
            d.setdefault((int(xcc), int(hw) & 0xFF00), []).append((int(mt), int(rt)))
        return {k: sorted(v)[len(v) // 2] for k, v in d.items()}

    ua, ub = by_unit(p0), by_unit(p1)
    pairs = {}
    for key in set(ua) & set(ub):
        dmt, drt = ub[key][0] - ua[key][0], ub[key][1] - ua[key][1]
        if drt > 0 and dmt > 0:
            pairs.setdefault(key[0], []).append(dmt / drt * 100.0)
    mhz = {k: round(statistics.median(v), 1) for k, v in sorted(pairs.items())}
    return (statistics.median(mhz.values()) if mhz else None), mhz


def first_trial(i: int, rank: int, world: int, batch: int) -> int:
    """Global index of the first trial of step slot i on `rank`: slot i of the
    job is world x batch consecutive trials, rank r's shard the r-th batch of
    them (weak scaling, disjoint shards; Philox keyed by global trial index)."""
    return (i * world + rank) * batch


def rank_ranges(base: int, steps: int, rank: int, world: int, batch: int) -> list:
    """The (first, count) trial ranges one rank resolves in the timed steps
    base .. base+steps-1: one contiguous range at world 1, one per step otherwise."""
    if world == 1:
        return [(first_trial(base, 0, 1, batch), batch * steps)]
    return [(first_trial(base + i, rank, world, batch), batch) for i in range(steps)]


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(gpus: int, argv: list, port: int) -> list:
    """The torch.distributed.run command bench.py starts for --gpus N > 1 when it
    was not launched by one: N local ranks, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def check_or_launch_world(gpus: int, argv: list, env) -> int | None:
    """None: run this process as a rank (or alone).  Otherwise the exit code to
    leave with: the launched job's, or 2 when a launcher's WORLD_SIZE disagrees
    with --gpus (the line would report a different n_gpus than asked)."""
    if gpus < 1:
        print(f"bench: --gpus {gpus} must be >= 1", file=sys.stderr, flush=True)
        return 2
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench: WORLD_SIZE={ws} but --gpus {gpus}: launch one rank per GPU asked for",
                  file=sys.stderr, flush=True)
            return 2
        return None
    if gpus == 1:
        return None
    import subprocess
    cmd = launch_cmd(gpus, argv, free_port())
    child_env = dict(env)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=child_env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="trials per GPU per step")
    ap.add_argument("--fmax", type=int, default=-1)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xBA5EED)
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "levels"])
    ap.add_argument("--warm-s", type=float, default=1.0,
                    help="common warm-up: back-to-back steps before any timed pass")
    ap.add_argument("--cpu-budget-s", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--inputs-in-kernel", action="store_true",
                    help="draw faulty sets/orders inside the timed kernel (no staging)")
    ap.add_argument("--streams", type=int, default=2,
                    help="steps in flight: step i runs on stream (and ctx) i %% streams, so the next "
                         "step's waves fill the SIMDs a finishing step leaves idle")
    args = ap.parse_args()

    # --gpus N: one process per GPU.  Launched without a launcher (no WORLD_SIZE),
    # N > 1 starts torch.distributed.run on N local ranks as a CHILD process and
    # exits with its code; nothing here has touched the GPU yet.  Under a launcher
    # the world it made must be the one asked for.
    rc = check_or_launch_world(args.gpus, sys.argv[1:], os.environ)
    if rc is not None:
        raise SystemExit(rc)

    import torch
    from ba_amd import lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = comm = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # rendezvous, barriers, wall-time max; RCCL is in the C ABI
    # BA_BENCH_DEVICE: put every rank on one device (a multi-rank rehearsal on a
    # one-GPU box; RCCL refuses two ranks on one GPU, so the counters then go
    # through the gloo fallback)
    local = int(os.environ.get("BA_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n, m, B = args.n, args.m, args.batch
    fmax = L.default_fmax(n) if args.fmax < 0 else args.fmax
    engine_id = {"auto": L.ENGINE_AUTO, "fused": L.ENGINE_FUSED, "levels": L.ENGINE_LEVELS}[args.engine]
    NS = max(1, args.streams)
    # the steps' ctxs, created one after another before anything else makes streams
    # (RCCL does): consecutive ctx streams land on different hardware queues
    engines = [L.Engine(dev.index) for _ in range(NS)]
    eng = engines[0]
    collective = None
    if world > 1:
        from ba_amd import dist as D
        try:
            comm = D.init_comm(eng)
            collective = "rccl (libba_hip ba_comm_allreduce_device)"
            if os.environ.get("BA_RCCL_LIB"):  # test-only replacement (tests/native/fake_rccl.c)
                collective = ("rccl API of BA_RCCL_LIB=" + os.path.basename(os.environ["BA_RCCL_LIB"]) +
                              " (libba_hip ba_comm_allreduce_device; a test stand-in, not RCCL)")
        except L.BAError as e:  # reported in the JSON line, never silent
            print(f"bench: RCCL communicator failed ({e}); counters all-reduced over gloo",
                  file=sys.stderr, flush=True)
            collective = f"gloo fallback (RCCL failed: {e})"
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    # dedicated (non-null) streams, one library ctx each (a ctx orders its own calls,
    # so steps overlap only across ctxs); every ctx adds its run counters into cnt
    # (atomic sums).  Stream 0 carries the HIP events and the collectives.
    # The steps run on the ctxs' own streams: ctxs created one after another get
    # streams on different hardware queues (two torch pool streams can share one
    # queue, which serialises them: rocprofv3 showed both on queue 4).
    streams = [torch.cuda.ExternalStream(e.stream(), device=dev) for e in engines]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    decs = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(NS)]
    outs = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(NS)]

    def first_of(i):
        return first_trial(i, rank, world, B)

    # every step's inputs staged in HBM and every step's params built before timing
    n_warm_slots = args.warmup + 2
    n_total = n_warm_slots + 3 * args.steps
    staged_params, gen_params, staged = [], [], []
    if not args.inputs_in_kernel:
        fbuf = torch.empty((n_total, B), dtype=torch.int32, device=dev)
        obuf = torch.empty((n_total, B), dtype=torch.uint8, device=dev)
    for i in range(n_total):
        gp = L.make_params(n, m, args.seed, L.LIE_PHILOX, L.FAULTY_RANDOM, fmax, L.ORDER_RANDOM,
                           L.ATTACK, engine_id, first_of(i))
        gen_params.append(gp)
        if not args.inputs_in_kernel:
            eng.gen_inputs_device(gp, B, d_faulty=fbuf[i].data_ptr(), d_order=obuf[i].data_ptr(),
                                  stream=sp)
            staged.append((fbuf[i].data_ptr(), obuf[i].data_ptr()))
            staged_params.append(L.make_params(n, m, args.seed, L.LIE_PHILOX, L.FAULTY_GIVEN, fmax,
                                               L.ORDER_GIVEN, L.ATTACK, engine_id, first_of(i)))
    torch.cuda.synchronize(dev)
    cptr = cnt.data_ptr()

    def step(i, in_kernel, ns=NS):
        j = i % ns
        e, st = engines[j], streams[j].cuda_stream
        dptr, optr = decs[j].data_ptr(), outs[j].data_ptr()
        if in_kernel:
            e.run_device(gen_params[i], B, d_decisions=dptr, d_outcome=optr, d_counters=cptr,
                         stream=st)
        else:
            fp, op = staged[i]
            e.run_device(staged_params[i], B, d_faulty=fp, d_order=op, d_decisions=dptr,
                         d_outcome=optr, d_counters=cptr, stream=st)

    # common warm-up: >= warm_s of back-to-back steps (both modes) before any timing,
    # so the first timed pass does not pay the clock / power ramp
    # (the warm-up walks every staged step, so its dispatches read inputs as cold
    # as the timed ones do: a rocprofv3 average over all dispatches then agrees
    # with the HIP-event figure below)
    t_w = time.perf_counter()
    k = 0
    while True:
        for i in range(n_total):
            step(i, args.inputs_in_kernel)
            if not args.inputs_in_kernel and i % 4 == 0:
                step(i, True)
        torch.cuda.synchronize(dev)
        k += 1
        if time.perf_counter() - t_w >= args.warm_s and k >= 1:
            break
    warm_s = time.perf_counter() - t_w

    bar = torch.zeros(16, dtype=torch.int64, device=dev)  # RCCL barrier operand
    local_cnt = torch.zeros(16, dtype=torch.int64, device=dev)  # this rank's counters, pre all-reduce
    probes = torch.zeros((2, L.PROBE_BLOCKS, 4), dtype=torch.int64, device=dev)

    host_enq = [0.0]  # ms from t0 until every step was enqueued (the last timed pass)

    def timed(base, in_kernel, ns=NS, probe=False):
        cnt.zero_()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
            if comm is not None:  # release every rank together: a device-side RCCL barrier
                comm.allreduce_device(bar.data_ptr(), stream=sp)
        torch.cuda.synchronize(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        if probe:  # the clock pass (untimed): one probe before the steps, one after
            eng.clock_probe_device(probes[0].data_ptr(), stream=sp)
        ev0.record(stream)
        for j in range(1, ns):
            streams[j].wait_event(ev0)
        for i in range(args.steps):
            step(base + i, in_kernel, ns)
        for j in range(1, ns):
            stream.wait_stream(streams[j])
        ev1.record(stream)
        if probe:
            eng.clock_probe_device(probes[1].data_ptr(), stream=sp)
        if comm is not None:
            local_cnt.copy_(cnt)  # 128 B on the stream: the rank's own tallies (cpu_baseline)
            # the only collective: the run counters (RCCL).  It is also the closing
            # barrier: it completes on a rank only after every rank's steps ended.
            comm.allreduce_device(cptr, stream=sp)
        t_enq = time.perf_counter()
        # (a host loop polling an event here slowed the GPU's own steps by ~7%:
        # tools/host_overhead.py, profiles/r04d_host_overhead.log)
        torch.cuda.synchronize(dev)
        if dist and comm is None:  # gloo fallback: host all-reduce, then a host barrier
            host = cnt.cpu()
            local_cnt.copy_(host)
            dist.all_reduce(host)
            cnt.copy_(host)
            dist.barrier()
        wall = time.perf_counter() - t0
        if not dist:  # bookkeeping for cpu_baseline, outside the timed wall
            local_cnt.copy_(cnt)
        host_enq[0] = (t_enq - t0) * 1e3
        elapsed = torch.tensor([wall], dtype=torch.float64)
        if dist:
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        return float(elapsed.item()), ev0.elapsed_time(ev1)

    total_trials = B * args.steps * world
    base = n_warm_slots
    # one untimed rehearsal of the timed region itself: its cross-stream event
    # waits are the first of the process, and the first one costs ~0.1 ms of
    # one-time setup that no later region pays
    timed(base, args.inputs_in_kernel)
    T, gpu_ms = timed(base, args.inputs_in_kernel)
    enq_ms = host_enq[0]
    counters = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
    local_counters = dict(zip(L.COUNTER_NAMES, [int(x) for x in local_cnt.cpu().tolist()]))
    value = total_trials / T
    value_gen = gen_ms = None
    if not args.inputs_in_kernel:
        T2, gen_ms = timed(base, True)  # same trials, inputs drawn in the kernel
        counters2 = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
        if counters2 != counters:
            raise SystemExit(f"staged-input and in-kernel-input runs disagree: {counters} vs {counters2}")
        value_gen = total_trials / T2
    # the same steps one at a time on one stream: the single-stream rate, and (one launch
    # per step) the kernel's own average launch time for the roofline below
    T1, gpu_ms_1 = timed(base, args.inputs_in_kernel, 1)
    counters1 = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
    if counters1 != counters:
        raise SystemExit(f"{NS}-stream and one-stream runs disagree: {counters} vs {counters1}")
    value_1 = total_trials / T1
    # the clock pass: the timed region's steps again (untimed), bracketed by two
    # engine-clock probes on the launch stream (attributes a run's
    # rate to the clock it ran at)
    Tc, gpu_ms_c = timed(base, args.inputs_in_kernel, NS, probe=True)
    pr = probes.cpu().numpy()
    sclk, sclk_xcd = clock_from_probes(pr[0], pr[1])

    # per-kernel HIP-event timing on the launch stream (a further pass of new steps)
    kernels, roof, valu_roof, compute_roof, side = {}, None, None, None, None
    staged_mode = not args.inputs_in_kernel
    if not args.no_profile:
        eng.profile(True)
        for i in range(args.steps):
            step(base + args.steps + i, args.inputs_in_kernel, 1)
        torch.cuda.synchronize(dev)
        kernels = eng.profile_read()
        eng.profile(False)
    avg_src = None
    if kernels:
        name, (nl, ms) = max(kernels.items(), key=lambda kv: kv[1][1])
        avg_ms = ms / nl
        avg_src = "per-launch HIP events (profiling pass)"
        if len(kernels) == 1 and nl == args.steps:
            # a step is exactly one launch of this kernel: its average duration is the
            # one-stream timed region's HIP-event time over the steps (the per-launch
            # event pairs of the profiling pass add ~3 us of event overhead to each)
            avg_ms = gpu_ms_1 / args.steps
            avg_src = "one-stream timed-region HIP events / steps (one launch per step)"
        digest = so_digest()
        pmc, pmc_src, same_build = pmc_for(n, m, B, args.engine, name, digest)
        io = kernel_io_bytes(name, n, m, B, staged_mode)
        achieved = io / (avg_ms * 1e-3) / 1e9
        traffic = pmc["traffic_bytes"] if pmc else None
        roof = {"bound": "hbm", "kernel": name, "avg_ms": round(avg_ms, 4), "avg_ms_source": avg_src,
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": round(traffic) if traffic else None,
                "traffic_frac": round(traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "algorithmic_bytes_per_launch": io,
                "algorithmic_bytes_per_trial": io / B,
                "traffic_source": pmc_src, "traffic_same_build": same_build,
                "note": ("bytes the kernel must move: per-trial inputs (5 B, staged) and outputs "
                         "(9 B); the OM tree lives in LDS/registers, so HBM is not this kernel's "
                         "bound -- valu_roofline is") if name.startswith(("k_om", "k_fused")) else
                        ("bytes the kernel must move through the LEVELS arrays (kernel_io_bytes); "
                         "it draws its leaf levels from Philox in registers, so it is VALU-bound")}
        if pmc and pmc.get("counters", {}).get("SQ_INSTS_VALU"):
            insts = pmc["counters"]["SQ_INSTS_VALU"]
            cycles = avg_ms * 1e-3 * CLOCK_GHZ * 1e9
            valu_roof = {"bound": "valu", "kernel": name,
                         "achieved": round(insts * VALU_ISSUE_CYCLES / (avg_ms * 1e-3) / 1e9, 1),
                         "peak": round(SIMDS * CLOCK_GHZ, 1), "unit": "G SIMD-cycles/s",
                         "frac": round(insts * VALU_ISSUE_CYCLES / (SIMDS * cycles), 4),
                         "valu_insts_per_launch": insts,
                         "formula": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x avg launch)",
                         "source": pmc_src, "same_build": same_build}
        words = (B + 63) // 64
        calls = philox_calls_per_trial_word(n, m) * words
        rate = calls / (avg_ms * 1e-3)
        peaks = philox_peaks()
        wps = 2 if name.startswith("k_om") else max(peaks)
        peak = peaks.get(wps, max(peaks.values()))
        compute_roof = {"bound": "valu (Philox4x32-10 lie draws)", "kernel": name,
                        "achieved": round(rate / 1e9, 2), "peak": round(peak / 1e9, 2),
                        "unit": "G Philox calls/s", "frac": round(rate / peak, 4),
                        "peak_waves_per_simd": wps,
                        "peaks_by_waves_per_simd": {str(k): round(v / 1e9, 2) for k, v in sorted(peaks.items())},
                        "calls_per_launch": calls, "floor_ms": round(calls / peak * 1e3, 4),
                        "peak_source": PHILOX_PEAK_SRC}
        if valu_roof:
            # the kernel's VALU issue rate against the rate the Philox bench sustains at
            # the same occupancy (its calls are 40 VOP3 instructions: 10 rounds x 2
            # v_mad_u64_u32 + 2 v_bitop3), i.e. what this instruction mix can issue
            bench_rate = peak * PHILOX_BENCH_INSTS_PER_CALL / 64
            kern_rate = valu_roof["valu_insts_per_launch"] / (avg_ms * 1e-3)
            compute_roof["valu_issue_rate_frac_of_philox_bench"] = round(kern_rate / bench_rate, 4)
        if NS > 1 and len(kernels) == 1 and nl == args.steps:
            # with NS steps in flight a launch spans ~NS x its one-stream time (rocprofv3
            # reports that span), while the GPU completes one step per eff_ms: the
            # throughput-side figures of the same kernel
            eff_ms = gpu_ms / args.steps
            roof["effective_ms_per_step"] = round(eff_ms, 4)
            roof["achieved_effective"] = round(io / (eff_ms * 1e-3) / 1e9, 1)
            roof["frac_effective"] = round(io / (eff_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if valu_roof:
                valu_roof["frac_effective"] = round(
                    valu_roof["valu_insts_per_launch"] * VALU_ISSUE_CYCLES /
                    (SIMDS * eff_ms * 1e-3 * CLOCK_GHZ * 1e9), 4)
            wps_eff = min(NS * wps, max(peaks))
            peak_eff = peaks.get(wps_eff, max(peaks.values()))
            compute_roof["effective"] = {
                "ms_per_step": round(eff_ms, 4), "achieved": round(calls / (eff_ms * 1e-3) / 1e9, 2),
                "peak": round(peak_eff / 1e9, 2), "peak_waves_per_simd": wps_eff,
                "frac": round(calls / (eff_ms * 1e-3) / peak_eff, 4)}
        lsb = level_synchronous_bytes_per_trial(n, m) * B
        side = {"bytes_per_launch": lsb, "bytes_per_trial": lsb / B,
                "equivalent_gbs": round(lsb / (avg_ms * 1e-3) / 1e9, 1),
                "note": "SURVEY.md 8d's level-synchronous bytes (each bit-packed tree level written "
                        "once and read once): moved by the LEVELS engine, NOT by this kernel; a "
                        "comparison figure only"}
    cpu = None
    if rank == 0 and not args.no_cpu:
        # this rank's timed steps: trials [first_of(i), first_of(i) + B) for i in the
        # timed slots (contiguous at world 1); checked against its pre-all-reduce counters
        cpu = run_cpu_baseline(n, m, args.seed, fmax, args.cpu_budget_s,
                               rank_ranges(base, args.steps, rank, world, B), local_counters,
                               first_trial(n_total, 0, world, B))

    if rank == 0:
        line = {
            "metric": "OM(m) trial-decisions/sec (whole node) at n=10,m=3; achieved HBM GB/s",
            "value": round(value, 1), "unit": "trial-decisions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(T * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (Philox-generated faulty sets and orders staged in HBM, lies drawn in-kernel)",
            "config": {"workload": f"OM({m}) n={n}, {B} trials/GPU/step, f~U{{0..{fmax}}}, "
                                   f"random order, decisions+outcome written",
                       "n": n, "m": m, "trials_per_gpu_step": B, "engine": args.engine,
                       "parallelism": f"trial-dp{world}"},
            "collective": collective,
            "inputs": "in-kernel Philox draws" if args.inputs_in_kernel else
                      "staged in HBM before the timed region (ba_gen_inputs_device); lies drawn in-kernel",
            "schedule": (f"step i on stream/ctx i % {NS}: up to {NS} steps in flight, each a full "
                         "1M-trial pass with its own outputs; every step's counters summed and checked"
                         if NS > 1 else "one step at a time on one stream"),
            "ms_per_step_gpu_events": round(gpu_ms / args.steps, 4),
            "host_enqueue_ms_per_step": round(enq_ms / args.steps, 4),
            "value_gpu_events": round(B * args.steps / (gpu_ms * 1e-3), 1),
            "streams": NS,
            "value_single_stream": round(value_1, 1),
            "ms_per_step_single_stream_gpu_events": round(gpu_ms_1 / args.steps, 4),
            "value_with_input_generation": round(value_gen, 1) if value_gen else None,
            "ms_per_step_with_input_generation_gpu_events": round(gen_ms / args.steps, 4) if gen_ms else None,
            "warm_up_s": round(warm_s, 2),
            "sclk_mhz_timed": sclk,
            "clock": {"sclk_mhz_median_xcd": sclk, "per_xcd_mhz": {str(k): v for k, v in sclk_xcd.items()},
                      "ms_per_step_gpu_events_clock_pass": round(gpu_ms_c / args.steps, 4),
                      "value_at_2400mhz": round(value * 2400.0 / sclk, 1) if sclk else None,
                      "note": "engine clock over a replica of the timed region (same steps, streams "
                              "and schedule, untimed), from two s_memtime/s_memrealtime probes "
                              "bracketing it (ba_clock_probe_device); value_at_2400mhz = value x "
                              "2400 / sclk: a labelled side figure, not a measurement"},
            "kernels_ms": {k: round(v[1] / v[0], 4) for k, v in kernels.items()},
            "roofline": roof,
            "valu_roofline": valu_roof,
            "compute_roofline": compute_roof,
            "level_synchronous_equivalent": side,
            "cpu_baseline": cpu,
            "counters": counters,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist:
        dist.destroy_process_group()
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
