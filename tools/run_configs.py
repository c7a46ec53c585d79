"""BASELINE.json configs 1 and 3-5 (the non-headline ones) through the C ABI
(configs 3-5 through its multi-GPU entries, ba_run_trials_multi and
ba_run_instance_split_multi; ba_amd.dist does the rendezvous).

    python tools/run_configs.py [--only 1,3,4,5]                      # one GPU
    python -m torch.distributed.run --nproc-per-node N tools/run_configs.py  # N GPUs

  1  ba.py-exact mode at batch scale: OM(1) at n=4 and n=10, 1M trials, each
     trial its own ba.py round -- random.seed(seed_t), then the round's coins in
     ba.py's draw order (ba.py:45, 269) -- with random faulty sets, stale-primary
     polls (ba.py:171) and orders.  The coin table is built by ba_mt_table (C++,
     every host thread) and by ba_mt_table_device (one GPU thread per trial; the
     two tables must be equal); k_table (ba_run_trials_device, BA_LIE_TABLE)
     resolves the trials from it.  The kernel's rate, each table's generation time
     and both end-to-end rates are reported (one GPU, rank 0 only).

  3  n=13, m=4, 64M trials, trial-DP across ranks (counters all-reduced)
  4  n=10, m=3 faulty-count sweep f = 0..n/3+1, exactly f faulty, 1M trials each:
     agreement (IC1) / validity (IC2) / quorum-outcome breakdown curve
  5  n=16, m=5: one instance split by first-hop subtree (--split-level 2:
     second-hop subtree) (latency), and a batch of 1024 instances (throughput),
     votes all-gathered across ranks

Rank 0 prints one JSON line per config.  Timings bracket the device work with
torch.cuda.synchronize() (+ a gloo barrier across ranks) and take the max over
ranks; the collectives themselves are RCCL inside libba_hip.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ba_amd import dist as D  # noqa: E402
from ba_amd import lib as L  # noqa: E402


def timed(fn, world, dev):
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize(dev)
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return out, float(dt.item())


def counters(t):
    if isinstance(t, dict):
        return t
    return dict(zip(L.COUNTER_NAMES, [int(x) for x in t.cpu().tolist()]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="3,4,5")
    ap.add_argument("--trials1", type=int, default=1 << 20)
    ap.add_argument("--trials3", type=int, default=64 << 20)
    ap.add_argument("--trials4", type=int, default=1 << 20)
    ap.add_argument("--batch5", type=int, default=1024)
    ap.add_argument("--split-level", type=int, default=1,
                    help="config 5 split: 1 = first-hop subtrees, 2 = second-hop subtrees")
    a = ap.parse_args()
    which = {int(x) for x in a.only.split(",")}
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo")  # rendezvous + barriers; RCCL runs inside the C ABI
    eng = L.Engine(local)
    comm = D.init_comm(eng)  # a one-rank communicator on one GPU
    out = []

    if 1 in which and rank == 0:
        import numpy as np
        for n in (4, 10):
            T = a.trials1
            rng = np.random.default_rng(1000 + n)
            seeds = np.arange(T, dtype=np.uint64) + np.uint64(n << 32)
            # faulty sets: k ~ U{0..f_max+1} generals (the commander included) chosen
            # uniformly, so some trials exceed the OM(1) bound
            fmax = (n - 1) // 3 + 1
            k = rng.integers(0, fmax + 1, T)
            order_g = np.argsort(rng.random((T, n)), axis=1)
            faulty = np.zeros(T, np.uint32)
            for j in range(fmax):
                faulty |= np.where(k > j, np.uint32(1) << order_g[:, j].astype(np.uint32), 0).astype(np.uint32)
            poll = (rng.integers(0, 1 << n, T) & ~1).astype(np.uint32)  # stale primaries
            order = rng.choice(np.array([0, 1, 2], np.uint8), T, p=[0.45, 0.45, 0.1])
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
            t0 = time.perf_counter()
            tab, _ = L.mt_table(n, 1, seeds, faulty, poll, threads=threads)
            t_tab = time.perf_counter() - t0
            t0 = time.perf_counter()
            d_tab = torch.from_numpy(tab.view(np.int32)).to(dev)
            d_f = torch.from_numpy(faulty.view(np.int32)).to(dev)
            d_p = torch.from_numpy(poll.view(np.int32)).to(dev)
            d_o = torch.from_numpy(order).to(dev)
            torch.cuda.synchronize(dev)
            t_h2d = time.perf_counter() - t0
            dec = torch.empty(T, dtype=torch.int64, device=dev)
            outc = torch.empty(T, dtype=torch.uint8, device=dev)
            cnt = torch.zeros(16, dtype=torch.int64, device=dev)
            p = L.make_params(n, 1, 0, L.LIE_TABLE, L.FAULTY_GIVEN, 0, L.ORDER_GIVEN, L.ATTACK,
                              L.ENGINE_AUTO, 0, tab.shape[1])
            st = torch.cuda.Stream(dev)

            def call1():
                eng.run_device(p, T, d_faulty=d_f.data_ptr(), d_order=d_o.data_ptr(),
                               d_table=d_tab.data_ptr(), d_poll=d_p.data_ptr(),
                               d_decisions=dec.data_ptr(), d_outcome=outc.data_ptr(),
                               d_counters=cnt.data_ptr(), stream=st.cuda_stream)
            call1()
            torch.cuda.synchronize(dev)
            first = counters(cnt)
            reps = 20
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cnt.zero_()
            torch.cuda.synchronize(dev)
            e0.record(st)
            for _ in range(reps):
                call1()
            e1.record(st)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            if any(v != first[c] * reps for c, v in counters(cnt).items()):
                raise SystemExit("config 1: repeated calls disagree")
            # the same table generated on the device (ba_mt_table_device: CPython's
            # MT19937 seeded per trial, one thread each), timed with HIP events;
            # its rows must equal the host table's
            d_seeds = torch.from_numpy(seeds.view(np.int64)).to(dev)
            d_tab2 = torch.empty_like(d_tab)

            def gen_dev():
                eng.mt_table_device(n, 1, T, d_seeds.data_ptr(), d_f.data_ptr(), tab.shape[1],
                                    d_tab2.data_ptr(), d_poll=d_p.data_ptr(), stream=st.cuda_stream)
            gen_dev()
            torch.cuda.synchronize(dev)
            if not torch.equal(d_tab2, d_tab):
                raise SystemExit("config 1: device coin table differs from the host table")
            e0.record(st)
            for _ in range(5):
                gen_dev()
            e1.record(st)
            torch.cuda.synchronize(dev)
            ms_gen = e0.elapsed_time(e1) / 5

            def both():  # table generation + the trials, back to back on the stream
                gen_dev()
                eng.run_device(p, T, d_faulty=d_f.data_ptr(), d_order=d_o.data_ptr(),
                               d_table=d_tab2.data_ptr(), d_poll=d_p.data_ptr(),
                               d_decisions=dec.data_ptr(), d_outcome=outc.data_ptr(),
                               d_counters=cnt.data_ptr(), stream=st.cuda_stream)
            cnt.zero_()
            e0.record(st)
            for _ in range(5):
                both()
            e1.record(st)
            torch.cuda.synchronize(dev)
            ms_both = e0.elapsed_time(e1) / 5
            if any(v != first[c] * 5 for c, v in counters(cnt).items()):
                raise SystemExit("config 1: device-table runs disagree")
            import config1_prof
            mt_roof = config1_prof.mt_roofline(n, T, tab.shape[1], ms_gen * 1e-3)
            out.append({"config": 1, "workload": f"ba.py OM(1) bit-exact, n={n}, {T} trials, one "
                        "MT19937 seed per trial (random.seed + the round's coins in ba.py's draw "
                        "order), random faulty sets / stale-primary polls / orders",
                        "n": n, "m": 1, "trials": T,
                        "kernel_trial_decisions_per_s": T / (ms * 1e-3), "kernel_ms_per_call": ms,
                        "kernel_timing": "HIP events over 20 back-to-back k_table calls on one "
                                         "stream, table and inputs resident in HBM",
                        "table_generation_s": t_tab, "table_generation_trials_per_s": T / t_tab,
                        "table_threads": threads or os.cpu_count(),
                        "table_bytes": int(tab.nbytes), "h2d_s": t_h2d,
                        "end_to_end_trials_per_s": T / (t_tab + t_h2d + ms * 1e-3),
                        "end_to_end_note": "host table (ba_mt_table) + H2D + kernel",
                        "device_table_ms": ms_gen,
                        "device_table_trials_per_s": T / (ms_gen * 1e-3),
                        "device_end_to_end_trials_per_s": T / (ms_both * 1e-3),
                        "device_end_to_end_note": "ba_mt_table_device + k_table back to back on "
                                                  "one stream (seeds, faulty sets, polls, orders in "
                                                  "HBM; HIP events), table equal to the host's",
                        "n_gpus": 1, "counters": first, "roofline": mt_roof})
            del d_tab, d_tab2, d_seeds, d_f, d_p, d_o, dec, outc

    if 3 in which:
        n, m, T = 13, 4, a.trials3
        D.run_trials_dp(comm, n, m, 1 << 16, f=4)  # warm-up: geometry, scratch
        cnt, dt = timed(lambda: D.run_trials_dp(comm, n, m, T, f=4), world, dev)
        rec = {"config": 3, "workload": f"OM({m}) n={n}, {T} trials, f~U{{0..4}}, "
               f"trial-DP over {world} GPU(s), counters all-reduced",
               "trials_per_s": T / dt, "seconds": dt, "n_gpus": world,
               "counters": counters(cnt)}
        if world == 1:
            # the same trials with their inputs staged in HBM before timing (as
            # bench.py): one ba_run_trials_device call of all T trials on a stream;
            # its counters must equal the in-kernel-draw run's
            p = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 4, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_AUTO, 0)
            pg = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 4, L.ORDER_GIVEN,
                               L.ATTACK, L.ENGINE_AUTO, 0)
            st = torch.cuda.Stream(dev)
            fb = torch.empty(T, dtype=torch.int32, device=dev)
            ob = torch.empty(T, dtype=torch.uint8, device=dev)
            sd = torch.empty(T, dtype=torch.int64, device=dev)
            so = torch.empty(T, dtype=torch.uint8, device=dev)
            sc = torch.zeros(16, dtype=torch.int64, device=dev)
            eng.gen_inputs_device(p, T, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                  stream=st.cuda_stream)

            def call3():
                eng.run_device(pg, T, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                               d_decisions=sd.data_ptr(), d_outcome=so.data_ptr(),
                               d_counters=sc.data_ptr(), stream=st.cuda_stream)
            call3()  # warm-up
            torch.cuda.synchronize(dev)
            sc.zero_()
            torch.cuda.synchronize(dev)
            _, sdt = timed(call3, world, dev)
            if counters(sc) != counters(cnt):
                raise SystemExit("config 3: staged-input counters differ from the in-kernel run")
            rec["trials_per_s_staged"] = T / sdt
            rec["seconds_staged"] = sdt
            rec["staged_note"] = ("inputs staged in HBM before timing (as bench.py), one "
                                  "ba_run_trials_device call; counters equal the in-kernel run")
            # one rank's share at N=8 (8,388,608 trials, the launch the committed
            # rocprofv3 trace and PMC of k_om4w<13> cover: tools/config3_prof.py),
            # timed with HIP events over back-to-back calls on one stream, and its
            # three rooflines from the same-build PMC
            import config3_prof
            T8 = min(T, 8 << 20)
            sc.zero_()

            def call8():
                eng.run_device(pg, T8, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                               d_decisions=sd.data_ptr(), d_outcome=so.data_ptr(),
                               d_counters=sc.data_ptr(), stream=st.cuda_stream)
            call8()
            torch.cuda.synchronize(dev)
            s8 = config3_prof.ev_time(call8, 10, torch.cuda.ExternalStream(st.cuda_stream, device=dev))
            roof, valu, comp = config3_prof.rooflines(n, m, T8, s8, True, engine="auto/staged")
            rec["rank_share_trials"] = T8
            rec["rank_share_us_per_call"] = round(s8 * 1e6, 2)
            rec["rank_share_trials_per_s"] = T8 / s8
            rec["roofline"], rec["valu_roofline"], rec["compute_roofline"] = roof, valu, comp
            rec["roofline_note"] = (f"one k_om4w<13> launch over {T8} staged trials (one rank's share "
                                    "of 64M at N=8), HIP events; traffic / VALU from the committed "
                                    "PMC of the same build (same_build)")
            del fb, ob, sd, so
        out.append(rec)

    if 4 in which:
        n, m, T = 10, 3, a.trials4
        D.run_trials_dp(comm, n, m, 1 << 16, f=1)  # warm-up
        rows = []
        for f in range(0, (n - 1) // 3 + 2):
            cnt, dt = timed(lambda: D.run_trials_dp(comm, n, m, T, f=f, faulty_mode=L.FAULTY_EXACT,
                                                    base_trial=T * f), world, dev)
            c = counters(cnt)
            rows.append({"f": f, "agreement": c["agreement"] / T,
                         "validity": c["validity"] / max(1, c["validity_applicable"]),
                         "quorum_attack": c["quorum_attack"] / T,
                         "quorum_retreat": c["quorum_retreat"] / T,
                         "quorum_undetermined": c["quorum_undetermined"] / T,
                         "undefined_decisions_per_trial": c["undefined_decisions"] / T,
                         "bound_violations": c["bound_violations"], "trials_per_s": T / dt})
        out.append({"config": 4, "workload": f"OM({m}) n={n}, exactly f faulty, {T} trials "
                    "per point", "n_gpus": world, "sweep": rows})

    if 5 in which:
        n, m = 16, 5
        res = {}
        for B in (1, a.batch5):
            p = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_LEVELS, 0)
            lv = a.split_level
            D.run_instance_split(comm, p, B, dev, level=lv)  # warm-up
            reps = 10 if B == 1 else 3
            (dec, o, cnt), dt = timed(lambda: [D.run_instance_split(comm, p, B, dev, level=lv)
                                               for _ in range(reps)][-1], world, dev)
            res[B] = {"seconds_per_call": dt / reps, "instances_per_s": B * reps / dt,
                      "counters": counters(cnt)}
            # the same call replayed from hipGraphs (D.InstanceSplitGraphs, its own ctx)
            g = D.InstanceSplitGraphs(dev, p, B, comm if world > 1 else None, level=lv)
            reps_g = 50 if B == 1 else 10
            (gd, go, gc), gdt = timed(lambda: [g.replay() for _ in range(reps_g)][-1], world, dev)
            if not (torch.equal(gd, dec) and torch.equal(go, o) and counters(gc) == counters(cnt)):
                raise SystemExit("config 5: graph replay differs from the eager split")
            res[B]["graph_seconds_per_call"] = gdt / reps_g
            res[B]["graph_instances_per_s"] = B * reps_g / gdt
            g.close()
            if world == 1:
                # sustained stream of calls, inputs staged in HBM before timing (as
                # bench.py): the same instances, every call launched back to back on
                # one stream (no host sync between calls; the unsplit pass is what
                # the one-rank split runs)
                fb = torch.empty(B, dtype=torch.int32, device=dev)
                ob = torch.empty(B, dtype=torch.uint8, device=dev)
                st = torch.cuda.Stream(dev)
                eng.gen_inputs_device(p, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                      stream=st.cuda_stream)
                pg = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 5, L.ORDER_GIVEN,
                                   L.ATTACK, L.ENGINE_LEVELS, 0)
                sd = torch.empty(B, dtype=torch.int64, device=dev)
                so = torch.empty(B, dtype=torch.uint8, device=dev)
                sc = torch.zeros(16, dtype=torch.int64, device=dev)

                def call():
                    eng.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                   d_decisions=sd.data_ptr(), d_outcome=so.data_ptr(),
                                   d_counters=sc.data_ptr(), stream=st.cuda_stream)
                call()  # warm-up (geometry, scratch)
                torch.cuda.synchronize(dev)
                sc.zero_()
                call()
                torch.cuda.synchronize(dev)
                if not (torch.equal(sd, dec) and torch.equal(so, o) and counters(sc) == counters(cnt)):
                    raise SystemExit("config 5: staged-input call differs from the split")
                reps_s = 20 if B == 1 else 50
                _, sdt = timed(lambda: [call() for _ in range(reps_s)], world, dev)
                res[B]["stream_seconds_per_call"] = sdt / reps_s
                res[B]["stream_instances_per_s"] = B * reps_s / sdt
                # two calls in flight: call i on ctx i % 2, each ctx on its own stream
                # (ctx streams sit on different hardware queues) with its own outputs,
                # so one call's short latency-bound launches overlap the other's leaf
                # kernel; the counters of every call are summed and checked
                eng2 = L.Engine(local)
                ctxs = [(eng, eng.stream()), (eng2, eng2.stream())]
                outs2 = [(torch.empty(B, dtype=torch.int64, device=dev),
                          torch.empty(B, dtype=torch.uint8, device=dev)) for _ in ctxs]

                def call2(i):
                    e, s2 = ctxs[i % 2]
                    d2, o2 = outs2[i % 2]
                    e.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                 d_decisions=d2.data_ptr(), d_outcome=o2.data_ptr(),
                                 d_counters=sc.data_ptr(), stream=s2)
                for i in range(4):  # warm-up of both ctxs
                    call2(i)
                torch.cuda.synchronize(dev)
                sc.zero_()
                torch.cuda.synchronize(dev)
                _, s2dt = timed(lambda: [call2(i) for i in range(reps_s)], world, dev)
                c2 = counters(sc)
                if c2["trials"] != B * reps_s or any(v != counters(cnt)[k] * reps_s for k, v in c2.items()):
                    raise SystemExit("config 5: two-stream calls' counters differ")
                if not (torch.equal(outs2[0][0], dec) and torch.equal(outs2[1][1], o)):
                    raise SystemExit("config 5: two-stream outputs differ from the split")
                res[B]["stream2_seconds_per_call"] = s2dt / reps_s
                res[B]["stream2_instances_per_s"] = B * reps_s / s2dt
                eng2.close()
        out.append({"config": 5, "workload": f"OM({m}) n={n} (3,999,675 tree slots), "
                    f"{'first' if a.split_level == 1 else 'second'}-hop subtree split over "
                    f"{world} GPU(s), votes all-gathered", "split_level": a.split_level,
                    "latency_one_instance_ms": res[1]["seconds_per_call"] * 1e3,
                    "latency_one_instance_ms_graph": res[1]["graph_seconds_per_call"] * 1e3,
                    "batch": a.batch5, "throughput_instances_per_s": res[a.batch5]["instances_per_s"],
                    "throughput_instances_per_s_graph": res[a.batch5]["graph_instances_per_s"],
                    "latency_one_instance_ms_stream": res[1].get("stream_seconds_per_call", 0) * 1e3,
                    "throughput_instances_per_s_stream": res[a.batch5].get("stream_instances_per_s"),
                    "latency_one_instance_ms_stream2": res[1].get("stream2_seconds_per_call", 0) * 1e3,
                    "throughput_instances_per_s_stream2": res[a.batch5].get("stream2_instances_per_s"),
                    "stream_note": "staged inputs, calls launched back to back on one stream; "
                                   "stream2: two calls in flight on two ctx streams (one rank only)",
                    "n_gpus": world, "counters_batch": res[a.batch5]["counters"]})
        # the Philox roofline of the batch call on one stream (tools/config5_prof.py
        # has the same figure per process, for rocprofv3 runs of one batch size)
        sec = res[a.batch5].get("stream_seconds_per_call")
        if sec:
            import bench  # philox_calls_per_trial_word, philox_peaks
            calls = bench.philox_calls_per_trial_word(n, m) * ((a.batch5 + 63) // 64)
            peaks = bench.philox_peaks()
            pk = peaks.get(2, max(peaks.values()))
            out[-1]["compute_roofline"] = {
                "bound": "valu (Philox4x32-10 lie draws, ba.py:42-57 at every relay level)",
                "unit": "G Philox calls/s", "calls_per_call": calls,
                "achieved": round(calls / sec / 1e9, 2), "peak": round(pk / 1e9, 2),
                "peak_waves_per_simd": 2, "frac": round(calls / sec / pk, 4),
                "floor_us": round(calls / pk * 1e6, 2), "peak_source": bench.PHILOX_PEAK_SRC,
                "timing": "batch call on one stream (stream_seconds_per_call)"}

    if rank == 0:
        for line in out:
            print(json.dumps(line), flush=True)
    comm.close()
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
