"""Lab: where the bench's wall time goes outside the GPU events (one GPU).

bench.py's `value` is wall time from t0 (after a synchronize) to the closing
synchronize; its HIP events bracket only the GPU work.  This times the pieces
of that gap on the bench workload (n=10, m=3, 1M trials, staged inputs), with
`reps` repetitions each, and prints one JSON line per variant:
  empty        t0 -> record ev0, ev1 -> close (no steps)
  steps_K      K steps as bench.py's timed region (NS streams), close = poll the
               last event, then synchronize
  steps_K_sync the same, close = a plain synchronize
  enqueue      host time to enqueue K steps (no wait)
Each line: wall us, GPU-event us, and their difference.

--sched spin|yield|blocking|auto sets the HIP runtime's wait mode
(hipSetDeviceFlags: hipDeviceScheduleSpin / Yield / BlockingSync / Auto) before
the process's first device call, for an A/B of the close (`default`: untouched).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))

import torch  # noqa: E402

from ba_amd import lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--sched", default="default", choices=["default", "auto", "spin", "yield", "blocking"])
    a = ap.parse_args()
    if a.sched != "default":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL) if hasattr(os, "RTLD_NOLOAD") else None
        flags = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}[a.sched]
        rc = hip.hipSetDeviceFlags(flags)
        print(json.dumps({"sched": a.sched, "hipSetDeviceFlags_rc": rc}), flush=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, m, B, NS, K = 10, 3, 1 << 20, a.streams, a.steps
    engines = [L.Engine(0) for _ in range(NS)]
    streams = [torch.cuda.ExternalStream(e.stream(), device=dev) for e in engines]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    fb = torch.empty((K, B), dtype=torch.int32, device=dev)
    ob = torch.empty((K, B), dtype=torch.uint8, device=dev)
    for i in range(K):
        engines[0].gen_inputs_device(L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3,
                                                   L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, i * B),
                                     B, d_faulty=fb[i].data_ptr(), d_order=ob[i].data_ptr(),
                                     stream=stream.cuda_stream)
    params = [L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 3, L.ORDER_GIVEN, L.ATTACK,
                            L.ENGINE_AUTO, i * B) for i in range(K)]
    decs = [torch.empty(B, dtype=torch.int64, device=dev) for _ in range(NS)]
    outs = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(NS)]
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)

    def step(i):
        j = i % NS
        engines[j].run_device(params[i], B, d_faulty=fb[i].data_ptr(), d_order=ob[i].data_ptr(),
                              d_decisions=decs[j].data_ptr(), d_outcome=outs[j].data_ptr(),
                              d_counters=cnt.data_ptr(), stream=streams[j].cuda_stream)

    def region(nsteps, poll=True):
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for j in range(1, NS):
            streams[j].wait_event(ev0)
        for i in range(nsteps):
            step(i)
        for j in range(1, NS):
            stream.wait_stream(streams[j])
        ev1.record(stream)
        t1 = time.perf_counter()
        if poll:
            while not ev1.query():
                pass
        t2 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        return {"wall": (t3 - t0) * 1e6, "enqueue": (t1 - t0) * 1e6, "poll": (t2 - t1) * 1e6,
                "sync": (t3 - t2) * 1e6, "gpu": ev0.elapsed_time(ev1) * 1e3}

    # bench.py's warm-up: >= 1 s of back-to-back steps on both streams, no
    # cross-stream event waits; then the FIRST timed-region-shaped pass alone
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < 1.0:
        for i in range(K):
            step(i)
        torch.cuda.synchronize(dev)
    first = region(K, False)
    print(json.dumps({"variant": f"first_region_{K}_sync", "streams": NS,
                      "us": {k: round(v, 1) for k, v in first.items()},
                      "gap_us": round(first["wall"] - first["gpu"], 1)}), flush=True)
    second = region(K, False)
    print(json.dumps({"variant": f"second_region_{K}_sync", "streams": NS,
                      "us": {k: round(v, 1) for k, v in second.items()},
                      "gap_us": round(second["wall"] - second["gpu"], 1)}), flush=True)
    for _ in range(3):  # warm-up
        region(K)
    for name, ns, poll in (("empty", 0, True), (f"steps_{K}", K, True), (f"steps_{K}_sync", K, False),
                           ("steps_1", 1, True), ("steps_2", 2, True)):
        rs = [region(ns, poll) for _ in range(a.reps)]
        med = {k: round(statistics.median(r[k] for r in rs), 1) for k in rs[0]}
        mn = {k: round(min(r[k] for r in rs), 1) for k in rs[0]}
        print(json.dumps({"variant": name, "sched": a.sched, "streams": NS, "median_us": med, "min_us": mn,
                          "gap_median_us": round(med["wall"] - med["gpu"], 1)}), flush=True)
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
