"""Config 5 (n=16, m=5) measurement on one GPU: the one-launch cascade at ONE
batch size per process (so a rocprofv3 --kernel-trace --stats run of it averages
one shape only), and the per-rank share of the subtree split.

    python tools/config5_prof.py --batch 1024 [--reps 200] [--split]

Prints JSON lines:
  {"what": "cascade", ...}  calls launched back to back on one stream (staged
      inputs, HIP events around `reps` calls): us per call, instances/s, and the
      Philox roofline -- the fewest Philox4x32-10 calls that yield every lie bit
      of the tree (sum_k ceil(|L_k|/2) per 64-instance word, ba.py:42-57 relay
      lies at every level) per second against the issue ceiling tools/philox_bench
      measured (profiles/*philox_bench.jsonl) at 2 and 4 waves per SIMD.
  {"what": "split_share", ...} (--split) ba_split_votes_device over the largest
      8-rank share -- 2 of 15 first hops (level 1), 27 of 210 second hops
      (level 2) -- and ba_root_from_split_votes_device over the gathered votes:
      a ONE-GPU share measurement (what one rank of 8 runs), not a multi-GPU run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402  (philox_peaks, philox_calls_per_trial_word)
from ba_amd import lib as L  # noqa: E402

N, M = 16, 5


def ev_time(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps  # seconds per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--split", action="store_true")
    ap.add_argument("--no-inflight", action="store_true",
                    help="calls on one stream only (clean per-kernel rocprofv3 averages)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = L.Engine(0)
    st = torch.cuda.ExternalStream(eng.stream(), device=dev)
    s = st.cuda_stream
    B = a.batch
    pd = L.make_params(N, M, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    pg = L.make_params(N, M, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 5, L.ORDER_GIVEN, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    fb = torch.empty(B, dtype=torch.int32, device=dev)
    ob = torch.empty(B, dtype=torch.uint8, device=dev)
    eng.gen_inputs_device(pd, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)

    def call():
        eng.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), d_decisions=dec.data_ptr(),
                       d_outcome=out.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
    for _ in range(max(20, a.reps // 5)):  # warm-up: scratch, counters, clocks
        call()
    torch.cuda.synchronize()
    cnt.zero_()
    call()
    torch.cuda.synchronize()
    one = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
    sec = ev_time(call, a.reps, st)
    words = (B + 63) // 64
    calls = bench.philox_calls_per_trial_word(N, M) * words
    peaks = bench.philox_peaks()
    rate = calls / sec
    rec = {"what": "cascade", "n": N, "m": M, "batch": B, "reps": a.reps,
           "us_per_call": round(sec * 1e6, 2), "instances_per_s": round(B / sec, 1),
           "philox_calls_per_call": calls, "philox_calls_per_s": round(rate, 1),
           "roofline": {"bound": "valu (Philox4x32-10 lie draws)", "unit": "G Philox calls/s",
                        "achieved": round(rate / 1e9, 2),
                        "peak_2w": round(peaks.get(2, max(peaks.values())) / 1e9, 2),
                        "frac_2w": round(rate / peaks.get(2, max(peaks.values())), 4),
                        "peak_4w": round(peaks.get(4, max(peaks.values())) / 1e9, 2),
                        "frac_4w": round(rate / peaks.get(4, max(peaks.values())), 4),
                        "floor_us_2w": round(calls / peaks.get(2, max(peaks.values())) * 1e6, 2),
                        "peak_source": bench.PHILOX_PEAK_SRC},
           "counters_one_call": one, "lib_sha16": bench.so_digest()}
    # k calls in flight (k = 2, 3): call i on ctx i % k (each ctx on its own stream,
    # own outputs), one HIP-event pair bracketing all of them on the first stream
    for k, name in (() if a.no_inflight else ((2, "two"), (3, "three"))):
        extra = [L.Engine(0) for _ in range(k - 1)]
        sts = [st] + [torch.cuda.ExternalStream(e.stream(), device=dev) for e in extra]
        decs = [dec] + [torch.empty(B, dtype=torch.int64, device=dev) for _ in extra]
        outs = [out] + [torch.empty(B, dtype=torch.uint8, device=dev) for _ in extra]
        engs = [eng] + extra

        def callk(i):
            j = i % k
            if j == 0:
                call()
            else:
                engs[j].run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                   d_decisions=decs[j].data_ptr(), d_outcome=outs[j].data_ptr(),
                                   d_counters=cnt.data_ptr(), stream=sts[j].cuda_stream)
        for i in range(20):
            callk(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for x in sts[1:]:
            x.wait_event(e0)
        for i in range(a.reps):
            callk(i)
        for x in sts[1:]:
            st.wait_stream(x)
        e1.record(st)
        torch.cuda.synchronize()
        seck = e0.elapsed_time(e1) * 1e-3 / a.reps
        rec[f"us_per_call_{name}_in_flight"] = round(seck * 1e6, 2)
        rec[f"instances_per_s_{name}_in_flight"] = round(B / seck, 1)
        for e in extra:
            e.close()
    print(json.dumps(rec), flush=True)

    if a.split:
        W = words
        for level, (ub, ue) in ((1, (0, 2)), (2, (0, 27))):
            units = L.split_units(N, M, level)
            per = N - 1 - level
            full = torch.zeros((L.split_vote_slots(N, M, level, 0, units), W), dtype=torch.int64,
                               device=dev)
            # every unit's votes once (the all-gather's result), then the share alone
            eng.split_votes_device(pg, B, level, 0, units, full.data_ptr(), d_faulty=fb.data_ptr(),
                                   d_order=ob.data_ptr(), stream=s)
            part = full[ub * per:]

            def share():
                eng.split_votes_device(pg, B, level, ub, ue, part.data_ptr(), d_faulty=fb.data_ptr(),
                                       d_order=ob.data_ptr(), stream=s)

            def root():
                eng.root_from_split_votes_device(pg, B, level, full.data_ptr(), cnt.data_ptr(),
                                                 d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                                 d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s)
            for _ in range(10):
                share()
                root()
            torch.cuda.synchronize()
            cnt.zero_()
            root()
            torch.cuda.synchronize()
            got = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
            if got != one:
                raise SystemExit(f"split level {level}: root pass counters differ from the unsplit call")
            reps = max(20, a.reps // 2)
            ts = ev_time(share, reps, st)
            tr = ev_time(root, reps, st)
            print(json.dumps({"what": "split_share", "n": N, "m": M, "batch": B, "level": level,
                              "share": [ub, ue], "units": units,
                              "share_frac_of_tree": round((ue - ub) / units, 4),
                              "us_share_votes": round(ts * 1e6, 2), "us_root_pass": round(tr * 1e6, 2),
                              "us_share_plus_root": round((ts + tr) * 1e6, 2),
                              "note": "one GPU running the largest 8-rank share of the split, then the "
                                      "root pass every rank runs after the all-gather (not timed: the "
                                      "RCCL exchange itself)"}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
