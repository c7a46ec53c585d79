"""Config 3 (n=13, m=4) measurement on one GPU: one k_om4w<13> launch over a
rank's share of the 64M trials (8,388,608 = 64M / 8 ranks), with the same
roofline contract bench.py gives config 2.

    python tools/config3_prof.py [--trials 8388608] [--reps 20] [--mode staged,inkernel]

Each mode is one ba_run_trials_device call per rep (a hipMemsetAsync of the task
counter + ONE k_om4w launch), launched back to back on the ctx stream and timed
with HIP events on that stream:
  staged    faulty sets / orders written to HBM first by ba_gen_inputs_device
            (FAULTY_GIVEN / ORDER_GIVEN: the k_om4w<13, true> specialisation)
  inkernel  the same trials drawn inside the kernel (FAULTY_RANDOM / ORDER_RANDOM)
The two modes' counters must be equal (same seed, same trials).

Prints one JSON line per mode with three rooflines of the launch (rooflines()):
  roofline          HBM: the 14 B/trial of per-trial I/O (5 B staged inputs read,
                    8 B decision + 1 B outcome written; the tree stays on chip)
                    over the launch, `traffic` from the committed same-build PMC
  valu_roofline     SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x launch)
  compute_roofline  the fewest Philox4x32-10 calls of the tree (54,192 per 64-trial
                    word at n=13, m=4) per second against tools/philox_bench's
                    2-waves-per-SIMD ceiling
The PMC summary is looked up in profiles/*pmc*.json by (n, m, batch, engine) and
the library's sha256 (bench.pmc_for), so a stale build's counters are flagged
`same_build: false`.
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

import bench  # noqa: E402
from ba_amd import lib as L  # noqa: E402

N, M, F = 13, 4, 4
SEED = 0xBA5EED
KERNEL = "k_om4w"


def ev_time(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps  # seconds per call


def rooflines(n, m, batch, sec, staged, kernel=KERNEL, engine="auto"):
    """(roofline, valu_roofline, compute_roofline) of one WAVE launch of `batch`
    trials lasting `sec` seconds, with the committed same-build PMC of it."""
    digest = bench.so_digest()
    pmc, src, same = bench.pmc_for(n, m, batch, engine, kernel, digest)
    io = bench.kernel_io_bytes(kernel, n, m, batch, staged)
    traffic = pmc["traffic_bytes"] if pmc else None
    roof = {"bound": "hbm", "kernel": kernel, "avg_ms": round(sec * 1e3, 4),
            "achieved": round(io / sec / 1e9, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(io / sec / 1e9 / bench.HBM_PEAK_GBS, 4),
            "traffic": round(traffic) if traffic else None,
            "traffic_over_algorithmic": round(traffic / io, 4) if traffic else None,
            "algorithmic_bytes_per_launch": io, "algorithmic_bytes_per_trial": io / batch,
            "source": src, "same_build": same}
    valu = None
    if pmc and pmc.get("counters", {}).get("SQ_INSTS_VALU"):
        insts = pmc["counters"]["SQ_INSTS_VALU"]
        valu = {"bound": "valu", "kernel": kernel, "valu_insts_per_launch": insts,
                "achieved": round(insts * bench.VALU_ISSUE_CYCLES / sec / 1e9, 1),
                "peak": round(bench.SIMDS * bench.CLOCK_GHZ, 1), "unit": "G SIMD-cycles/s",
                "frac": round(insts * bench.VALU_ISSUE_CYCLES / (bench.SIMDS * sec * bench.CLOCK_GHZ * 1e9), 4),
                "formula": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x launch)",
                "source": src, "same_build": same}
        c = pmc["counters"]
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"):
            if k in c:
                valu[k] = c[k]
    calls = bench.philox_calls_per_trial_word(n, m) * ((batch + 63) // 64)
    peaks = bench.philox_peaks()
    pk = peaks.get(2, max(peaks.values()))
    comp = {"bound": "valu (Philox4x32-10 lie draws, ba.py:42-57 at every relay level)",
            "kernel": kernel, "unit": "G Philox calls/s", "calls_per_launch": calls,
            "achieved": round(calls / sec / 1e9, 2), "peak": round(pk / 1e9, 2),
            "peak_waves_per_simd": 2, "frac": round(calls / sec / pk, 4),
            "floor_ms": round(calls / pk * 1e3, 4), "peak_source": bench.PHILOX_PEAK_SRC}
    if valu:
        comp["valu_issue_rate_frac_of_philox_bench"] = round(
            valu["valu_insts_per_launch"] / sec / (pk * bench.PHILOX_BENCH_INSTS_PER_CALL / 64), 4)
    return roof, valu, comp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--mode", default="staged,inkernel")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = L.Engine(0)
    st = torch.cuda.ExternalStream(eng.stream(), device=dev)
    s = st.cuda_stream
    T = a.trials
    pr = L.make_params(N, M, SEED, L.LIE_PHILOX, L.FAULTY_RANDOM, F, L.ORDER_RANDOM, L.ATTACK,
                       L.ENGINE_AUTO, 0)
    pg = L.make_params(N, M, SEED, L.LIE_PHILOX, L.FAULTY_GIVEN, F, L.ORDER_GIVEN, L.ATTACK,
                       L.ENGINE_AUTO, 0)
    fb = torch.empty(T, dtype=torch.int32, device=dev)
    ob = torch.empty(T, dtype=torch.uint8, device=dev)
    dec = torch.empty(T, dtype=torch.int64, device=dev)
    oc = torch.empty(T, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    eng.gen_inputs_device(pr, T, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s)
    first = {}
    for mode in a.mode.split(","):
        staged = mode == "staged"
        p = pg if staged else pr

        def call():
            eng.run_device(p, T, d_faulty=fb.data_ptr() if staged else 0,
                           d_order=ob.data_ptr() if staged else 0, d_decisions=dec.data_ptr(),
                           d_outcome=oc.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
        cnt.zero_()
        torch.cuda.synchronize()
        call()  # warm-up; its counters are the mode's reference
        torch.cuda.synchronize()
        c1 = [int(x) for x in cnt.cpu().tolist()]
        first[mode] = c1
        cnt.zero_()
        torch.cuda.synchronize()
        sec = ev_time(call, a.reps, st)
        cr = [int(x) for x in cnt.cpu().tolist()]
        if any(v != c * a.reps for v, c in zip(cr, c1)):
            raise SystemExit(f"config 3 {mode}: repeated calls disagree")
        if c1[L.COUNTER_NAMES.index("trials")] != T:
            raise SystemExit(f"config 3 {mode}: trial count {c1[0]} != {T}")
        roof, valu, comp = rooflines(N, M, T, sec, staged, engine=f"auto/{mode}")
        print(json.dumps({"what": "config3", "mode": mode, "n": N, "m": M, "trials": T,
                          "workload": f"OM({M}) n={N}, {T} trials (one rank's share of 64M at N=8), "
                                      f"f~U{{0..{F}}}, seed {SEED:#x}",
                          "us_per_call": round(sec * 1e6, 2), "trials_per_s": T / sec,
                          "timing": f"HIP events over {a.reps} back-to-back ba_run_trials_device "
                                    "calls on the ctx stream (task-counter memset + one k_om4w launch)",
                          "roofline": roof, "valu_roofline": valu, "compute_roofline": comp,
                          "counters": dict(zip(L.COUNTER_NAMES, c1))}), flush=True)
    if len(first) == 2 and first["staged"] != first["inkernel"]:
        raise SystemExit("config 3: staged and in-kernel counters differ")
    eng.close()


if __name__ == "__main__":
    main()
