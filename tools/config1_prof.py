"""Config 1 at batch scale (ba.py-exact OM(1), one MT19937 seed per trial) on one
GPU: the device coin table k_mt_table (ba_mt_table_device) and the table-mode
trials k_table, one n per process, so a rocprofv3 --kernel-trace --stats or
--pmc run of it averages one shape only.

    python tools/config1_prof.py --n 4 [--trials 1048576] [--reps 20]

The inputs are run_configs.py's config-1 inputs (same generator and seeds):
seeds n<<32 + t, random faulty sets of up to (n-1)//3+1 generals, random
stale-primary polls, orders.  Prints one JSON line: per-call times (HIP events
over back-to-back calls on one stream), and the HBM roofline of k_mt_table on
the bytes it must move -- per trial its seed (8 B), faulty mask (4 B) and poll
mask (4 B) read, its coin-table row (4 x stride B) written -- with the
same-build PMC's measured traffic (profiles/*pmc*.json, matched by n and the
library's sha256) beside it: the MT19937 state between random.seed and the
draws is scratch that a kernel holding it on chip would not move.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ba_amd import lib as L  # noqa: E402


def config1_inputs(n: int, T: int):
    """run_configs.py config 1: (seeds, faulty, poll, order) as numpy arrays."""
    rng = np.random.default_rng(1000 + n)
    seeds = np.arange(T, dtype=np.uint64) + np.uint64(n << 32)
    fmax = (n - 1) // 3 + 1
    k = rng.integers(0, fmax + 1, T)
    order_g = np.argsort(rng.random((T, n)), axis=1)
    faulty = np.zeros(T, np.uint32)
    for j in range(fmax):
        faulty |= np.where(k > j, np.uint32(1) << order_g[:, j].astype(np.uint32), 0).astype(np.uint32)
    poll = (rng.integers(0, 1 << n, T) & ~1).astype(np.uint32)
    order = rng.choice(np.array([0, 1, 2], np.uint8), T, p=[0.45, 0.45, 0.1])
    return seeds, faulty, poll, order


def mt_roofline(n: int, T: int, stride: int, sec: float) -> dict:
    """HBM roofline of one k_mt_table launch over T trials lasting `sec`: the bytes
    it must move (seed 8 B + faulty 4 B + poll 4 B read, 4 x stride B of coin row
    written, per trial), with the committed same-build PMC's traffic and VALU
    issue beside it (bench.pmc_for: matched by n, T, "mt_table" and the library's
    sha256)."""
    io = (8 + 4 + 4 + 4 * stride) * T
    pmc, src, same = bench.pmc_for(n, 1, T, "mt_table", "k_mt_table", bench.so_digest())
    traffic = pmc["traffic_bytes"] if pmc else None
    roof = {"bound": "hbm", "kernel": "k_mt_table", "avg_ms": round(sec * 1e3, 4),
            "achieved": round(io / sec / 1e9, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(io / sec / 1e9 / bench.HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_trial": io / T, "algorithmic_bytes_per_launch": io,
            "traffic": round(traffic) if traffic else None,
            "traffic_per_trial": round(traffic / T, 1) if traffic else None,
            "traffic_GBps": round(traffic / sec / 1e9, 1) if traffic else None,
            "source": src, "same_build": same,
            "note": "the MT19937 state between random.seed and the draws is scratch (a window "
                    "per wave, DESIGN.md section 4): traffic above the algorithmic bytes; the "
                    "kernel is bound by the seeding recurrences (valu_frac)"}
    if pmc and pmc.get("counters", {}).get("SQ_INSTS_VALU"):
        insts = pmc["counters"]["SQ_INSTS_VALU"]
        roof["valu_frac"] = round(insts * bench.VALU_ISSUE_CYCLES / (bench.SIMDS * sec * bench.CLOCK_GHZ * 1e9), 4)
        roof["valu_insts_per_launch"] = insts
    return roof


def ev_time(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--trials", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, T = a.n, a.trials
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = L.Engine(0)
    st = torch.cuda.ExternalStream(eng.stream(), device=dev)
    s = st.cuda_stream
    seeds, faulty, poll, order = config1_inputs(n, T)
    stride = L.table_stride(n)
    d_s = torch.from_numpy(seeds.view(np.int64)).to(dev)
    d_f = torch.from_numpy(faulty.view(np.int32)).to(dev)
    d_p = torch.from_numpy(poll.view(np.int32)).to(dev)
    d_o = torch.from_numpy(order).to(dev)
    tab = torch.empty((T, stride), dtype=torch.int32, device=dev)
    dec = torch.empty(T, dtype=torch.int64, device=dev)
    outc = torch.empty(T, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    p = L.make_params(n, 1, 0, L.LIE_TABLE, L.FAULTY_GIVEN, 0, L.ORDER_GIVEN, L.ATTACK, L.ENGINE_AUTO, 0, stride)

    def gen():
        eng.mt_table_device(n, 1, T, d_s.data_ptr(), d_f.data_ptr(), stride, tab.data_ptr(),
                            d_poll=d_p.data_ptr(), stream=s)

    def trials():
        eng.run_device(p, T, d_faulty=d_f.data_ptr(), d_order=d_o.data_ptr(), d_table=tab.data_ptr(),
                       d_poll=d_p.data_ptr(), d_decisions=dec.data_ptr(), d_outcome=outc.data_ptr(),
                       d_counters=cnt.data_ptr(), stream=s)
    gen()
    trials()
    torch.cuda.synchronize()
    # the device table equals the host replay (ba_mt_table, pinned on ba.py's fixtures)
    # on a sample of rows
    idx = np.random.default_rng(n).choice(T, 4096, replace=False)
    htab, _ = L.mt_table(n, 1, seeds[idx], faulty[idx], poll[idx])
    if not np.array_equal(tab.cpu().numpy().view(np.uint32)[idx], htab):
        raise SystemExit(f"config 1 n={n}: device coin table differs from the host replay")
    t_gen = ev_time(gen, a.reps, st)
    t_tab = ev_time(trials, a.reps, st)
    roof = mt_roofline(n, T, stride, t_gen)
    print(json.dumps({"what": "config1", "n": n, "trials": T, "table_stride": stride,
                      "device_table_ms": round(t_gen * 1e3, 4), "k_table_ms": round(t_tab * 1e3, 4),
                      "device_table_trials_per_s": T / t_gen,
                      "device_end_to_end_trials_per_s": T / (t_gen + t_tab),
                      "timing": f"HIP events over {a.reps} back-to-back calls on the ctx stream",
                      "mt_table_roofline": roof}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
