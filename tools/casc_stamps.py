"""Lab: where a config-5 units launch (k_cascade<16,5,2>, the first of the two
launches) spends its time, from the per-wave phase stamps of the lab library
(tools/casc_stamps.sh builds it; BA_HIP_LIB selects it):

    BA_HIP_LIB=$PWD/labbuild/libba_hip_stamps.so python tools/casc_stamps.py --batch 1024

Phases (s_memtime cycles per wave, ba_cascade.hip CASC_STAMP):
  draws    staged-input loads issued, the leaf block's diagonal lies and the
           relay-chain lies (no inputs needed)
  slice    the block's input planes bit-sliced into LDS
  barrier  the block barrier after slicing
  relay    path unranking + relay_apply (the unit's L_0 .. L_{me-2})
  leaf     the leaf block: 55 Philox calls + carry-save columns (S = 11)
  up       transpose through LDS, the level-(me-2) majority, sc1 store
  drain    waiting for the sc1 stores (lab only: the product does not drain here)
Also the launch's wall span from s_memrealtime (entry of the first wave to exit
of the last), the engine clock per wave, and how many waves each SIMD ran.
One JSON line; the stamps themselves cost ~11% (MI355X_MICROARCH.md)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))

import torch  # noqa: E402

from ba_amd import lib as L  # noqa: E402

PHASES = ["draws", "slice", "barrier", "relay", "leaf", "up", "drain"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--co", action="store_true",
                    help="one CO launch (BA_CASC_CO=1): the fan-in blocks' rows follow the units blocks'")
    a = ap.parse_args()
    if a.co:
        os.environ["BA_CASC_CO"] = "1"
    n, m, B = 16, 5, a.batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = L.Engine(0)
    lib = eng.lib
    lib.ba_lab_casc_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    s = torch.cuda.ExternalStream(eng.stream(), device=dev)
    pd = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    pg = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 5, L.ORDER_GIVEN, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    fb = torch.empty(B, dtype=torch.int32, device=dev)
    ob = torch.empty(B, dtype=torch.uint8, device=dev)
    eng.gen_inputs_device(pd, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s.cuda_stream)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)

    def call():
        eng.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), d_decisions=dec.data_ptr(),
                       d_outcome=out.data_ptr(), d_counters=cnt.data_ptr(), stream=s.cuda_stream)
    for _ in range(a.reps):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        call()
    e1.record(s)
    torch.cuda.synchronize()
    us_call = e0.elapsed_time(e1) * 1e3 / a.reps
    lib.ba_lab_mtop_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert lib.ba_lab_stamps_clear() == 0
    call()  # the stamped call: every row written by this call alone
    torch.cuda.synchronize()
    # the last call's units launch: W words x 2730 units, 20 per block of 4 waves
    W = (B + 63) // 64
    units = W * 15 * 14 * 13
    waves = (units + 19) // 20 * 4
    buf = np.zeros((1 << 16, 12), np.uint64)
    assert lib.ba_lab_casc_stamps_read(buf.ctypes.data, buf.nbytes) == 0
    st = buf[:waves].astype(np.int64)
    act = (st[:, 11] >> 32) == 1
    t = st[act]
    d = np.diff(t[:, :8], axis=1)
    per = {p: {"mean_cycles": float(d[:, i].mean()), "p50": float(np.median(d[:, i])),
               "p99": float(np.percentile(d[:, i], 99))} for i, p in enumerate(PHASES)}
    tot = d.sum(axis=1)
    rt0, rt1 = t[:, 8], t[:, 9]
    span_us = (rt1.max() - rt0.min()) / 100.0  # s_memrealtime: 100 MHz
    life_us = (rt1 - rt0) / 100.0
    mhz = (t[:, 7] - t[:, 0]) / np.maximum(1, rt1 - rt0) * 100.0
    hw = t[:, 10]
    simd = ((hw >> 4) & 3) | (((hw >> 8) & 0xF) << 2) | (((hw >> 12) & 1) << 6) | (((hw >> 13) & 7) << 7) | \
           (((hw >> 32) & 7) << 10)
    per_simd = np.bincount(np.unique(simd, return_inverse=True)[1])
    # the fan-in launch (k_cascade_mtop): one block per (word, first hop s0)
    mb = np.zeros((1 << 16, 16), np.uint64)
    assert lib.ba_lab_mtop_stamps_read(mb.ctypes.data, mb.nbytes) == 0
    blocks = W * 15
    nub = (units + 19) // 20 if a.co else 0  # CO: the fan-in blocks follow the units blocks
    mt = mb[nub:nub + blocks].astype(np.int64)
    mph = (["draws+inputs", "barrier", "poll_units", "stepQ+barrier", "relay_q1_apply", "store", "drain",
            "arrive"] if a.co else
           ["kids+inputs+draws", "barrier1", "stepQ", "barrier2", "relay_q1", "store", "drain", "arrive"])
    md = np.diff(mt[:, :9], axis=1)
    lastb = mt[:, 11] != 0
    root = {}
    if lastb.any():
        r = mt[lastb]
        root = {"root_kids+relay": float((r[:, 9] - r[:, 8]).mean()),
                "root_majority+epilogue": float((r[:, 10] - r[:, 9]).mean()),
                "sink": float((r[:, 11] - r[:, 10]).mean())}
    mtop = {"blocks": int(blocks), "phase_cycles_mean": {p: float(md[:, i].mean()) for i, p in enumerate(mph)},
            "phase_cycles_max": {p: float(md[:, i].max()) for i, p in enumerate(mph)},
            "root_step_cycles": root,
            "gap_units_last_exit_to_mtop_first_entry_us": round(float((mt[:, 14].min() - rt1.max()) / 100.0), 2),
            "gap_units_last_exit_to_mtop_last_entry_us": round(float((mt[:, 14].max() - rt1.max()) / 100.0), 2),
            "mtop_span_us": round(float((mt[:, 15].max() - mt[:, 14].min()) / 100.0), 2),
            "units_first_entry_to_mtop_last_exit_us": round(float((mt[:, 15].max() - rt0.min()) / 100.0), 2)}
    if a.co:  # the wait: wave 0's children all fresh (s_memrealtime) vs the units' last exit
        mtop["co_wait_done_minus_units_last_exit_us"] = {
            "min": round(float((mt[:, 12].min() - rt1.max()) / 100.0), 2),
            "max": round(float((mt[:, 12].max() - rt1.max()) / 100.0), 2)}
        mtop["co_granule_polls"] = {"mean": float(mt[:, 13].mean()), "max": int(mt[:, 13].max())}
    print(json.dumps({"mtop": mtop, "co": a.co,
        "batch": B, "units": units, "waves": int(waves), "active_waves": int(act.sum()),
        "us_per_call_stamped_lib": round(us_call, 2), "units_launch_span_us": round(float(span_us), 2),
        "wave_life_us": {"mean": round(float(life_us.mean()), 2), "p50": round(float(np.median(life_us)), 2),
                         "max": round(float(life_us.max()), 2)},
        "clock_mhz_median": round(float(np.median(mhz)), 1),
        "phase_cycles": per,
        "phase_share": {p: round(float(d[:, i].sum() / tot.sum()), 4) for i, p in enumerate(PHASES)},
        "simds_used": int(len(per_simd)), "waves_per_simd": {"max": int(per_simd.max()),
                                                              "mean": round(float(per_simd.mean()), 2)},
        "first_entry_to_last_entry_us": round(float((rt0.max() - rt0.min()) / 100.0), 2),
    }), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
