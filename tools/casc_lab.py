"""Lab: time k_cascade (n=16, m=5) ablations (BA_CASC_DIAG, ba_cascade.hip; the
ablated results are wrong by design).  One JSON line per (batch, diag):
average time per call of `reps` calls back to back on one stream.

    python tools/casc_lab.py [--batches 1,1024] [--diags 0,2,4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))

import torch  # noqa: E402

from ba_amd import lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,1024")
    ap.add_argument("--diags", default="0,2,4")
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--m", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = L.Engine(0)
    s = torch.cuda.ExternalStream(eng.stream(), device=dev)
    pd = L.make_params(a.n, a.m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, (a.n - 1) // 3,
                       L.ORDER_RANDOM, L.ATTACK, L.ENGINE_LEVELS, 0)
    pg = L.make_params(a.n, a.m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 5, L.ORDER_GIVEN,
                       L.ATTACK, L.ENGINE_LEVELS, 0)
    for B in [int(x) for x in a.batches.split(",")]:
        fb = torch.empty(B, dtype=torch.int32, device=dev)
        ob = torch.empty(B, dtype=torch.uint8, device=dev)
        eng.gen_inputs_device(pd, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), stream=s.cuda_stream)
        dec = torch.empty(B, dtype=torch.int64, device=dev)
        out = torch.empty(B, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(16, dtype=torch.int64, device=dev)
        for d in a.diags.split(","):
            os.environ["BA_CASC_DIAG"] = d

            def call():
                eng.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                               d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                               d_counters=cnt.data_ptr(), stream=s.cuda_stream)
            for _ in range(20):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                call()
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            print(json.dumps({"n": a.n, "m": a.m, "batch": B, "diag": int(d), "us_per_call": round(ms * 1e3, 2)}),
                  flush=True)
    os.environ.pop("BA_CASC_DIAG", None)
    eng.close()


if __name__ == "__main__":
    main()
