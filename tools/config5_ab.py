"""Config 5 (n=16, m=5, one GPU) A/B of the LEVELS launch-fusion switches
(default: the one-launch k_cascade; no_cascade: the multi-launch pipeline).

    python tools/config5_ab.py [--batches 1,1024] [--reps 200]

For each batch, input mode (staged in HBM before timing, or drawn in-kernel)
and switch setting: the per-kernel HIP-event times of eager calls
(ba_profile_*) and the average time per call of `reps` calls launched back to
back on one stream (HIP events around them).  Every setting's outputs and
counters must equal the default's (the switches change launches, not results).
Prints one JSON line per (batch, inputs, setting).
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

SETTINGS = {
    "default": {},
    "no_cascade": {"BA_NO_CASCADE": "1"},
    "no_input": {"BA_NO_INPUT_FUSION": "1"},
    "no_tail": {"BA_NO_TAIL": "1"},
    "no_input_no_tail": {"BA_NO_INPUT_FUSION": "1", "BA_NO_TAIL": "1"},
    "no_leaf_up": {"BA_NO_LEAF_UP": "1"},
}
SWITCHES = ("BA_NO_CASCADE", "BA_NO_LEAF_UP", "BA_NO_INPUT_FUSION", "BA_NO_TAIL")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,1024")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--settings", default=",".join(SETTINGS))
    ap.add_argument("--inputs", default="staged,drawn")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pd = L.make_params(16, 5, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    pg = L.make_params(16, 5, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_GIVEN, 5, L.ORDER_GIVEN, L.ATTACK,
                       L.ENGINE_LEVELS, 0)
    ref = {}
    for B in [int(x) for x in a.batches.split(",")]:
        fb = torch.empty(B, dtype=torch.int32, device=dev)
        ob = torch.empty(B, dtype=torch.uint8, device=dev)
        for inputs in a.inputs.split(","):
            for name in a.settings.split(","):
                for k in SWITCHES:
                    os.environ.pop(k, None)
                os.environ.update(SETTINGS[name])
                eng = L.Engine(0)
                s = torch.cuda.Stream(dev)
                eng.gen_inputs_device(pd, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                      stream=s.cuda_stream)
                dec = torch.empty(B, dtype=torch.int64, device=dev)
                out = torch.empty(B, dtype=torch.uint8, device=dev)
                cnt = torch.zeros(16, dtype=torch.int64, device=dev)

                def call():
                    if inputs == "staged":
                        eng.run_device(pg, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                                       d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                       d_counters=cnt.data_ptr(), stream=s.cuda_stream)
                    else:
                        eng.run_device(pd, B, d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                       d_counters=cnt.data_ptr(), stream=s.cuda_stream)

                with torch.cuda.stream(s):
                    call()  # warm-up: geometry, scratch
                    torch.cuda.synchronize()
                    eng.profile(True)
                    for _ in range(20):
                        call()
                    torch.cuda.synchronize()
                    prof = {k: round(v[1] / v[0] * 1e3, 2) for k, v in eng.profile_read().items()}
                    eng.profile(False)
                    cnt.zero_()
                    call()
                    torch.cuda.synchronize()
                    c = [int(x) for x in cnt.cpu().tolist()][:12]
                    reps = a.reps if B <= 64 else max(20, a.reps // 4)
                    for _ in range(10):
                        call()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(reps):  # back to back, no host sync between calls
                        call()
                    e1.record(s)
                    torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                if B not in ref:
                    ref[B] = (c, dec.cpu(), out.cpu())
                same = c == ref[B][0] and torch.equal(dec.cpu(), ref[B][1]) and torch.equal(out.cpu(), ref[B][2])
                print(json.dumps({"setting": name, "inputs": inputs, "batch": B,
                                  "stream_ms": round(ms, 4), "instances_per_s": B / ms * 1e3,
                                  "kernel_us_eager": prof, "same_as_default": same}), flush=True)
                eng.close()
                if not same:
                    raise SystemExit(f"{name} {inputs} batch {B}: results differ from the default")


if __name__ == "__main__":
    main()
