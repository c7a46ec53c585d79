"""Summarise rocprofv3 --pmc passes (tools/gpu_session.sh `pmc` stage) per kernel.

usage: python tools/pmc_summary.py <pmc dir> <out.json> [--workload TEXT]
                                  [--config n,m,batch,engine,kernel]

Per kernel: the mean per dispatch of every counter, plus the derived figures
DESIGN.md §Measurement uses:
  hbm_read_bytes   = 2 x FETCH_SIZE KiB x 1024  (gfx950 tallies 128-B requests at
                     64 B: MI355X_MICROARCH.md §HBM, "double it")
  hbm_write_bytes  = WRITE_SIZE KiB x 1024
  traffic_bytes    = read + write, per launch
  valu_util        = SQ_INSTS_VALU x 2 cyc / (SIMDs x kernel cycles), the share of
                     the VALU issue slots used (wave64 VALU issues over 2 cycles
                     on a 32-lane SIMD); kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs
"""
from __future__ import annotations

import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("BA_HIP_LIB") or os.path.join(ROOT, "byzantine-agreement_amd", "ba_amd", "libba_hip.so")

SIMDS = 256 * 4


def main():
    d, out = sys.argv[1], sys.argv[2]
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else ""
    config = None
    if "--config" in sys.argv:
        n, m, batch, engine, kernel = sys.argv[sys.argv.index("--config") + 1].split(",")
        config = {"n": int(n), "m": int(m), "batch": int(batch), "engine": engine, "kernel": kernel}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"dispatches": max(len(v) for v in cs.values()), "counters": mean}
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            rd = 2 * mean["FETCH_SIZE"] * 1024
            wr = mean["WRITE_SIZE"] * 1024
            e.update(hbm_read_bytes=rd, hbm_write_bytes=wr, traffic_bytes=rd + wr)
        if "SQ_INSTS_VALU" in mean and "GRBM_GUI_ACTIVE" in mean:
            cyc = mean["GRBM_GUI_ACTIVE"] / 8
            e["kernel_cycles"] = cyc
            e["valu_util"] = mean["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc)
        res[k] = e
    # the build these counters belong to (bench.py matches it before quoting them)
    sha = hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16] if os.path.exists(LIB) else None
    json.dump({"source": d, "workload": workload, "config": config, "lib_sha16": sha,
               "kernels": res}, open(out, "w"), indent=1)
    for k, e in res.items():
        print(k[:50], {x: e[x] for x in e if x not in ("counters",)})


if __name__ == "__main__":
    main()
