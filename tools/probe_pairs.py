"""Lab: which rows of the two clock probes give consistent s_memtime differences.
Probes bracket back-to-back device work (no host sync in between, as bench.py's
clock pass); per XCD, the clock from rows keyed by CU (HW_ID & 0xFF00), by shader
engine + array (& 0xF000), by shader engine (& 0xE000), and by XCD only."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))

import torch  # noqa: E402

from ba_amd import lib as L  # noqa: E402


def clocks(p0, p1, mask):
    def by(rows):
        d = {}
        for x, hw, mt, rt in rows:
            d.setdefault((x, hw & mask), []).append((mt, rt))
        return d
    a, b = by(p0), by(p1)
    out = {}
    for k in set(a) & set(b):
        for m0, r0 in a[k]:
            for m1, r1 in b[k]:
                if r1 > r0:
                    out.setdefault(k[0], []).append((m1 - m0) / (r1 - r0) * 100.0)
    return {x: (round(min(v)), round(statistics.median(v)), round(max(v)), len(v)) for x, v in sorted(out.items())}


def main():
    dev = torch.device("cuda", 0)
    eng = L.Engine(0)
    s = eng.stream()
    B = 1 << 20
    p = L.make_params(10, 3, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, 0)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    for t in range(4):
        probes = torch.zeros((2, L.PROBE_BLOCKS, 4), dtype=torch.int64, device=dev)
        eng.clock_probe_device(probes[0].data_ptr(), stream=s)
        for i in range(20):
            eng.run_device(p, B, d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
        eng.clock_probe_device(probes[1].data_ptr(), stream=s)
        torch.cuda.synchronize()
        rows = probes.cpu().tolist()
        if t == 0:
            print({"hw_ids_probe0": sorted({(r[0], hex(r[1] & 0xFFFF)) for r in rows[0]})[:16]}, flush=True)
        for name, mask in (("cu_simd", 0xFF30), ("cu", 0xFF00), ("se", 0xE000)):
            print({"pair": t, "key": name, "per_xcd_min_med_max_n": clocks(rows[0], rows[1], mask)}, flush=True)
    eng.close()


if __name__ == "__main__":
    main()
