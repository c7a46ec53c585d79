"""Per-kernel achieved HBM bandwidth: rocprofv3 --stats average duration
(kernel_stats.csv) joined with PMC traffic per dispatch (tools/pmc_summary.py
json: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md), against the 8.0 TB/s
MI355X HBM peak.

usage: python tools/kernel_hbm.py <run_kernel_stats.csv> <pmc_summary.json>
"""
import csv
import json
import sys

PEAK_GBS = 8000.0


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")


def main():
    stats = {short(r["Name"]): r for r in csv.DictReader(open(sys.argv[1]))}
    pmc = {short(k): v for k, v in json.load(open(sys.argv[2]))["kernels"].items()}
    rows = []
    for k, r in stats.items():
        if not k.startswith("ba::"):
            continue
        avg_ns = float(r["AverageNs"])
        e = pmc.get(k, {})
        traffic = e.get("traffic_bytes")
        gbs = traffic / avg_ns if traffic else None  # bytes/ns == GB/s
        rows.append({"kernel": k, "calls": int(r["Calls"]), "avg_us": round(avg_ns / 1e3, 3),
                     "share": float(r["Percentage"]), "hbm_bytes_per_dispatch": traffic,
                     "achieved_GBs": round(gbs, 1) if gbs else None,
                     "frac_of_peak": round(gbs / PEAK_GBS, 4) if gbs else None})
    rows.sort(key=lambda x: -x["share"])
    print(json.dumps({"peak_GBs": PEAK_GBS, "kernels": rows}, indent=1))


if __name__ == "__main__":
    main()
