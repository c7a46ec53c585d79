"""Print the last N kernels of a rocprofv3 kernel trace with start offset, duration and launch shape."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} {r['Kernel_Name'][:40]:40s} "
          f"grid={r['Grid_Size_X']} vgpr={r['VGPR_Count']}")
