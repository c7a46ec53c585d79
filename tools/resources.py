"""Per-kernel register/LDS/occupancy table from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", "-o", "/tmp/_res.o",
       src, "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r['name'][:60]:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
          f"sgpr={r.get('SGPRs','?'):>4} vspill={r.get('VGPRs Spill','?'):>3} "
          f"sspill={r.get('SGPRs Spill','?'):>3} lds={r.get('LDS Size [bytes/block]','?'):>5} "
          f"occ={r.get('Occupancy [waves/SIMD]','?')} scratch={r.get('ScratchSize [bytes/lane]','?')}")
