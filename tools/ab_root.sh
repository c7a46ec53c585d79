# Root-pass A/B: abx/libba_base.so (no prefetch) vs the tree's library, split tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dist.py tests/test_gpu_cascade.py -m gpu -k "split or second_hop or subtree or fanin or handoff" > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for rep in 1 2; do for b in 1 1024; do for lib in abx/libba_base.so byzantine-agreement_amd/ba_amd/libba_hip.so; do
  echo "lib=$lib batch=$b rep=$rep" >> gpurun_out/ab.log
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 300 --split >> gpurun_out/ab.log 2>&1 || exit 1
done; done; done
python - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("lib="): print(l.strip(), end=" |")
    elif l.startswith("{"):
        d = json.loads(l)
        if d["what"] == "cascade": print(f" whole {d['us_per_call']}", end="")
        else: print(f" L{d['level']} share {d['us_share_votes']} root {d['us_root_pass']}", end="" if d["level"] == 1 else "\n")
PY
