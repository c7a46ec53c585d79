# Split-share A/B: the range mode in one launch (BA_CASC_TWO=0) or two (units +
# k_cascade_mtop), the units normal or in latency mode (BA_CASC_LAT), after the
# cascade and split GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cascade.py tests/test_dist.py -m gpu > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for rep in 1 2; do for b in 1 64 1024; do for mode in "0 0" "1 0" "1 1"; do
  set -- $mode
  echo "two=$1 lat=$2 batch=$b rep=$rep" >> gpurun_out/ab.log
  BA_CASC_TWO=$1 BA_CASC_LAT=$2 timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 200 --split >> gpurun_out/ab.log 2>&1 || exit 1
done; done; done
python - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("two="): print(l.strip(), end=" |")
    elif l.startswith("{"):
        d = json.loads(l)
        if d["what"] == "cascade": print(f" whole {d['us_per_call']}", end="")
        else: print(f" L{d['level']} share {d['us_share_votes']} root {d['us_root_pass']}", end="" if d["level"] == 1 else "\n")
PY
