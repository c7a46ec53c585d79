# Generic library A/B on config 5: bash tools/ab_libs.sh "<pytest -k expr>" "<batches>" lib1 lib2 ...
# (parity subset under each library first; then config5_prof.py --split, A B A B).
set -o pipefail
mkdir -p gpurun_out
K="$1"; BATCHES="$2"; shift 2
for lib in "$@"; do
  BA_HIP_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cascade.py tests/test_dist.py -m gpu -k "$K" > gpurun_out/tests_$(basename $lib).log 2>&1 || { tail -30 gpurun_out/tests_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/tests_$(basename $lib).log)"
done
for rep in 1 2; do for b in $BATCHES; do for lib in "$@"; do
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
