# Philox grouping (every group on the asm path) A/B: abx/libba_base.so (before) vs the
# tree's library vs abx/libba_minb4.so (+ units at 4 waves/SIMD); parity first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cascade.py tests/test_gpu.py -m gpu > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
BA_HIP_LIB=$PWD/abx/libba_minb4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cascade.py -m gpu -k "two_launch_equals or fuzz" > gpurun_out/tests_minb4.log 2>&1 || { tail -30 gpurun_out/tests_minb4.log; exit 1; }
tail -1 gpurun_out/tests_minb4.log
for rep in 1 2; do for b in 1024 1; do for lib in abx/libba_base.so byzantine-agreement_amd/ba_amd/libba_hip.so abx/libba_minb4.so; do
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
        else: print(f" L{d['level']} share {d['us_share_votes']}", end="" if d["level"] == 1 else "\n")
PY
