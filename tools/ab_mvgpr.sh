# Philox multipliers as VGPR operands (-DBA_PHILOX_MVGPR): philox_bench both ways,
# then the bench and config 5 with abx/libba_mv.so vs the tree's library, A B A B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./abx/philox_bench_s > gpurun_out/philox_s.jsonl 2>&1 || exit 1
timeout -k 10 120 ./abx/philox_bench_v > gpurun_out/philox_v.jsonl 2>&1 || exit 1
BA_HIP_LIB=$PWD/abx/libba_mv.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "fuzz or wave" > gpurun_out/tests_mv.log 2>&1 || { tail -30 gpurun_out/tests_mv.log; exit 1; }
tail -1 gpurun_out/tests_mv.log
for rep in 1 2 3; do for lib in byzantine-agreement_amd/ba_amd/libba_hip.so abx/libba_mv.so; do
  echo "lib=$lib rep=$rep" >> gpurun_out/ab.log
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --cpu-budget-s 0 >> gpurun_out/ab.log 2>&1 || exit 1
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch 1024 --reps 300 >> gpurun_out/ab.log 2>&1 || exit 1
done; done
python - <<'PY'
import json
for f in ("gpurun_out/philox_s.jsonl", "gpurun_out/philox_v.jsonl"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            if "vgpr_keys" in d["variant"]: print(f[-8:-6], d["variant"], d["waves_per_simd"], "%.3e" % d["philox_calls_per_s"])
for l in open("gpurun_out/ab.log"):
    if l.startswith("lib="): print(l.strip(), end=" |")
    elif l.startswith("{"):
        d = json.loads(l)
        if "metric" in d: print(f" value {d['value']:.4e} gpu_ms {d['ms_per_step_gpu_events']} single {d['value_single_stream']:.4e} sclk {d['sclk_mhz_timed']}", end="")
        elif d.get("what") == "cascade": print(f" c5 {d['us_per_call']}")
PY
