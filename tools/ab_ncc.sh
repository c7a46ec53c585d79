# Carry-out SGPR rotation A/B (tools/gen_philox_asm.py PHILOX_ASM_NCC=1/2/4): philox_bench
# builds abx/philox_bench_cc{1,2,4}, then bench + config 5 with abx/libba_cc4.so vs the tree's.
set -o pipefail
mkdir -p gpurun_out
for n in 1 2 4 1 2 4; do
  timeout -k 10 120 ./abx/philox_bench_cc$n > gpurun_out/philox_cc$n.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/philox_cc$n.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        if d['variant'] == 'kernel_shape_vgpr_keys': print('cc$n', d['waves_per_simd'], '%.4e' % d['philox_calls_per_s'])
" | tee -a gpurun_out/philox_summary.txt
done
BA_HIP_LIB=$PWD/abx/libba_cc4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu -k "fuzz or wave" > gpurun_out/tests_cc4.log 2>&1 || { tail -30 gpurun_out/tests_cc4.log; exit 1; }
tail -1 gpurun_out/tests_cc4.log
for rep in 1 2 3; do for lib in byzantine-agreement_amd/ba_amd/libba_hip.so abx/libba_cc4.so; do
  echo "lib=$lib rep=$rep" >> gpurun_out/ab.log
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --cpu-budget-s 0 >> gpurun_out/ab.log 2>&1 || exit 1
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch 1024 --reps 300 >> gpurun_out/ab.log 2>&1 || exit 1
done; done
python - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("lib="): print(l.strip(), end=" |")
    elif l.startswith("{"):
        d = json.loads(l)
        if "metric" in d: print(f" value {d['value']:.4e} gpu_ms {d['ms_per_step_gpu_events']} single {d['value_single_stream']:.4e} sclk {d['sclk_mhz_timed']}", end="")
        elif d.get("what") == "cascade": print(f" c5 {d['us_per_call']}")
PY
