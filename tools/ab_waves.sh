# Cascade waves-per-block A/B (abx/libba_w1.so, libba_w2.so: -DBA_CASC_WAVES=1/2) vs the
# 4-wave product library; parity subset under each A/B library first.
set -o pipefail
mkdir -p gpurun_out
for lib in abx/libba_w1.so abx/libba_w2.so; do
  BA_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cascade.py -k "two_launch_equals or fuzz or latency_mode_units" > gpurun_out/tests_$(basename $lib).log 2>&1 || { tail -30 gpurun_out/tests_$(basename $lib).log; exit 1; }
  tail -1 gpurun_out/tests_$(basename $lib).log
done
for rep in 1 2; do for b in 1024 1; do for lib in byzantine-agreement_amd/ba_amd/libba_hip.so abx/libba_w1.so abx/libba_w2.so; do
  echo "lib=$lib batch=$b rep=$rep" >> gpurun_out/ab.log
  BA_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 300 >> gpurun_out/ab.log 2>&1 || exit 1
done; done; done
grep -E "^lib|us_per_call" gpurun_out/ab.log | sed -E 's/.*"us_per_call": ([0-9.]+).*/  \1 us/' | paste - -
