# Latency-mode A/B (BA_CASC_LAT=1/0) for n=16 m=5 after the cascade GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cascade.py > gpurun_out/casc.log 2>&1 || { tail -40 gpurun_out/casc.log; exit 1; }
tail -2 gpurun_out/casc.log
for rep in 1 2; do for b in 1 64 128 256 512; do for lat in 1 0; do
  echo "lat=$lat batch=$b rep=$rep" >> gpurun_out/ab.log
  BA_CASC_LAT=$lat timeout -k 10 120 python tools/config5_prof.py --batch $b --reps 300 >> gpurun_out/ab.log 2>&1 || exit 1
done; done; done
grep -E "^lat|us_per_call" gpurun_out/ab.log | sed -E 's/.*"us_per_call": ([0-9.]+).*/  \1 us/' | paste - -
