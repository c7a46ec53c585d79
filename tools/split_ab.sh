set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "split_halves or om3_wave_block" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_split.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sp in 0 2 3; do
    timeout -k 10 300 env BA_WAVE_SPLIT=$sp python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_split${sp}_$r.log 2>&1 || exit 1
    python3 -c "
import json
b=json.loads(open('gpurun_out/bench_split${sp}_$r.log').read().strip().splitlines()[-1])
print('split=$sp rep=$r value %.4g single %.4g single_ms %.4f kernels %s' % (b['value'], b['value_single_stream'], b['ms_per_step_single_stream_gpu_events'], b.get('kernels_ms')))"
  done
done
for sp in 0 2 3; do
  (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/prof_split$sp" && \
   timeout -k 10 300 env BA_WAVE_SPLIT=$sp rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$ROOT/gpurun_out/prof_split$sp" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 \
     --warm-s 0.3 --no-cpu --no-profile --streams 1 > "$ROOT/gpurun_out/prof_split$sp.log" 2>&1) || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_split$sp/run_kernel_stats.csv')):
    if 'k_om3' in r['Name']: print('split=$sp', r['Name'][:30], r['Calls'], r['AverageNs'])"
done
