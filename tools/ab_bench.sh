# bench A/B of libraries on one lease, A B A B ...: bash tools/ab_bench.sh out.log lib1 lib2 ...
set -o pipefail
out=$1; shift
for r in 1 2 3; do for lib in "$@"; do
  BA_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-profile 2>/dev/null | grep '^{"metric"' | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$lib', 'rep', $r, 'value', round(d['value']/1e10,4), 'ev_ms', d['ms_per_step_gpu_events'], 'single', round(d['value_single_stream']/1e10,4), 'single_ms', d['ms_per_step_single_stream_gpu_events'], 'sclk', round(d['sclk_mhz_timed']))" | tee -a $out || exit 1
done; done
