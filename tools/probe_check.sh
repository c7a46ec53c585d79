# Clock-probe check: the probe's GPU test, then three bench runs' clock fields.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_probe.py -m gpu > gpurun_out/probe.log 2>&1 || { tail -30 gpurun_out/probe.log; exit 1; }
tail -2 gpurun_out/probe.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --cpu-budget-s 0 > gpurun_out/bench$i.log 2>&1 || exit 1
  grep "^{" gpurun_out/bench$i.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['value'], d['sclk_mhz_timed'], d['clock']['per_xcd_mhz'])"
done
