set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_cascade.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_casc.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_casc.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in ab/libba_r03i.so ab/libba_cascpre.so; do
    timeout -k 10 300 env BA_HIP_LIB=$(pwd)/$lib python -u tools/run_configs.py --only 5 > gpurun_out/c5_$(basename $lib .so)_$r.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/c5_$(basename $lib .so)_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib', $r, 'lat_stream %.4f ms' % d['latency_one_instance_ms_stream'], 'stream %.4g' % d['throughput_instances_per_s_stream'], 'stream2 %.4g' % d['throughput_instances_per_s_stream2'], 'graph_lat %.4f' % d['latency_one_instance_ms_graph'])"
  done
done
