#!/bin/bash
# A/B of two builds of libba_hip.so on one box (BA_HIP_LIB selects the library):
# the bench (two steps in flight and one at a time), config 3, config 5, and a
# rocprofv3 kernel-stats pass per library; runs alternate A, B, A, B.
# usage: tools/ab_libs.sh <reps> <lib> [<lib> ...]   (tags A, B, C, ... in that order)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
REPS=$1; shift; LIBS=("$@"); TAGS=(A B C D E F)
mkdir -p gpurun_out/ab
for r in $(seq 1 $REPS); do
  for i in "${!LIBS[@]}"; do
    tag=${TAGS[$i]}; lib=${LIBS[$i]}
    timeout -k 10 300 env BA_HIP_LIB=$ROOT/$lib python -u bench.py --steps 20 --warmup 3 --no-cpu \
      > gpurun_out/ab/bench_${tag}_$r.log 2>&1 || { echo "bench $tag $r failed"; exit 1; }
    timeout -k 10 300 env BA_HIP_LIB=$ROOT/$lib python -u tools/run_configs.py --only 3,5 \
      > gpurun_out/ab/configs_${tag}_$r.log 2>&1 || { echo "configs $tag $r failed"; exit 1; }
    python3 - "$tag" "$r" <<'PY'
import json, sys
tag, r = sys.argv[1], sys.argv[2]
b = json.loads(open(f"gpurun_out/ab/bench_{tag}_{r}.log").read().strip().splitlines()[-1])
print(tag, r, "value %.4g single %.4g single_ms %.4f" % (b["value"], b["value_single_stream"], b["ms_per_step_single_stream_gpu_events"]))
for ln in open(f"gpurun_out/ab/configs_{tag}_{r}.log"):
    if ln.startswith("{"):
        c = json.loads(ln)
        print(tag, r, "config", c["config"], {k: "%.4g" % v for k, v in c.items() if "per_s" in k and v})
PY
  done
done
for i in "${!LIBS[@]}"; do
  tag=${TAGS[$i]}; lib=${LIBS[$i]}
  (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/ab/prof_$tag" && \
   timeout -k 10 300 env BA_HIP_LIB=$ROOT/$lib rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$ROOT/gpurun_out/ab/prof_$tag" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 \
     --warm-s 0.3 --no-cpu --no-profile --streams 1 > "$ROOT/gpurun_out/ab/prof_$tag.log" 2>&1) || { echo "prof $tag failed"; exit 1; }
  python3 -c "import csv,sys; [print('$tag', r['Name'][:40], r['Calls'], r['AverageNs']) for r in csv.DictReader(open('gpurun_out/ab/prof_$tag/run_kernel_stats.csv')) if 'k_om3w' in r['Name']]"
done
echo "ab done"
