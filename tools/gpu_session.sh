#!/bin/bash
# GPU-box session: every GPU step has its own time limit; a fault, abort or
# timeout ends the session (no retries).  Logs land in gpurun_out/.
# usage: tools/gpu_session.sh [tests] [smoke] [bench] [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
STAGES="${*:-tests smoke bench prof}"
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }  # 1 = ordinary test failure
for s in $STAGES; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?; fatal $rc && exit $rc ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python -u bench.py --steps 20 --warmup 3 || exit $? ;;
    bench_levels) run bench_levels 600 python -u bench.py --steps 20 --warmup 3 --engine levels --no-cpu || exit $? ;;
    bench_fused) run bench_fused 600 python -u bench.py --steps 20 --warmup 3 --engine fused --no-cpu || exit $? ;;
    prof) (cd /tmp && export TMPDIR=/tmp && run_dir="$ROOT/gpurun_out/prof" && mkdir -p "$run_dir" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$run_dir" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-profile > "$ROOT/gpurun_out/prof.log" 2>&1); rc=$?
          echo "prof rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
echo "session done"
