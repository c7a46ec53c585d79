#!/bin/bash
# LEVELS engine (level-synchronous relay / majority kernels, the north star's
# original design) on the bench workload: rocprofv3 kernel stats plus PMC
# HBM traffic per kernel, combined by tools/kernel_hbm.py into achieved GB/s
# per kernel against the MI355X HBM peak.  Output: gpurun_out/levels${TAG}_*.
# usage: [TAG=_n16m5 WL="--n 16 --m 5 --batch 1024" CONFIG=16,5,1024,levels,k_leaf] tools/levels_profile.sh
set -u
TAG=${TAG:-}
WL=${WL:-}
CONFIG=${CONFIG:-10,3,1048576,levels,k_leaf}  # n,m,batch,engine,kernel (bench.py traffic lookup)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/levels${TAG}_prof gpurun_out/levels${TAG}_pmc
CMD="$ROOT/bench.py --steps 5 --warmup 1 --no-cpu --no-profile --engine levels --inputs-in-kernel $WL"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$ROOT/gpurun_out/levels${TAG}_prof" -o run -- python3 $CMD > "$ROOT/gpurun_out/levels${TAG}_prof.log" 2>&1) || exit $?
for pass in "FETCH_SIZE" "WRITE_SIZE"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv \
     -d "$ROOT/gpurun_out/levels${TAG}_pmc" -o "$pass" -- python3 $CMD > "$ROOT/gpurun_out/levels${TAG}_pmc_$pass.log" 2>&1) || exit $?
done
python3 tools/pmc_summary.py gpurun_out/levels${TAG}_pmc gpurun_out/levels${TAG}_pmc_summary.json \
  --workload "bench.py --engine levels $WL" --config "$CONFIG" > gpurun_out/levels${TAG}_pmc_summary.log 2>&1
python3 tools/kernel_hbm.py gpurun_out/levels${TAG}_prof/run_kernel_stats.csv gpurun_out/levels${TAG}_pmc_summary.json \
  > gpurun_out/levels${TAG}_kernel_hbm.json
cat gpurun_out/levels${TAG}_kernel_hbm.json
