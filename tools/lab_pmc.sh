#!/bin/bash
# PMC passes over a lab binary (one rocprofv3 run per counter group, each under
# its own time limit), summarised per kernel by tools/pmc_summary.py.
# usage: tools/lab_pmc.sh <binary> [args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
BIN=$(readlink -f "$1"); shift
mkdir -p gpurun_out/labpmc
pass() {  # name counters...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv \
     -d "$ROOT/gpurun_out/labpmc" -o "$name" -- "$BIN" $ARGS > "$ROOT/gpurun_out/labpmc_$name.log" 2>&1)
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
ARGS="$*"
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit $?
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
python3 tools/pmc_summary.py gpurun_out/labpmc gpurun_out/labpmc_summary.json > gpurun_out/labpmc_summary.log 2>&1
cat gpurun_out/labpmc_summary.log
