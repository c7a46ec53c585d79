#!/bin/bash
# GPU-box session: every GPU step has its own time limit; a fault, abort or
# timeout ends the session (no retries).  Logs land in gpurun_out/.
# usage: tools/gpu_session.sh [stage ...]
#   tests smoke bench bench2 bench_levels bench_fused prof prof1 pmc philox configs sched
#   (prof: the default bench command, two steps in flight, so each k_om3w launch
#   spans ~2x its own time; prof1: --streams 1, the launch time the roofline uses)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
STAGES="${*:-tests smoke bench prof}"
# heartbeat: a step that prints nothing for minutes (a multi-rank launch importing
# torch on a fresh box) must not look hung
(while true; do date +%T >> gpurun_out/heartbeat.txt; sleep 30; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }  # 1 = ordinary test failure
BENCH_PMC="$ROOT/bench.py --steps 3 --warmup 1 --warm-s 0 --no-cpu --no-profile --streams 1"
pmc_pass() {  # name counters...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv \
     -d "$ROOT/gpurun_out/pmc" -o "$name" -- python3 $BENCH_PMC > "$ROOT/gpurun_out/pmc_$name.log" 2>&1)
  local rc=$?; echo "pmc $name rc=$rc" | tee -a gpurun_out/steps.log; return $rc
}
for s in $STAGES; do
  case $s in
    tests) run pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?; fatal $rc && exit $rc ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 600 python -u bench.py --steps 20 --warmup 3 || exit $? ;;
    bench2) run bench2 600 env BA_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 20 --warmup 3 --cpu-budget-s 4 || exit $? ;;
    benchreps) for r in 1 2 3; do run bench_rep$r 300 python -u bench.py --steps 20 --warmup 5 --no-cpu || exit $?; done ;;
    configs2) run configs_l2 600 python -u tools/run_configs.py --only 5 --split-level 2 || exit $? ;;
    bench_levels) run bench_levels 600 python -u bench.py --steps 20 --warmup 3 --engine levels --no-cpu || exit $? ;;
    bench_fused) run bench_fused 600 python -u bench.py --steps 20 --warmup 3 --engine fused --no-cpu || exit $? ;;
    philox) run philox 120 ./tools/philox_bench || exit $? ;;
    lab) run lab 300 ./tools/om3_lab || exit $? ;;
    prof) (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/prof" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 2 --warm-s 0.3 --no-cpu --no-profile > "$ROOT/gpurun_out/prof.log" 2>&1); rc=$?
          echo "prof rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc ;;
    prof1) (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/prof1" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof1" -o run -- \
             python3 "$ROOT/bench.py" --steps 10 --warmup 2 --warm-s 0.3 --no-cpu --no-profile --streams 1 > "$ROOT/gpurun_out/prof1.log" 2>&1); rc=$?
          echo "prof1 rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/prof1.log; [ $rc -eq 0 ] || exit $rc ;;
    pmc) pmc_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit $?
         pmc_pass fetch FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
         pmc_pass write WRITE_SIZE || exit $?
         pmc_pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit $?
         python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_summary.json \
           --workload "bench.py default: n=10 m=3, 1048576 trials/step" --config 10,3,1048576,auto,k_om3w > gpurun_out/pmc_summary.log 2>&1 ;;
    sched) for m in default spin yield blocking default spin; do
             run sched_$m 300 python -u tools/host_overhead.py --sched $m || exit $?
             cat gpurun_out/sched_$m.log >> gpurun_out/sched_all.jsonl
           done ;;
    configs) run configs 600 python -u tools/run_configs.py || exit $? ;;
    configs1) run configs1 600 python -u tools/run_configs.py --only 1,3,4,5 || exit $? ;;
    c5) run c5_1024 300 python -u tools/config5_prof.py --batch 1024 --split || exit $?
        run c5_1 300 python -u tools/config5_prof.py --batch 1 --reps 500 --split || exit $? ;;
    multirank) run pytest_multirank 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_dist.py -m gpu -v --timeout 420 --timeout-method thread; rc=$?; fatal $rc && exit $rc ;;
    mt) run pytest_mt 300 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_fullsize.py -m gpu -v -k "mt or table or config1" --timeout 200 --timeout-method thread; rc=$?; fatal $rc && exit $rc
        run config1 300 python -u tools/run_configs.py --only 1 || exit $? ;;
    c1) for nn in 4 10; do run config1_n$nn 200 python -u tools/config1_prof.py --n $nn || exit $?; done ;;
    c1ab) for nn in 4 10; do run config1_r05_n$nn 200 env BA_HIP_LIB=$ROOT/labbuild/mt_r05.so python -u tools/config1_prof.py --n $nn || exit $?
          run config1_cur_n$nn 200 python -u tools/config1_prof.py --n $nn || exit $?; done ;;
    c1prof) for nn in 4 10; do
          (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/c1prof_$nn" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/c1prof_$nn" -o run -- \
             python3 "$ROOT/tools/config1_prof.py" --n $nn > "$ROOT/gpurun_out/c1prof_$nn.log" 2>&1); rc=$?
          echo "c1prof $nn rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc; done ;;
    c1pmc) for nn in 4 10; do
         C1="$ROOT/tools/config1_prof.py --n $nn --reps 3"
         # C1PMC_TAG / BA_HIP_LIB (optional): the same passes over a lab library (round-5 kernel)
         for pass in "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
                     "lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                     "fetch:FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "write:WRITE_SIZE"; do
           name=${pass%%:*}; ctrs=${pass#*:}
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv \
              -d "$ROOT/gpurun_out/c1pmc${C1PMC_TAG:-}_$nn" -o "$name" -- python3 $C1 > "$ROOT/gpurun_out/c1pmc${C1PMC_TAG:-}_${nn}_$name.log" 2>&1)
           rc=$?; echo "c1pmc $nn $name rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc
         done
         python3 tools/pmc_summary.py gpurun_out/c1pmc${C1PMC_TAG:-}_$nn gpurun_out/c1pmc${C1PMC_TAG:-}_${nn}_summary.json \
           --workload "tools/config1_prof.py --n $nn: ba.py-exact OM(1), 1048576 trials" \
           --config $nn,1,1048576,mt_table${C1PMC_TAG:-},k_mt_table > gpurun_out/c1pmc${C1PMC_TAG:-}_${nn}_summary.log 2>&1
       done ;;
    c1var) for lib in $C1LIBS; do
             run mttest_$(basename $lib .so) 200 env BA_HIP_LIB=$ROOT/$lib python -u -m pytest tests/test_gpu_mt.py -m gpu -q --timeout 100 --timeout-method thread || exit $?
           done
           for rep in 1 2; do for nn in 4 10; do for lib in $C1LIBS; do
             echo "lib=$lib n=$nn rep=$rep $(BA_HIP_LIB=$ROOT/$lib timeout -k 10 120 python tools/config1_prof.py --n $nn 2>/dev/null | grep '^{')" >> gpurun_out/c1var.log || exit $?
           done; done; done ;;
    bank) for lib in $BANKLIBS; do
            nm=$(basename $lib .so)
            (cd /tmp && export TMPDIR=/tmp BA_HIP_LIB=$ROOT/$lib && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv \
               -d "$ROOT/gpurun_out/bank_$nm" -o pmc -- python3 $ROOT/tools/om3w_launch.py > "$ROOT/gpurun_out/bank_$nm.log" 2>&1); rc=$?
            echo "bank $nm rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc
            python3 tools/pmc_summary.py gpurun_out/bank_$nm gpurun_out/bank_${nm}_summary.json --workload "bench.py --streams 1 with $lib" > /dev/null 2>&1
          done
          [ -n "${BANKBENCH:-}" ] && for rep in 1 2; do for lib in $BANKLIBS; do
            echo "lib=$lib rep=$rep $(BA_HIP_LIB=$ROOT/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-profile 2>/dev/null | grep '^{')" >> gpurun_out/bank_bench.log || exit $?
          done; done; true ;;
    om4ab) for lib in $OM4LIBS; do
             run c3test_$(basename $lib .so) 300 env BA_HIP_LIB=$ROOT/$lib python -u -m pytest tests/test_gpu.py tests/test_gpu_fullsize.py -m gpu -q -k "om4 or wave4 or config3 or depth4 or m4" --timeout 200 --timeout-method thread || exit $?
           done
           for rep in 1 2; do for lib in $OM4LIBS; do
             echo "lib=$lib rep=$rep $(BA_HIP_LIB=$ROOT/$lib timeout -k 10 200 python tools/config3_prof.py --mode staged,inkernel --reps 10 2>/dev/null | grep '^{' | python3 -c 'import sys,json; print(" ".join("%s=%.4g" % (d["mode"], d["trials_per_s"]) for d in map(json.loads, sys.stdin)))')" >> gpurun_out/om4ab.log || exit $?
           done; done ;;
    mcab) for rep in 1 2; do for lib in $MCLIBS; do
            echo "lib=$lib rep=$rep" >> gpurun_out/mcab.log
            BA_HIP_LIB=$ROOT/$lib timeout -k 10 200 python tools/run_configs.py --only 5 2>/dev/null | grep '^{' >> gpurun_out/mcab.log || exit $?
          done; done ;;
    handoff) run pytest_handoff 300 python -u -m pytest tests/test_gpu_handoff.py -m gpu -v --timeout 120 --timeout-method thread; rc=$?; fatal $rc && exit $rc ;;
    casc) run pytest_casc 600 python -u -m pytest tests/test_gpu_cascade.py tests/test_dist.py -m gpu -v --timeout 200 --timeout-method thread; rc=$?; fatal $rc && exit $rc ;;
    c5prof) for b in 1024 1; do
          (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/c5prof_$b" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/c5prof_$b" -o run -- \
             python3 "$ROOT/tools/config5_prof.py" --batch $b --reps 300 --no-inflight > "$ROOT/gpurun_out/c5prof_$b.log" 2>&1); rc=$?
          echo "c5prof $b rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc; done ;;
    c3) run config3 300 python -u tools/config3_prof.py || exit $? ;;
    c3prof) for md in staged inkernel; do
          (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out/c3prof_$md" && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/c3prof_$md" -o run -- \
             python3 "$ROOT/tools/config3_prof.py" --mode $md --reps 20 > "$ROOT/gpurun_out/c3prof_$md.log" 2>&1); rc=$?
          echo "c3prof $md rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc; done ;;
    c3pmc) for md in staged inkernel; do
         C3="$ROOT/tools/config3_prof.py --mode $md --reps 3"
         for pass in "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
                     "lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                     "fetch:FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "write:WRITE_SIZE"; do
           name=${pass%%:*}; ctrs=${pass#*:}
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv \
              -d "$ROOT/gpurun_out/c3pmc_$md" -o "$name" -- python3 $C3 > "$ROOT/gpurun_out/c3pmc_${md}_$name.log" 2>&1)
           rc=$?; echo "c3pmc $md $name rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc
         done
         python3 tools/pmc_summary.py gpurun_out/c3pmc_$md gpurun_out/c3pmc_${md}_summary.json \
           --workload "tools/config3_prof.py --mode $md: n=13 m=4, 8388608 trials per launch" \
           --config 13,4,8388608,auto/$md,k_om4w > gpurun_out/c3pmc_${md}_summary.log 2>&1
       done ;;
    c5pmc) C5="$ROOT/tools/config5_prof.py --batch 1024 --reps 50"
         for pass in "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
                     "lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                     "fetch:FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "write:WRITE_SIZE"; do
           name=${pass%%:*}; ctrs=${pass#*:}
           (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv \
              -d "$ROOT/gpurun_out/c5pmc" -o "$name" -- python3 $C5 > "$ROOT/gpurun_out/c5pmc_$name.log" 2>&1)
           rc=$?; echo "c5pmc $name rc=$rc" | tee -a gpurun_out/steps.log; [ $rc -eq 0 ] || exit $rc
         done ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
echo "session done"
